#!/usr/bin/env python3
"""Experiment: output-layout cost on c4.  Times decode / encode with the implicit slot layout (16-B
region stores) against explicit destinations packed back to back (per-lane dword stores), and the
per-string symbols' call latency.  Prints JSON lines."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))


def main():
    import torch

    from bench_configs import packed_huffman, timed
    from h2o_amd import codec, synth

    torch.cuda.set_device(0)
    b = synth.make_batch_torch("c4", seed=7)
    n, P = b["n"], int(b["total"])
    off32 = b["off"].to(torch.int32)
    lens = (b["off"][1:] - b["off"][:-1])
    huff, h_off, n_ok, H, P_ok = packed_huffman(torch, codec, b)
    d_len = torch.empty(n_ok, dtype=torch.int32, device="cuda")
    d_st = torch.empty(n_ok, dtype=torch.uint8, device="cuda")
    d_out = torch.empty(codec.decode_slot_size(H), dtype=torch.uint8, device="cuda")
    codec.decode_batch(huff, h_off, n_ok, out=d_out, out_len=d_len, status=d_st, in_size=H)
    # packed destinations from the decoded lengths
    pl = torch.where(d_len >= 0, d_len, torch.zeros_like(d_len)).to(torch.int64)
    p_off = torch.zeros(n_ok + 1, dtype=torch.int64, device="cuda")
    p_off[1:] = torch.cumsum(pl, 0)
    p_out = torch.empty(int(p_off[-1].item()) + 64, dtype=torch.uint8, device="cuda")
    h_start = h_off[:-1].contiguous()
    h_len = (h_off[1:] - h_off[:-1]).contiguous()
    p_off32 = p_off[:-1].to(torch.int32).contiguous()
    res = {}
    res["dec_region_ms"] = timed(torch, lambda: codec.decode_batch(huff, h_off, n_ok, out=d_out, out_len=d_len,
                                                                  status=d_st, in_size=H))
    res["dec_pairs_slots_ms"] = timed(torch, lambda: codec.decode_batch(huff, h_start, n_ok, in_len=h_len, out=d_out,
                                                                       out_len=d_len, status=d_st, in_size=H))
    res["dec_packed_dst_ms"] = timed(torch, lambda: codec.decode_batch(huff, h_start, n_ok, in_len=h_len, out=p_out,
                                                                      out_off=p_off32, out_len=d_len, status=d_st,
                                                                      in_size=H))
    e_out = torch.empty(P + 16, dtype=torch.uint8, device="cuda")
    e_len = torch.empty(n, dtype=torch.int32, device="cuda")
    e_st = torch.empty(n, dtype=torch.uint8, device="cuda")
    codec.encode_batch(b["data"], off32, n, out=e_out, out_len=e_len, status=e_st, in_size=P)
    el = torch.where(e_len >= 0, e_len, torch.zeros_like(e_len)).to(torch.int64)
    q_off = torch.zeros(n + 1, dtype=torch.int64, device="cuda")
    q_off[1:] = torch.cumsum(el, 0)
    q_out = torch.empty(P + 64, dtype=torch.uint8, device="cuda")
    q_off32 = q_off[:-1].to(torch.int32).contiguous()
    starts = off32[:-1].contiguous()
    l32 = lens.to(torch.int32).contiguous()
    res["enc_region_ms"] = timed(torch, lambda: codec.encode_batch(b["data"], off32, n, out=e_out, out_len=e_len,
                                                                  status=e_st, in_size=P))
    res["enc_packed_dst_ms"] = timed(torch, lambda: codec.encode_batch(b["data"], starts, n, in_len=l32, out=q_out,
                                                                      out_off=q_off32, out_len=e_len, status=e_st,
                                                                      in_size=P))
    pk_out = torch.empty(codec.decode_slot_size(H), dtype=torch.uint8, device="cuda")
    pk_off = torch.empty(n_ok + 1, dtype=torch.int32, device="cuda")
    res["dec_packed_ms"] = timed(torch, lambda: codec.decode_batch_packed(huff, h_off, n_ok, out=pk_out, out_off=pk_off,
                                                                         out_len=d_len, status=d_st, in_size=H))
    pe_off = torch.empty(n + 1, dtype=torch.int32, device="cuda")
    res["enc_packed_ms"] = timed(torch, lambda: codec.encode_batch_packed(b["data"], off32, n, out=q_out, out_off=pe_off,
                                                                         out_len=e_len, status=e_st, in_size=P))
    print(json.dumps({k: round(v, 4) for k, v in res.items()}), flush=True)
    # per-string symbol latency
    s = b"www.example.com" * 3
    hs = codec.encode_huffman(s)
    for name, fn in (("encode_huffman", lambda: codec.encode_huffman(s)),
                     ("decode_huffman", lambda: codec.decode_huffman(hs, False))):
        for _ in range(50):
            fn()
        t = []
        for _ in range(2000):
            t0 = time.perf_counter()
            fn()
            t.append(time.perf_counter() - t0)
        t.sort()
        print(json.dumps({"per_string": name, "median_us": round(t[len(t) // 2] * 1e6, 2),
                          "p99_us": round(t[int(len(t) * 0.99)] * 1e6, 2)}), flush=True)


if __name__ == "__main__":
    main()
