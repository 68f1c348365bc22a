#!/usr/bin/env python3
"""A/B of the decode kernel choice in one process (hhuff_set_decode_kernel): for each config the Huffman wire of
the config's batch is decoded with mode A and mode B in interleaved rounds (HIP events on the launch stream,
median), outputs checked equal.  usage: tools/dec_mode_ab.py [A B [configs...]]   (default 0 1 c3 c5)"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))


def main():
    import torch

    from bench_configs import packed_huffman
    from h2o_amd import codec, dist as hd, synth

    a, b = (int(x) for x in sys.argv[1:3]) if len(sys.argv) > 2 else (0, 1)
    cfgs = sys.argv[3:] or ["c3", "c5"]
    torch.cuda.set_device(0)
    for cfg in cfgs:
        bt = synth.make_batch_torch(cfg, seed=1000)
        huff, h_off, m, H, P_ok = packed_huffman(torch, codec, bt)
        ok = None
        names = None if os.environ.get("NO_NAMES") else hd.bool_to_bits(torch.rand(m, device="cuda") < 0.3)
        outs = {}
        for mode in (a, b):
            out = torch.empty(codec.decode_slot_size(H), dtype=torch.uint8, device="cuda")
            ol = torch.empty(m, dtype=torch.int32, device="cuda")
            st = torch.empty(m, dtype=torch.uint8, device="cuda")
            outs[mode] = (out, ol, st)
        t = {a: [], b: []}
        for r in range(24):
            for mode in (a, b) if r % 2 == 0 else (b, a):
                codec.set_decode_kernel(mode)
                out, ol, st = outs[mode]
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                codec.decode_batch(huff, h_off, m, is_name_bits=names, out=out, out_len=ol, status=st, in_size=H)
                e1.record()
                torch.cuda.synchronize()
                if r >= 4:
                    t[mode].append(e0.elapsed_time(e1))
        la, lb = outs[a][1], outs[b][1]
        ok = bool((la == lb).all()) and bool((outs[a][2] == outs[b][2]).all())
        slots = (h_off[:-1].to(torch.int64) * 8) // 5
        keep = la.to(torch.int64).clamp(min=0)
        same = ok and bool((hd.compact_results(outs[a][0], slots, la)[1] == hd.compact_results(outs[b][0], slots, lb)[1]).all())
        med = {k: sorted(v)[len(v) // 2] for k, v in t.items()}
        B = H + P_ok + 9 * m + 4 + (m + 7) // 8
        print(json.dumps({"lib": os.path.basename(codec.LIB_PATH), "names": names is not None, "config": cfg, "strings": m, "huffman_bytes": H, "mode_a": a, "mode_b": b,
                          "ms_a": round(med[a], 4), "ms_b": round(med[b], 4),
                          "frac_a": round(B / (med[a] * 1e-3) / 8e12, 4), "frac_b": round(B / (med[b] * 1e-3) / 8e12, 4),
                          "equal": same, "decoded": int((keep > 0).sum())}), flush=True)
    codec.set_decode_kernel(1)


if __name__ == "__main__":
    main()
