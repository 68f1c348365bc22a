#!/usr/bin/env python3
"""Secondary measurements for the other BASELINE.json configurations (the headline is bench.py, config 4):
  c2  1M strings mean 32 B, decode only
  c3  1M strings Zipf 8..512 B, encode + decode round trip, P / (t_enc + t_dec)
  c5  512K QPACK values mean 512 B (cookie/URI charset), encode only with flatten_string(prefix 7) framing
  hpenc[N]   f4 encode half: HTTP/2 responses of N connections (default 65536) flattened with their encoder
             tables (hhuff_hpack_flatten_responses)
  reqenc[N]  the same for the client's requests (h2o_hpack_flatten_request)
  blocks[N]  f4: N synthetic HPACK connections (default 65536), header blocks decoded with a dynamic
      table per connection; CPU baselines: the reference (1 thread) and the restatement (16 threads)
  lit 16M c4 strings framed as HPACK literals (h2o_hpack_encode_string), then decoded as literals
      (decode_string: header integer, Huffman or raw + validation); round trip checked on the device
Prints one JSON line per config.  Device-resident, HIP-event timing on the launch stream."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
GIB = float(1 << 30)


def timed_b2b(torch, fn, steps=20, warmup=3, reps=5):
    """device time per call with `steps` calls enqueued back to back between one event pair (the median of `reps`
    such runs): a server's sustained rate, without the gap an event pair around every call adds (2-4 us, which is
    a tenth of a c2 call)"""
    for _ in range(warmup):
        fn()
    t = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        a.record()
        for _ in range(steps):
            fn()
        b.record()
        torch.cuda.synchronize()
        t.append(a.elapsed_time(b) / steps)
    t.sort()
    return t[len(t) // 2]


def timed(torch, fn, steps=20, warmup=3):
    for _ in range(warmup):
        fn()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
    torch.cuda.synchronize()
    for a, b in ev:
        a.record()
        fn()
        b.record()
    torch.cuda.synchronize()
    t = sorted(a.elapsed_time(b) for a, b in ev)
    return t[len(t) // 2]


def packed_huffman(torch, codec, b):
    """encode once, keep the compressible strings packed contiguously (the wire)"""
    n, P = b["n"], int(b["total"])
    off32 = b["off"].to(torch.int32)
    lens = b["off"][1:] - b["off"][:-1]
    _, el, _ = codec.encode_batch(b["data"], off32, n, in_size=P)
    idx = torch.nonzero(el != -1).squeeze(1)
    hl = el[idx].to(torch.int64)
    h_off = torch.zeros(idx.numel() + 1, dtype=torch.int64, device="cuda")
    h_off[1:] = torch.cumsum(hl, 0)
    H = int(h_off[-1].item())
    huff = torch.empty(H + 16, dtype=torch.uint8, device="cuda")
    codec.encode_batch(b["data"], off32[idx].contiguous(), idx.numel(), in_len=lens[idx].to(torch.int32).contiguous(),
                       out=huff, out_off=h_off[:-1].to(torch.int32).contiguous(), in_size=P)
    return huff, h_off.to(torch.int32), int(idx.numel()), H, int(lens[idx].sum().item())


def literals_line(torch, codec, synth):
    b = synth.make_batch_torch("c4", seed=9)
    n, P = b["n"], int(b["total"])
    off32 = b["off"].to(torch.int32)
    f_out = torch.empty(P + 11 * n + 16, dtype=torch.uint8, device="cuda")
    f_len = torch.empty(n, dtype=torch.int32, device="cuda")
    codec.flatten_batch(b["data"], off32, n, 7, out=f_out, out_len=f_len, in_size=P)  # h2o_hpack_encode_string
    # pack the literals back to back, as they sit in header blocks
    fl = f_len.to(torch.int64)
    dense_off = torch.zeros(n + 1, dtype=torch.int64, device="cuda")
    dense_off[1:] = torch.cumsum(fl, 0)
    W = int(dense_off[-1].item())
    src = torch.repeat_interleave(b["off"][:-1] + 11 * torch.arange(n, device="cuda"), fl)
    src = src + torch.arange(W, device="cuda") - torch.repeat_interleave(dense_off[:-1], fl)
    wire = torch.empty(W + 16, dtype=torch.uint8, device="cuda")
    wire[:W] = f_out[src]
    f_out = wire
    lit_off = dense_off[:-1].to(torch.int32)
    lit_end = dense_off[1:].to(torch.int32)
    names = b["is_name_bits"]
    out = torch.empty((W * 8) // 5 + 16, dtype=torch.uint8, device="cuda")
    res = {}

    def run():
        res["r"] = codec.decode_literals(f_out, lit_off, lit_end, n, 7, is_name_bits=names, out=out, in_size=W)

    t = timed(torch, run)
    o, ol, po, cons, st = res["r"]
    ok = ol != -1
    # round trip on the device: every successfully decoded literal reproduces its plain string
    lens = (b["off"][1:] - b["off"][:-1])
    slot = (po.to(torch.int64) * 8) // 5
    seg = torch.repeat_interleave(torch.arange(n, device="cuda"), lens)
    pos = torch.arange(P, device="cuda") - torch.repeat_interleave(b["off"][:-1], lens)
    got = o[torch.repeat_interleave(slot, lens) + pos]
    good_str = ok & (ol.to(torch.int64) == lens)
    match = bool((got[good_str[seg]] == b["data"][good_str[seg]]).all())
    return {"config": "lit", "literals": n, "plain_bytes": P, "wire_bytes": int(f_len.to(torch.int64).sum().item()),
            "decode_literals_ms": round(t, 4), "decode_literals_gibps": round(P / GIB / (t * 1e-3), 2),
            "ok_literals": int(ok.sum().item()), "round_trip_match": match,
            "consumed_matches_wire": bool((cons[ok].to(torch.int64) == f_len[ok].to(torch.int64)).all())}


def blocks_line(torch, codec, nconn=65536):
    """f4: HPACK header blocks of synthetic browser-like connections (h2o_amd/hpack_synth.py, 1-8 requests
    each, 1 % adversarial), decoded with a dynamic table per connection; the CPU baselines run the same
    batch through the reference's h2o_hpack_decode_header (oracle/_ref, 1 thread) and the restatement
    (16 threads)"""
    import time

    from h2o_amd import hpack_synth as HS

    b = HS.make_connections(nconn, seed=5, adversarial_frac=0.01)
    dev = lambda a: torch.from_numpy(np.ascontiguousarray(a).copy()).cuda()  # noqa: E731
    d, bo, cf = dev(b["data"]), dev(b["blk_off"].view(np.int32)), dev(b["conn_first"].view(np.int32))
    # arena: 16 decoded bytes per block byte + 1 KiB (the browser-like blocks decode to ~3x their size);
    # codec.default_arena_off's worst case (every 4 block bytes an indexed copy of a whole table entry)
    # would put most blocks past the 4 GiB reach of the u32 field offsets at these connection counts
    L = np.diff(b["blk_off"].astype(np.int64))
    ao = dev(np.concatenate([[0], np.cumsum(16 * L + 1024)]).astype(np.int64))
    res = {}

    def run():
        res["r"] = codec.hpack_decode_blocks(d, bo, cf, 4096, arena_off=ao, in_size=int(b["data"].size))

    t = timed(torch, run, steps=10, warmup=2)

    def run_req():  # the same blocks through h2o_hpack_parse_request's rules (hhuff_hpack_parse_requests)
        res["q"] = codec.hpack_decode_blocks(d, bo, cf, 4096, arena_off=ao, in_size=int(b["data"].size), requests=True)

    tq = timed(torch, run_req, steps=10, warmup=2) if hasattr(codec.lib(), "hhuff_hpack_parse_requests") else float("nan")
    r = res["r"]
    nblk = len(b["blk_off"]) - 1
    nf = int(r["nfields"][:nblk].to(torch.int64).sum().item())
    out_bytes = int((r["name_len"].to(torch.int64) * 0).sum().item())
    ok = int((r["bstatus"][:nblk] == 0).sum().item())
    arena_fail = int((r["bstatus"][:nblk] == -300).sum().item())
    W = int(b["data"].size)
    line = {"config": "blocks", "connections": nconn, "blocks": nblk, "fields": nf, "block_bytes": W, "ok_blocks": ok,
            "arena_fail_blocks": arena_fail, "decode_ms": round(t, 4), "blocks_per_s": round(nblk / (t * 1e-3), 1),
            "fields_per_s": round(nf / (t * 1e-3), 1), "block_gibps": round(W / GIB / (t * 1e-3), 3),
            "parse_requests_ms": round(tq, 4), "parse_requests_blocks_per_s": round(nblk / (tq * 1e-3), 1)}
    del out_bytes
    try:
        sys.path.insert(0, ROOT)
        from oracle import oracle as O

        cpu = {}
        if O.ref_available():
            m = min(nconn, 4096)
            k = int(b["conn_first"][m])
            sub = (b["data"][:int(b["blk_off"][k])], b["blk_off"][:k + 1], b["conn_first"][:m + 1])
            t0 = time.perf_counter()
            O.ref().hpack_decode_blocks(*sub, 4096)
            dt = time.perf_counter() - t0
            cpu["reference_1thread_blocks_per_s"] = round(k / dt, 1)
            cpu["reference_1thread_gibps"] = round(int(sub[1][-1]) / GIB / dt, 4)
        threads = min(16, len(os.sched_getaffinity(0)))
        t0 = time.perf_counter()
        O.oracle().hpack_decode_blocks(b["data"], b["blk_off"], b["conn_first"], 4096, nthreads=threads)
        dt = time.perf_counter() - t0
        cpu["restatement_%dthreads_blocks_per_s" % threads] = round(nblk / dt, 1)
        line["cpu"] = cpu
    except Exception as e:  # the CPU baseline is a report, not a gate
        line["cpu_error"] = str(e)
    return line


def qpack_line(torch, codec, nconn=65536):
    """f4 (QPACK half): one decoder step of synthetic HTTP/3 connections (h2o_amd/qpack_synth.py: 1-4 requests
    each, encoder-stream inserts then field sections, 1 % adversarial) -- encoder streams one lane per
    connection, then sections one lane per section; the CPU baselines run the same step through the
    reference's h2o_qpack_decoder_handle_input + decode_header (oracle/_ref, 1 thread, first 4096
    connections) and the restatement (1 thread)"""
    import time

    from h2o_amd import qpack_synth as QS

    st = QS.make_session(nconn, steps=1, seed=9, adversarial_frac=0.01)[0]
    L = np.diff(st["sec_off"].astype(np.uint64))  # arena slice: 8/5 per literal byte, 64x per line byte
    ao_np = np.concatenate([[0], np.cumsum((L * 8) // 5 + L * np.uint64(64) + np.uint64(512))]).astype(np.uint64)
    dev = lambda a: torch.from_numpy(np.ascontiguousarray(a).copy()).cuda()  # noqa: E731
    u32 = lambda a: dev(np.asarray(a, np.uint32).view(np.int32))  # noqa: E731
    d, eo, el, so, cf = dev(st["data"]), u32(st["enc_off"]), u32(st["enc_len"]), u32(st["sec_off"]), u32(st["conn_first"])
    ao = dev(ao_np.view(np.int64))
    nsec = int(st["conn_first"][-1])
    scratch = torch.empty(int(codec.lib().hhuff_qpack_scratch_size(nconn, 4096)), dtype=torch.uint8, device="cuda")
    res = {}

    def run():
        res["r"] = codec.qpack_decode(d, eo, el, so, cf, nsec, 4096, 100, arena_off=ao, in_size=int(st["data"].size),
                                      scratch=scratch)

    t = timed(torch, run, steps=10, warmup=2)
    r = res["r"]
    nf = int(r["nfields"][:nsec].to(torch.int64).sum().item())
    W = int(st["data"].size)
    line = {"config": "qpack", "connections": nconn, "sections": nsec, "fields": nf, "input_bytes": W,
            "encoder_stream_bytes": int(st["enc_len"].sum()),
            "ok_sections": int((r["sstatus"][:nsec] == 0).sum().item()),
            "arena_short_sections": int((r["sstatus"][:nsec] == -300).sum().item()), "decode_ms": round(t, 4),
            "sections_per_s": round(nsec / (t * 1e-3), 1), "fields_per_s": round(nf / (t * 1e-3), 1),
            "input_gibps": round(W / GIB / (t * 1e-3), 3)}
    # the same step as HTTP/3 requests: h2o_qpack_parse_request per section (hhuff_qpack_parse_requests)
    sid = dev(np.arange(nsec, dtype=np.int64) * 4)

    def run_req():
        res["q"] = codec.qpack_decode(d, eo, el, so, cf, nsec, 4096, 100, arena_off=ao, in_size=int(st["data"].size),
                                      scratch=scratch, stream_id=sid)

    t_req = timed(torch, run_req, steps=10, warmup=2)
    q = res["q"]
    line.update(requests_ms=round(t_req, 4), requests_sections_per_s=round(nsec / (t_req * 1e-3), 1),
                ok_requests=int((q["sstatus"][:nsec] == 0).sum().item()),
                acks=int((q["req"][:nsec, 52] != 0).sum().item()))
    try:
        sys.path.insert(0, ROOT)
        from oracle import oracle as O

        cpu = {}
        m = min(nconn, 4096)
        k = int(st["conn_first"][m])
        sub = dict(data=st["data"], enc_off=st["enc_off"][:m], enc_len=st["enc_len"][:m], sec_off=st["sec_off"][:k + 1],
                   conn_first=st["conn_first"][:m + 1], arena_off=ao_np[:k + 1])
        for kind, lib in (("reference", O.ref() if O.ref_available() else None), ("restatement", O.oracle())):
            if lib is None:
                continue
            s = O.QpackSession(lib, m, 4096, 100)
            t0 = time.perf_counter()
            s.step(sub["data"], sub["enc_off"], sub["enc_len"], sub["sec_off"], sub["conn_first"], sub["arena_off"])
            dt = time.perf_counter() - t0
            s.close()
            cpu[kind + "_1thread_sections_per_s"] = round(k / dt, 1)
        line["cpu"] = cpu
    except Exception as e:  # the CPU baseline is a report, not a gate
        line["cpu_error"] = str(e)
    return line


def hpenc_line(torch, codec, nconn=65536, requests=False):
    """f4 encode half: HTTP/2 response header blocks (h2o_amd/hpenc_synth.py: 4,096 synthetic connections of 1-8
    responses tiled to nconn, 1 % edge cases) flattened as h2o_hpack_flatten_response / _trailers do, one encoder
    table per connection; the CPU baselines run the 4,096 distinct connections through the reference's
    h2o_hpack_flatten_response (oracle/_ref, 1 thread) and the restatement (1 thread).  requests=True: the
    client's requests instead (make_request_session, h2o_hpack_flatten_request)"""
    import time

    from h2o_amd import hpenc_synth as HE

    big = float(os.environ.get("HHUFF_HPENC_BIG", "0.001"))  # A/B knob: share of responses past max_frame_size
    base = (HE.make_request_session(4096, seed=13, big_frac=big) if requests else HE.make_session(4096, seed=13, big_frac=big))[0]
    b = HE.tile(base, max(1, nconn // 4096))
    dev = lambda a: torch.from_numpy(np.ascontiguousarray(a).copy()).cuda()  # noqa: E731
    d, hd, rs = dev(b["data"]), dev(b["hdr"].view(np.uint8)), dev(b["res"].view(np.uint8))
    cf, oo = dev(b["conn_first"].view(np.int32)), dev(b["out_off"].view(np.int64))
    nres, nhdr, nc = int(b["res"].size), int(b["hdr"].size), int(b["conn_first"].size - 1)
    out = torch.empty(int(b["out_off"][-1]), dtype=torch.uint8, device="cuda")
    scratch = torch.empty(int(codec.lib().hhuff_hpack_enc_scratch_size(nc)), dtype=torch.uint8, device="cuda")
    res = {}

    def run():
        res["r"] = codec.hpack_flatten_responses(d, hd, rs, cf, nres, oo, b["server_off"], b["server_len"],
                                                 in_size=int(b["data"].size), out=out, scratch=scratch)

    t = timed(torch, run, steps=10, warmup=2)
    r = res["r"]
    frame_bytes = int(r["out_len"][:nres].to(torch.int64).sum().item())
    field_bytes = int(b["hdr"]["name_len"].astype(np.int64).sum() + b["hdr"]["value_len"].astype(np.int64).sum())
    line = {"config": "reqenc" if requests else "hpenc", "connections": nc, ("requests" if requests else "responses"): nres, "fields": nhdr, "field_bytes": field_bytes,
            "frame_bytes": frame_bytes, ("ok_requests" if requests else "ok_responses"): int((r["rstatus"][:nres] == 0).sum().item()),
            "flatten_ms": round(t, 4), ("requests_per_s" if requests else "responses_per_s"): round(nres / (t * 1e-3), 1),
            "fields_per_s": round(nhdr / (t * 1e-3), 1), "field_gibps": round(field_bytes / GIB / (t * 1e-3), 3)}
    try:
        sys.path.insert(0, ROOT)
        from oracle import oracle as O

        cpu = {}
        n0 = int(base["res"].size)
        args = (base["data"], base["hdr"], base["res"], base["conn_first"], base["out_off"], base["server_off"],
                base["server_len"])
        for kind, lib in (("reference", O.ref() if O.ref_available() else None), ("restatement", O.oracle())):
            if lib is None:
                continue
            s = O.HpeSession(lib, 4096)
            t0 = time.perf_counter()
            s.step(*args)
            dt = time.perf_counter() - t0
            s.close()
            cpu[kind + ("_1thread_requests_per_s" if requests else "_1thread_responses_per_s")] = round(n0 / dt, 1)
        line["cpu"] = cpu
    except Exception as e:  # the CPU baseline is a report, not a gate
        line["cpu_error"] = str(e)
    return line


def responses_line(torch, codec, nconn=65536):
    """f4, client side: HTTP/2 response blocks as h2o's client receives them (h2o_amd/hpack_synth.py
    make_response_connections: 1-8 response heads per connection, a tenth of them trailers, 1 % adversarial)
    through h2o_hpack_parse_response's rules (hhuff_hpack_parse_responses); the CPU baseline runs 4,096 of the
    connections through the reference's h2o_hpack_parse_response (oracle/_ref, 1 thread)"""
    import time

    from h2o_amd import hpack_synth as HS

    b = HS.make_response_connections(nconn, seed=9, adversarial_frac=0.01, rule_frac=0.0, trailer_frac=0.1)
    dev = lambda a: torch.from_numpy(np.ascontiguousarray(a).copy()).cuda()  # noqa: E731
    d, bo, cf, tr = dev(b["data"]), dev(b["blk_off"].view(np.int32)), dev(b["conn_first"].view(np.int32)), dev(b["trailers"])
    L = np.diff(b["blk_off"].astype(np.int64))
    ao = dev(np.concatenate([[0], np.cumsum(16 * L + 1024)]).astype(np.int64))
    res = {}

    def run():
        res["r"] = codec.hpack_decode_blocks(d, bo, cf, 4096, arena_off=ao, in_size=int(b["data"].size), responses=True,
                                             trailers=tr)

    t = timed(torch, run, steps=10, warmup=2)
    r = res["r"]
    nblk = len(b["blk_off"]) - 1
    nf = int(r["nfields"][:nblk].to(torch.int64).sum().item())
    W = int(b["data"].size)
    line = {"config": "responses", "connections": nconn, "blocks": nblk, "trailer_blocks": int(b["trailers"].sum()),
            "fields": nf, "block_bytes": W, "ok_blocks": int((r["bstatus"][:nblk] == 0).sum().item()),
            "parse_responses_ms": round(t, 4), "blocks_per_s": round(nblk / (t * 1e-3), 1),
            "fields_per_s": round(nf / (t * 1e-3), 1), "block_gibps": round(W / GIB / (t * 1e-3), 3)}
    try:
        sys.path.insert(0, ROOT)
        from oracle import oracle as O

        if O.ref_available():
            m = min(nconn, 4096)
            k = int(b["conn_first"][m])
            t0 = time.perf_counter()
            O.ref().hpack_decode_blocks(b["data"][:int(b["blk_off"][k])], b["blk_off"][:k + 1], b["conn_first"][:m + 1],
                                        4096, responses=True, trailers=b["trailers"][:k])
            dt = time.perf_counter() - t0
            line["cpu"] = {"reference_1thread_blocks_per_s": round(k / dt, 1)}
    except Exception as e:  # the CPU baseline is a report, not a gate
        line["cpu_error"] = str(e)
    return line


def main():
    import torch

    from h2o_amd import codec, synth

    torch.cuda.set_device(0)
    if os.environ.get("HHUFF_AB_LIB"):  # A/B: time another build of the library (tools/ab.py build NAME)
        codec.LIB_PATH = os.environ["HHUFF_AB_LIB"]
    cfgs = sys.argv[1:] or ["c2", "c3", "c5", "lit"]
    for cfg in cfgs:
        if cfg == "lit":
            print(json.dumps(literals_line(torch, codec, synth)), flush=True)
            continue
        if cfg.startswith("qpack"):
            n = int(cfg[5:]) if len(cfg) > 5 else 65536
            print(json.dumps(qpack_line(torch, codec, n)), flush=True)
            continue
        if cfg.startswith("reqenc"):
            n = int(cfg[6:]) if len(cfg) > 6 else 65536
            print(json.dumps(hpenc_line(torch, codec, n, requests=True)), flush=True)
            continue
        if cfg.startswith("hpenc"):
            n = int(cfg[5:]) if len(cfg) > 5 else 65536
            print(json.dumps(hpenc_line(torch, codec, n)), flush=True)
            continue
        if cfg.startswith("resp"):
            n = int(cfg[4:]) if len(cfg) > 4 else 65536
            print(json.dumps(responses_line(torch, codec, n)), flush=True)
            continue
        if cfg.startswith("blocks"):
            n = int(cfg[6:]) if len(cfg) > 6 else 65536
            print(json.dumps(blocks_line(torch, codec, n)), flush=True)
            continue
        if cfg[5:].startswith("u") and cfg[6:].isdigit():  # flat_u<L>: fixed-length strings (A/B only)
            synth.CONFIGS.setdefault(cfg[5:], dict(n=1 << 20, lengths=("uniform", int(cfg[6:]), int(cfg[6:])),
                                                   alphabet="header"))
        flat = cfg.startswith("flat_")  # flat_<config>: flatten_string (prefix 7) over that config's strings
        b = synth.make_batch_torch(cfg[5:] if flat else cfg, seed=7)
        n, P = b["n"], int(b["total"])
        off32 = b["off"].to(torch.int32)
        line = {"config": cfg, "strings": n, "plain_bytes": P}
        if cfg in ("c2", "c3") and not flat:
            huff, h_off, n_ok, H, P_ok = packed_huffman(torch, codec, b)
            d_out = torch.empty(codec.decode_slot_size(H), dtype=torch.uint8, device="cuda")
            d_len = torch.empty(n_ok, dtype=torch.int32, device="cuda")
            d_st = torch.empty(n_ok, dtype=torch.uint8, device="cuda")
            t_dec = timed(torch, lambda: codec.decode_batch(huff, h_off, n_ok, out=d_out, out_len=d_len, status=d_st,
                                                            in_size=H))
            line.update(decode_ms=round(t_dec, 4), decode_gibps=round(P_ok / GIB / (t_dec * 1e-3), 2),
                        huffman_bytes=H)
            if cfg == "c3":
                e_out = torch.empty(P + 16, dtype=torch.uint8, device="cuda")
                e_len = torch.empty(n, dtype=torch.int32, device="cuda")
                e_st = torch.empty(n, dtype=torch.uint8, device="cuda")
                t_enc = timed(torch, lambda: codec.encode_batch(b["data"], off32, n, out=e_out, out_len=e_len,
                                                                status=e_st, in_size=P))
                line.update(encode_ms=round(t_enc, 4), encode_gibps=round(P / GIB / (t_enc * 1e-3), 2),
                            round_trip_gibps=round(P / GIB / ((t_enc + t_dec) * 1e-3), 2))
        elif cfg == "lit":
            pass
        else:
            f_out = torch.empty(P + 11 * n + 16, dtype=torch.uint8, device="cuda")
            f_len = torch.empty(n, dtype=torch.int32, device="cuda")
            t = timed(torch, lambda: codec.flatten_batch(b["data"], off32, n, 7, out=f_out, out_len=f_len, in_size=P))
            line.update(flatten_ms=round(t, 4), flatten_gibps=round(P / GIB / (t * 1e-3), 2),
                        framed_bytes=int(f_len.to(torch.int64).sum().item()))
        print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
