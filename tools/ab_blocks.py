#!/usr/bin/env python3
"""In-process A/B of hpack_blocks_kernel between builds (interleaved rounds, one process):

    python tools/ab_blocks.py [nconn] build/ab/libhhuff_A.so ...   # the in-tree library is always timed too
"""
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch

    from h2o_amd import codec
    from h2o_amd import hpack_synth as HS

    args = sys.argv[1:]
    nconn = int(args.pop(0)) if args and args[0].isdigit() else 65536
    paths = [codec.LIB_PATH] + args
    codec.lib()
    torch.cuda.set_device(0)
    b = HS.make_connections(nconn, seed=5, adversarial_frac=0.01)
    dev = lambda a: torch.from_numpy(np.ascontiguousarray(a).copy()).cuda()  # noqa: E731
    d, bo, cf = dev(b["data"]), dev(b["blk_off"].view(np.int32)), dev(b["conn_first"].view(np.int32))
    L = np.diff(b["blk_off"].astype(np.int64))
    fa, fb = (int(x) for x in os.environ.get("HHUFF_AB_ARENA", "16,1024").split(","))  # arena bytes per block: fa L + fb
    ao = dev(np.concatenate([[0], np.cumsum(fa * L + fb)]).astype(np.int64))
    nblk = len(L)
    nslots = int(b["blk_off"][-1])
    out = {k: torch.empty(nslots, dtype=torch.int32, device="cuda") for k in ("no", "nl", "vo", "vl")}
    ff = torch.empty(nslots, dtype=torch.uint8, device="cuda")
    nf = torch.empty(nblk, dtype=torch.int32, device="cuda")
    bs = torch.empty(nblk, dtype=torch.int32, device="cuda")
    arena = torch.empty(int(ao[-1].item()), dtype=torch.uint8, device="cuda")
    vp = ctypes.c_void_p
    libs = []
    for p in paths:
        L_ = ctypes.CDLL(p)
        L_.hhuff_hpack_scratch_size.restype = ctypes.c_uint64
        L_.hhuff_hpack_scratch_size.argtypes = [ctypes.c_uint32, ctypes.c_uint32]
        f = L_.hhuff_hpack_decode_blocks
        f.restype = ctypes.c_int
        f.argtypes = [vp, ctypes.c_uint64, vp, vp, ctypes.c_uint32, ctypes.c_uint32] + [vp] * 10 + \
            [ctypes.c_uint64, ctypes.c_uint, vp]
        libs.append((os.path.basename(p), L_))
    ss = int(libs[0][1].hhuff_hpack_scratch_size(nconn, 4096))
    scratch = torch.empty(ss, dtype=torch.uint8, device="cuda")
    P = lambda t: t.data_ptr()  # noqa: E731
    st = torch.cuda.current_stream().cuda_stream

    def call(L_):
        rc = L_.hhuff_hpack_decode_blocks(P(d), d.numel(), P(bo), P(cf), nconn, 4096, P(arena), P(ao), P(out["no"]),
                                          P(out["nl"]), P(out["vo"]), P(out["vl"]), P(ff), P(nf), P(bs), P(scratch),
                                          ss, 0, st)
        assert rc == 0

    times = {n: [] for n, _ in libs}
    for rnd in range(5):
        for n, L_ in libs:
            call(L_)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(5):
                call(L_)
            e1.record()
            torch.cuda.synchronize()
            times[n].append(e0.elapsed_time(e1) / 5)
            if rnd == 0:
                print(json.dumps({"lib": n, "ok_blocks": int((bs == 0).sum().item()), "fields": int(nf.sum().item())}))
    for n, t in times.items():
        print(json.dumps({"lib": n, "nconn": nconn, "ms_min": round(min(t), 4), "ms_med": round(sorted(t)[2], 4),
                          "block_gibps": round(d.numel() / 2 ** 30 / (min(t) * 1e-3), 3)}))


if __name__ == "__main__":
    main()
