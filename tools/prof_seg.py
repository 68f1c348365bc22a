#!/usr/bin/env python3
"""Per-phase shader cycles of decode_seg_kernel (profile build, -DHHUFF_PROFILE) on the configs' Huffman wires.

    python tools/ab.py build prof -DHHUFF_PROFILE     # build/ab/libhhuff_prof.so
    python tools/prof_seg.py [cfg ...]                 # default c3 c5
"""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
PHASES = ["setup+stage", "lead", "walk bulk", "walk checked+verify", "places+moves", "copy-out+results", "fallback", "-"]


def main():
    import torch

    from bench_configs import packed_huffman
    from h2o_amd import codec, synth

    codec.LIB_PATH = os.path.join(ROOT, "build", "ab", "libhhuff_prof.so")
    L = codec.lib()
    L.hhuff_debug_prof.argtypes = [ctypes.c_void_p, ctypes.c_int]
    torch.cuda.set_device(0)
    codec.set_decode_kernel(2)
    buf = (ctypes.c_ulonglong * 16)()
    for cfg in sys.argv[1:] or ["c3", "c5"]:
        b = synth.make_batch_torch(cfg, seed=7)
        huff, h_off, n_ok, H, _ = packed_huffman(torch, codec, b)
        fn = lambda: codec.decode_batch(huff, h_off, n_ok, in_size=H)  # noqa: E731
        fn()
        torch.cuda.synchronize()
        L.hhuff_debug_prof(buf, 1)
        fn()
        torch.cuda.synchronize()
        L.hhuff_debug_prof(buf, 1)
        row = list(buf)[0:8]
        tot = float(sum(row)) or 1.0
        print(json.dumps({"config": cfg, "cycles_sum": int(tot),
                          "phases": {PHASES[k]: round(row[k] / tot, 4) for k in range(8) if row[k]}}), flush=True)


if __name__ == "__main__":
    main()
