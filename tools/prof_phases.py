#!/usr/bin/env python3
"""Per-phase shader cycles of the staged kernels (profile build, -DHHUFF_PROFILE), slot layout vs packed.

    python tools/ab.py build prof -DHHUFF_PROFILE     # build/ab/libhhuff_prof.so
    python tools/prof_phases.py [cfg]
"""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
PHASES = ["plan+issue", "steps", "verdicts/compaction", "commit+plan", "out copy", "len/status", "direct", "-"]
FLAT_PHASES = ["stage issue", "shares+stage wait", "pass 1 (count)", "header+pass 2", "raw copies", "copy-out",
               "direct", "lengths"]


def main():
    import torch

    from bench_configs import packed_huffman
    from h2o_amd import codec, synth

    cfg = sys.argv[1] if len(sys.argv) > 1 else "c4"
    codec.LIB_PATH = os.path.join(ROOT, "build", "ab", "libhhuff_prof.so")
    L = codec.lib()
    L.hhuff_debug_prof.argtypes = [ctypes.c_void_p, ctypes.c_int]
    torch.cuda.set_device(0)
    b = synth.make_batch_torch(cfg, seed=7)
    n, P = b["n"], int(b["total"])
    off32 = b["off"].to(torch.int32)
    huff, h_off, n_ok, H, _ = packed_huffman(torch, codec, b)
    buf = (ctypes.c_ulonglong * 16)()
    runs = {
        "dec_slot": lambda: codec.decode_batch(huff, h_off, n_ok, in_size=H),
        "dec_packed": lambda: codec.decode_batch_packed(huff, h_off, n_ok, in_size=H),
        "enc_slot": lambda: codec.encode_batch(b["data"], off32, n, in_size=P),
        "enc_packed": lambda: codec.encode_batch_packed(b["data"], off32, n, in_size=P),
    }
    if cfg == "c5":  # the QPACK framing (flatten_pl_kernel), its own phases
        runs = {"flatten": lambda: codec.flatten_batch(b["data"], off32, n, 7, in_size=P), **runs}
    for name, fn in runs.items():
        fn()
        torch.cuda.synchronize()
        L.hhuff_debug_prof(buf, 1)
        fn()
        torch.cuda.synchronize()
        L.hhuff_debug_prof(buf, 1)
        row = list(buf)[0:8] if name.startswith("dec") else list(buf)[8:16]
        tot = float(sum(row)) or 1.0
        names = FLAT_PHASES if name == "flatten" else PHASES
        print(json.dumps({"run": name, "cycles_sum": int(tot),
                          "phases": {names[k]: round(row[k] / tot, 4) for k in range(8) if row[k]},
                          "cycles": {names[k]: int(row[k]) for k in range(8) if row[k]}}), flush=True)


if __name__ == "__main__":
    main()
