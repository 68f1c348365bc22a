#!/usr/bin/env python3
"""Per-phase lane cycles of hpack_blocks_kernel (profile build, -DHHUFF_PROFILE):

    python tools/ab.py build prof -DHHUFF_PROFILE     # build/ab/libhhuff_prof.so
    python tools/prof_blocks.py [nconn] [variant]     # build/ab/libhhuff_<variant>.so, default prof
"""
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
PHASES = ["representation", "static copy", "dynamic copy", "name literal", "value literal", "table add",
          "request rules", "block total"]


def main():
    import torch

    from h2o_amd import codec
    from h2o_amd import hpack_synth as HS

    nconn = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
    variant = sys.argv[2] if len(sys.argv) > 2 else "prof"
    codec.LIB_PATH = os.path.join(ROOT, "build", "ab", "libhhuff_%s.so" % variant)
    L = codec.lib()
    L.hhuff_debug_prof_blocks.argtypes = [ctypes.c_void_p, ctypes.c_int]
    torch.cuda.set_device(0)
    b = HS.make_connections(nconn, seed=5, adversarial_frac=0.01)
    dev = lambda a: torch.from_numpy(np.ascontiguousarray(a).copy()).cuda()  # noqa: E731
    d, bo, cf = dev(b["data"]), dev(b["blk_off"].view(np.int32)), dev(b["conn_first"].view(np.int32))
    Lb = np.diff(b["blk_off"].astype(np.int64))
    ao = dev(np.concatenate([[0], np.cumsum(16 * Lb + 1024)]).astype(np.int64))
    buf = (ctypes.c_ulonglong * 8)()
    for req in (False, True):
        codec.hpack_decode_blocks(d, bo, cf, 4096, arena_off=ao, requests=req)
        torch.cuda.synchronize()
        L.hhuff_debug_prof_blocks(buf, 1)
        codec.hpack_decode_blocks(d, bo, cf, 4096, arena_off=ao, requests=req)
        torch.cuda.synchronize()
        L.hhuff_debug_prof_blocks(buf, 1)
        row = list(buf)
        tot = float(row[7]) or 1.0
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(3):
            codec.hpack_decode_blocks(d, bo, cf, 4096, arena_off=ao, requests=req)
        e1.record()
        torch.cuda.synchronize()
        print(json.dumps({"variant": variant, "requests": req, "nconn": nconn, "ms": round(e0.elapsed_time(e1) / 3, 3),
                          "lane_cycles_total": int(tot),
                          "share": {PHASES[k]: round(row[k] / tot, 4) for k in range(7)},
                          "per_block_cycles": round(tot / (len(Lb)), 1)}), flush=True)


if __name__ == "__main__":
    main()
