#!/usr/bin/env python3
"""Long-string decode: libhhuff builds interleaved in one process (split_decode_kernel against one lane per
string).  Batches of long header values: 512 x 4-64 KB, 64 x 256 KB, one string of 100 KB / 1 MB / 2 KB, 8 x 3 KB.

    python tools/split_bench.py NAME1 NAME2 ...   (libraries from build/ab)
"""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
ABDIR = os.path.join(ROOT, "build", "ab")


def main(names, rounds=5, steps=10):
    import numpy as np
    import torch

    from h2o_amd import synth
    from oracle import oracle as O

    torch.cuda.set_device(0)
    vp = ctypes.c_void_p
    libs = {}
    for nm in names:
        L = ctypes.CDLL(os.path.join(ABDIR, "libhhuff_%s.so" % nm))
        L.hhuff_decode_batch.argtypes = [vp, ctypes.c_uint64, vp, vp, ctypes.c_uint32, vp, vp, vp, vp, vp, vp]
        libs[nm] = L
    o = O.oracle()
    rng = np.random.default_rng(9)
    syms, p = synth.header_alphabet()
    cases = {"512x4-64K": [int(x) for x in rng.integers(4096, 65536, 512)], "64x256K": [262144] * 64,
             "1x100K": [100000], "1x1M": [1 << 20], "1x2K": [2000], "8x3K": [3000] * 8, "1x16K": [16384], "4x8K": [8192] * 4}
    s = torch.cuda.current_stream().cuda_stream
    res = {}
    for cname, lens in cases.items():
        plain = [bytes(rng.choice(syms, int(L * 1.3), p=p)) for L in lens]
        data, off = synth.pack(plain)
        enc, el, _ = o.encode_batch(data, off, len(plain), nthreads=8)
        huff = [enc[int(off[i]):int(off[i]) + int(el[i])].tobytes() for i in range(len(plain))]
        hdata, hoff = synth.pack(huff)
        n = len(huff)
        d = torch.from_numpy(hdata.copy()).cuda()
        doff = torch.from_numpy(hoff.astype(np.int32)).cuda()
        out = torch.empty(hdata.size * 8 // 5 + 64, dtype=torch.uint8, device="cuda")
        ol = torch.empty(n, dtype=torch.int32, device="cuda")
        st = torch.empty(n, dtype=torch.uint8, device="cuda")
        ref = None
        for nm in names:  # same results from every build
            libs[nm].hhuff_decode_batch(d.data_ptr(), hdata.size, doff.data_ptr(), None, n, None, out.data_ptr(), None,
                                        ol.data_ptr(), st.data_ptr(), s)
            torch.cuda.synchronize()
            got = (ol.cpu().numpy().tobytes(), out.cpu().numpy().tobytes())
            assert ref is None or got == ref, (cname, nm)
            ref = got
        assert (ol.cpu().numpy() >= 0).all()
        t = {nm: [] for nm in names}
        for _ in range(rounds):
            for nm in names:
                L = libs[nm]
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                L.hhuff_decode_batch(d.data_ptr(), hdata.size, doff.data_ptr(), None, n, None, out.data_ptr(), None,
                                     ol.data_ptr(), st.data_ptr(), s)
                e0.record()
                for _ in range(steps):
                    L.hhuff_decode_batch(d.data_ptr(), hdata.size, doff.data_ptr(), None, n, None, out.data_ptr(),
                                         None, ol.data_ptr(), st.data_ptr(), s)
                e1.record()
                torch.cuda.synchronize()
                t[nm].append(e0.elapsed_time(e1) / steps)
        res[cname] = {nm: {"ms": min(v), "GiB/s": hdata.size / (min(v) * 1e-3) / 2**30} for nm, v in t.items()}
        res[cname]["bytes"] = int(hdata.size)
        print(json.dumps({cname: res[cname]}), flush=True)


if __name__ == "__main__":
    main(sys.argv[1:])
