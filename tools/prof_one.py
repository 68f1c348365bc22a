#!/usr/bin/env python3
"""Run one direction of one A/B build a few times (for rocprofv3 --pmc / --kernel-trace runs).

    python tools/prof_one.py NAME [enc|dec] [cfg] [iters]      # build/ab/libhhuff_NAME.so
"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch

    from h2o_amd import synth

    name = sys.argv[1]
    kind = sys.argv[2] if len(sys.argv) > 2 else "enc"
    cfg = sys.argv[3] if len(sys.argv) > 3 else "c4"
    iters = int(sys.argv[4]) if len(sys.argv) > 4 else 5
    synth.CONFIGS.setdefault("c4u", dict(n=1 << 24, lengths=("uniform", 48, 48), alphabet="header"))
    torch.cuda.set_device(0)
    vp = ctypes.c_void_p
    L = ctypes.CDLL(os.path.join(ROOT, "build", "ab", "libhhuff_%s.so" % name))
    L.hhuff_decode_batch.argtypes = [vp, ctypes.c_uint64, vp, vp, ctypes.c_uint32, vp, vp, vp, vp, vp, vp]
    L.hhuff_encode_batch.argtypes = [vp, ctypes.c_uint64, vp, vp, ctypes.c_uint32, vp, vp, vp, vp, vp]
    b = synth.make_batch_torch(cfg, seed=5)
    n, P = b["n"], int(b["total"])
    off32 = b["off"].to(torch.int32)
    e_out = torch.empty(P + 16, dtype=torch.uint8, device="cuda")
    e_len = torch.empty(n, dtype=torch.int32, device="cuda")
    e_st = torch.empty(n, dtype=torch.uint8, device="cuda")
    s = torch.cuda.current_stream().cuda_stream

    def enc():
        assert L.hhuff_encode_batch(b["data"].data_ptr(), P, off32.data_ptr(), None, n, e_out.data_ptr(), None,
                                    e_len.data_ptr(), e_st.data_ptr(), s) == 0

    enc()
    torch.cuda.synchronize()
    if kind == "dec":
        idx = torch.nonzero(e_len != -1).squeeze(1)
        n_ok = int(idx.numel())
        hl = e_len[idx].to(torch.int64)
        h_off = torch.zeros(n_ok + 1, dtype=torch.int64, device="cuda")
        h_off[1:] = torch.cumsum(hl, 0)
        H = int(h_off[-1].item())
        lens = (b["off"][1:] - b["off"][:-1])[idx].to(torch.int32).contiguous()
        huff = torch.empty(H + 16, dtype=torch.uint8, device="cuda")
        tmp = torch.empty(n_ok, dtype=torch.int32, device="cuda")
        assert L.hhuff_encode_batch(b["data"].data_ptr(), P, off32[idx].contiguous().data_ptr(), lens.data_ptr(), n_ok,
                                    huff.data_ptr(), h_off[:-1].to(torch.int32).contiguous().data_ptr(), tmp.data_ptr(),
                                    None, s) == 0
        hoff = h_off.to(torch.int32).contiguous()
        d_out = torch.empty(H * 8 // 5 + 16, dtype=torch.uint8, device="cuda")
        d_len = torch.empty(n_ok, dtype=torch.int32, device="cuda")
        d_st = torch.empty(n_ok, dtype=torch.uint8, device="cuda")
        for _ in range(iters):
            assert L.hhuff_decode_batch(huff.data_ptr(), H, hoff.data_ptr(), None, n_ok, None, d_out.data_ptr(), None,
                                        d_len.data_ptr(), d_st.data_ptr(), s) == 0
    else:
        for _ in range(iters):
            enc()
    torch.cuda.synchronize()
    print("ok", name, kind, cfg)


if __name__ == "__main__":
    main()
