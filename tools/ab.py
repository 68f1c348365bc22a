#!/usr/bin/env python3
"""In-process A/B timing of libhhuff builds (MI355X methodology rule: interleaved rounds, one process).

    python tools/ab.py build NAME -DFLAG ...     # hipcc the library into build/ab/libhhuff_NAME.so
                                                  # (-DHHUFF_AB_VARIANTS=1: with the tools/ab variant kernels)
    python tools/ab.py run NAME1 NAME2 ...        # time c4 encode + decode for each build, interleaved
"""
import ctypes
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
ABDIR = os.path.join(ROOT, "build", "ab")


def build(name, flags):
    from h2o_amd import build as hb

    os.makedirs(ABDIR, exist_ok=True)
    out = os.path.join(ABDIR, "libhhuff_%s.so" % name)
    # tools/ab holds the variant kernels that are not in libhhuff.so (-DHHUFF_AB_VARIANTS=1 or a flag selecting one)
    cmd = ["/opt/rocm/bin/hipcc", "-shared"] + hb.HIPCC_FLAGS + flags + ["-I" + os.path.join(ROOT, "include"), "-I" + hb.CSRC,
                                                                         "-I" + os.path.join(ROOT, "tools", "ab")] + \
        hb.sources() + ["-o", out]
    subprocess.run(cmd, check=True)
    print(out)


def run(names, cfg="c4", rounds=5, steps=10):
    import torch

    from h2o_amd import synth

    # ablation configs (not product configs): fixed-length strings isolate lane imbalance
    synth.CONFIGS.setdefault("c4u", dict(n=1 << 24, lengths=("uniform", 48, 48), alphabet="header"))
    synth.CONFIGS.setdefault("c3desc", dict(n=1 << 20, lengths=("zipf_desc", 8, 512), alphabet="header"))
    # c3's two halves at their c3 counts (the zipf's conditional lengths): what a length partition could reach
    synth.CONFIGS.setdefault("c3lo", dict(n=643000, lengths=("zipf", 8, 96), alphabet="header"))
    synth.CONFIGS.setdefault("c3hi", dict(n=405000, lengths=("zipf", 97, 512), alphabet="header"))
    synth.CONFIGS.setdefault("c3hid", dict(n=405000, lengths=("zipf_desc", 97, 512), alphabet="header"))
    synth.CONFIGS.setdefault("u250", dict(n=405000, lengths=("uniform", 250, 250), alphabet="header"))
    # mixed-length batches near the staged / stream boundary (the select test's two distributions)
    synth.CONFIGS.setdefault("m120", dict(n=1 << 20, lengths=("uniform", 110, 130), alphabet="header"))
    synth.CONFIGS.setdefault("m60", dict(n=1 << 20, lengths=("uniform", 40, 100), alphabet="header"))
    for L in (64, 80, 96, 120, 200, 400):  # fixed lengths at the c3 scale: what length-sorted tiles could reach
        synth.CONFIGS.setdefault("u%d" % L, dict(n=1 << 20, lengths=("uniform", L, L), alphabet="header"))
    torch.cuda.set_device(0)
    libs = {}
    vp = ctypes.c_void_p
    for nm in names:
        L = ctypes.CDLL(os.path.join(ABDIR, "libhhuff_%s.so" % nm))
        L.hhuff_decode_batch.argtypes = [vp, ctypes.c_uint64, vp, vp, ctypes.c_uint32, vp, vp, vp, vp, vp, vp]
        L.hhuff_encode_batch.argtypes = [vp, ctypes.c_uint64, vp, vp, ctypes.c_uint32, vp, vp, vp, vp, vp]
        L.hhuff_flatten_batch.argtypes = [vp, ctypes.c_uint64, vp, vp, ctypes.c_uint32, vp, ctypes.c_uint32, vp, vp, vp,
                                          vp, vp]
        libs[nm] = L
    b = synth.make_batch_torch(cfg, seed=5)
    n, P = b["n"], int(b["total"])
    off32 = b["off"].to(torch.int32)
    lens = b["off"][1:] - b["off"][:-1]
    e_out = torch.empty(P + 16, dtype=torch.uint8, device="cuda")
    e_len = torch.empty(n, dtype=torch.int32, device="cuda")
    e_st = torch.empty(n, dtype=torch.uint8, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    L0 = libs[names[0]]
    L0.hhuff_encode_batch(b["data"].data_ptr(), P, off32.data_ptr(), None, n, e_out.data_ptr(), None,
                          e_len.data_ptr(), e_st.data_ptr(), s)
    idx = torch.nonzero(e_len != -1).squeeze(1)
    n_ok = int(idx.numel())
    hl = e_len[idx].to(torch.int64)
    h_off = torch.zeros(n_ok + 1, dtype=torch.int64, device="cuda")
    h_off[1:] = torch.cumsum(hl, 0)
    H = int(h_off[-1].item())
    huff = torch.empty(H + 16, dtype=torch.uint8, device="cuda")
    tmp = torch.empty(n_ok, dtype=torch.int32, device="cuda")
    ho32 = h_off[:-1].to(torch.int32).contiguous()
    L0.hhuff_encode_batch(b["data"].data_ptr(), P, off32[idx].contiguous().data_ptr(),
                          lens[idx].to(torch.int32).contiguous().data_ptr(), n_ok, huff.data_ptr(), ho32.data_ptr(),
                          tmp.data_ptr(), None, s)
    hoff = h_off.to(torch.int32).contiguous()
    d_out = torch.empty(H * 8 // 5 + 16, dtype=torch.uint8, device="cuda")
    d_len = torch.empty(n_ok, dtype=torch.int32, device="cuda")
    d_st = torch.empty(n_ok, dtype=torch.uint8, device="cuda")
    ref = None
    res = {nm: {"enc": [], "dec": [], "flat": []} for nm in names}
    f_out = torch.empty(P + 11 * n + 16, dtype=torch.uint8, device="cuda")
    f_len = torch.empty(n, dtype=torch.int32, device="cuda")
    kinds = ("enc", "dec", "flat") if os.environ.get("AB_FLAT") else ("enc", "dec")

    def positions(starts, lens_):  # byte positions covered by [start, start + len) slots
        lens_ = lens_.to(torch.int64)
        tot = int(lens_.sum().item())
        rep = torch.repeat_interleave(starts.to(torch.int64), lens_)
        first = torch.repeat_interleave(torch.cumsum(lens_, 0) - lens_, lens_)
        return rep + torch.arange(tot, device="cuda", dtype=torch.int64) - first

    def content_sum(buf, pos):
        v = buf[pos].to(torch.int64)
        return int((v * (torch.arange(v.numel(), device="cuda", dtype=torch.int64) % 251 + 1)).sum().item())
    for r in range(rounds):
        for nm in names:
            L = libs[nm]
            for kind in kinds:
                ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
                for i in range(steps + 2):
                    if i == 2:
                        ev[0].record()
                    if kind == "flat":  # QPACK flatten_string framing (prefix 7), c5's own operation
                        rc = L.hhuff_flatten_batch(b["data"].data_ptr(), P, off32.data_ptr(), None, n, None, 7, None,
                                                   f_out.data_ptr(), None, f_len.data_ptr(), s)
                    elif kind == "enc":
                        rc = L.hhuff_encode_batch(b["data"].data_ptr(), P, off32.data_ptr(), None, n, e_out.data_ptr(),
                                                  None, e_len.data_ptr(), e_st.data_ptr(), s)
                    else:
                        rc = L.hhuff_decode_batch(huff.data_ptr(), H, hoff.data_ptr(), None, n_ok, None,
                                                  d_out.data_ptr(), None, d_len.data_ptr(), d_st.data_ptr(), s)
                    assert rc == 0, (nm, kind, rc)  # a launch that failed leaves the last build's outputs
                ev[1].record()
                torch.cuda.synchronize()
                res[nm][kind].append(ev[0].elapsed_time(ev[1]) / steps)
            # correctness: compare outputs with the first build
            # lengths and the bytes inside each output slot must agree (slot tails are unspecified)
            ar = torch.arange(n, device="cuda", dtype=torch.int64)
            chk = (int(e_len.to(torch.int64).sum().item()), int(d_len.to(torch.int64).sum().item()),
                   int((e_len.to(torch.int64) * (ar % 977 + 1)).sum().item()),
                   int((d_len.to(torch.int64) * (ar[:n_ok] % 977 + 1)).sum().item()))
            ok_e = e_len != -1
            e_pos = positions(b["off"][:-1][ok_e], e_len[ok_e])
            ok_d = d_len != -1
            d_pos = positions((hoff[:-1].to(torch.int64) * 8 // 5)[ok_d], d_len[ok_d])
            chk = chk + (content_sum(e_out, e_pos), content_sum(d_out, d_pos))
            if "flat" in kinds:  # framed literals at in_off[i] + 11 i, f_len bytes each
                f_pos = positions(b["off"][:-1] + 11 * torch.arange(n, device="cuda"), f_len)
                chk = chk + (int(f_len.to(torch.int64).sum().item()), content_sum(f_out, f_pos))
            if ref is None:
                ref = chk
            assert chk == ref or nm.startswith("x_"), (nm, chk, ref)  # x_*: ablation builds, output not checked
    # profile builds (-DHHUFF_PROFILE): per-phase shader cycles of one launch of each kernel
    phases = ["plan+issue", "steps", "verdicts/bswap", "commit", "out copy", "len/status", "direct", "plan next"]
    for nm in names:
        L = libs[nm]
        if not hasattr(L, "hhuff_debug_prof"):
            continue
        buf = (ctypes.c_ulonglong * 16)()
        L.hhuff_debug_prof(buf, 1)
        for kind in ("dec", "enc"):
            if kind == "enc":
                L.hhuff_encode_batch(b["data"].data_ptr(), P, off32.data_ptr(), None, n, e_out.data_ptr(), None,
                                     e_len.data_ptr(), e_st.data_ptr(), s)
            else:
                L.hhuff_decode_batch(huff.data_ptr(), H, hoff.data_ptr(), None, n_ok, None, d_out.data_ptr(), None,
                                     d_len.data_ptr(), d_st.data_ptr(), s)
            torch.cuda.synchronize()
            L.hhuff_debug_prof(buf, 1)
            row = list(buf)[0:8] if kind == "dec" else list(buf)[8:16]
            tot = float(sum(row)) or 1.0
            print(json.dumps({"build": nm, "kernel": kind, "cycles_per_wave": round(tot / 4096),
                              "phases": {phases[k]: round(row[k] / tot, 4) for k in range(8) if row[k]}}))
    for nm in names:
        e = sorted(res[nm]["enc"])
        d = sorted(res[nm]["dec"])
        line = {"build": nm, "cfg": cfg, "enc_ms_median": round(e[len(e) // 2], 4), "enc_ms_min": round(e[0], 4),
                "dec_ms_median": round(d[len(d) // 2], 4), "dec_ms_min": round(d[0], 4)}
        if res[nm]["flat"]:
            f = sorted(res[nm]["flat"])
            line.update(flat_ms_median=round(f[len(f) // 2], 4), flat_ms_min=round(f[0], 4))
        print(json.dumps(line))


if __name__ == "__main__":
    if sys.argv[1] == "build":
        build(sys.argv[2], sys.argv[3:])
    else:
        args = sys.argv[2:]
        cfg = "c4"
        if args and args[0].startswith("cfg="):
            cfg = args.pop(0)[4:]
        run(args, cfg=cfg)
