#!/usr/bin/env python3
"""Scalar emulation of split_decode_kernel (one wave = 64 lanes, run one after another), for checking the
segment / synchronisation logic on the CPU against the oracle.  Mirrors seg_walk over the same tables
(13-bit window LUT, long-code tables) and the kernel's agree-with-the-lane-before loop.

    python tools/emu_split.py [n] [seed] [min_len] [max_len]   (plain lengths)
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))

from emu_decode import M32, long_entry, tables  # noqa: E402

LEAD = 256
EOS = 256


def seg_walk(T, data, s, TB, p0, kstart, pstop, emit):
    """-> dict(f, e, cnt, flags, first, last, eos, end_ok, out)"""
    lut = T[0]
    bits = int.from_bytes(bytes(data[s:s + TB // 8]) + b"\0" * 8, "big")
    nbits = TB + 64
    r = dict(f=None, e=0, cnt=0, flags=0, first=0, last=0, eos=False, end_ok=False, out=[])

    def take(p, sym, fl):
        if p < kstart:
            return
        r["f"] = p if r["f"] is None else min(r["f"], p)
        if r["cnt"] == 0:
            r["first"] = sym
        r["last"] = sym
        r["cnt"] += 1
        r["flags"] |= fl
        if emit:
            r["out"].append(sym)

    def window(p):  # 32 bits at p
        return (bits >> (nbits - p - 32)) & M32

    p = p0
    while p < pstop:
        R = TB - p
        w = window(p)
        e = lut[w >> 19]
        if e >> 31:
            le = long_entry(T, w)
            L = (le >> 9) & 31
            if L > R:
                break
            sym = le & 0x1FF
            if sym == EOS and p >= kstart:
                r["eos"] = True
                break
            if sym != EOS:
                take(p, sym, (le >> 14) & 3)
            p += L
        else:
            L1 = (e >> 8) & 15
            if L1 > R:
                break
            L12 = (e >> 12) & 15
            take(p, e & 0xFF, (e >> 24) & 3)
            two = bool((e >> 30) & 1) and L12 <= R and p + L1 < pstop
            if two:
                take(p + L1, (e >> 16) & 0xFF, (e >> 26) & 3)
            p += L12 if two else L1
    r["e"] = p
    if r["f"] is None:
        r["f"] = p
    if pstop >= TB:
        R = TB - p
        top = window(p) >> 24
        r["end_ok"] = (not r["eos"]) and R <= 7 and ((top | (0xFF >> R)) & 0xFF) == 0xFF
    return r


def split_decode(T, data, s, length, nseg=64, minseg=32):
    """-> (decoded bytes or None, rewalks).  nseg=64: split_decode_wave; nseg=64 W, minseg=128:
    split_decode_block (W waves)"""
    TB = 8 * length
    if TB == 0:  # an empty string decodes to nothing
        return b"", 0
    seg = max(((TB + nseg * 32 - 1) // (nseg * 32)) * 32, minseg)
    W = []
    for lane in range(nseg):
        ks = lane * seg
        act = ks < TB
        pstop = TB if (act and ks + seg >= TB) else ks + seg
        lead = 64 if seg <= 64 else (128 if seg <= 256 else LEAD)
        W.append(seg_walk(T, data, s, TB, max(ks - lead, 0), ks, pstop, False) if act else None)
    rewalks = 0
    for _ in range(nseg):
        bad = [lane for lane in range(1, nseg) if W[lane] is not None and W[lane]["f"] != W[lane - 1]["e"]]
        if not bad:
            break
        pe = {lane: W[lane - 1]["e"] for lane in bad}
        for lane in bad:
            ks = lane * seg
            pstop = TB if ks + seg >= TB else ks + seg
            W[lane] = seg_walk(T, data, s, TB, pe[lane], pe[lane], pstop, False)
            rewalks += 1
    act = [w for w in W if w is not None]
    eos = any(w["eos"] for w in act)
    end_ok = act[-1]["end_ok"]
    if eos or not end_ok:
        return None, rewalks
    out = []
    for lane, w in enumerate(W):
        if w is None or not w["cnt"]:
            continue
        ks = lane * seg
        pstop = TB if ks + seg >= TB else ks + seg
        out += seg_walk(T, data, s, TB, w["f"], w["f"], pstop, True)["out"]
        assert len(out) == sum(x["cnt"] for x in W[:lane + 1] if x is not None)
    return bytes(out), rewalks


def main():
    import numpy as np

    from h2o_amd import synth
    from oracle import oracle as O

    n = int(sys.argv[1]) if len(sys.argv) > 1 else 24
    seed = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from test_gpu_parity import _long_huffman_strings

    T = tables()
    o = O.oracle()
    rng = np.random.default_rng(seed)
    lo = int(sys.argv[3]) if len(sys.argv) > 3 else 5200
    hi = int(sys.argv[4]) if len(sys.argv) > 4 else 12000
    huff = _long_huffman_strings(o, rng, [int(x) for x in rng.integers(lo, hi, n)])
    bad = 0
    for i, h in enumerate(huff):
        ref, _ = o.decode(h)
        got, rw = split_decode(T, h, 0, len(h))
        print(i, len(h), "ok" if ref is not None else "fail", "rewalks", rw, "MISMATCH" if got != ref else "")
        bad += got != ref
    print("checked", len(huff), "mismatches", bad)


if __name__ == "__main__":
    main()
