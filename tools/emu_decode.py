#!/usr/bin/env python3
"""Scalar emulation of the GPU decode step functions (one lane), for debugging kernel logic on the CPU.

Emulates decode_staged_lane_v7 (bulk + tail) over a big-endian dword view of the input, with the
lock-step details that matter for one lane: the long-code detour runs only on every other step
(HHUFF_DEC_LONG2) and the step parity restarts at the tail.  Bytes past the buffer read as `fill`.

    python tools/emu_decode.py [cfg] [n] [seed]    # compares against the CPU oracle (pairs layout)
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))

import gen_tables as G  # noqa: E402

M32 = 0xFFFFFFFF


def tables():
    lens = G.code_lengths()
    codes, order = G.canonical_codes(lens)
    root = G.build_tree(lens, codes)
    lut = G.window_lut(root)
    kinfo, ones = G.ones_tables(lens, codes)
    return lut, kinfo, ones


def s32(x):
    x &= M32
    return x - (1 << 32) if x >> 31 else x


def alignbit(x0, x1, s):
    s &= 31
    return (((x0 << 32) | x1) >> s) & M32


class Lane:
    def __init__(self, T, data, start, length, fill=0):
        self.lut, self.kinfo, self.ones = T
        self.data, self.fill = data, fill

    def word(self, q):  # big-endian dword q of the stream
        b = bytes(self.data[4 * q + k] if 0 <= 4 * q + k < len(self.data) else self.fill for k in range(4))
        return int.from_bytes(b, "big")


def clz32(x):
    return 32 - x.bit_length() if x else 32


def long_entry(T, w):
    lut, kinfo, ones = T
    k = min(clz32((~w | 1) & M32), 30)
    ki = kinfo[k]
    idx = (ki & 0xFFFF) + ((((w << (k + 1)) & M32) >> 1) >> (31 - (ki >> 16)))
    return ones[idx]


def decode_v7(T, data, start, length, fill=0):
    """-> (ok, out bytes, flags) following decode_staged_lane_v7"""
    lut = T[0]
    ln = Lane(T, data, start, length, fill)
    pm = 8 * start - 1
    end = 8 * (start + length)
    out = []
    fail = False
    flags = 0
    parked = False
    lim = end - 26
    step_i = 0
    # bulk
    while pm < lim:
        longchk = step_i % 2 == 1
        step_i += 1
        q = pm >> 5
        w = alignbit(ln.word(q), ln.word(q + 1), ~pm)
        e = lut[w >> 19]
        cons = 0
        if not e >> 31:
            out.append(e & 0xFF)
            if (e >> 30) & 1:
                out.append((e >> 16) & 0xFF)
            flags |= e
            cons = (e >> 12) & 15
            wb = (w << cons) & M32
            eb = lut[wb >> 19]
            if not eb >> 31:
                out.append(eb & 0xFF)
                if (eb >> 30) & 1:
                    out.append((eb >> 16) & 0xFF)
                flags |= eb
                cons += (eb >> 12) & 15
        elif longchk:
            le = long_entry(T, w)
            L = (le >> 9) & 31
            fits = L + pm - end < 0
            eos = (le & 0x1FF) == 256
            if fits and eos:
                fail = True
            if fits and not eos:
                out.append(le & 0xFF)
                flags |= ((le >> 14) & 3) << 24
                cons = L
            else:
                parked = True
                lim = -(1 << 31)
        pm += cons
    # tail: step(true), then pairs (false, true) until no lane progressed on a long-code step
    c = 0x40000000 if parked else pm - end
    step_i = 0
    while True:
        longchk = step_i % 2 == 0
        step_i += 1
        q = pm >> 5
        w = alignbit(ln.word(q), ln.word(q + 1), ~pm)
        e = lut[w >> 19]
        L1, L12 = (e >> 8) & 15, (e >> 12) & 15
        m1 = (not e >> 31) and L1 + c < 0
        m2 = bool((e >> 30) & 1) and L12 + c < 0
        cons = L12 if m2 else (L1 if m1 else 0)
        if m1:
            out.append(e & 0xFF)
            flags |= e & (3 << 24)
        if m2:
            out.append((e >> 16) & 0xFF)
            flags |= e & (3 << 26)
        wb = (w << cons) & M32
        eb = lut[wb >> 19]
        cb = c + cons
        L1b, L12b = (eb >> 8) & 15, (eb >> 12) & 15
        m1b = (not eb >> 31) and L1b + cb < 0
        m2b = bool((eb >> 30) & 1) and L12b + cb < 0
        if m1b:
            out.append(eb & 0xFF)
            flags |= eb & (3 << 24)
        if m2b:
            out.append((eb >> 16) & 0xFF)
            flags |= eb & (3 << 26)
        cons += L12b if m2b else (L1b if m1b else 0)
        lact = (e >> 31) and L1 + c < 0
        if longchk and lact:
            le = long_entry(T, w)
            L = (le >> 9) & 31
            fits = L + c < 0
            eos = (le & 0x1FF) == 256
            if fits and eos:
                fail = True
            if fits and not eos:
                out.append(le & 0xFF)
                flags |= ((le >> 14) & 3) << 24
                cons = L
            else:
                c = 0x40000000
        c += cons
        pm += cons
        if cons == 0 and longchk:
            break
        if cons == 0 and not lact:
            break
    R = (~c) & M32
    q = pm >> 5
    w = alignbit(ln.word(q), ln.word(q + 1), ~pm)
    ok = (not fail) and R <= 7 and (w | (M32 >> (R & 31))) == M32
    f = ((flags >> 24) | (flags >> 26)) & 3
    return ok, bytes(out), f


def main():
    import numpy as np

    from h2o_amd import synth
    from oracle import oracle as O

    cfg = sys.argv[1] if len(sys.argv) > 1 else "c2"
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 20000
    seed = int(sys.argv[3]) if len(sys.argv) > 3 else 1
    T = tables()
    o = O.oracle()
    b = synth.make_batch(cfg, n=n, seed=seed, adversarial_frac=0.02)
    enc, el, _ = o.encode_batch(b["data"], b["off"], n)
    lens = np.where(el != O.FAIL, el, 0).astype(np.uint32)
    bad = 0
    for i in range(n):
        s, ln = int(b["off"][i]), int(lens[i])
        src = bytes(enc[s:s + ln])
        ref, _ = o.decode(src)
        ok, out, _ = decode_v7(T, enc, s, ln)
        got = out if ok else None
        if got != ref:
            bad += 1
            if bad <= 5:
                print("mismatch", i, "len", ln, "ref", None if ref is None else len(ref), "got",
                      None if got is None else len(got), src.hex())
    print("checked", n, "mismatches", bad)


if __name__ == "__main__":
    main()
