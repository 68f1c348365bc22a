#!/usr/bin/env python3
"""CPU replay of encode_inplace_lane / encode_redo (hhuff_kernels.hip, HHUFF_ENC_INPLACE): one chunk's stage as
32-bit words, the strings' lanes run in lock step (one word step of every lane, in a seeded lane order, per
round), checked against a plain encoder (hpack.c:774-804).  Test infrastructure for the kernel's algorithm."""
import os
import random
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from h2o_amd.tables import ENC_CODE, ENC_NBITS  # noqa: E402

FAIL = 0xFFFFFFFF


def ref_encode(s):
    """h2o_hpack_encode_huffman: bytes, or None when not shorter"""
    acc = nb = 0
    out = bytearray()
    for b in s:
        acc = (acc << ENC_NBITS[b]) | ENC_CODE[b]
        nb += ENC_NBITS[b]
        while nb >= 8:
            nb -= 8
            out.append((acc >> nb) & 0xFF)
        if len(out) >= len(s):
            return None
    if nb:
        out.append(((acc << (8 - nb)) | ((1 << (8 - nb)) - 1)) & 0xFF)
    return bytes(out) if len(out) < len(s) else None


class Stage:
    def __init__(self, data):
        self.w = [int.from_bytes(data[i:i + 4].ljust(4, b"\0"), "big") for i in range(0, len(data), 4)]  # (committed swapped)

    def fetch_and(self, i, m):
        old = self.w[i]
        self.w[i] = old & m
        return old

    def orw(self, i, v):
        self.w[i] |= v & 0xFFFFFFFF

    def place(self, tb, c, n):  # place_bits: MSB-first words
        if n == 0:
            return
        t = (c << (64 - n)) & (2**64 - 1)
        sh = tb & 31
        u = t >> sh
        a = tb >> 5
        self.orw(a, u >> 32)
        self.orw(a + 1, u)
        if sh + n > 64:
            self.orw(a + 2, (t << (32 - sh)))


def lane(st, last, start, length, limit):
    """generator: one yield per word step (the kernel's lock-step points); returns (bits or FAIL, redo)"""
    end = start + length
    a0 = start & ~3
    a0w, lastw = a0 >> 2, last >> 2
    ndw = (end - a0 + 3) >> 2
    jl = (end - a0) >> 2
    mfirst = 0xFFFFFFFF >> (8 * (start & 3))  # big-endian words: string byte k at bits 31 - 8k
    mlast = (0xFFFFFFFF << ((32 - 8 * (end & 3)) & 31)) & 0xFFFFFFFF

    def mo(q):
        m = (mfirst if q == 0 else 0xFFFFFFFF) & (mlast if q + 1 == ndw else 0xFFFFFFFF)
        return m if q < ndw else 0

    def rc(q):
        return st.fetch_and(min(a0w + q, lastw), ~mo(q) & 0xFFFFFFFF)

    startbit, base = 8 * start, 32 * a0w
    E = dict(tb=startbit, tlim=startbit + limit, live=True, fail=False, haz=False)

    def put(codes, on, rlim):
        n = sum(nb for _, nb in codes)
        if on and E["live"] and E["tb"] + n >= E["tlim"]:
            E["fail"], E["live"] = True, False
        if on and E["live"] and E["tb"] + n > rlim:
            E["haz"] = True
        if on and E["live"] and not E["haz"]:
            tb = E["tb"]
            for c, nb in codes:
                st.place(tb, c, nb)
                tb += nb
        if on and E["live"]:
            E["tb"] += n

    def codes_of(w, vm):
        return [(ENC_CODE[(w >> (24 - 8 * k)) & 0xFF], ENC_NBITS[(w >> (24 - 8 * k)) & 0xFF])
                if (vm >> (24 - 8 * k)) & 0xFF else (0, 0) for k in range(4)]

    w0 = rc(0)
    wn = rc(1)
    wt = wn
    put(codes_of(w0, mo(0)), ndw != 0, base + 32 * min(2, ndw))
    yield
    jlv = jl if E["live"] else 0
    for j in range(1, jlv):
        w = wn
        wn = rc(j + 1)
        if j + 1 == jl:
            wt = wn
        put(codes_of(w, 0xFFFFFFFF), True, base + 32 * min(j + 2, ndw))  # the bulk's own checks are the same
        yield
    if E["live"] and E["tb"] >= E["tlim"]:
        E["fail"], E["live"] = True, False
    if (end & 3) and jl >= 1:
        put(codes_of(wt, mlast), True, base + 32 * ndw)
    if E["fail"]:
        return FAIL, False
    if E["haz"]:
        return E["tb"] - startbit, True
    p = (-E["tb"]) & 7
    st.place(E["tb"], (1 << p) - 1, p)
    return E["tb"] - startbit, False


def redo(st, data, start, length):
    end = start + length
    a0w, ndw = start >> 2, (end - (start & ~3) + 3) >> 2
    mfirst = 0xFFFFFFFF >> (8 * (start & 3))
    mlast = (0xFFFFFFFF << ((32 - 8 * (end & 3)) & 31)) & 0xFFFFFFFF
    for q in range(ndw):
        m = (mfirst if q == 0 else 0xFFFFFFFF) & (mlast if q + 1 == ndw else 0xFFFFFFFF)
        st.fetch_and(a0w + q, ~m & 0xFFFFFFFF)
    tb = 8 * start
    for b in data[start:end]:
        st.place(tb, ENC_CODE[b], ENC_NBITS[b])
        tb += ENC_NBITS[b]
    p = (-tb) & 7
    st.place(tb, (1 << p) - 1, p)


def run_chunk(strings, rng):
    data = b"".join(strings)
    span = (len(data) + 15) & ~15
    st = Stage(data.ljust(span + 32, b"\0"))
    offs, o = [], 0
    for s in strings:
        offs.append(o)
        o += len(s)
    gens, res = {}, {}
    for i, s in enumerate(strings):
        if s:
            gens[i] = lane(st, span - 4, offs[i], len(s), 8 * len(s) - 7)
    while gens:  # lock step: every live lane takes one word step per round, in a random order
        order = list(gens)
        rng.shuffle(order)
        for i in order:
            try:
                next(gens[i])
            except StopIteration as e:
                res[i] = e.value
                del gens[i]
    for i, (bits, rd) in res.items():
        if rd:
            redo(st, data, offs[i], len(strings[i]))
    raw = b"".join(w.to_bytes(4, "big") for w in st.w)  # the copy-out's byte swap
    nredo = 0
    for i, s in enumerate(strings):
        want = ref_encode(s)
        if not s:
            continue
        bits, rd = res[i]
        nredo += rd
        if want is None:
            assert bits == FAIL, (i, s, bits)
            continue
        assert bits != FAIL and (bits + 7) // 8 == len(want), (i, s, bits, len(want))
        got = raw[offs[i]:offs[i] + len(want)]
        assert got == want, (i, s, got.hex(), want.hex())
    return nredo


def main(rounds=200, seed=1):
    rng = random.Random(seed)
    alpha = b"abcdefghijklmnopqrstuvwxyz0123456789-_./=;, ABCDEFGHIJKLMNOPQRSTUVWXYZ\"{}<>?@[]^|~"
    tot = nred = 0
    for _ in range(rounds):
        strings = []
        for _ in range(rng.randint(1, 64)):
            L = rng.choice([rng.randint(0, 8), rng.randint(24, 72), rng.randint(1, 200)])
            if rng.random() < 0.05:
                s = bytes(rng.randrange(256) for _ in range(L))  # random bytes: fail
            elif rng.random() < 0.1:
                s = bytes(rng.choice(b"{}<>?@[]^|~\\") for _ in range(min(L, 6))) + \
                    bytes(rng.choice(alpha) for _ in range(max(0, L - 6)))  # long codes first: redo
            else:
                s = bytes(rng.choice(alpha) for _ in range(L))
            strings.append(s)
        nred += run_chunk(strings, rng)
        tot += len(strings)
    print("strings %d, redone %d: all equal to the plain encoder" % (tot, nred))


if __name__ == "__main__":
    main()
