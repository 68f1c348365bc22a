#!/usr/bin/env python3
"""Scalar emulation of encode_long_kernel (hhuff_kernels.hip): 16-KB rounds of 1,024 threads x 16 bytes, a block
scan of the threads' code bits, the early verdict, 64-bit accumulators OR-ed a word at a time into a stage whose
word 0 carries the previous round's partial word, whole words out, then the EOS-prefix padding."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

CHUNK = 16384


def table():
    from h2o_amd import tables
    return tables.ENC_CODE, tables.ENC_NBITS


def encode_long(code, nbits, data, chunk=CHUNK, threads=1024):
    n = len(data)
    lim = 8 * n - 8 if n else 0
    if n == 0:
        return None
    out = {}  # output word index -> MSB-first word
    P, carry = 0, 0
    for c0 in range(0, n, chunk):
        cl = min(chunk, n - c0)
        per = [data[c0 + 16 * t:c0 + min(16 * t + 16, cl)] if 16 * t < cl else b"" for t in range(threads)]
        bits = [sum(nbits[b] for b in seg) for seg in per]
        T = sum(bits)
        if P + T > lim:
            return None
        base = P & 31
        st = [0] * ((chunk * 30) // 32 + 8)
        st[0] = carry
        pre = 0
        for t, seg in enumerate(per):
            pos = base + pre
            pre += bits[t]
            wp, fill, acc = pos >> 5, pos & 31, 0
            for b in seg:
                acc |= code[b] << (64 - fill - nbits[b])
                fill += nbits[b]
                if fill >= 32:
                    st[wp] |= acc >> 32
                    wp += 1
                    acc = (acc << 32) & ((1 << 64) - 1)
                    fill -= 32
            if fill:
                st[wp] |= acc >> 32
        nfull = (base + T) >> 5
        for k in range(nfull):
            out[(P >> 5) + k] = st[k]
        carry = st[nfull]
        P += T
    p = (-P) & 7
    sh = P & 31
    w = carry
    if p:
        w |= (0xFFFFFFFF >> sh) & ~(0 if sh + p >= 32 else 0xFFFFFFFF >> (sh + p)) & 0xFFFFFFFF
    if sh:
        out[P >> 5] = w
    nbytes = (P + 7) >> 3
    raw = b"".join(out.get(k, 0).to_bytes(4, "big") for k in range((nbytes + 3) // 4))
    return raw[:nbytes]
