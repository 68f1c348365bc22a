"""CPU check of the split decoder's algorithm (split_decode_wave, hhuff_kernels.hip): the scalar emulation in
tools/emu_split.py -- 64 segments, leads of 64/128/256 bits by segment size, the agree-with-the-lane-before
fix-up, the prefix-summed second pass -- against the oracle on header text, long-code mixes, periodic text
that never resynchronises and corrupted strings (EOS, flipped bits, truncation, bad padding)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))


def test_split_algorithm_matches_oracle(oracle_codec):
    import emu_split as E
    from test_gpu_parity import _long_huffman_strings

    T = E.tables()
    rng = np.random.default_rng(17)
    lengths = [int(x) for x in rng.integers(40, 900, 24)] + [int(x) for x in rng.integers(900, 6000, 12)]
    huff = _long_huffman_strings(oracle_codec, rng, lengths)
    rewalked = 0
    for h in huff:
        ref, _ = oracle_codec.decode(h)
        got, rw = E.split_decode(T, h, 0, len(h))
        assert got == ref, (len(h), None if ref is None else len(ref))
        rewalked += rw > 0
    assert rewalked > 0  # the periodic strings exercise the fix-up
    assert E.split_decode(T, b"", 0, 0)[0] == b"" == oracle_codec.decode(b"")[0]


def test_split_block_algorithm_matches_oracle(oracle_codec):
    """split_decode_block's parameters: 64 W = 1024 or 256 segments of at least 128 bits (lead 128 up to 256-bit
    segments), the fix-up crossing waves."""
    import emu_split as E
    from test_gpu_parity import _long_huffman_strings

    T = E.tables()
    rng = np.random.default_rng(29)
    lengths = [4096, 4500, 9000, 16384, 20000, 33000] + [int(x) for x in rng.integers(4096, 12000, 6)]
    huff = _long_huffman_strings(oracle_codec, rng, lengths)
    rewalked = 0
    for h in huff:
        ref, _ = oracle_codec.decode(h)
        for nseg in (1024, 256):  # split_decode_kernel's block list (16 waves), one_string_kernel (4 waves)
            got, rw = E.split_decode(T, h, 0, len(h), nseg=nseg, minseg=128)
            assert got == ref, (nseg, len(h), None if ref is None else len(ref))
            rewalked += rw > 0
    assert rewalked > 0


def test_encode_long_algorithm_matches_oracle(oracle_codec):
    """encode_long_kernel's algorithm (tools/emu_encode_long.py, 16-KB rounds and a carried partial word; small
    rounds here so that several are crossed quickly) against the oracle, with the verdict at its edge"""
    import emu_encode_long as L

    code, nbits = L.table()
    rng = np.random.default_rng(41)
    from h2o_amd import synth
    syms, p = synth.header_alphabet()
    cases = [b"&" * 4000 + b"aaa", b"&" * 4000 + b"aa", b"0e" * 3000, bytes(rng.integers(0, 256, 3000, dtype=np.uint8)),
             b"a" * 1023 + b"&" * 1025 + b"aaa" + b"z" * 7, bytes(rng.choice(syms, 9000, p=p)), b"a", b"&"]
    for s in cases:
        for chunk, threads in ((1024, 64), (512, 32), (16384, 1024)):
            assert L.encode_long(code, nbits, s, chunk=chunk, threads=threads) == oracle_codec.encode(s), \
                (len(s), chunk)


def test_encode_inplace_algorithm_matches_plain_encoder():
    """encode_inplace_kernel's lane algorithm (tools/emu_encode_inplace.py): strings encoded over their own input
    words with the lanes in a random lock-step order, long-code prefixes re-encoded, random bytes failing --
    byte for byte equal to a plain encoder of hpack.c:774-804"""
    import random

    import emu_encode_inplace as emu

    rng = random.Random(7)
    alpha = b"abcdefghijklmnopqrstuvwxyz0123456789-_./=;, ABCDEFGHIJKLMNOPQRSTUVWXYZ\"{}<>?@[]^|~"
    redone = 0
    for _ in range(40):
        strings = []
        for _ in range(rng.randint(1, 48)):
            L = rng.choice([rng.randint(0, 8), rng.randint(24, 72), rng.randint(1, 160)])
            r = rng.random()
            if r < 0.05:
                s = bytes(rng.randrange(256) for _ in range(L))
            elif r < 0.15:
                s = bytes(rng.choice(b"{}<>?@[]^|~\\") for _ in range(min(L, 6))) + \
                    bytes(rng.choice(alpha) for _ in range(max(0, L - 6)))
            else:
                s = bytes(rng.choice(alpha) for _ in range(L))
            strings.append(s)
        redone += emu.run_chunk(strings, rng)
    assert redone > 0  # the re-encode path ran
