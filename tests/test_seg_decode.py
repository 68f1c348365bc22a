"""decode_seg_kernel (segment decode: a tile's bits shared evenly over the lanes, tools/ab/hhuff_ab_decoders.h) against
the CPU restatement.  The segment decoder lost its A/B (DESIGN (e)) and is not in libhhuff.so: these tests skip on the
product library and run against an A/B build (HHUFF_AB_LIB=build/ab/libhhuff_NAME.so, built with
-DHHUFF_AB_VARIANTS=1).  hhuff_set_decode_kernel(2) sends every contiguous batch to it, so the golden sets and short-string
batches run through it too; the cases below aim at its own edges: tiles of more than 64 strings (sub-tiles),
lanes closing more strings than they can record (the one-lane fallback), empty strings at tile and span ends,
last strings just under / over the 640-byte keep limit (split lists or one lane), batches not starting at offset
0, periodic text on which a lane that starts off the symbol boundaries never resynchronises (re-walk rounds),
and corrupted strings (EOS, flipped bits, truncation, bad padding) at every position in a segment."""
import contextlib

import numpy as np
import pytest

from conftest import GOLDEN_SETS, compact, load_golden
from h2o_amd import synth
from test_gpu_parity import _long_huffman_strings, gpu_decode, torch_cuda  # noqa: F401

pytestmark = pytest.mark.gpu

FAIL = 0xFFFFFFFF


@contextlib.contextmanager
def decode_kernel(mode):
    from h2o_amd import codec

    try:
        prev = codec.set_decode_kernel(mode)
    except codec.HhuffError:  # the segment decoder is A/B-only: run these against such a build via HHUFF_AB_LIB
        pytest.skip("segment decoder not in this library (tools/ab.py build NAME -DHHUFF_AB_VARIANTS=1)")
    try:
        yield
    finally:
        codec.set_decode_kernel(prev)


def check_decode(torch, oracle_codec, data, off, n, names=None, base=0):
    """decode data[off[i]:off[i+1]] on the GPU and with the restatement; compare lengths, statuses and bytes"""
    g = gpu_decode(torch, data, off, n, is_name_bits=names)
    o = oracle_codec.decode_batch(data, off, n, is_name_bits=names, nthreads=8)
    np.testing.assert_array_equal(g[1], o[1])
    np.testing.assert_array_equal(g[2], o[2])
    slots = (off[:n].astype(np.uint64) * 8) // 5
    assert compact(g[0], slots, g[1]) == compact(o[0], slots, o[1])
    return g


def huffman_of(oracle_codec, plain):
    data, off = synth.pack(plain)
    o_out, o_len, _ = oracle_codec.encode_batch(data, off, len(plain), nthreads=8)
    return [o_out[int(off[i]):int(off[i]) + int(o_len[i])].tobytes() if o_len[i] != FAIL else plain[i]
            for i in range(len(plain))]


@pytest.mark.parametrize("name", GOLDEN_SETS)
def test_seg_golden(torch_cuda, name):  # noqa: F811
    g = load_golden(name)
    if "dec_len" not in g:
        pytest.skip("no decode vectors")
    n = len(g["dec_len"])
    with decode_kernel(2):
        out, out_len, status = gpu_decode(torch_cuda, g["dec_in"], g["dec_in_off"], n, is_name_bits=g["is_name_bits"])
    np.testing.assert_array_equal(out_len, g["dec_len"])
    np.testing.assert_array_equal(status, g["dec_status"])
    slots = (g["dec_in_off"][:n].astype(np.uint64) * 8) // 5
    assert compact(out, slots, out_len) == g["dec_out"].tobytes()


@pytest.mark.parametrize("cfg,n,seed", [("c2", 60000, 1), ("c3", 40000, 2), ("c4", 60000, 3), ("c5", 6000, 4)])
def test_seg_random_batches(torch_cuda, oracle_codec, cfg, n, seed):  # noqa: F811
    """every config's Huffman strings packed back to back (with 2 % corrupted), and the plain strings read as
    Huffman (mostly invalid: EOS, bad padding, long codes at every offset)"""
    b = synth.make_batch(cfg, n=n, seed=seed, adversarial_frac=0.02)
    rng = np.random.default_rng(seed)
    huff = huffman_of(oracle_codec, synth.unpack(b["data"], b["off"]))
    for j in rng.choice(n, n // 50, replace=False):
        h = bytearray(huff[j])
        k = int(rng.integers(4))
        if k == 0 and len(h) > 1:
            h = h[:int(rng.integers(1, len(h)))]
        elif k == 1 and h:
            h[int(rng.integers(len(h)))] ^= 1 << int(rng.integers(8))
        elif k == 2:
            h += b"\xff\xff\xff\xff"
        else:
            h += b"\x00"
        huff[j] = bytes(h)
    hdata, hoff = synth.pack(huff)
    with decode_kernel(2):
        g = check_decode(torch_cuda, oracle_codec, hdata, hoff, n, b["is_name_bits"])
        assert (g[1] != FAIL).sum() > 0.9 * n
        check_decode(torch_cuda, oracle_codec, b["data"], b["off"], n, b["is_name_bits"])


def test_seg_structure_edges(torch_cuda, oracle_codec):  # noqa: F811
    """tiles of many tiny strings (sub-tiles of 64, record overflow -> one lane per string), runs of empty
    strings (inside segments, at segment and span ends, whole tiles of them), last strings of 639..642 and
    thousands of bytes (kept, listed or decoded by one lane), periodic text"""
    rng = np.random.default_rng(41)
    syms, p = synth.header_alphabet()
    plain = []
    for blk in range(60):
        kind = blk % 6
        if kind == 0:  # 300 tiny strings (1..6 B): > 64 strings per tile, > 8 closes per lane
            plain += [bytes(rng.choice(syms, int(rng.integers(1, 7)), p=p)) for _ in range(300)]
        elif kind == 1:  # empties between, and in runs of 100
            for _ in range(40):
                plain += [b""] * int(rng.integers(0, 4))
                plain.append(bytes(rng.choice(syms, int(rng.integers(20, 300)), p=p)))
            plain += [b""] * 100
        elif kind == 2:  # strings around the 640-byte keep limit (Huffman), header text
            for L in (840, 850, 856, 860, 2000, 6000):
                plain.append(bytes(rng.choice(syms, L, p=p)))
                plain += [bytes(rng.choice(syms, int(rng.integers(30, 200)), p=p)) for _ in range(5)]
        elif kind == 3:  # periodic text: 5-bit codes in a fixed phase
            plain += [(b"a" * int(rng.integers(200, 700))), (b"0e" * int(rng.integers(100, 350))), b"aeiost" * 60]
        elif kind == 4:  # long codes only
            plain += [bytes(rng.choice(np.frombuffer(b"{}~^|<>\\\x00\x7f", np.uint8), int(rng.integers(10, 400))))
                      for _ in range(20)]
        else:  # Zipf lengths
            L = np.arange(8, 513)
            w = 1.0 / L
            plain += [bytes(rng.choice(syms, int(x), p=p)) for x in rng.choice(L, 200, p=w / w.sum())]
    huff = huffman_of(oracle_codec, plain)
    hdata, hoff = synth.pack(huff)
    n = len(huff)
    names = synth.bits_from_bools(rng.random(n) < 0.3)
    lens = np.diff(hoff)
    assert (lens > 640).sum() > 10 and (lens == 0).sum() > 500
    for mode in (2, 1):
        with decode_kernel(mode):
            g = check_decode(torch_cuda, oracle_codec, hdata, hoff, n, names)
    assert (g[1] != FAIL).sum() > 0.75 * n  # tiny strings often stay plain (not shorter): invalid Huffman
    # the same strings at a batch offset of 37 bytes, with a buffer longer than the strings
    pad = np.concatenate([rng.integers(0, 256, 37, dtype=np.uint8), hdata,
                          rng.integers(0, 256, 5000, dtype=np.uint8)]).astype(np.uint8)
    with decode_kernel(2):
        check_decode(torch_cuda, oracle_codec, pad, (hoff + 37).astype(np.uint32), n, names)


def test_seg_long_mixed_and_split_lists(torch_cuda, oracle_codec):  # noqa: F811
    """mean above 128 B (the split lists exist): strings of 4 KB - 370 KB among 0-900 B ones, corrupted
    long strings, periodic ones"""
    rng = np.random.default_rng(43)
    longs = _long_huffman_strings(oracle_codec, rng, [5200, 9000, 40000, 150000, 370000] +
                                  [int(x) for x in rng.integers(700, 30000, 30)])
    syms, p = synth.header_alphabet()
    short = huffman_of(oracle_codec, [bytes(rng.choice(syms, int(rng.integers(0, 900)), p=p)) for _ in range(3000)])
    mix = short[:1000] + longs[:15] + short[1000:2000] + longs[15:] + short[2000:]
    hdata, hoff = synth.pack(mix)
    n = len(mix)
    assert hdata.size // n > 128
    for mode in (1, 2):
        with decode_kernel(mode):
            check_decode(torch_cuda, oracle_codec, hdata, hoff, n, synth.bits_from_bools(rng.random(n) < 0.3))


def test_default_mode_c3(torch_cuda, oracle_codec):  # noqa: F811
    """mode 0 -- the default -- is the staged / stream choice; the segment kernel (modes 1, 2) is opt-in"""
    b = synth.make_batch("c3", n=30000, seed=5)
    huff = huffman_of(oracle_codec, synth.unpack(b["data"], b["off"]))
    hdata, hoff = synth.pack(huff)
    from h2o_amd import codec

    with decode_kernel(0):
        assert codec.set_decode_kernel(0) == 0
        check_decode(torch_cuda, oracle_codec, hdata, hoff, len(huff), b["is_name_bits"])
    with pytest.raises(codec.HhuffError):
        codec.set_decode_kernel(3)
