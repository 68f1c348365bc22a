"""Pin the CPU restatement (oracle/huff_oracle.c) to the reference's golden vectors (tests/golden/,
produced by the compiled reference via oracle/gen_golden.py), and to the reference itself when present."""
import numpy as np
import pytest

from conftest import GOLDEN_SETS, load_golden
from h2o_amd import synth


def _golden_out(g, prefix):
    return synth.unpack(g[prefix + "_out"], g[prefix + "_out_off"])


@pytest.mark.parametrize("name", GOLDEN_SETS)
def test_oracle_decode_matches_golden(oracle_codec, name):
    g = load_golden(name)
    if "dec_len" not in g:
        pytest.skip("no decode vectors")
    n = len(g["dec_len"])
    out, out_len, status = oracle_codec.decode_batch(g["dec_in"], g["dec_in_off"], n, is_name_bits=g["is_name_bits"],
                                                     nthreads=4)
    np.testing.assert_array_equal(out_len, g["dec_len"])
    np.testing.assert_array_equal(status, g["dec_status"])
    slots = (g["dec_in_off"][:n].astype(np.uint64) * 8) // 5
    got = [out[s:s + L].tobytes() for s, L in zip(slots, out_len) if L != 0xFFFFFFFF]
    assert got == _golden_out(g, "dec")


@pytest.mark.parametrize("name", GOLDEN_SETS)
def test_oracle_encode_matches_golden(oracle_codec, name):
    g = load_golden(name)
    if "enc_len" not in g:
        pytest.skip("no encode vectors")
    n = len(g["enc_len"])
    out, out_len, status = oracle_codec.encode_batch(g["enc_in"], g["enc_in_off"], n, nthreads=4)
    np.testing.assert_array_equal(out_len, g["enc_len"])
    np.testing.assert_array_equal(status, np.where(g["enc_len"] == 0xFFFFFFFF, 0x80, 0).astype(np.uint8))
    got = [out[s:s + L].tobytes() for s, L in zip(g["enc_in_off"][:n], out_len) if L != 0xFFFFFFFF]
    assert got == _golden_out(g, "enc")


def test_oracle_soft_errors_are_or_accumulated(oracle_codec):
    """*soft_errors is OR-ed, never cleared, and untouched on SIZE_MAX (hpack.c:117-156)."""
    g = load_golden("adversarial")
    strings = synth.unpack(g["dec_in"], g["dec_in_off"])
    names = np.unpackbits(g["is_name_bits"].view(np.uint8), bitorder="little")[:len(strings)]
    for s, nm, exp in list(zip(strings, names, g["dec_soft_preset"]))[:2000]:
        _, soft = oracle_codec.decode(s, bool(nm), soft_in=0x2 if nm else 0x1)
        assert soft == exp


def test_oracle_kats(oracle_codec):
    o = oracle_codec
    assert o.decode(bytes.fromhex("f1e3c2e5f23a6ba0ab90f4ff")) == (b"www.example.com", 0)
    assert o.encode(b"www.example.com") == bytes.fromhex("f1e3c2e5f23a6ba0ab90f4ff")
    assert o.encode(b"aaa") == bytes.fromhex("18c7")
    assert o.encode(b"ABCDEFGH") == bytes.fromhex("86edebf830e2c7")
    assert o.encode(b"") is None and o.encode(b"a") is None and o.encode(b"XXXXXXXX") is None
    assert o.decode(b"", True) == (b"", 1)
    assert o.decode(b"\xff") == (None, 0)
    assert o.decode(b"\x1f") == (b"a", 0)
    assert o.decode(bytes.fromhex("5071ff")) == (b" ab", 2)


def test_oracle_framing_matches_golden(oracle_codec):
    g = load_golden("framing")
    strings = synth.unpack(g["fr_in"], g["fr_in_off"])
    hp = synth.unpack(g["hpack_out"], g["hpack_out_off"])
    qp = synth.unpack(g["qpack_out"], g["qpack_out_off"])
    for s, pb, fb, raw, h, q in zip(strings, g["fr_prefix"], g["fr_first"], g["fr_raw"], hp, qp):
        assert oracle_codec.encode_string(s) == h
        assert oracle_codec.flatten_string(s, int(pb), int(fb), bool(raw)) == q
    ints = synth.unpack(g["int_out"], g["int_out_off"])
    k = 0
    for pb in (3, 4, 5, 6, 7):
        for v in g["int_values"]:
            enc = oracle_codec.encode_int(int(v), pb)
            assert enc == ints[k]
            assert oracle_codec.decode_int(enc, pb) == (int(v), len(enc))
            k += 1


def test_oracle_matches_reference_directly():
    """Fresh seeded strings through both the restatement and the compiled reference (container only)."""
    from oracle import oracle as O

    if not O.ref_available():
        pytest.skip("oracle/_ref not built (no /root/reference here)")
    o, r = O.oracle(), O.ref()
    b = synth.make_batch("c3", n=3000, seed=909, adversarial_frac=0.1)
    n = b["n"]
    eo, el, _ = o.encode_batch(b["data"], b["off"], n)
    ro, rl, _ = r.encode_batch(b["data"], b["off"], n)
    np.testing.assert_array_equal(el, rl)
    ok = el != 0xFFFFFFFF
    for i in np.nonzero(ok)[0]:
        s = b["off"][i]
        assert eo[s:s + el[i]].tobytes() == ro[s:s + rl[i]].tobytes()
    for data, off in ((eo, b["off"]), (b["data"], b["off"])):
        lens = np.where(ok, el, 0).astype(np.uint32) if data is eo else None
        d1 = o.decode_batch(data, off[:-1].copy() if lens is not None else off, n, in_len=lens,
                            is_name_bits=b["is_name_bits"])
        d2 = r.decode_batch(data, off[:-1].copy() if lens is not None else off, n, in_len=lens,
                            is_name_bits=b["is_name_bits"])
        np.testing.assert_array_equal(d1[1], d2[1])
        np.testing.assert_array_equal(d1[2], d2[2])


# ------------------------------------------------------------------------------------------------
# string literals (decode_string / QPACK literal decode), tests/golden/literals.npz
# ------------------------------------------------------------------------------------------------
def literal_cases(g):
    """(name, in, lit_off, lit_end, prefix_bits, qpack, names, expected dict) for every literal set"""
    n = len(g["h_out_len"])
    yield ("hpack", g["lit_in"], g["lit_off"], g["lit_end"], 7, False, g["lit_names"],
           dict(out_len=g["h_out_len"], pay_off=g["h_pay_off"], consumed=g["h_consumed"], status=g["h_status"],
                out=g["h_out"]), n)
    for pb in (3, 5, 7):
        k = "q%d_" % pb
        yield ("qpack%d" % pb, g["q_in"], g[k + "off"], g[k + "end"], pb, True, g[k + "names"],
               dict(out_len=g[k + "out_len"], pay_off=g[k + "pay_off"], consumed=g[k + "consumed"],
                    status=g[k + "status"], out=g[k + "out"]), len(g[k + "off"]))


def literal_concat(out, pay_off, out_len):
    slots = (pay_off.astype(np.uint64) * 8) // 5
    return b"".join(out[int(a):int(a) + int(L)].tobytes() for a, L in zip(slots, out_len) if L != 0xFFFFFFFF)


def test_oracle_literals_match_golden(oracle_codec):
    g = load_golden("literals")
    assert int(g["n_corpus"][0]) > 40000  # every literal of the fuzz corpus's HPACK blocks
    for name, data, off, end, pb, qp, names, exp, n in literal_cases(g):
        out, ol, po, cons, st = oracle_codec.literals_batch(data, off, end, n, pb, qpack=qp, is_name_bits=names,
                                                            nthreads=4)
        np.testing.assert_array_equal(ol, exp["out_len"], err_msg=name)
        np.testing.assert_array_equal(po, exp["pay_off"], err_msg=name)
        np.testing.assert_array_equal(cons, exp["consumed"], err_msg=name)
        np.testing.assert_array_equal(st, exp["status"], err_msg=name)
        assert literal_concat(out, po, ol) == exp["out"].tobytes(), name
    # every verdict the API defines is exercised by the fixture
    codes = set(((g["h_status"][g["h_status"] >= 0x80] >> 2) & 7).tolist())
    assert {1, 2, 3, 4, 5} <= codes


def test_adversarial_encode_fixture_covers_the_rules():
    """the reference's encode verdicts in adversarial.npz: every 'X'-only string stays raw ('X' is an 8-bit code,
    never shorter: t/40http3/test.pl:194), and both sides of hpack.c:799-800's edge occur (a string whose code
    bits are 8 len - 8 compresses to len - 1 bytes, one at 8 len - 7 .. 8 len does not)"""
    g = load_golden("adversarial")
    strings = synth.unpack(g["enc_in"], g["enc_in_off"])
    el = g["enc_len"]
    xs = [i for i, s in enumerate(strings) if s and set(s) == {ord("X")}]
    assert len(xs) > 10 and all(el[i] == 0xFFFFFFFF for i in xs)
    from h2o_amd import tables as T

    nb = np.asarray(T.ENC_NBITS)
    edge_ok = edge_fail = 0
    for s, L in zip(strings, el):
        if not s:
            continue
        bits = int(nb[np.frombuffer(s, np.uint8)].sum())
        if bits == 8 * len(s) - 8:
            assert L == len(s) - 1
            edge_ok += 1
        elif 8 * len(s) - 7 <= bits <= 8 * len(s):
            assert L == 0xFFFFFFFF
            edge_fail += 1
    assert edge_ok > 0 and edge_fail > 0
