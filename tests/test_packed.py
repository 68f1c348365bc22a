"""Packed output (include/hhuff.h hhuff_{de,en}code_batch_packed): the wave-prefix-compacted layout against
the reference's golden vectors and the CPU restatement, its tile structure, and that no byte outside the
outputs is written."""
import numpy as np
import pytest

from conftest import GOLDEN_SETS, compact, load_golden
from h2o_amd import synth

pytestmark = pytest.mark.gpu

FAIL = 0xFFFFFFFF
SENTINEL = 0xA5


@pytest.fixture(scope="module")
def torch_cuda():
    import torch

    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    return torch


def _dev(torch, a):
    a = np.ascontiguousarray(a)
    if a.dtype == np.uint32:
        a = a.view(np.int32)
    if a.size == 0:
        a = np.zeros(1, a.dtype)
    return torch.from_numpy(a.copy()).cuda()


def check_layout(in_off, n, out_len, out_off, dec):
    """tile t's run starts at its bound position and its strings follow each other back to back"""
    in_off = np.asarray(in_off, np.uint64)
    keep = np.where(out_len != FAIL, out_len, 0).astype(np.uint64)
    off = out_off.astype(np.uint64)
    bound = (in_off * 8) // 5 if dec else in_off
    for t0 in range(0, n, 64):
        t1 = min(n, t0 + 64)
        assert off[t0] == bound[t0], ("tile start", t0)
        exp = off[t0] + np.concatenate([[0], np.cumsum(keep[t0:t1])])
        assert (off[t0:t1] == exp[:-1]).all(), ("places", t0)
        if t1 == n:
            assert off[n] == exp[-1], "out_off[n]"
        else:  # runs never overlap the next tile's
            assert exp[-1] <= bound[t1]


def untouched(buf, out_off, out_len):
    mask = np.ones(buf.size, bool)
    for o, L in zip(out_off, out_len):
        if L != FAIL:
            mask[int(o):int(o) + int(L)] = False
    return bool((buf[mask] == SENTINEL).all())


def gpu_decode_packed(torch, data, off, n, names=None):
    from h2o_amd import codec

    size = int(np.asarray(data).size)
    out = torch.full((codec.decode_slot_size(size),), SENTINEL, dtype=torch.uint8, device="cuda")
    o, oo, ol, st = codec.decode_batch_packed(_dev(torch, data), _dev(torch, off), n,
                                              is_name_bits=None if names is None else _dev(torch, names), out=out,
                                              in_size=size)
    torch.cuda.synchronize()
    return (o.cpu().numpy(), oo.cpu().numpy().view(np.uint32)[:n + 1], ol.cpu().numpy().view(np.uint32)[:n],
            st.cpu().numpy()[:n])


def gpu_encode_packed(torch, data, off, n):
    from h2o_amd import codec

    size = int(np.asarray(data).size)
    out = torch.full((size + 16,), SENTINEL, dtype=torch.uint8, device="cuda")
    o, oo, ol, st = codec.encode_batch_packed(_dev(torch, data), _dev(torch, off), n, out=out, in_size=size)
    torch.cuda.synchronize()
    return (o.cpu().numpy(), oo.cpu().numpy().view(np.uint32)[:n + 1], ol.cpu().numpy().view(np.uint32)[:n],
            st.cpu().numpy()[:n])


@pytest.mark.parametrize("name", GOLDEN_SETS)
def test_packed_golden(torch_cuda, name):
    g = load_golden(name)
    if "dec_len" in g:
        n = len(g["dec_len"])
        out, oo, ol, st = gpu_decode_packed(torch_cuda, g["dec_in"], g["dec_in_off"], n, g["is_name_bits"])
        np.testing.assert_array_equal(ol, g["dec_len"])
        np.testing.assert_array_equal(st, g["dec_status"])
        assert compact(out, oo[:n], ol) == g["dec_out"].tobytes()
        check_layout(g["dec_in_off"], n, ol, oo, True)
        assert untouched(out, oo[:n], ol)
    if "enc_len" in g:
        n = len(g["enc_len"])
        out, oo, ol, st = gpu_encode_packed(torch_cuda, g["enc_in"], g["enc_in_off"], n)
        np.testing.assert_array_equal(ol, g["enc_len"])
        assert compact(out, oo[:n], ol) == g["enc_out"].tobytes()
        check_layout(g["enc_in_off"], n, ol, oo, False)
        assert untouched(out, oo[:n], ol)


# c3 / c5 / long strings reach the staged kernels with long stages and the scratch + pack_tiles path
@pytest.mark.parametrize("cfg,n,seed", [("c2", 60000, 1), ("c3", 30000, 2), ("c4", 60000, 3), ("c5", 4000, 4),
                                        (dict(n=3000, lengths=("uniform", 200, 900), alphabet="header"), 3000, 5)])
def test_packed_vs_oracle(torch_cuda, oracle_codec, cfg, n, seed):
    b = synth.make_batch(cfg, n=n, seed=seed, adversarial_frac=0.02)
    o_out, o_len, o_st = oracle_codec.encode_batch(b["data"], b["off"], n, nthreads=8)
    out, oo, ol, st = gpu_encode_packed(torch_cuda, b["data"], b["off"], n)
    np.testing.assert_array_equal(ol, o_len)
    np.testing.assert_array_equal(st, o_st)
    assert compact(out, oo[:n], ol) == compact(o_out, b["off"][:n], o_len)
    check_layout(b["off"], n, ol, oo, False)
    assert untouched(out, oo[:n], ol)
    # the wire: compressible strings back to back, decoded packed
    ok = np.nonzero(o_len != FAIL)[0]
    huff = [o_out[int(b["off"][i]):int(b["off"][i]) + int(o_len[i])].tobytes() for i in ok]
    rng = np.random.default_rng(seed)
    for j in rng.choice(len(huff), len(huff) // 50, replace=False):  # some invalid ones
        huff[j] = huff[j] + b"\x00" if j % 2 else huff[j][:-1]
    hdata, hoff = synth.pack(huff)
    m = len(huff)
    names = synth.bits_from_bools(rng.random(m) < 0.3)
    d = oracle_codec.decode_batch(hdata, hoff, m, is_name_bits=names, nthreads=8)
    out, oo, ol, st = gpu_decode_packed(torch_cuda, hdata, hoff, m, names)
    np.testing.assert_array_equal(ol, d[1])
    np.testing.assert_array_equal(st, d[2])
    slots = (hoff[:m].astype(np.uint64) * 8) // 5
    assert compact(out, oo[:m], ol) == compact(d[0], slots, d[1])
    check_layout(hoff, m, ol, oo, True)
    assert untouched(out, oo[:m], ol)


def test_packed_tiles_past_the_stage(torch_cuda, oracle_codec):
    """a tile whose input does not fit the LDS stage takes the count-then-place direct path: a few very long
    strings among short ones (mean length below the long-string threshold)"""
    rng = np.random.default_rng(9)
    syms, p = synth.header_alphabet()
    strings = [bytes(rng.choice(syms, int(rng.choice([5, 20, 40]) if i % 97 else 5000), p=p)) for i in range(20000)]
    strings[7] = b""
    data, off = synth.pack(strings)
    n = len(strings)
    o_out, o_len, _ = oracle_codec.encode_batch(data, off, n)
    out, oo, ol, _ = gpu_encode_packed(torch_cuda, data, off, n)
    np.testing.assert_array_equal(ol, o_len)
    assert compact(out, oo[:n], ol) == compact(o_out, off[:n], o_len)
    check_layout(off, n, ol, oo, False)
    assert untouched(out, oo[:n], ol)
    ok = np.nonzero(o_len != FAIL)[0]
    hdata, hoff = synth.pack([o_out[int(off[i]):int(off[i]) + int(o_len[i])].tobytes() for i in ok])
    m = len(ok)
    d = oracle_codec.decode_batch(hdata, hoff, m)
    out, oo, ol, st = gpu_decode_packed(torch_cuda, hdata, hoff, m)
    np.testing.assert_array_equal(ol, d[1])
    np.testing.assert_array_equal(st, d[2])
    assert compact(out, oo[:m], ol) == compact(d[0], (hoff[:m].astype(np.uint64) * 8) // 5, d[1])
    check_layout(hoff, m, ol, oo, True)


def test_packed_c4_full_size(torch_cuda):
    """16M strings: packed encode equals the slot-layout encode string by string; the packed wire decodes
    back to the plain strings (device-side checks)"""
    import torch

    from h2o_amd import codec

    b = synth.make_batch_torch("c4", seed=77)
    n, P = b["n"], int(b["total"])
    off32 = b["off"].to(torch.int32)
    lens = b["off"][1:] - b["off"][:-1]
    s_out, s_len, _ = codec.encode_batch(b["data"], off32, n, in_size=P)
    p_out, p_off, p_len, _ = codec.encode_batch_packed(b["data"], off32, n, in_size=P)
    assert bool((s_len == p_len).all())
    ok = s_len != -1
    keep = torch.where(ok, s_len, torch.zeros_like(s_len)).to(torch.int64)
    tot = int(keep.sum().item())
    seg = torch.repeat_interleave(torch.arange(n, device="cuda"), keep)
    rel = torch.arange(tot, device="cuda") - torch.repeat_interleave(torch.cumsum(keep, 0) - keep, keep)
    a = s_out[torch.repeat_interleave(b["off"][:-1], keep) + rel]
    pk = p_off.to(torch.int64) & 0xFFFFFFFF
    c = p_out[torch.repeat_interleave(pk[:-1], keep) + rel]
    assert bool((a == c).all())
    # tile structure: out_off[64 t] == in_off[64 t], places are the prefix sums inside a tile
    assert bool((pk[:-1][::64] == b["off"][:-1][::64]).all())
    # decode the compressible strings packed back to back (the wire) and compare with the plain input
    h_off = torch.zeros(int(ok.sum().item()) + 1, dtype=torch.int64, device="cuda")
    h_off[1:] = torch.cumsum(keep[ok], 0)
    wire = torch.empty(int(h_off[-1].item()) + 16, dtype=torch.uint8, device="cuda")
    wire[:tot] = c
    m = int(ok.sum().item())
    d_out, d_off, d_len, d_st = codec.decode_batch_packed(wire, h_off.to(torch.int32), m, in_size=tot)
    plain_len = lens[ok]
    assert bool((d_len.to(torch.int64) == plain_len).all())
    dk = plain_len
    dtot = int(dk.sum().item())
    drel = torch.arange(dtot, device="cuda") - torch.repeat_interleave(torch.cumsum(dk, 0) - dk, dk)
    got = d_out[torch.repeat_interleave(d_off[:-1].to(torch.int64) & 0xFFFFFFFF, dk) + drel]
    exp = b["data"][torch.repeat_interleave(b["off"][:-1][ok], dk) + drel]
    assert bool((got == exp).all())


def test_packed_edges_deferred(torch_cuda, oracle_codec):
    """the packed kernels with their shared 16-B chunks deferred to edge records and edge_fix_kernel
    (hhuff_set_edge_defer_min(0)); the default stores them in the kernels, one byte a lane"""
    from h2o_amd import codec

    prev = codec.set_edge_defer_min(0)
    try:
        for cfg, n, seed in [("c2", 20000, 11), ("c4", 20000, 13), ("c3", 8000, 12)]:
            test_packed_vs_oracle(torch_cuda, oracle_codec, cfg, n, seed)
        test_packed_tiles_past_the_stage(torch_cuda, oracle_codec)
    finally:
        codec.set_edge_defer_min(prev)
