"""The multi-device batch (include/hhuff.h (3d), hhuff_{de,en}code_batch_multi): one batch over several GPUs of
one process, for h2o's C callers (lib/http2/hpack.c:241, lib/http3/qpack.c:228) -- SURVEY 2 new component 5, 8e.

CPU: the native byte-balanced cut (hhuff_shard_bounds) against the torch.distributed path's split
(h2o_amd/dist.py byte_balanced_bounds) for 1..8 shards, and its tile alignment.  GPU: every mode (device arrays
in place, device arrays through the peer-copy path -- HHUFF_MULTI_COPY=1 routes the source device's own shards
through it on a one-GPU box --, host arrays) equals the one-device call byte for byte, and the oracle."""
import os

import numpy as np
import pytest

from h2o_amd import synth

FAIL = 0xFFFFFFFF


def _offsets(rng, n, lo, hi, empty_frac=0.0):
    L = rng.integers(lo, hi + 1, n)
    L[rng.random(n) < empty_frac] = 0
    off = np.zeros(n + 1, np.uint32)
    off[1:] = np.cumsum(L)
    return off


@pytest.mark.parametrize("nshards", range(1, 9))
def test_shard_bounds_match_dist_split(nshards):
    import torch

    from h2o_amd import codec
    from h2o_amd import dist as hd

    rng = np.random.default_rng(100 + nshards)
    for n, lo, hi, ef in ((1, 5, 5, 0), (7, 0, 3, 0.5), (1000, 8, 512, 0), (5000, 24, 72, 0.1), (64, 0, 0, 0)):
        off = _offsets(rng, n, lo, hi, ef)
        got = codec.shard_bounds(off, n, nshards, align=1)
        want = hd.byte_balanced_bounds(torch.from_numpy(off.astype(np.int64)), nshards).numpy()
        np.testing.assert_array_equal(got.astype(np.int64), want, err_msg=str((n, lo, hi, nshards)))


def test_shard_bounds_tile_aligned_and_balanced():
    from h2o_amd import codec

    rng = np.random.default_rng(7)
    off = _offsets(rng, 1 << 20, 24, 72)
    n = off.size - 1
    for ns in (2, 3, 4, 5, 8):
        b = codec.shard_bounds(off, n, ns, align=64)
        assert b[0] == 0 and b[-1] == n and (np.diff(b.astype(np.int64)) >= 0).all()
        assert (b[1:-1] % 64 == 0).all()
        shard_bytes = np.diff(off[b].astype(np.int64))
        # one tile of at most 64 x 72 bytes off the exact quantile
        assert np.abs(shard_bytes - off[-1] / ns).max() <= 2 * 64 * 72
    # a batch with a start offset: the quantiles are of its own bytes
    off2 = (off[1000:2001] + 12345).astype(np.uint32)
    b = codec.shard_bounds(off2, 1000, 4, align=1)
    assert b[0] == 0 and b[-1] == 1000 and 200 < b[2] < 800


def test_multi_rejects_bad_arguments_without_a_gpu():
    from h2o_amd import codec

    L = codec.lib()
    p = 1 << 20
    assert L.hhuff_decode_batch_multi(0, None, -1, p, 1, p, 1, None, p, 16, p, p, None) == -1
    assert L.hhuff_encode_batch_multi(65, None, -1, p, 1, p, 1, p, 16, p, p, None) == -1
    assert b"ndev" in L.hhuff_last_error_string()
    assert L.hhuff_shard_bounds(None, 1, 2, 64, p) == -1
    assert L.hhuff_shard_bounds(p, 1, 0, 64, p) == -1


# ---------------------------------------------------------------------------------------------------
@pytest.fixture(scope="module")
def torch_cuda():
    import torch

    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    return torch


def _batch(cfg, n, seed):
    b = synth.make_batch(cfg, n=n, seed=seed, adversarial_frac=0.02)
    return b["data"], b["off"], b["is_name_bits"], b["n"]


def _kept(out, off, ln, decode):
    ok = ln != FAIL
    st = (off[:-1].astype(np.int64) * 8) // 5 if decode else off[:-1].astype(np.int64)
    return b"".join(out[s:s + L].tobytes() for s, L in zip(st[ok], ln[ok].astype(np.int64)))


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["device", "device_copy", "host"])
@pytest.mark.parametrize("devices", [[0], [0, 0], [0, 0, 0, 0, 0]])
def test_multi_equals_one_device(torch_cuda, oracle_codec, mode, devices):
    from h2o_amd import codec

    torch = torch_cuda
    data, off, names, n = _batch("c3", 40000, 5 + len(devices))
    P = int(off[n])
    dev = lambda a: torch.from_numpy(a.view(np.int32) if a.dtype == np.uint32 else a).cuda()  # noqa: E731
    e1, el1, es1 = codec.encode_batch(dev(data), dev(off), n)
    torch.cuda.synchronize()
    el1 = el1.cpu().numpy().view(np.uint32)[:n]
    e1 = e1.cpu().numpy()
    if mode == "device_copy":
        os.environ["HHUFF_MULTI_COPY"] = "1"
    try:
        if mode == "host":
            e2, el2, es2 = codec.encode_batch_multi(devices, data, off, n)
        else:
            e2, el2, es2 = codec.encode_batch_multi(devices, dev(data), dev(off), n)
            torch.cuda.synchronize()
            e2, el2, es2 = e2.cpu().numpy(), el2.cpu().numpy().view(np.uint32)[:n], es2.cpu().numpy()[:n]
        np.testing.assert_array_equal(el2, el1)
        np.testing.assert_array_equal(es2, es1.cpu().numpy()[:n])
        assert _kept(e2, off, el2, False) == _kept(e1, off, el1, False)
        oe, oel, _ = oracle_codec.encode_batch(data, off, n, nthreads=8)
        np.testing.assert_array_equal(el2, oel)
        assert _kept(e2, off, el2, False) == _kept(oe, off, oel, False)
        # decode of the wire (the compressible strings back to back) the same way
        ok = np.nonzero(el1 != FAIL)[0]
        huff = np.frombuffer(_kept(e1, off, el1, False), np.uint8).copy()
        h_off = np.zeros(ok.size + 1, np.uint32)
        h_off[1:] = np.cumsum(el1[ok].astype(np.int64))
        m = ok.size
        hn = synth.bits_from_bools(np.random.default_rng(9).random(m) < 0.3)
        d1, dl1, ds1 = codec.decode_batch(dev(huff), dev(h_off), m, is_name_bits=dev(hn))
        torch.cuda.synchronize()
        d1, dl1, ds1 = d1.cpu().numpy(), dl1.cpu().numpy().view(np.uint32)[:m], ds1.cpu().numpy()[:m]
        if mode == "host":
            d2, dl2, ds2 = codec.decode_batch_multi(devices, huff, h_off, m, is_name_bits=hn)
        else:
            d2, dl2, ds2 = codec.decode_batch_multi(devices, dev(huff), dev(h_off), m, is_name_bits=dev(hn))
            torch.cuda.synchronize()
            d2, dl2, ds2 = d2.cpu().numpy(), dl2.cpu().numpy().view(np.uint32)[:m], ds2.cpu().numpy()[:m]
        np.testing.assert_array_equal(dl2, dl1)
        np.testing.assert_array_equal(ds2, ds1)
        got = _kept(d2, h_off, dl2, True)
        assert got == _kept(d1, h_off, dl1, True)
        assert got == b"".join(data[off[i]:off[i + 1]].tobytes() for i in ok)
    finally:
        os.environ.pop("HHUFF_MULTI_COPY", None)


@pytest.mark.gpu
def test_multi_device_mode_is_stream_ordered(torch_cuda):
    """device mode returns once enqueued: the caller's stream waits for every shard (a copy queued behind the call
    on the same stream sees the results)"""
    from h2o_amd import codec

    torch = torch_cuda
    data, off, names, n = _batch("c4", 1 << 18, 77)
    d, o = torch.from_numpy(data).cuda(), torch.from_numpy(off.view(np.int32)).cuda()
    s = torch.cuda.Stream()
    os.environ["HHUFF_MULTI_COPY"] = "1"
    try:
        with torch.cuda.stream(s):
            out, ol, st = codec.encode_batch_multi([0, 0, 0], d, o, n, stream=s)
            snap = ol.clone()  # queued on s behind the multi call
    finally:
        os.environ.pop("HHUFF_MULTI_COPY", None)
    s.synchronize()
    ref = codec.encode_batch(d, o, n)[1]
    torch.cuda.synchronize()
    assert torch.equal(snap[:n], ref[:n])


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["device", "device_copy", "host"])
def test_multi_sub_batch_and_small_batches(torch_cuda, mode):
    """offsets that do not start at 0 (a sub-range of a larger buffer), batches smaller than a shard's 64-string
    unit (everything lands on the last device), and an encode without status: the one-device call's results"""
    from h2o_amd import codec

    torch = torch_cuda
    data, off, names, n = _batch("c2", 5000, 41)
    dev = lambda a: torch.from_numpy(a.view(np.int32) if a.dtype == np.uint32 else a).cuda()  # noqa: E731
    if mode == "device_copy":
        os.environ["HHUFF_MULTI_COPY"] = "1"
    try:
        for lo, m in ((37, 4000), (1000, 50), (0, 1), (4999, 1)):
            sub = np.ascontiguousarray(off[lo:lo + m + 1])
            e1, el1, _ = codec.encode_batch(dev(data), dev(sub), m, in_size=data.size)
            torch.cuda.synchronize()
            el1 = el1.cpu().numpy().view(np.uint32)[:m]
            e1 = e1.cpu().numpy()
            if mode == "host":
                out = np.zeros(data.size + 16, np.uint8)
                ln = np.zeros(m, np.uint32)
                rc = codec.lib().hhuff_encode_batch_multi(3, codec._devs([0, 0, 0])[1], codec.HOST_MEMORY,
                                                          data.ctypes.data, data.size, sub.ctypes.data, m,
                                                          out.ctypes.data, out.size, ln.ctypes.data, None, None)
                assert rc == 0, codec.lib().hhuff_last_error_string()
                e2, el2 = out, ln
            else:
                d_out = torch.empty(data.size + 16, dtype=torch.uint8, device="cuda")
                d_ln = torch.empty(m, dtype=torch.int32, device="cuda")
                dd, ds = dev(data), dev(sub)
                rc = codec.lib().hhuff_encode_batch_multi(3, codec._devs([0, 0, 0])[1], 0, dd.data_ptr(), data.size,
                                                          ds.data_ptr(), m, d_out.data_ptr(), d_out.numel(),
                                                          d_ln.data_ptr(), None, torch.cuda.current_stream().cuda_stream)
                assert rc == 0, codec.lib().hhuff_last_error_string()
                torch.cuda.synchronize()
                e2, el2 = d_out.cpu().numpy(), d_ln.cpu().numpy().view(np.uint32)
            np.testing.assert_array_equal(el2, el1)
            assert _kept(e2, sub, el2, False) == _kept(e1, sub, el1, False)
    finally:
        os.environ.pop("HHUFF_MULTI_COPY", None)
