"""Response header blocks as h2o's clients parse them (client side):
h2o_hpack_parse_response (lib/http2/hpack.c:642-750) per HPACK block -- response heads and trailers, as
lib/common/http2client.c:332 / :421 call it -- and h2o_qpack_parse_response (lib/http3/qpack.c:860-882) per
QPACK section, as lib/common/http3client.c:542 calls it.
CPU: the restatement (oracle/hpack_block.c orc_rs_field, oracle/qpack_decode.c) against tests/golden/resp.npz
(written by oracle/gen_golden.py resp_set from the reference's own functions, every QPACK section also checked
against the real h2o_qpack_parse_response) and, where oracle/_ref exists, against the reference on fresh
synthetic connections.  GPU: hhuff_hpack_parse_responses / hhuff_qpack_parse_responses through the C-ABI
against the same fixtures (verdicts, records -- status, header count, err_desc code, datagram flow id, Section
Acknowledgment -- and every field's name, value and flags) and against the restatement field by field."""
import numpy as np
import pytest

from conftest import load_golden
from h2o_amd import hpack_synth as HS
from h2o_amd import qpack_synth as QS

HSETS = ["h", "h256"]
DF = 0x30200  # H2O_HTTP3_ERROR_QPACK_DECOMPRESSION_FAILED


def hset(g, name):
    p = name + "_"
    return {k[len(p):]: v for k, v in g.items() if k.startswith(p)}


def qsteps(g):
    nconn, hts, mb, nsteps = (int(x) for x in g["q_meta"])
    steps = []
    for k in range(nsteps):
        p = "q_%d_" % k
        steps.append({key[len(p):]: v for key, v in g.items() if key.startswith(p)})
    return nconn, hts, mb, g["q_num_blocked"], steps


def fields_of(res, off, n):
    names, values, fl = [], [], []
    a = res["arena"]
    for k in range(n):
        s = int(off[k])
        for f in range(s, s + int(res["nfields"][k])):
            no, nl, vo, vl = (int(res[x][f]) for x in ("name_off", "name_len", "value_off", "value_len"))
            names.append(a[no:no + nl].tobytes())
            values.append(a[vo:vo + vl].tobytes())
            fl.append(int(res["fflags"][f]))
    return names, values, np.asarray(fl, np.uint8)


def expected_fields(s):
    n = len(s["fld_name_off"]) - 1
    names = [s["fld_name"][s["fld_name_off"][i]:s["fld_name_off"][i + 1]].tobytes() for i in range(n)]
    values = [s["fld_value"][s["fld_value_off"][i]:s["fld_value_off"][i + 1]].tobytes() for i in range(n)]
    return names, values, s["fflags"]


def words(rec, n, w):
    """records as [n, w] u32 words (numpy records or raw int32 / uint8 device rows)"""
    return np.ascontiguousarray(np.asarray(rec)[:n]).view(np.uint8).reshape(n, 4 * w).view(np.uint32)


def check_hpack(res, s):
    nb = len(s["blk_off"]) - 1
    np.testing.assert_array_equal(np.asarray(res["nfields"][:nb]).astype(np.uint32), s["nfields"], err_msg="nfields")
    np.testing.assert_array_equal(np.asarray(res["bstatus"][:nb]).astype(np.int32), s["bstatus"], err_msg="bstatus")
    np.testing.assert_array_equal(words(res["res"], nb, 4), s["res"], err_msg="response records")
    names, values, fl = fields_of(res, s["blk_off"], nb)
    en, ev, ef = expected_fields(s)
    assert names == en
    assert values == ev
    np.testing.assert_array_equal(fl, ef, err_msg="field flags (soft bits | HHUFF_FIELD_HEADER)")


def check_qpack_step(res, st, nconn):
    ns = len(st["sec_off"]) - 1
    for k in ("nfields", "sstatus", "req_insert_count"):
        np.testing.assert_array_equal(np.asarray(res[k][:ns]).astype(st[k].dtype), st[k], err_msg=k)
    for k in ("enc_status", "enc_consumed", "insert_count"):
        np.testing.assert_array_equal(np.asarray(res[k][:nconn]).astype(st[k].dtype), st[k], err_msg=k)
    np.testing.assert_array_equal(words(res["res"], ns, 10), st["res"], err_msg="response records")
    names, values, fl = fields_of(res, st["sec_off"], ns)
    en, ev, ef = expected_fields(st)
    assert names == en
    assert values == ev
    np.testing.assert_array_equal(fl, ef, err_msg="field flags")


def oracle_qpack(codec_lib, nconn, hts, mb, nbl, steps):
    from oracle import oracle as O

    s = O.QpackSession(codec_lib, nconn, hts, mb)
    try:
        return [s.step(st["data"], st["enc_off"], st["enc_len"], st["sec_off"], st["conn_first"], st["arena_off"], nbl,
                       stream_id=st["stream_id"], responses=True) for st in steps]
    finally:
        s.close()


# ---------------------------------------------------------------------------------------------- CPU
@pytest.mark.parametrize("name", HSETS)
def test_restatement_matches_reference_fixtures_hpack(oracle_codec, name):
    s = hset(load_golden("resp"), name)
    res = oracle_codec.hpack_decode_blocks(s["data"], s["blk_off"], s["conn_first"], int(s["table_size"][0]),
                                           nthreads=8, responses=True, trailers=s["trailers"])
    check_hpack(res, s)


def test_restatement_matches_reference_fixtures_qpack(oracle_codec):
    nconn, hts, mb, nbl, steps = qsteps(load_golden("resp"))
    for res, st in zip(oracle_qpack(oracle_codec, nconn, hts, mb, nbl, steps), steps):
        check_qpack_step(res, st, nconn)


def test_fixtures_cover_the_rules():
    g = load_golden("resp")
    s = hset(g, "h")
    rec = s["res"]
    errs = set(rec[:, 2].tolist())
    for e in (0, 1, 2, 3, 4, 6, 7, 9):  # HHUFF_HERR_*: none, soft name/value, too long, pseudo, conn-specific,
        assert e in errs, e            # upper-case raw name, missing :status
    st = set(s["bstatus"].tolist())
    for v in (0, -254, -1, -9, -301):
        assert v in st, v
    tr = s["trailers"] != 0
    assert tr.sum() > 100 and (rec[tr, 0] == 0).all()  # trailers never carry a status
    heads_ok = (~tr) & (s["bstatus"] == 0)
    assert set(rec[heads_ok, 0].tolist()) >= {200, 204, 304, 404, 500}
    # a :status that failed after its first digits keeps them (PARSE_DIGIT); an empty trailers block fails in
    # decode_header (COMPRESSION)
    assert ((s["bstatus"] == -1) & (rec[:, 0] != 0) & (rec[:, 2] == 4)).any()
    empty = np.diff(s["blk_off"].astype(np.int64)) == 0
    assert (empty & tr & (s["bstatus"] == -9)).any() and (empty & ~tr & (rec[:, 2] == 9)).any()
    assert int(s["nfields"].max()) > 1000
    # HTTP/3: acks only after a clean parse, soft errors without one, normalised hard errors
    _, _, _, _, steps = qsteps(g)
    q = np.concatenate([st["res"] for st in steps])
    qs = np.concatenate([st["sstatus"] for st in steps])
    assert ((qs == 0) & (q[:, 4] > 0)).any() and (q[qs != 0, 4] == 0).all()
    assert (qs == -254).any() and (qs == DF).any() and (qs == -302).any()
    assert ((q[:, 3].astype(np.int32)) >= 0).any()  # a datagram flow id stored
    assert set(q[:, 2].tolist()) >= {0, 2, 4, 6, 9}


def test_restatement_matches_compiled_reference_on_fresh_connections(oracle_codec):
    from oracle import oracle as O

    if not O.ref_available():
        pytest.skip("oracle/_ref not built (no /root/reference here)")
    for seed, ts in ((51, 4096), (52, 256), (53, 0)):
        b = HS.make_response_connections(1200, seed=seed, table_size=ts, adversarial_frac=0.1, rule_frac=0.3)
        r1 = O.ref().hpack_decode_blocks(b["data"], b["blk_off"], b["conn_first"], ts, responses=True,
                                         trailers=b["trailers"])
        r2 = oracle_codec.hpack_decode_blocks(b["data"], b["blk_off"], b["conn_first"], ts, nthreads=8,
                                              responses=True, trailers=b["trailers"])
        nb = len(b["blk_off"]) - 1
        for k in ("nfields", "bstatus"):
            np.testing.assert_array_equal(r1[k][:nb], r2[k][:nb], err_msg=k)
        np.testing.assert_array_equal(words(r1["res"], nb, 4), words(r2["res"], nb, 4))
        assert fields_of(r1, b["blk_off"], nb)[2].tolist() == fields_of(r2, b["blk_off"], nb)[2].tolist()
    nconn = 300
    steps = QS.make_session(nconn, steps=3, seed=54, adversarial_frac=0.1, request_frac=0.4, responses=True)
    for k, st in enumerate(steps):
        st["arena_off"] = QS.arena_offsets(st["sec_off"], 4096)
        st["stream_id"] = np.arange(len(st["sec_off"]) - 1, dtype=np.uint64) * 4 + 4096 * k
    nbl = (np.arange(nconn) % 3).astype(np.uint32)
    for a, b_, st in zip(oracle_qpack(O.ref(), nconn, 4096, 2, nbl, steps),
                         oracle_qpack(oracle_codec, nconn, 4096, 2, nbl, steps), steps):
        ns = len(st["sec_off"]) - 1
        for key in ("nfields", "sstatus", "req_insert_count"):
            np.testing.assert_array_equal(a[key][:ns], b_[key][:ns], err_msg=key)
        np.testing.assert_array_equal(words(a["res"], ns, 10), words(b_["res"], ns, 10))


# ---------------------------------------------------------------------------------------------- GPU
@pytest.fixture(scope="module")
def torch_cuda():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch


def _dev(torch, a):
    return torch.from_numpy(np.ascontiguousarray(a).copy()).cuda()


def gpu_hpack(torch, data, blk_off, conn_first, table_size, trailers):
    from h2o_amd import codec

    d = _dev(torch, data if data.size else np.zeros(1, np.uint8))
    r = codec.hpack_decode_blocks(d, _dev(torch, blk_off.view(np.int32)), _dev(torch, conn_first.view(np.int32)),
                                  table_size, in_size=int(data.size), responses=True,
                                  trailers=None if trailers is None else _dev(torch, trailers))
    torch.cuda.synchronize()
    out = {}
    for k, v in r.items():
        if k == "scratch":
            continue
        a = v.cpu().numpy()
        out[k] = a.view(np.uint32) if k in ("name_off", "name_len", "value_off", "value_len", "nfields") else a
    return out


def gpu_qpack(torch, nconn, hts, mb, nbl, steps):
    from h2o_amd import codec

    u32 = lambda a: _dev(torch, np.asarray(a, np.uint32).view(np.int32))  # noqa: E731
    out, scratch = [], None
    for k, st in enumerate(steps):
        data = st["data"] if st["data"].size else np.zeros(1, np.uint8)
        r = codec.qpack_decode(_dev(torch, data), u32(st["enc_off"]), u32(st["enc_len"]), u32(st["sec_off"]),
                               u32(st["conn_first"]), int(st["conn_first"][-1]), hts, mb, num_blocked=u32(nbl),
                               arena_off=_dev(torch, np.asarray(st["arena_off"], np.uint64).view(np.int64)),
                               in_size=int(st["data"].size), scratch=scratch, cont=k > 0,
                               stream_id=_dev(torch, np.asarray(st["stream_id"], np.uint64).view(np.int64)),
                               responses=True)
        torch.cuda.synchronize()
        scratch = r["scratch"]
        h = {}
        for key, v in r.items():
            if key == "scratch":
                continue
            a = v.cpu().numpy()
            if key in ("name_off", "name_len", "value_off", "value_len", "nfields", "enc_consumed"):
                a = a.view(np.uint32)
            elif key in ("req_insert_count", "insert_count"):
                a = a.view(np.uint64)
            h[key] = a
        out.append(h)
    return out


@pytest.mark.gpu
@pytest.mark.parametrize("name", HSETS)
def test_gpu_hpack_responses_match_reference_fixtures(torch_cuda, name):
    s = hset(load_golden("resp"), name)
    res = gpu_hpack(torch_cuda, s["data"], s["blk_off"], s["conn_first"], int(s["table_size"][0]), s["trailers"])
    check_hpack(res, s)


@pytest.mark.gpu
def test_gpu_qpack_responses_match_reference_fixtures(torch_cuda):
    nconn, hts, mb, nbl, steps = qsteps(load_golden("resp"))
    for res, st in zip(gpu_qpack(torch_cuda, nconn, hts, mb, nbl, steps), steps):
        check_qpack_step(res, st, nconn)


@pytest.mark.gpu
@pytest.mark.parametrize("seed,table_size,trailers", [(61, 4096, True), (62, 256, True), (63, 0, False)])
def test_gpu_hpack_responses_match_restatement(torch_cuda, oracle_codec, seed, table_size, trailers):
    b = HS.make_response_connections(3000, seed=seed, table_size=table_size, adversarial_frac=0.1, rule_frac=0.3)
    tr = b["trailers"] if trailers else None
    ro = oracle_codec.hpack_decode_blocks(b["data"], b["blk_off"], b["conn_first"], table_size, nthreads=8,
                                          responses=True, trailers=tr)
    rg = gpu_hpack(torch_cuda, b["data"], b["blk_off"], b["conn_first"], table_size, tr)
    nb = len(b["blk_off"]) - 1
    for k in ("nfields", "bstatus"):
        np.testing.assert_array_equal(rg[k][:nb], ro[k][:nb], err_msg=k)
    np.testing.assert_array_equal(words(rg["res"], nb, 4), words(ro["res"], nb, 4))
    for blk in range(nb):
        s0, n = int(b["blk_off"][blk]), int(ro["nfields"][blk])
        for k in ("name_off", "name_len", "value_off", "value_len", "fflags"):
            np.testing.assert_array_equal(rg[k][s0:s0 + n], ro[k][s0:s0 + n], err_msg="%s block %d" % (k, blk))


@pytest.mark.gpu
def test_gpu_qpack_responses_match_restatement(torch_cuda, oracle_codec):
    nconn, hts, mb = 1500, 4096, 2
    steps = QS.make_session(nconn, steps=3, seed=64, header_table_size=hts, adversarial_frac=0.1, request_frac=0.4,
                            responses=True)
    for k, st in enumerate(steps):
        st["arena_off"] = QS.arena_offsets(st["sec_off"], hts)
        st["stream_id"] = (np.arange(len(st["sec_off"]) - 1, dtype=np.uint64) * 4 + (1 << 20) * k) << (7 * (k % 3))
    nbl = (np.arange(nconn) % 4).astype(np.uint32)
    ro = oracle_qpack(oracle_codec, nconn, hts, mb, nbl, steps)
    rg = gpu_qpack(torch_cuda, nconn, hts, mb, nbl, steps)
    for a, g, st in zip(ro, rg, steps):
        ns = len(st["sec_off"]) - 1
        for k in ("nfields", "sstatus", "req_insert_count"):
            np.testing.assert_array_equal(g[k][:ns], a[k][:ns], err_msg=k)
        np.testing.assert_array_equal(words(g["res"], ns, 10), words(a["res"], ns, 10))
        for s_ in range(ns):
            o, n = int(st["sec_off"][s_]), int(a["nfields"][s_])
            for k in ("name_off", "name_len", "value_off", "value_len", "fflags"):
                np.testing.assert_array_equal(g[k][o:o + n], a[k][o:o + n], err_msg="%s section %d" % (k, s_))
