"""QPACK decoder (QPACK half): h2o_qpack_decoder_handle_input over each connection's encoder
stream, then its field sections the way h2o_qpack_parse_request reads them (parse_decode_context,
check_decode_context_blocked, decode_header field after field), one dynamic table per connection kept across
steps.  CPU: the restatement (oracle/qpack_decode.c) against the reference's outputs (tests/golden/qpack.npz,
written by oracle/gen_golden.py from h2o's own qpack.c) and, where oracle/_ref exists, against the reference
directly on fresh synthetic sessions.  GPU: hhuff_qpack_decode through the C-ABI against the same fixtures
(every step, tables carried over with HHUFF_QPK_CONTINUE) and against the restatement field by field.
HTTP/3 requests (hhuff_qpack_parse_requests): every section also through h2o_qpack_parse_request
(qpack.c:830-858) -- the fixtures' rq_* arrays come from the reference harness, which checks each section
against the real function -- verdicts, request records (hhuff_qpack_request_t), Section Acknowledgments and
the fields' header-list flags."""
import numpy as np
import pytest

from conftest import load_golden
from h2o_amd import qpack_synth as QS

SESSIONS = ["q4096", "q256", "q0", "qreq", "qedge"]
DF = 0x30200  # H2O_HTTP3_ERROR_QPACK_DECOMPRESSION_FAILED
SEC_KEYS = ("nfields", "sstatus", "req_insert_count")
CONN_KEYS = ("enc_status", "enc_consumed", "insert_count")


def soft_code(bits):
    """decode_header reports one soft error per field (err_desc, qpack.c:744-749): name first"""
    bits = np.asarray(bits)
    return np.where(bits & 1, 1, np.where(bits & 2, 2, 0)).astype(np.uint8)


def fields_of(res, sec_off, nsec):
    names, values, soft = [], [], []
    a = res["arena"]
    for k in range(nsec):
        s = int(sec_off[k])
        for f in range(s, s + int(res["nfields"][k])):
            no, nl, vo, vl = (int(res[x][f]) for x in ("name_off", "name_len", "value_off", "value_len"))
            names.append(a[no:no + nl].tobytes())
            values.append(a[vo:vo + vl].tobytes())
            soft.append(int(res["fflags"][f]))
    return names, values, np.asarray(soft, np.uint8)


def golden_steps(g, name):
    nconn, hts, mb, nsteps = (int(x) for x in g[name + "_meta"])
    steps = []
    for k in range(nsteps):
        p = "%s_%d_" % (name, k)
        steps.append({key[len(p):]: v for key, v in g.items() if key.startswith(p)})
    return nconn, hts, mb, g[name + "_num_blocked"], steps


def check_step(res, st, nconn):
    ns = len(st["sec_off"]) - 1
    for k in SEC_KEYS:
        np.testing.assert_array_equal(np.asarray(res[k][:ns]).astype(st[k].dtype), st[k], err_msg=k)
    for k in CONN_KEYS:
        np.testing.assert_array_equal(np.asarray(res[k][:nconn]).astype(st[k].dtype), st[k], err_msg=k)
    names, values, soft = fields_of(res, st["sec_off"], ns)
    n = len(st["fld_name_off"]) - 1
    en = [st["fld_name"][st["fld_name_off"][i]:st["fld_name_off"][i + 1]].tobytes() for i in range(n)]
    ev = [st["fld_value"][st["fld_value_off"][i]:st["fld_value_off"][i + 1]].tobytes() for i in range(n)]
    assert names == en
    assert values == ev
    np.testing.assert_array_equal(soft_code(soft), st["fld_soft"])


def run_oracle_session(codec_lib, nconn, hts, mb, nbl, steps, requests=False):
    from oracle import oracle as O

    s = O.QpackSession(codec_lib, nconn, hts, mb)
    try:
        return [s.step(st["data"], st["enc_off"], st["enc_len"], st["sec_off"], st["conn_first"], st["arena_off"], nbl,
                       stream_id=st["rq_stream_id"] if requests else None)
                for st in steps]
    finally:
        s.close()


def req_words(req, ns):
    """request records as [ns, 18] u32 words (from QREQ_DTYPE records or raw 72-byte rows)"""
    a = np.ascontiguousarray(np.asarray(req)[:ns])
    return a.view(np.uint8).reshape(ns, 72).view(np.uint32)


def check_request_step(res, st):
    ns = len(st["sec_off"]) - 1
    np.testing.assert_array_equal(np.asarray(res["nfields"][:ns]).astype(np.uint32), st["rq_nfields"], err_msg="nfields")
    np.testing.assert_array_equal(np.asarray(res["sstatus"][:ns]).astype(np.int32), st["rq_sstatus"], err_msg="sstatus")
    got = req_words(res["req"], ns)
    for k in range(ns):  # the record; unset fields of a section that never reached the rules are as reset
        np.testing.assert_array_equal(got[k], st["rq_req"][k], err_msg="request record of section %d" % k)
    fl = []
    for k in range(ns):
        o = int(st["sec_off"][k])
        fl += list(np.asarray(res["fflags"][o:o + int(st["rq_nfields"][k])]))
    np.testing.assert_array_equal(np.asarray(fl, np.uint8), st["rq_fflags"], err_msg="fflags")


@pytest.mark.parametrize("name", SESSIONS)
def test_restatement_requests_match_reference_fixtures(oracle_codec, name):
    nconn, hts, mb, nbl, steps = golden_steps(load_golden("qpack"), name)
    for res, st in zip(run_oracle_session(oracle_codec, nconn, hts, mb, nbl, steps, requests=True), steps):
        check_request_step(res, st)


def test_request_fixtures_cover_the_rules():
    """every h2o_qpack_parse_request outcome the reference produced: all verdicts, the err_desc codes of the
    rules (soft name / value, headers too long, invalid pseudo-header, content-length, connection-specific
    -- cache-digest included for HTTP/3 -- and decode_header's own), all scheme kinds, stored
    datagram-flow-ids, and acknowledgments of 1 to 9 bytes"""
    g = load_golden("qpack")
    st, err, sk, acks, dfid, hdr = set(), set(), set(), set(), 0, 0
    for name in SESSIONS:
        _, _, _, _, steps = golden_steps(g, name)
        for s in steps:
            st |= set(int(x) for x in s["rq_sstatus"])
            w = s["rq_req"]
            err |= set(int(x) for x in w[:, 10])
            sk |= set(int(x) for x in w[:, 11])
            acks |= set(int(x) for x in w[:, 13])
            dfid += int((w[:, 12].view(np.int32) >= 0).sum())
            hdr += int(((s["rq_fflags"] & 4) != 0).sum())
    assert {0, -254, DF, -301, -302} <= st
    assert {0, 1, 2, 3, 4, 5, 6, 8} <= err
    assert {0, 1, 2, 3} <= sk
    assert set(range(10)) <= acks
    assert dfid > 0 and hdr > 10000


def test_restatement_requests_match_compiled_reference_on_fresh_sessions():
    from oracle import oracle as O

    if not O.ref_available():
        pytest.skip("oracle/_ref not built (no /root/reference here)")
    for seed, hts, mb in ((91, 4096, 4), (92, 256, 1), (93, 0, 0)):
        nconn = 150
        steps = QS.make_session(nconn, steps=3, seed=seed, header_table_size=hts, adversarial_frac=0.1, request_frac=0.4)
        for k, st in enumerate(steps):
            st["arena_off"] = QS.arena_offsets(st["sec_off"], hts)
            st["rq_stream_id"] = np.arange(len(st["sec_off"]) - 1, dtype=np.uint64) * 4 + 4000 * k
        nbl = (np.arange(nconn) % 5).astype(np.uint32)
        ro = run_oracle_session(O.oracle(), nconn, hts, mb, nbl, steps, requests=True)
        rr = run_oracle_session(O.ref(), nconn, hts, mb, nbl, steps, requests=True)  # checked against the real function
        for a, b, st in zip(ro, rr, steps):
            ns = len(st["sec_off"]) - 1
            for k in ("nfields", "sstatus"):
                np.testing.assert_array_equal(a[k][:ns], b[k][:ns])
            np.testing.assert_array_equal(req_words(a["req"], ns), req_words(b["req"], ns))
            for s_ in range(ns):
                o, n = int(st["sec_off"][s_]), int(a["nfields"][s_])
                np.testing.assert_array_equal(a["fflags"][o:o + n] & 4, b["fflags"][o:o + n] & 4)


@pytest.mark.parametrize("name", SESSIONS)
def test_restatement_matches_reference_fixtures(oracle_codec, name):
    nconn, hts, mb, nbl, steps = golden_steps(load_golden("qpack"), name)
    for res, st in zip(run_oracle_session(oracle_codec, nconn, hts, mb, nbl, steps), steps):
        check_step(res, st, nconn)


def test_fixtures_cover_the_paths():
    g = load_golden("qpack")
    st, es, soft, nf = set(), set(), [], 0
    for name in SESSIONS:
        _, _, _, _, steps = golden_steps(g, name)
        for s in steps:
            st |= set(int(x) for x in s["sstatus"])
            es |= set(int(x) for x in s["enc_status"])
            soft += list(s["fld_soft"])
            nf += int(s["nfields"].sum())
    assert {0, DF, -301, -302} <= st  # ok, decompression failed, skipped after an encoder error, blocked
    assert {0, DF, -301} <= es
    assert 1 in soft and 2 in soft
    assert nf > 30000


def test_restatement_matches_compiled_reference_on_fresh_sessions():
    from oracle import oracle as O

    if not O.ref_available():
        pytest.skip("oracle/_ref not built (no /root/reference here)")
    for seed, hts, mb in ((71, 4096, 4), (72, 256, 1), (73, 0, 0), (74, 65536, 16)):
        nconn = 120
        steps = QS.make_session(nconn, steps=3, seed=seed, header_table_size=hts, adversarial_frac=0.3)
        for st in steps:
            st["arena_off"] = QS.arena_offsets(st["sec_off"], hts)
        nbl = (np.arange(nconn) % 5).astype(np.uint32)
        ro = run_oracle_session(O.oracle(), nconn, hts, mb, nbl, steps)
        rr = run_oracle_session(O.ref(), nconn, hts, mb, nbl, steps)
        for a, b, st in zip(ro, rr, steps):
            ns = len(st["sec_off"]) - 1
            for k in SEC_KEYS:
                np.testing.assert_array_equal(a[k][:ns], b[k][:ns])
            for k in CONN_KEYS:
                np.testing.assert_array_equal(a[k][:nconn], b[k][:nconn])
            fa, fb = fields_of(a, st["sec_off"], ns), fields_of(b, st["sec_off"], ns)
            assert fa[0] == fb[0] and fa[1] == fb[1]
            np.testing.assert_array_equal(soft_code(fa[2]), fb[2])


# ---------------------------------------------------------------------------------------------------
# GPU
# ---------------------------------------------------------------------------------------------------
@pytest.fixture(scope="module")
def torch_cuda():
    import torch

    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    return torch


def gpu_session(torch, nconn, hts, mb, nbl, steps, move=False, requests=False):
    """every step through hhuff_qpack_decode, the tables carried over in the scratch -> list of host dicts
    (move: the scratch is copied to a new buffer between steps and the old one overwritten)"""
    from h2o_amd import codec

    dev = lambda a: torch.from_numpy(np.ascontiguousarray(a).copy()).cuda()  # noqa: E731
    u32 = lambda a: dev(np.asarray(a, np.uint32).view(np.int32))  # noqa: E731
    out, scratch = [], None
    nb = u32(nbl) if nbl is not None else None
    for k, st in enumerate(steps):
        data = st["data"] if st["data"].size else np.zeros(1, np.uint8)
        r = codec.qpack_decode(dev(data), u32(st["enc_off"]), u32(st["enc_len"]), u32(st["sec_off"]),
                               u32(st["conn_first"]), int(st["conn_first"][-1]), hts, mb, num_blocked=nb,
                               arena_off=dev(np.asarray(st["arena_off"], np.uint64).view(np.int64)),
                               in_size=int(st["data"].size), scratch=scratch, cont=k > 0,
                               stream_id=dev(np.asarray(st["rq_stream_id"], np.uint64).view(np.int64)) if requests else None)
        torch.cuda.synchronize()
        scratch = r["scratch"]
        if move:
            moved = torch.empty_like(scratch)
            moved.copy_(scratch)
            scratch.fill_(0x5A)  # stays allocated: a stale address would read this
            old, scratch = scratch, moved  # noqa: F841
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
@pytest.mark.parametrize("name", SESSIONS)
def test_gpu_matches_reference_fixtures(torch_cuda, name):
    nconn, hts, mb, nbl, steps = golden_steps(load_golden("qpack"), name)
    for res, st in zip(gpu_session(torch_cuda, nconn, hts, mb, nbl, steps), steps):
        check_step(res, st, nconn)


@pytest.mark.gpu
@pytest.mark.parametrize("name", SESSIONS)
def test_gpu_requests_match_reference_fixtures(torch_cuda, name):
    """hhuff_qpack_parse_requests against h2o_qpack_parse_request's outputs (verdicts, records, acks, flags)"""
    nconn, hts, mb, nbl, steps = golden_steps(load_golden("qpack"), name)
    for res, st in zip(gpu_session(torch_cuda, nconn, hts, mb, nbl, steps, requests=True), steps):
        check_request_step(res, st)


@pytest.mark.gpu
@pytest.mark.parametrize("seed,hts,mb", [(95, 4096, 4), (96, 256, 1)])
def test_gpu_requests_match_restatement(torch_cuda, oracle_codec, seed, hts, mb):
    nconn = 1500
    steps = QS.make_session(nconn, steps=3, seed=seed, header_table_size=hts, adversarial_frac=0.1, request_frac=0.4)
    for k, st in enumerate(steps):
        st["arena_off"] = QS.arena_offsets(st["sec_off"], hts)
        st["rq_stream_id"] = (np.arange(len(st["sec_off"]) - 1, dtype=np.uint64) * 4 + (1 << 20) * k) << (7 * (k % 3))
    nbl = (np.arange(nconn) % 5).astype(np.uint32)
    ro = run_oracle_session(oracle_codec, nconn, hts, mb, nbl, steps, requests=True)
    rg = gpu_session(torch_cuda, nconn, hts, mb, nbl, steps, requests=True)
    for a, g, st in zip(ro, rg, steps):
        ns = len(st["sec_off"]) - 1
        for k in ("nfields", "sstatus", "req_insert_count"):
            np.testing.assert_array_equal(g[k][:ns], a[k][:ns], err_msg=k)
        np.testing.assert_array_equal(req_words(g["req"], ns), req_words(a["req"], ns))
        for s_ in range(ns):
            o, n = int(st["sec_off"][s_]), int(a["nfields"][s_])
            for k in ("name_off", "name_len", "value_off", "value_len", "fflags"):
                np.testing.assert_array_equal(g[k][o:o + n], a[k][o:o + n], err_msg="%s section %d" % (k, s_))


@pytest.mark.gpu
@pytest.mark.parametrize("seed,hts,mb", [(81, 4096, 4), (82, 256, 1), (83, 0, 0), (84, 65536, 16)])
def test_gpu_matches_restatement_field_by_field(torch_cuda, oracle_codec, seed, hts, mb):
    nconn = 1500
    steps = QS.make_session(nconn, steps=3, seed=seed, header_table_size=hts, adversarial_frac=0.3)
    for st in steps:
        st["arena_off"] = QS.arena_offsets(st["sec_off"], hts)
    nbl = (np.arange(nconn) % 5).astype(np.uint32)
    ro = run_oracle_session(oracle_codec, nconn, hts, mb, nbl, steps)
    rg = gpu_session(torch_cuda, nconn, hts, mb, nbl, steps)
    for a, g, st in zip(ro, rg, steps):
        ns = len(st["sec_off"]) - 1
        for k in SEC_KEYS:
            np.testing.assert_array_equal(g[k][:ns], a[k][:ns], err_msg=k)
        for k in CONN_KEYS:
            np.testing.assert_array_equal(g[k][:nconn], a[k][:nconn], err_msg=k)
        for s in range(ns):  # same arena offsets, lengths and full soft bits in every used slot
            o, n = int(st["sec_off"][s]), int(a["nfields"][s])
            for k in ("name_off", "name_len", "value_off", "value_len", "fflags"):
                np.testing.assert_array_equal(g[k][o:o + n], a[k][o:o + n], err_msg="%s section %d" % (k, s))
        fg, fa = fields_of(g, st["sec_off"], ns), fields_of(a, st["sec_off"], ns)
        assert fg[0] == fa[0] and fg[1] == fa[1]


@pytest.mark.gpu
def test_gpu_scratch_moves_between_steps(torch_cuda, oracle_codec):
    """the tables hold scratch offsets: a scratch copied to another buffer between steps continues exactly"""
    nconn = 1000
    steps = QS.make_session(nconn, steps=3, seed=87, adversarial_frac=0.05)
    for st in steps:
        st["arena_off"] = QS.arena_offsets(st["sec_off"], 4096)
    ro = run_oracle_session(oracle_codec, nconn, 4096, 8, None, steps)
    rg = gpu_session(torch_cuda, nconn, 4096, 8, None, steps, move=True)
    for a, g, st in zip(ro, rg, steps):
        ns = len(st["sec_off"]) - 1
        for k in SEC_KEYS:
            np.testing.assert_array_equal(g[k][:ns], a[k][:ns], err_msg=k)
        for k in CONN_KEYS:
            np.testing.assert_array_equal(g[k][:nconn], a[k][:nconn], err_msg=k)
        fg, fa = fields_of(g, st["sec_off"], ns), fields_of(a, st["sec_off"], ns)
        assert fg[0] == fa[0] and fg[1] == fa[1]


@pytest.mark.gpu
def test_gpu_arena_limit_and_no_blocked_slots_match_restatement(torch_cuda, oracle_codec):
    """tight arena slices (HHUFF_QPK_ARENA exactly where the restatement reports it) and num_blocked NULL"""
    nconn = 800
    steps = QS.make_session(nconn, steps=2, seed=85, adversarial_frac=0.1)
    rng = np.random.default_rng(86)
    for st in steps:
        L = np.diff(st["sec_off"].astype(np.uint64))
        cap = (L * rng.uniform(0.5, 4.0, size=L.size)).astype(np.uint64)
        st["arena_off"] = np.concatenate([[0], np.cumsum(cap)]).astype(np.uint64)
    ro = run_oracle_session(oracle_codec, nconn, 4096, 0, None, steps)
    rg = gpu_session(torch_cuda, nconn, 4096, 0, None, steps)
    assert any((a["sstatus"] == -300).any() for a in ro)
    for a, g, st in zip(ro, rg, steps):
        ns = len(st["sec_off"]) - 1
        for k in SEC_KEYS:
            np.testing.assert_array_equal(g[k][:ns], a[k][:ns], err_msg=k)
        fg, fa = fields_of(g, st["sec_off"], ns), fields_of(a, st["sec_off"], ns)
        assert fg[0] == fa[0] and fg[1] == fa[1]
        np.testing.assert_array_equal(fg[2], fa[2])
