"""HTTP/3 response HEADERS frames (QPACK encode half): h2o_qpack_flatten_response
(lib/http3/qpack.c:1352-1399) as h2o's HTTP/3 server calls it (lib/http3/server.c:1680-1683, no encoder-stream
buffer: the encoder's dynamic table stays empty and every response stands alone).
CPU: the rule used for h2o_qpack_lookup_static against every generated lookup function (reference), the
restatement (oracle/qpack_encode.c) against the reference's frames (tests/golden/qpenc.npz, from
oracle/ref_shim.c ref_qpe_step) and against the reference directly on fresh responses, and a round trip: every
section decoded again by the QPACK decoder restatement gives back the response's fields.
GPU: hhuff_qpack_flatten_responses through the C-ABI against the fixtures, fresh edge-heavy responses against
the restatement, and a bench-sized batch (about 290,000 responses) byte for byte.
Requests (HHUFF_QRES_REQUEST): h2o_qpack_flatten_request (:1312-1350) as h2o's HTTP/3 client calls it
(lib/common/http3client.c:792) -- fixtures, the reference directly (incl. the request of the reference's own
t/00unit/lib/http3/qpack.c:65-67), a round trip through the decoder restatement, the GPU against all three."""
import numpy as np
import pytest

from conftest import load_golden
from h2o_amd import codec as C
from h2o_amd import hpenc_synth as HE

SETS = ["q1", "qedge", "qerr", "qrq", "qrqerr"]
KEYS = ("out_len", "header_len", "rstatus")


def golden(g, name):
    p = name + "_"
    q = {k[len(p):]: v for k, v in g.items() if k.startswith(p)}
    q["hdr"] = q["hdr"].view(C.HPE_HEADER_DTYPE)
    q["res"] = q["res"].view(C.QPE_RESPONSE_DTYPE)
    q["server_off"], q["server_len"] = (int(x) for x in q["server"])
    return q


def frames_of(out, out_off, out_len):
    return b"".join(np.asarray(out)[int(o):int(o) + int(L)].tobytes() for o, L in zip(out_off, out_len))


def check(r, q, want=None):
    n = q["res"].size
    want = q if want is None else want
    for k in KEYS:
        np.testing.assert_array_equal(np.asarray(r[k][:n]).astype(np.int64), np.asarray(want[k][:n]).astype(np.int64),
                                      err_msg=k)
    if want is q:
        wf = q["frames"].tobytes()
        ends = np.concatenate([[0], np.cumsum(q["out_len"].astype(np.int64))])
        wants = [wf[ends[k]:ends[k + 1]] for k in range(n)]
    else:
        wants = [np.asarray(want["out"])[int(o):int(o) + int(L)].tobytes() for o, L in zip(q["out_off"], want["out_len"])]
    gots = [np.asarray(r["out"])[int(o):int(o) + int(L)].tobytes() for o, L in zip(q["out_off"], r["out_len"][:n])]
    bad = [k for k in range(n) if gots[k] != wants[k]]
    assert not bad, "%d responses differ; first %d: got %s want %s" % (len(bad), bad[0], gots[bad[0]][:48].hex(),
                                                                       wants[bad[0]][:48].hex())


def ostep(codec, q):
    from oracle import oracle as O

    return O.qpe_step(codec, q["data"], q["hdr"], q["res"], q["out_off"], q["server_off"], q["server_len"])


def test_lookup_rule(oracle_codec):
    from oracle import oracle as O

    if not O.ref_available():
        pytest.skip("oracle/_ref not built (needs /root/reference)")
    assert O.ref().lib.ref_qpe_lookup_check() == 0


@pytest.mark.parametrize("name", SETS)
def test_restatement_golden(oracle_codec, name):
    from oracle import oracle as O

    q = golden(load_golden("qpenc"), name)
    check(ostep(O.oracle(), q), q)


@pytest.mark.parametrize("seed", [31, 32])
def test_restatement_vs_reference(oracle_codec, seed):
    from oracle import oracle as O

    if not O.ref_available():
        pytest.skip("oracle/_ref not built (needs /root/reference)")
    q = HE.to_qpack(HE.make_session(200, seed=seed, big_frac=0.01, notoken_frac=0.1, dont_compress_frac=0.1)[0],
                    seed=seed, dfid_frac=0.2, odd_status_frac=0.1)
    check(ostep(O.oracle(), q), q, want=ostep(O.ref(), q))


def unit_request():
    """t/00unit/lib/http3/qpack.c:61-67: GET https example.com /foobar, dnt: 1 and x-hoge: A added by string
    (h2o_add_header_by_str with maybe_token 0: not tokens), no encoder stream (the enc_stream == NULL case)"""
    TOK = C.HDR_TOKEN
    own = [(b":method", b"GET", TOK), (b":scheme", b"https", TOK), (b":authority", b"example.com", TOK),
           (b":path", b"/foobar", TOK)]
    b = HE.build_batch([[dict(status=4, flags=C.RES_REQUEST, headers=own + [(b"dnt", b"1", 0), (b"x-hoge", b"A", 0)])]])
    return HE.to_qpack_requests(b, dfid_frac=0.0)


@pytest.mark.parametrize("seed", [33, 34])
def test_requests_restatement_vs_reference(oracle_codec, seed):
    from oracle import oracle as O

    if not O.ref_available():
        pytest.skip("oracle/_ref not built (needs /root/reference)")
    b = HE.make_request_session(200, seed=seed, big_frac=0.01, notoken_frac=0.1, dont_compress_frac=0.1)[0]
    q = HE.to_qpack_requests(b, seed=seed, dfid_frac=0.2)
    check(ostep(O.oracle(), q), q, want=ostep(O.ref(), q))
    u = unit_request()
    check(ostep(O.oracle(), u), u, want=ostep(O.ref(), u))


def test_unit_request_bytes(oracle_codec):
    """the unit test's request: :method GET (17), :scheme https (23) static; :authority (0) and :path (1) name
    references with Huffman values; dnt and x-hoge literals with literal names"""
    from oracle import oracle as O

    u = unit_request()
    r = ostep(O.oracle(), u)
    f = r["out"][:int(r["out_len"][0])].tobytes()
    n, p = _varint(f, 1)
    sec = f[p:]
    assert sec[:4] == bytes([0, 0, 0xC0 | 17, 0xC0 | 23])
    assert sec[4] == 0x50 and sec[5] & 0x80  # :authority (static 0), Huffman value
    assert n == len(sec) == r["header_len"][0]


def _varint(b, p):
    n = 1 << (b[p] >> 6)
    v = b[p] & 0x3F
    for k in range(1, n):
        v = (v << 8) | b[p + k]
    return v, p + n


def test_round_trip(oracle_codec):
    """every HEADERS frame's field section, decoded by the QPACK decoder restatement (oracle/qpack_decode.c),
    is the response: :status, server, content-length, the headers in order, datagram-flow-id"""
    from oracle import oracle as O

    b = HE.make_session(120, seed=41, big_frac=0.0, dont_compress_frac=0.1)[0]
    q = HE.to_qpack(b, seed=41, dfid_frac=0.2, odd_status_frac=0.1)
    r = ostep(O.oracle(), q)
    data = q["data"].tobytes()
    sections, want = [], []
    for k in range(q["res"].size):
        f = r["out"][int(q["out_off"][k]):int(q["out_off"][k]) + int(r["out_len"][k])].tobytes()
        assert f[0] == 1
        n, p = _varint(f, 1)
        assert len(f) == p + n and n == r["header_len"][k]
        sections.append(f[p:])
        R = q["res"][k]
        st = int(R["status"]) & 0xFFFF
        fl = [(b":status", b"%d" % st)]
        if R["flags"] & C.RES_SERVER:
            fl.append((b"server", data[q["server_off"]:q["server_off"] + q["server_len"]]))
        if R["content_length"] != 0xFFFFFFFFFFFFFFFF:
            fl.append((b"content-length", b"%d" % int(R["content_length"])))
        for h in q["hdr"][int(R["hdr_first"]):int(R["hdr_first"]) + int(R["nhdr"])]:
            fl.append((data[h["name_off"]:h["name_off"] + h["name_len"]], data[h["value_off"]:h["value_off"] + h["value_len"]]))
        if R["flags"] & C.QRES_DATAGRAM:
            fl.append((b"datagram-flow-id", data[R["dfid_off"]:R["dfid_off"] + R["dfid_len"]]))
        want.append(fl)
    blob = b"".join(sections)
    sec_off = np.concatenate([[0], np.cumsum([len(s) for s in sections])]).astype(np.uint32)
    s = O.QpackSession(O.oracle(), 1)
    arena_off = np.concatenate([[0], np.cumsum([4 * len(x) + 256 for x in sections])]).astype(np.uint64)
    d = s.step(np.frombuffer(blob, np.uint8), np.zeros(1, np.uint32), np.zeros(1, np.uint32), sec_off,
               np.array([0, len(sections)], np.uint32), arena_off)
    assert (d["sstatus"][:len(sections)] == 0).all()
    a = d["arena"]
    for k, fl in enumerate(want):
        got = []
        for f in range(int(sec_off[k]), int(sec_off[k]) + int(d["nfields"][k])):
            got.append((a[d["name_off"][f]:d["name_off"][f] + d["name_len"][f]].tobytes(),
                        a[d["value_off"][f]:d["value_off"][f] + d["value_len"][f]].tobytes()))
        assert got == fl, k


def test_requests_round_trip(oracle_codec):
    """request sections decoded by the QPACK decoder restatement give back the own fields, the headers and the
    datagram-flow-id, in order"""
    from oracle import oracle as O

    b = HE.make_request_session(150, seed=43, big_frac=0.0, dont_compress_frac=0.1)[0]
    q = HE.to_qpack_requests(b, seed=43, dfid_frac=0.2)
    r = ostep(O.oracle(), q)
    data = q["data"].tobytes()
    sections, want = [], []
    for k in range(q["res"].size):
        f = r["out"][int(q["out_off"][k]):int(q["out_off"][k]) + int(r["out_len"][k])].tobytes()
        n, p = _varint(f, 1)
        sections.append(f[p:])
        R = q["res"][k]
        fl = [(data[h["name_off"]:h["name_off"] + h["name_len"]], data[h["value_off"]:h["value_off"] + h["value_len"]])
              for h in q["hdr"][int(R["hdr_first"]):int(R["hdr_first"]) + int(R["nhdr"])]]
        if R["flags"] & C.QRES_DATAGRAM:
            fl.append((b"datagram-flow-id", data[R["dfid_off"]:R["dfid_off"] + R["dfid_len"]]))
        want.append(fl)
    blob = b"".join(sections)
    sec_off = np.concatenate([[0], np.cumsum([len(s) for s in sections])]).astype(np.uint32)
    arena_off = np.concatenate([[0], np.cumsum([4 * len(x) + 256 for x in sections])]).astype(np.uint64)
    d = O.QpackSession(O.oracle(), 1).step(np.frombuffer(blob, np.uint8), np.zeros(1, np.uint32), np.zeros(1, np.uint32),
                                           sec_off, np.array([0, len(sections)], np.uint32), arena_off)
    assert (d["sstatus"][:len(sections)] == 0).all()
    a = d["arena"]
    for k, fl in enumerate(want):
        got = [(a[d["name_off"][f]:d["name_off"][f] + d["name_len"][f]].tobytes(),
                a[d["value_off"][f]:d["value_off"][f] + d["value_len"][f]].tobytes())
               for f in range(int(sec_off[k]), int(sec_off[k]) + int(d["nfields"][k]))]
        assert got == fl, k


# ---------------------------------------------------------------------------------------------------
# GPU
# ---------------------------------------------------------------------------------------------------
@pytest.fixture(scope="module")
def torch_cuda():
    import torch

    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    from h2o_amd import build

    build.build(verbose=False)
    return torch


def gpu(torch, q):
    dev = lambda a: torch.from_numpy(np.ascontiguousarray(a).copy()).cuda()  # noqa: E731
    data = dev(q["data"] if q["data"].size else np.zeros(1, np.uint8))
    hdr = dev(q["hdr"].view(np.uint8) if q["hdr"].size else np.zeros(20, np.uint8))
    r = C.qpack_flatten_responses(data, hdr if q["hdr"].size else hdr[:0], dev(q["res"].view(np.uint8)),
                                  int(q["res"].size), dev(q["out_off"].view(np.int64)), q["server_off"], q["server_len"],
                                  in_size=int(q["data"].size))
    torch.cuda.synchronize()
    r = {k: v.cpu().numpy() for k, v in r.items()}
    r["out_len"], r["header_len"] = r["out_len"].view(np.uint32), r["header_len"].view(np.uint32)
    return r


@pytest.mark.gpu
@pytest.mark.parametrize("name", SETS)
def test_gpu_golden(torch_cuda, name):
    q = golden(load_golden("qpenc"), name)
    check(gpu(torch_cuda, q), q)


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [51, 52])
def test_gpu_vs_restatement(torch_cuda, oracle_codec, seed):
    from oracle import oracle as O

    q = HE.to_qpack(HE.make_session(600, seed=seed, big_frac=0.01, notoken_frac=0.1, dont_compress_frac=0.1)[0],
                    seed=seed, dfid_frac=0.2, odd_status_frac=0.1)
    check(gpu(torch_cuda, q), q, want=ostep(O.oracle(), q))


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [53, 54])
def test_gpu_requests_vs_restatement(torch_cuda, oracle_codec, seed):
    from oracle import oracle as O

    b = HE.make_request_session(600, seed=seed, big_frac=0.01, notoken_frac=0.1, dont_compress_frac=0.1)[0]
    q = HE.to_qpack_requests(b, seed=seed, dfid_frac=0.2)
    check(gpu(torch_cuda, q), q, want=ostep(O.oracle(), q))
    u = unit_request()
    check(gpu(torch_cuda, u), u, want=ostep(O.oracle(), u))


@pytest.mark.gpu
def test_gpu_edges(torch_cuda, oracle_codec):
    """no headers, empty names and values, content-length 0, a datagram flow id with an empty value, statuses
    that wrap at 16 bits, a section over 16383 bytes (a 4-byte frame length)"""
    from oracle import oracle as O

    T = C.HDR_TOKEN
    conns = [[dict(status=200)], [dict(status=65536 + 404, content_length=0, headers=[(b"", b"", 0), (b"x", b"", 0)])],
             [dict(status=7, headers=[(b"content-type", b"text/css", T), (b"content-type", b"text/x", T),
                                      (b"cache-control", b"no-cache", T | C.HDR_DONT_COMPRESS)])],
             [dict(status=200, headers=[(b"link", b"<x>" * 6000, T)])]]
    b = HE.build_batch(conns)
    q = HE.to_qpack(b, seed=1, dfid_frac=0.0, odd_status_frac=0.0)
    q["res"]["status"] = [200, 65536 + 404, 7, 200]
    q["res"]["flags"][0] |= C.QRES_DATAGRAM  # empty datagram flow id value
    q["res"]["dfid_off"][0], q["res"]["dfid_len"][0] = 0, 0
    q["out_off"] = HE.qpack_out_offsets(q["hdr"], q["res"], q["server_len"])
    check(gpu(torch_cuda, q), q, want=ostep(O.oracle(), q))


@pytest.mark.gpu
def test_gpu_bench_size(torch_cuda, oracle_codec):
    from oracle import oracle as O

    q = HE.to_qpack(HE.tile(HE.make_session(4096, seed=5)[0], 16), seed=5)
    r = gpu(torch_cuda, q)
    assert (r["rstatus"][:q["res"].size] == 0).all()
    check(r, q, want=ostep(O.oracle(), q))


@pytest.mark.gpu
def test_gpu_malformed_ranges(torch_cuda):
    """a response whose header range runs past the call's headers, or whose output region ends before it
    starts, is refused with HHUFF_RES_EINVAL; its neighbours are encoded as before"""
    T = C.HDR_TOKEN
    conns = [[dict(status=200, headers=[(b"date", b"now", T)])], [dict(status=404, headers=[(b"x-a", b"1", 0)])],
             [dict(status=200, headers=[(b"server", b"h2o", T)])], [dict(status=204)]]
    q = HE.to_qpack(HE.build_batch(conns), seed=1, dfid_frac=0.0, odd_status_frac=0.0)
    good = gpu(torch_cuda, q)
    assert (good["rstatus"] == 0).all()
    q["res"]["hdr_first"][1] = np.uint32(q["hdr"].size + 7)
    q["res"]["hdr_first"][2] = np.uint32(0xFFFFFFFF)
    q["out_off"][4] = q["out_off"][3] - 1  # response 3's region ends before it starts
    r = gpu(torch_cuda, q)
    assert list(r["rstatus"]) == [0, C.RES_EINVAL, C.RES_EINVAL, C.RES_EINVAL]
    assert r["out_len"][0] == good["out_len"][0] and r["header_len"][0] == good["header_len"][0]
