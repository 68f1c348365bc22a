"""HTTP/2 response header blocks, encode side (SURVEY.md 8 f4 encode half): h2o_hpack_flatten_response and
h2o_hpack_flatten_trailers (lib/http2/hpack.c:1137-1196) -- and the client's h2o_hpack_flatten_request
(:1044-1096, HHUFF_RES_REQUEST records) -- with one encoder dynamic table per connection
(do_encode_header :858-937) kept across steps.  Requests are also decoded again (the reference's own
request tests, t/00unit/lib/http2/hpack.c:395-450, are such round trips through h2o_hpack_parse_request).
CPU: the restatement (oracle/hpack_encode.c) against the reference's frames (tests/golden/hpenc.npz, written
by oracle/gen_golden.py from h2o's own hpack.c through oracle/ref_hpenc.c), against the reference directly
on fresh sessions where oracle/_ref exists, the token facts both rely on, and the known answers of the
reference's unit tests (t/00unit/lib/http2/hpack.c:308-333, :495-525, :629-645).
GPU: hhuff_hpack_flatten_responses through the C-ABI against the same fixtures (every step, tables carried
over with HHUFF_ENC_CONTINUE), the known answers, fresh edge-heavy sessions against the restatement, and the
bench-sized batch (65,536 connections) against the restatement byte for byte."""
import numpy as np
import pytest

from conftest import load_golden
from h2o_amd import codec as C
from h2o_amd import hpenc_synth as HE

SESSIONS = ["h4096", "hedge", "herr", "rq4096", "rqedge", "rqerr"]
KEYS = ("out_len", "headers_size", "rstatus")


def golden_steps(g, name):
    nconn, nsteps = (int(x) for x in g[name + "_meta"])
    steps = []
    for k in range(nsteps):
        p = "%s_%d_" % (name, k)
        st = {key[len(p):]: v for key, v in g.items() if key.startswith(p)}
        st["hdr"] = st["hdr"].view(C.HPE_HEADER_DTYPE)
        st["res"] = st["res"].view(C.HPE_RESPONSE_DTYPE)
        st["server_off"], st["server_len"] = (int(x) for x in st["server"])
        steps.append(st)
    return nconn, steps


def frames_of(out, out_off, out_len):
    return b"".join(np.asarray(out)[int(o):int(o) + int(L)].tobytes() for o, L in zip(out_off, out_len))


def check_step(r, st):
    n = st["res"].size
    for k in KEYS:
        np.testing.assert_array_equal(np.asarray(r[k][:n]).astype(st[k].dtype), st[k], err_msg=k)
    got = frames_of(r["out"], st["out_off"], st["out_len"])
    assert got == st["frames"].tobytes()


def oracle_step(sess, st):
    return sess.step(st["data"], st["hdr"], st["res"], st["conn_first"], st["out_off"], st["server_off"], st["server_len"])


# ---- known answers of the reference's unit tests ----
TOK = C.HDR_TOKEN


def kat_batch():
    """three connections: t/00unit/lib/http2/hpack.c:308-333 (302 then 307, Huffman, fully indexed on the
    second response), :495-525 (te: a token outside the static table, then indexed), :629-645 (a peer
    SETTINGS_HEADER_TABLE_SIZE of 1024 -> Dynamic Table Size Update, content-length 12345)"""
    c0 = [dict(status=302, headers=[(b"cache-control", b"private", TOK), (b"date", b"Mon, 21 Oct 2013 20:13:21 GMT", TOK),
                                    (b"location", b"https://www.example.com", TOK)]),
          dict(status=307, headers=[(b"cache-control", b"private", TOK), (b"date", b"Mon, 21 Oct 2013 20:13:21 GMT", TOK),
                                    (b"location", b"https://www.example.com", TOK)])]
    c1 = [dict(status=200, headers=[(b"te", b"test", TOK)]), dict(status=200, headers=[(b"te", b"test", TOK)])]
    c2 = [dict(status=200, header_table_size=1024, content_length=12345)]
    return HE.build_batch([c0, c1, c2])


KAT_PAYLOADS = [
    bytes.fromhex("0803333032" "5885aec3771a4b" "6196d07abe941054d444a8200595040b8166e082a62d1bff"
                  "6e919d29ad171863c78f0b97c8e9ae82ae43d3"),  # hpack.c:322-325
    bytes.fromhex("0803333037c0bfbe"),  # hpack.c:333
    b"\x88\x40\x02te\x83IP\x9f",  # hpack.c:508-512
    b"\x88\xbe",  # hpack.c:518-520
    b"\x3f\xe1\x07\x88\x0f\x0d\x0512345",  # hpack.c:634-644: size update 1024, :status 200, content-length
]


def check_kats(r, b):
    for k, want in enumerate(KAT_PAYLOADS):
        o = int(b["out_off"][k])
        frame = np.asarray(r["out"])[o:o + int(r["out_len"][k])].tobytes()
        assert frame[:9] == bytes([0, 0, len(want), 1, 4, 0, 0, 0, 1])
        assert frame[9:] == want, k


def test_kats_restatement(oracle_codec):
    from oracle import oracle as O

    b = kat_batch()
    s = O.HpeSession(O.oracle(), 3)
    check_kats(oracle_step(s, b), b)


def test_kats_reference(oracle_codec):
    from oracle import oracle as O

    if not O.ref_available():
        pytest.skip("oracle/_ref not built (needs /root/reference)")
    b = kat_batch()
    s = O.HpeSession(O.ref(), 3)
    check_kats(oracle_step(s, b), b)
    assert O.ref().lib.ref_hpe_token_check() == 0  # the token facts of lib/common/token_table.h


@pytest.mark.parametrize("name", SESSIONS)
def test_restatement_golden(oracle_codec, name):
    from oracle import oracle as O

    g = load_golden("hpenc")
    nconn, steps = golden_steps(g, name)
    s = O.HpeSession(O.oracle(), nconn)
    for st in steps:
        check_step(oracle_step(s, st), st)


@pytest.mark.parametrize("seed", [11, 12])
def test_restatement_vs_reference(oracle_codec, seed):
    from oracle import oracle as O

    if not O.ref_available():
        pytest.skip("oracle/_ref not built (needs /root/reference)")
    steps = HE.make_session(150, steps=3, seed=seed, small_table_frac=0.25, trailers_frac=0.08, big_frac=0.01,
                            notoken_frac=0.1, dont_compress_frac=0.1, frame_frac=0.2)
    a, b = O.HpeSession(O.oracle(), 150), O.HpeSession(O.ref(), 150)
    for st in steps:
        ra, rb = oracle_step(a, st), oracle_step(b, st)
        for k in KEYS:
            np.testing.assert_array_equal(ra[k], rb[k], err_msg=k)
        assert frames_of(ra["out"], st["out_off"], ra["out_len"]) == frames_of(rb["out"], st["out_off"], rb["out_len"])


@pytest.mark.parametrize("seed", [13, 14])
def test_requests_restatement_vs_reference(oracle_codec, seed):
    from oracle import oracle as O

    if not O.ref_available():
        pytest.skip("oracle/_ref not built (needs /root/reference)")
    steps = HE.make_request_session(150, steps=3, seed=seed, small_table_frac=0.25, big_frac=0.01, notoken_frac=0.1,
                                    dont_compress_frac=0.1, frame_frac=0.2)
    a, b = O.HpeSession(O.oracle(), 150), O.HpeSession(O.ref(), 150)
    for st in steps:
        ra, rb = oracle_step(a, st), oracle_step(b, st)
        for k in KEYS:
            np.testing.assert_array_equal(ra[k], rb[k], err_msg=k)
        assert frames_of(ra["out"], st["out_off"], ra["out_len"]) == frames_of(rb["out"], st["out_off"], rb["out_len"])


def request_blocks(st, r):
    """the header blocks of flattened requests (frame headers stripped) -> (data, blk_off)"""
    blocks = []
    for o, L in zip(st["out_off"], r["out_len"]):
        f = np.asarray(r["out"])[int(o):int(o) + int(L)].tobytes()
        p, b = 0, b""
        while p < len(f):
            n = int.from_bytes(f[p:p + 3], "big")
            b += f[p + 9:p + 9 + n]
            p += 9 + n
        blocks.append(b)
    blk_off = np.concatenate([[0], np.cumsum([len(b) for b in blocks])]).astype(np.uint32)
    return np.frombuffer(b"".join(blocks), np.uint8).copy(), blk_off


def check_request_roundtrip(st, blk_off, d):
    """every request decodes to its own fields and headers, in order, and passes h2o_hpack_parse_request.
    The sessions carry no dont_compress flags: for a header that is not a token, with dont_compress and a value
    under 20 bytes, h2o's do_encode_header writes 0x40 (literal WITH incremental indexing, hpack.c:906-907) but
    sends the value as-is without adding the entry to its own table (:908-910), so the peer's table gains an
    entry the encoder's lacks and later indices disagree -- the encoder (and this port, byte for byte, see the
    fixtures) does that; a round trip cannot hold across it."""
    assert (np.asarray(d["bstatus"])[:blk_off.size - 1] == 0).all()
    data, A = st["data"], np.asarray(d["arena"])
    for b, R in enumerate(st["res"]):
        want = [(data[h["name_off"]:h["name_off"] + h["name_len"]].tobytes(),
                 data[h["value_off"]:h["value_off"] + h["value_len"]].tobytes())
                for h in st["hdr"][R["hdr_first"]:R["hdr_first"] + R["nhdr"]]]
        s0 = int(blk_off[b])
        got = []
        for k in range(int(d["nfields"][b])):
            no, nl, vo, vl = (int(d[x][s0 + k]) for x in ("name_off", "name_len", "value_off", "value_len"))
            got.append((A[no:no + nl].tobytes(), A[vo:vo + vl].tobytes()))
        assert got == want, b


def test_requests_roundtrip_restatement(oracle_codec):
    from oracle import oracle as O

    st = HE.make_request_session(200, seed=9, big_frac=0.01, frame_frac=0.2, small_table_frac=0.2, dont_compress_frac=0.0)[0]
    r = oracle_step(O.HpeSession(O.oracle(), 200), st)
    assert (r["rstatus"] == 0).all()
    data, blk_off = request_blocks(st, r)
    d = O.oracle().hpack_decode_blocks(data, blk_off, st["conn_first"], requests=True)
    check_request_roundtrip(st, blk_off, d)


def request_edges(outside_reference=True):
    """own-field placement rules: the one-byte references apply to own fields (:method, :scheme, :path) and to
    accept-encoding among the headers only; an old-style CONNECT; :protocol; send_own_expect; server and
    content_length ignored.  outside_reference adds a connection whose records are no flatten_request call
    (the reference harness refuses them; the restatement defines them): accept-encoding counted as an own field,
    a request with no own fields, an own-field count past nhdr (HHUFF_RES_EINVAL, then the connection's next
    request SKIPPED)"""
    M, SC, AU, PA = b":method", b":scheme", b":authority", b":path"
    req = lambda own, hs, **k: dict(status=len(own), headers=[(n, v, TOK) for n, v in own] + hs,  # noqa: E731
                                    flags=C.RES_REQUEST | k.pop("fl", 0), **k)
    c0 = [req([(M, b"GET"), (SC, b"https"), (AU, b"a.example"), (PA, b"/")], [(b"accept-encoding", b"gzip, deflate", TOK)],
              fl=C.RES_END_STREAM | C.RES_SERVER, content_length=5),
          req([(M, b"POST"), (SC, b"http"), (AU, b"a.example"), (PA, b"/index.html"), (b"expect", b"100-continue")],
              [(b"content-length", b"3", TOK), (b":method", b"GET", TOK)]),
          req([(M, b"CONNECT"), (AU, b"proxy:443")], [(b"accept-encoding", b"gzip, deflate", 0)]),
          req([(M, b"CONNECT"), (SC, b"https"), (AU, b"b.example"), (PA, b"/chat"), (b":protocol", b"websocket")], [])]
    c1 = [req([(M, b"GET"), (SC, b"masque"), (AU, b"a.example"), (PA, b"/x"), (b"accept-encoding", b"gzip, deflate")], []),
          dict(status=0, flags=C.RES_REQUEST, headers=[(b"accept-encoding", b"gzip, deflate", TOK), (b"x-a", b"b", 0)]),
          dict(status=3, flags=C.RES_REQUEST, headers=[(M, b"GET", TOK)]),
          req([(M, b"GET"), (SC, b"https"), (AU, b"a"), (PA, b"/")], [])]
    c2 = [req([(M, b"GET"), (SC, b"https"), (AU, b"c.example"), (PA, b"/" + b"p" * 40)],
              [(b"cookie", b"k=" + b"v" * 20000, TOK)], header_table_size=256)]
    return HE.build_batch([c0, c1, c2] if outside_reference else [c0, c2])


def test_request_edges_reference(oracle_codec):
    from oracle import oracle as O

    if not O.ref_available():
        pytest.skip("oracle/_ref not built (needs /root/reference)")
    b = request_edges(outside_reference=False)
    ra = oracle_step(O.HpeSession(O.oracle(), 2), b)
    rb = oracle_step(O.HpeSession(O.ref(), 2), b)
    assert (ra["rstatus"] == 0).all()
    for k in KEYS:
        np.testing.assert_array_equal(ra[k], rb[k], err_msg=k)
    assert frames_of(ra["out"], b["out_off"], ra["out_len"]) == frames_of(rb["out"], b["out_off"], rb["out_len"])


def test_request_edges_restatement(oracle_codec):
    from oracle import oracle as O

    b = request_edges()
    r = oracle_step(O.HpeSession(O.oracle(), 3), b)
    assert list(r["rstatus"]) == [0, 0, 0, 0, 0, 0, C.RES_EINVAL, C.RES_SKIPPED, 0]
    f = lambda k: np.asarray(r["out"])[int(b["out_off"][k]) + 9:int(b["out_off"][k]) + int(r["out_len"][k])].tobytes()  # noqa
    assert f(0) == bytes([0x82, 0x87]) + f(0)[2:-1] + bytes([0x90])  # GET, https, ..., accept-encoding gzip, deflate
    assert f(0)[2] == 0x41  # :authority, indexed name 1, new entry
    assert f(1)[:1] == b"\x83" and b"\x85" in f(1)[1:6]  # POST, /index.html
    assert f(5)[:1] == b"\x90"  # accept-encoding at the head of the headers of a request without own fields


def test_bound_holds(oracle_codec):
    """hhuff_hpack_response_bound covers the worst representation: every header a new-name literal sent raw"""
    from oracle import oracle as O

    names = [bytes([0x7f - i]) * (1 + i) for i in range(30)]  # raw (Huffman longer than the input)
    conn = [dict(status=999, headers=[(n, n * 3, C.HDR_DONT_COMPRESS) for n in names], content_length=2 ** 64 - 2,
                 flags=C.RES_SERVER, header_table_size=0)]
    b = HE.build_batch([conn], server=b"\x7f" * 300)
    r = oracle_step(O.HpeSession(O.oracle(), 1), b)
    assert r["rstatus"][0] == 0
    assert r["out_len"][0] <= int(b["out_off"][1])


def test_tile():
    b = HE.make_session(20, seed=3)[0]
    t = HE.tile(b, 3)
    assert t["res"].size == 3 * b["res"].size and t["conn_first"][-1] == t["res"].size
    assert t["conn_first"].size == 3 * 20 + 1


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


def gpu_step(torch, st, scratch=None, cont=False):
    dev = lambda a: torch.from_numpy(np.ascontiguousarray(a).copy()).cuda()  # noqa: E731
    data = dev(st["data"] if st["data"].size else np.zeros(1, np.uint8))
    hdr = dev(st["hdr"].view(np.uint8) if st["hdr"].size else np.zeros(20, np.uint8))
    res = dev(st["res"].view(np.uint8))
    r = C.hpack_flatten_responses(data, hdr if st["hdr"].size else hdr[:0], res, dev(st["conn_first"].view(np.int32)),
                                  int(st["res"].size), dev(st["out_off"].view(np.int64)), st["server_off"],
                                  st["server_len"], in_size=int(st["data"].size), scratch=scratch, cont=cont)
    torch.cuda.synchronize()
    return {k: (v.cpu().numpy() if k != "scratch" else v) for k, v in r.items()}


def host(r):
    return dict(out=r["out"], out_len=r["out_len"].view(np.uint32), headers_size=r["headers_size"].view(np.uint32),
                rstatus=r["rstatus"], scratch=r["scratch"])


@pytest.mark.gpu
@pytest.mark.parametrize("name", SESSIONS)
def test_gpu_golden(torch_cuda, name):
    g = load_golden("hpenc")
    nconn, steps = golden_steps(g, name)
    scratch = None
    for k, st in enumerate(steps):
        r = host(gpu_step(torch_cuda, st, scratch=scratch, cont=k > 0))
        scratch = r["scratch"]
        check_step(r, st)


@pytest.mark.gpu
def test_gpu_kats(torch_cuda):
    b = kat_batch()
    check_kats(host(gpu_step(torch_cuda, b)), b)


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [21, 22])
def test_gpu_vs_restatement(torch_cuda, oracle_codec, seed):
    from oracle import oracle as O

    steps = HE.make_session(600, steps=3, seed=seed, small_table_frac=0.25, trailers_frac=0.08, big_frac=0.01,
                            notoken_frac=0.1, dont_compress_frac=0.1, frame_frac=0.2)
    s = O.HpeSession(O.oracle(), 600)
    scratch = None
    for k, st in enumerate(steps):
        q = oracle_step(s, st)
        r = host(gpu_step(torch_cuda, st, scratch=scratch, cont=k > 0))
        scratch = r["scratch"]
        for key in KEYS:
            np.testing.assert_array_equal(r[key], q[key], err_msg=key)
        assert frames_of(r["out"], st["out_off"], r["out_len"]) == frames_of(q["out"], st["out_off"], q["out_len"])


@pytest.mark.gpu
def test_gpu_empty_and_edges(torch_cuda, oracle_codec):
    """connections without responses, responses without headers, empty names and values, an all-evicting
    table size of 0, trailers only, a status outside the static table, a response about max_frame_size long"""
    from oracle import oracle as O

    filler = b"x" * (16384 - 1 - 3 - 1)  # :status 200 (1) + new-name literal 0x40, name "a" raw (2), value prefix
    conns = [[], [dict(status=200)], [dict(status=599, headers=[(b"", b"", 0), (b"x-empty", b"", 0), (b"", b"v", 0)])],
             [dict(status=200, header_table_size=0, headers=[(b"date", b"now", TOK)]),
              dict(status=200, headers=[(b"date", b"now", TOK)])],
             [dict(flags=C.RES_TRAILERS, headers=[(b"x-t", b"1", 0)])], [],
             [dict(status=200, headers=[(b"a", filler, C.HDR_DONT_COMPRESS)])]]
    b = HE.build_batch(conns)
    q = oracle_step(O.HpeSession(O.oracle(), len(conns)), b)
    r = host(gpu_step(torch_cuda, b))
    for key in KEYS:
        np.testing.assert_array_equal(r[key], q[key], err_msg=key)
    assert frames_of(r["out"], b["out_off"], r["out_len"]) == frames_of(q["out"], b["out_off"], q["out_len"])


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [23, 24])
def test_gpu_requests_vs_restatement(torch_cuda, oracle_codec, seed):
    from oracle import oracle as O

    steps = HE.make_request_session(600, steps=3, seed=seed, small_table_frac=0.25, big_frac=0.01, notoken_frac=0.1,
                                    dont_compress_frac=0.1, frame_frac=0.2)
    s = O.HpeSession(O.oracle(), 600)
    scratch = None
    for k, st in enumerate(steps):
        q = oracle_step(s, st)
        r = host(gpu_step(torch_cuda, st, scratch=scratch, cont=k > 0))
        scratch = r["scratch"]
        for key in KEYS:
            np.testing.assert_array_equal(r[key], q[key], err_msg=key)
        assert frames_of(r["out"], st["out_off"], r["out_len"]) == frames_of(q["out"], st["out_off"], q["out_len"])


@pytest.mark.gpu
def test_gpu_request_edges(torch_cuda, oracle_codec):
    from oracle import oracle as O

    b = request_edges()
    q = oracle_step(O.HpeSession(O.oracle(), 3), b)
    r = host(gpu_step(torch_cuda, b))
    for key in KEYS:
        np.testing.assert_array_equal(r[key], q[key], err_msg=key)
    assert frames_of(r["out"], b["out_off"], r["out_len"]) == frames_of(q["out"], b["out_off"], q["out_len"])


@pytest.mark.gpu
def test_gpu_request_roundtrip(torch_cuda):
    """GPU flatten -> GPU parse (hhuff_hpack_parse_requests): the fields come back, h2o's request rules pass"""
    torch = torch_cuda
    st = HE.make_request_session(2000, seed=31, big_frac=0.005, frame_frac=0.2, small_table_frac=0.2,
                                 dont_compress_frac=0.0)[0]
    r = host(gpu_step(torch, st))
    assert (r["rstatus"] == 0).all()
    data, blk_off = request_blocks(st, r)
    dev = lambda a: torch.from_numpy(np.ascontiguousarray(a).copy()).cuda()  # noqa: E731
    L = np.diff(blk_off.astype(np.int64))
    ao = np.concatenate([[0], np.cumsum(16 * L + 1024)]).astype(np.int64)  # 8/5 of a block is its longest decode
    d = C.hpack_decode_blocks(dev(data), dev(blk_off.view(np.int32)), dev(st["conn_first"].view(np.int32)),
                              arena_off=dev(ao), requests=True)
    torch.cuda.synchronize()
    h = {k: v.cpu().numpy() for k, v in d.items() if k != "scratch"}
    for k in ("name_off", "name_len", "value_off", "value_len", "nfields"):
        h[k] = h[k].view(np.uint32)  # u32 bits in int32 tensors
    check_request_roundtrip(st, blk_off, h)


@pytest.mark.gpu
def test_gpu_bench_size(torch_cuda, oracle_codec):
    """the bench's batch (65,536 connections: 4,096 synthetic ones tiled 16 times) byte for byte against the
    restatement"""
    from oracle import oracle as O

    b = HE.tile(HE.make_session(4096, seed=5)[0], 16)
    q = oracle_step(O.HpeSession(O.oracle(), 65536), b)
    r = host(gpu_step(torch_cuda, b))
    for key in KEYS:
        np.testing.assert_array_equal(r[key], q[key], err_msg=key)
    assert (r["rstatus"] == 0).all()
    assert frames_of(r["out"], b["out_off"], r["out_len"]) == frames_of(q["out"], b["out_off"], q["out_len"])


@pytest.mark.gpu
def test_gpu_malformed_ranges(torch_cuda):
    """a response whose header range runs past the call's headers, or whose output region ends before it
    starts, is refused with HHUFF_RES_EINVAL (the connection's later responses SKIPPED), and nothing is
    read or written outside the arrays; the other connections are unaffected"""
    conns = [[dict(status=200, headers=[(b"date", b"now", TOK)]), dict(status=200, headers=[(b"x-a", b"1", 0)]),
              dict(status=204)],
             [dict(status=200, headers=[(b"server", b"h2o", TOK)])],
             [dict(status=301, headers=[(b"location", b"/a", TOK)]), dict(status=200)]]
    b = HE.build_batch(conns)
    good = host(gpu_step(torch_cuda, b))
    assert (good["rstatus"] == 0).all()
    bad = {k: (v.copy() if isinstance(v, np.ndarray) else v) for k, v in b.items()}
    bad["res"]["hdr_first"][1] = np.uint32(b["hdr"].size + 1000)  # past nhdr
    bad["res"]["hdr_first"][3] = np.uint32(0xFFFFFFF0)  # wraps u32 with its nhdr
    bad["out_off"][5] = bad["out_off"][4] - 1  # connection 2's first region ends before it starts
    r = host(gpu_step(torch_cuda, bad))
    assert list(r["rstatus"]) == [0, C.RES_EINVAL, C.RES_SKIPPED, C.RES_EINVAL, C.RES_EINVAL, C.RES_SKIPPED]
    assert r["out_len"][0] == good["out_len"][0]
