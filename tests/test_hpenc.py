"""HTTP/2 response header blocks, encode side (SURVEY.md 8 f4 encode half): h2o_hpack_flatten_response and
h2o_hpack_flatten_trailers (lib/http2/hpack.c:1137-1196) with one encoder dynamic table per connection
(do_encode_header :858-937) kept across steps.
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

SESSIONS = ["h4096", "hedge", "herr"]
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
