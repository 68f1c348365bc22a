"""HPACK header blocks: h2o_hpack_decode_header over whole blocks with a dynamic table per
connection.  CPU: the restatement (oracle/hpack_block.c) against the reference's outputs (tests/golden/
blocks*.npz, written by oracle/gen_golden.py from h2o's own decoder) and, where oracle/_ref exists, against
the reference directly on fresh synthetic connections.  GPU: hhuff_hpack_decode_blocks through the C-ABI
against the same fixtures (bit-exact names, values, soft-error codes, field counts, block statuses) and
against the restatement field by field (arena offsets and full soft bits included)."""
import numpy as np
import pytest

from conftest import load_golden
from h2o_amd import hpack_synth as HS

BLOCK_SETS = ["blocks", "blocks_256"]


def soft_code(bits):
    """the reference reports one soft error per field (err_desc, hpack.c:427-431): name first"""
    bits = np.asarray(bits)
    return np.where(bits & 1, 1, np.where(bits & 2, 2, 0)).astype(np.uint8)


def fields_of(res, blk_off, nblk):
    """-> (names, values, soft bits) of every decoded field, in block order"""
    names, values, soft = [], [], []
    a = res["arena"]
    for b in range(nblk):
        s = int(blk_off[b])
        for f in range(s, s + int(res["nfields"][b])):
            no, nl, vo, vl = (int(res[k][f]) for k in ("name_off", "name_len", "value_off", "value_len"))
            names.append(a[no:no + nl].tobytes())
            values.append(a[vo:vo + vl].tobytes())
            soft.append(int(res["fflags"][f]))
    return names, values, np.asarray(soft, np.uint8)


def expected_fields(g):
    n = len(g["fld_name_off"]) - 1
    names = [g["fld_name"][g["fld_name_off"][i]:g["fld_name_off"][i + 1]].tobytes() for i in range(n)]
    values = [g["fld_value"][g["fld_value_off"][i]:g["fld_value_off"][i + 1]].tobytes() for i in range(n)]
    return names, values, g["fld_soft"]


def check_against_golden(res, g):
    nblk = len(g["blk_off"]) - 1
    np.testing.assert_array_equal(np.asarray(res["nfields"][:nblk], np.uint32), g["nfields"])
    np.testing.assert_array_equal(np.asarray(res["bstatus"][:nblk], np.int32), g["bstatus"])
    names, values, soft = fields_of(res, g["blk_off"], nblk)
    en, ev, es = expected_fields(g)
    assert names == en
    assert values == ev
    np.testing.assert_array_equal(soft_code(soft), es)


@pytest.mark.parametrize("name", BLOCK_SETS)
def test_restatement_matches_reference_fixtures(oracle_codec, name):
    g = load_golden(name)
    res = oracle_codec.hpack_decode_blocks(g["data"], g["blk_off"], g["conn_first"], int(g["table_size"][0]),
                                           nthreads=8)
    check_against_golden(res, g)


# ---- h2o_hpack_parse_request (hhuff_hpack_parse_requests) ----
W_SLOTS = slice(2, 8)  # method, scheme, authority, path, protocol, expect: field indices within the block
W_EXPECT = 7


def req_words(res, nblk):
    return np.ascontiguousarray(res["req"][:nblk]).view(np.uint32).reshape(nblk, 12)


def check_requests_against_golden(res, g):
    """verdicts, request records and field flags of h2o_hpack_parse_request (blocks.npz rq_*); the fields
    themselves are a prefix of the decode-only fixture fields of the same block"""
    nblk = len(g["blk_off"]) - 1
    np.testing.assert_array_equal(np.asarray(res["nfields"][:nblk], np.uint32), g["rq_nfields"])
    np.testing.assert_array_equal(np.asarray(res["bstatus"][:nblk], np.int32), g["rq_bstatus"])
    got, exp = req_words(res, nblk), g["rq_req"]
    # everything but `expect` word for word; expect (the last one wins in h2o) by the bytes it points at
    keep = np.ones(12, bool)
    keep[W_EXPECT] = False
    np.testing.assert_array_equal(got[:, keep], exp[:, keep])
    en, ev, _ = expected_fields(g)
    first = np.concatenate([[0], np.cumsum(g["nfields"])])
    a = res["arena"]
    flags = []
    for b in range(nblk):
        s0, k = int(g["blk_off"][b]), int(g["rq_nfields"][b])
        for f in range(k):
            gi = int(first[b]) + f
            no, nl, vo, vl = (int(res[x][s0 + f]) for x in ("name_off", "name_len", "value_off", "value_len"))
            assert a[no:no + nl].tobytes() == en[gi] and a[vo:vo + vl].tobytes() == ev[gi], (b, f)
            flags.append(int(res["fflags"][s0 + f]))
        ge, ee = int(got[b, W_EXPECT].view(np.int32)), int(exp[b, W_EXPECT].view(np.int32))
        assert (ge < 0) == (ee < 0), b
        if ge >= 0:
            assert ev[int(first[b]) + ge] == ev[int(first[b]) + ee], b
    fl = np.asarray(flags, np.uint8)
    np.testing.assert_array_equal(fl & 4, g["rq_fflags"] & 4)  # HHUFF_FIELD_HEADER
    np.testing.assert_array_equal(soft_code(fl & 3), soft_code(g["rq_fflags"] & 3))


def test_restatement_matches_reference_request_verdicts(oracle_codec):
    g = load_golden("blocks")
    res = oracle_codec.hpack_decode_blocks(g["data"], g["blk_off"], g["conn_first"], int(g["table_size"][0]),
                                           nthreads=8, requests=True)
    check_requests_against_golden(res, g)


def test_request_fixtures_cover_the_rules():
    g = load_golden("blocks")
    w = g["rq_req"]
    st = set(int(x) for x in g["rq_bstatus"])
    assert {0, -254, -1, -9, -301} <= st
    assert set(range(8)) <= set(int(x) for x in w[:, 10])  # every HHUFF_HERR_* (err_desc) value
    assert {0, 1, 2, 3} <= set(int(x) for x in w[:, 11])  # scheme unset / http / https / masque
    cl = w[:, 0].astype(np.uint64) | (w[:, 1].astype(np.uint64) << np.uint64(32))
    assert (cl != np.uint64(2 ** 64 - 1)).sum() > 10 and (cl == np.uint64(9999999999999999999)).any()
    assert (w[:, 9] == 100).any() and (w[:, 8] & 16).any()  # header-list limit reached; :protocol seen
    assert (w[:, W_EXPECT].view(np.int32) >= 0).any() and (g["rq_fflags"] & 4).any()
    assert (g["rq_nfields"] > 1000).any()


def test_restatement_matches_compiled_reference_on_fresh_requests():
    from oracle import oracle as O

    if not O.ref_available():
        pytest.skip("oracle/_ref not built (no /root/reference here)")
    for seed, ts in ((35, 4096), (36, 256), (37, 0)):
        b = HS.make_connections(800, seed=seed, table_size=ts, adversarial_frac=0.1, request_frac=0.3)
        ro = O.oracle().hpack_decode_blocks(b["data"], b["blk_off"], b["conn_first"], ts, requests=True)
        rr = O.ref().hpack_decode_blocks(b["data"], b["blk_off"], b["conn_first"], ts, requests=True)
        nblk = len(b["blk_off"]) - 1
        np.testing.assert_array_equal(ro["nfields"][:nblk], rr["nfields"][:nblk])
        np.testing.assert_array_equal(ro["bstatus"][:nblk], rr["bstatus"][:nblk])
        np.testing.assert_array_equal(req_words(ro, nblk), req_words(rr, nblk))
        for b_ in range(nblk):
            s0, k = int(b["blk_off"][b_]), int(ro["nfields"][b_])
            np.testing.assert_array_equal(ro["fflags"][s0:s0 + k] & 4, rr["fflags"][s0:s0 + k] & 4)


def test_fixtures_cover_the_paths():
    g = load_golden("blocks")
    st = set(int(x) for x in g["bstatus"])
    assert {0, -9, -1, -301} <= st  # ok, COMPRESSION, PROTOCOL, skipped after an error
    assert (g["fld_soft"] == 1).any() and (g["fld_soft"] == 2).any()
    assert int(g["nfields"].sum()) > 100000
    # the static-table sweep: indices 1..61 decode to RFC 7541 Appendix A (checked by the reference)
    en, ev, _ = expected_fields(g)
    from h2o_amd import tables

    k = int(g["nfields"][:6].sum())  # 6 request blocks of the unit test come first, then the sweep
    assert list(zip(en[k:k + 61], ev[k:k + 61])) == list(tables.STATIC_TABLE)


def test_restatement_matches_compiled_reference_on_fresh_connections():
    from oracle import oracle as O

    if not O.ref_available():
        pytest.skip("oracle/_ref not built (no /root/reference here)")
    for seed, ts in ((31, 4096), (32, 256), (33, 0), (34, 65536)):
        b = HS.make_connections(600, seed=seed, table_size=ts, adversarial_frac=0.3)
        ro = O.oracle().hpack_decode_blocks(b["data"], b["blk_off"], b["conn_first"], ts)
        rr = O.ref().hpack_decode_blocks(b["data"], b["blk_off"], b["conn_first"], ts)
        nblk = len(b["blk_off"]) - 1
        np.testing.assert_array_equal(ro["nfields"][:nblk], rr["nfields"][:nblk])
        np.testing.assert_array_equal(ro["bstatus"][:nblk], rr["bstatus"][:nblk])
        a, b2 = fields_of(ro, b["blk_off"], nblk), fields_of(rr, b["blk_off"], nblk)
        assert a[0] == b2[0] and a[1] == b2[1]
        np.testing.assert_array_equal(soft_code(a[2]), b2[2])


# ---------------------------------------------------------------------------------------------------
# GPU
# ---------------------------------------------------------------------------------------------------
@pytest.fixture(scope="module")
def torch_cuda():
    import torch

    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    return torch


def gpu_blocks(torch, data, blk_off, conn_first, table_size, arena_off=None, requests=False):
    from h2o_amd import codec

    dev = lambda a: torch.from_numpy(np.ascontiguousarray(a).copy()).cuda()  # noqa: E731
    d = dev(data if data.size else np.zeros(1, np.uint8))
    ao = None if arena_off is None else dev(np.asarray(arena_off, np.uint64).view(np.int64))
    r = codec.hpack_decode_blocks(d, dev(blk_off.view(np.int32)), dev(conn_first.view(np.int32)), table_size,
                                  arena_off=ao, in_size=int(data.size), requests=requests)
    torch.cuda.synchronize()
    out = {}
    for k, v in r.items():
        if k == "scratch":
            continue
        a = v.cpu().numpy()
        out[k] = a.view(np.uint32) if k in ("name_off", "name_len", "value_off", "value_len", "nfields") else a
    return out


@pytest.mark.gpu
@pytest.mark.parametrize("name", BLOCK_SETS)
def test_gpu_matches_reference_fixtures(torch_cuda, name):
    g = load_golden(name)
    res = gpu_blocks(torch_cuda, g["data"], g["blk_off"], g["conn_first"], int(g["table_size"][0]))
    check_against_golden(res, g)


@pytest.mark.gpu
@pytest.mark.parametrize("seed,table_size", [(41, 4096), (42, 256), (43, 0), (44, 65536)])
def test_gpu_matches_restatement_field_by_field(torch_cuda, oracle_codec, seed, table_size):
    b = HS.make_connections(3000, seed=seed, table_size=table_size, adversarial_frac=0.3)
    ro = oracle_codec.hpack_decode_blocks(b["data"], b["blk_off"], b["conn_first"], table_size, nthreads=8)
    rg = gpu_blocks(torch_cuda, b["data"], b["blk_off"], b["conn_first"], table_size)
    nblk = len(b["blk_off"]) - 1
    np.testing.assert_array_equal(rg["nfields"][:nblk], ro["nfields"][:nblk])
    np.testing.assert_array_equal(rg["bstatus"][:nblk], ro["bstatus"][:nblk])
    for b_ in range(nblk):  # same arena offsets, lengths and full soft bits in every used slot
        s, n = int(b["blk_off"][b_]), int(ro["nfields"][b_])
        for k in ("name_off", "name_len", "value_off", "value_len", "fflags"):
            np.testing.assert_array_equal(rg[k][s:s + n], ro[k][s:s + n], err_msg="%s block %d" % (k, b_))
    ga, oa = fields_of(rg, b["blk_off"], nblk), fields_of(ro, b["blk_off"], nblk)
    assert ga[0] == oa[0] and ga[1] == oa[1]


@pytest.mark.gpu
def test_gpu_arena_limit_matches_restatement(torch_cuda, oracle_codec):
    """tight arena slices: HHUFF_BLK_ARENA exactly where the restatement reports it"""
    b = HS.make_connections(800, seed=45, adversarial_frac=0.1)
    L = np.diff(b["blk_off"].astype(np.uint64))
    rng = np.random.default_rng(46)
    cap = (L * rng.uniform(0.3, 1.6, size=L.size)).astype(np.uint64)
    ao = np.zeros(L.size + 1, np.uint64)
    ao[1:] = np.cumsum(cap)
    ro = oracle_codec.hpack_decode_blocks(b["data"], b["blk_off"], b["conn_first"], 4096, arena_off=ao)
    rg = gpu_blocks(torch_cuda, b["data"], b["blk_off"], b["conn_first"], 4096, arena_off=ao)
    nblk = L.size
    assert (ro["bstatus"][:nblk] == -300).any()
    np.testing.assert_array_equal(rg["bstatus"][:nblk], ro["bstatus"][:nblk])
    np.testing.assert_array_equal(rg["nfields"][:nblk], ro["nfields"][:nblk])
    ga, oa = fields_of(rg, b["blk_off"], nblk), fields_of(ro, b["blk_off"], nblk)
    assert ga[0] == oa[0] and ga[1] == oa[1]
    np.testing.assert_array_equal(ga[2], oa[2])


@pytest.mark.gpu
def test_gpu_empty_and_degenerate_batches(torch_cuda, oracle_codec):
    conns = [[], [b""], [b"\x82", b""], [b"\x20"], [b"\x3f\xe1\x1f"], [b"\x80"], [b"\xbe"]]
    b = HS.pack_connections(conns)
    ro = oracle_codec.hpack_decode_blocks(b["data"], b["blk_off"], b["conn_first"], 4096)
    rg = gpu_blocks(torch_cuda, b["data"], b["blk_off"], b["conn_first"], 4096)
    nblk = len(b["blk_off"]) - 1
    np.testing.assert_array_equal(rg["bstatus"][:nblk], ro["bstatus"][:nblk])
    np.testing.assert_array_equal(rg["nfields"][:nblk], ro["nfields"][:nblk])


@pytest.mark.gpu
@pytest.mark.parametrize("move", [False, True])
def test_gpu_tables_carry_over_between_calls(torch_cuda, oracle_codec, move):
    """HHUFF_BLK_CONTINUE: each connection's blocks split over two calls sharing the scratch decode exactly
    like one call over all of them (dynamic tables and the failed state persist).  move: the scratch is
    copied to a new buffer between the calls and the old one overwritten (tables hold offsets, not addresses)"""
    from h2o_amd import codec

    b = HS.make_connections(2000, seed=47, adversarial_frac=0.2)
    conns = [[b["data"][b["blk_off"][k]:b["blk_off"][k + 1]].tobytes()
              for k in range(b["conn_first"][c], b["conn_first"][c + 1])] for c in range(len(b["conn_first"]) - 1)]
    first = HS.pack_connections([cb[:len(cb) // 2] for cb in conns])
    second = HS.pack_connections([cb[len(cb) // 2:] for cb in conns])
    ro = oracle_codec.hpack_decode_blocks(b["data"], b["blk_off"], b["conn_first"], 4096)
    want = fields_of(ro, b["blk_off"], len(b["blk_off"]) - 1)
    torch = torch_cuda
    dev = lambda a: torch.from_numpy(np.ascontiguousarray(a).copy()).cuda()  # noqa: E731
    got, st, nf = ([], [], []), [], []
    scratch = None
    for part, cont in ((first, False), (second, True)):
        r = codec.hpack_decode_blocks(dev(part["data"] if part["data"].size else np.zeros(1, np.uint8)),
                                      dev(part["blk_off"].view(np.int32)), dev(part["conn_first"].view(np.int32)),
                                      4096, in_size=int(part["data"].size), scratch=scratch, cont=cont)
        torch.cuda.synchronize()
        scratch = r["scratch"]
        if move:
            moved = torch.empty_like(scratch)
            moved.copy_(scratch)
            scratch.fill_(0x5A)  # stays allocated: a stale address would read this
            old, scratch = scratch, moved  # noqa: F841
        h = {k: v.cpu().numpy() for k, v in r.items() if k != "scratch"}
        for k in ("name_off", "name_len", "value_off", "value_len", "nfields"):
            h[k] = h[k].view(np.uint32)
        nb = len(part["blk_off"]) - 1
        st.append((part, h["bstatus"][:nb], h["nfields"][:nb]))
        f = fields_of(h, part["blk_off"], nb)
        got[0].extend(f[0])
        got[1].extend(f[1])
    # reassemble per connection in the original block order and compare statuses and fields
    exp_status = []
    for c, cb in enumerate(conns):
        k0 = int(b["conn_first"][c])
        exp_status += list(ro["bstatus"][k0:k0 + len(cb)])
    got_status = []
    p1, s1, _ = st[0]
    p2, s2, _ = st[1]
    for c, cb in enumerate(conns):
        got_status += list(s1[p1["conn_first"][c]:p1["conn_first"][c + 1]])
        got_status += list(s2[p2["conn_first"][c]:p2["conn_first"][c + 1]])
    assert got_status == exp_status
    # fields: compare as per-connection multisets of the ordered lists (calls interleave connections)
    def per_conn(part_stats, fields):
        out, i = {}, 0
        for part, _, nfields in part_stats:
            for c in range(len(part["conn_first"]) - 1):
                for k in range(part["conn_first"][c], part["conn_first"][c + 1]):
                    n = int(nfields[k])
                    out.setdefault(c, []).extend(zip(fields[0][i:i + n], fields[1][i:i + n]))
                    i += n
        return out
    exp, i = {}, 0
    for c in range(len(conns)):
        for k in range(b["conn_first"][c], b["conn_first"][c + 1]):
            n = int(ro["nfields"][k])
            exp.setdefault(c, []).extend(zip(want[0][i:i + n], want[1][i:i + n]))
            i += n
    assert per_conn(st, got) == exp


@pytest.mark.gpu
def test_gpu_request_verdicts_match_reference_fixtures(torch_cuda):
    g = load_golden("blocks")
    res = gpu_blocks(torch_cuda, g["data"], g["blk_off"], g["conn_first"], int(g["table_size"][0]), requests=True)
    check_requests_against_golden(res, g)


@pytest.mark.gpu
@pytest.mark.parametrize("seed,table_size", [(45, 4096), (46, 256), (47, 0)])
def test_gpu_request_verdicts_match_restatement(torch_cuda, oracle_codec, seed, table_size):
    b = HS.make_connections(3000, seed=seed, table_size=table_size, adversarial_frac=0.1, request_frac=0.3)
    ro = oracle_codec.hpack_decode_blocks(b["data"], b["blk_off"], b["conn_first"], table_size, nthreads=8,
                                          requests=True)
    rg = gpu_blocks(torch_cuda, b["data"], b["blk_off"], b["conn_first"], table_size, requests=True)
    nblk = len(b["blk_off"]) - 1
    np.testing.assert_array_equal(rg["nfields"][:nblk], ro["nfields"][:nblk])
    np.testing.assert_array_equal(rg["bstatus"][:nblk], ro["bstatus"][:nblk])
    np.testing.assert_array_equal(req_words(rg, nblk), req_words(ro, nblk))
    for b_ in range(nblk):
        s0, k = int(b["blk_off"][b_]), int(ro["nfields"][b_])
        np.testing.assert_array_equal(rg["fflags"][s0:s0 + k], ro["fflags"][s0:s0 + k])
