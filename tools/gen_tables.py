#!/usr/bin/env python3
"""Table generator for the hhuff HPACK/QPACK Huffman codec (build tooling, not the oracle).

Source of truth: the static Huffman code of RFC 7541 Appendix B (a public standard).  The code is
*canonical*: within each code length, codes are assigned in increasing symbol order, and the first
code of a length is the previous length's last code + 1, shifted left.  So the whole code table is
fixed by the 257 code lengths below; the codes are re-derived here and never transcribed.

The reference builds its tables with `misc/mkhufftbl.py` (tree :356-372, accept rule :374-381,
nibble transitions :386-407, flags :419-458) into `lib/http2/hpack_huffman_table.h`.  This script is
our own construction with the same semantics, emitting layouts chosen for the MI355X kernels:

  h2o_amd/csrc/hhuff_tables.h   product tables (GPU decode window LUT, canonical long-code tables,
                                 encode table, validity bitmaps)
  h2o_amd/tables.py              host-side code table + validity sets (synthetic data, framing)
  oracle/huff_tables.h           oracle tables (the reference's 256-state x 16-nibble FSM, restated in a
                                 packed u32 layout, plus the {code, nbits} symbol table)

Run:  python3 tools/gen_tables.py          (rewrites both headers; they are committed)
      python3 tools/gen_tables.py --check  (exit 1 if the committed headers are stale)
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

# RFC 7541 Appendix B code lengths for symbols 0..256 (256 = EOS), one letter per symbol:
# 'A' = 5 bits, 'B' = 6, ... 'Z' = 30.
_RFC7541_LENGTHS = (
    "ISXXXXXXXTZXXZXXXXXXXXZXXXXXXXXXBFFHIBDGFFDGDBBBAAABBBBBBBCDKBHFIBCCCCCCCCCCCCCCCCCCCCCCDCDIOIJB"
    "KABABABBBACCBBBABCBAABCCCCCKGJIXPRPPRRRSRSSSSSTSTTRSTSSSSQRSRSSTRQPRRSSQSRRTQRSSQQRQSRSSPRRRSRRSV"
    "VPORSRUVVVWWVTUOQVWWVWTQQVVXWWWPTPQRQQSRRUUTTVSVWVVWWWWWXWWWWWVZ"
)
EOS = 256
NSYM = 257

# RFC 7230 3.2.6 tchar minus upper-case letters (the reference's valid_h2_field_name_char,
# mkhufftbl.py:311-321 encodes the same set).
NAME_VALID = set(b"!#$%&'*+-.^_`|~0123456789abcdefghijklmnopqrstuvwxyz")
# RFC 7230 field-vchar + SP + HTAB + obs-text (mkhufftbl.py:323-333): everything except CTLs other
# than HTAB, and DEL.
VALUE_VALID = set([0x09] + list(range(0x20, 0x7F)) + list(range(0x80, 0x100)))

# oracle FSM flag bits (same meaning as the reference's nghttp2_huff_decode_flag enum,
# hpack_huffman_table.h:73-81)
F_ACCEPTED = 1
F_SYM = 2
F_FAIL = 4
F_INV_NAME = 8
F_INV_VALUE = 16
F_UPPER = 32

LUT_BITS = 13  # GPU decode window

# RFC 7541 Appendix A static table (index 1..61): (name, value).  The reference holds the same table in
# lib/common/token_table.h (h2o_hpack_static_table); tests/test_hpack_blocks.py checks every index
# against the reference's decoding of it.
STATIC_TABLE = [
    (":authority", ""), (":method", "GET"), (":method", "POST"), (":path", "/"), (":path", "/index.html"),
    (":scheme", "http"), (":scheme", "https"), (":status", "200"), (":status", "204"), (":status", "206"),
    (":status", "304"), (":status", "400"), (":status", "404"), (":status", "500"), ("accept-charset", ""),
    ("accept-encoding", "gzip, deflate"), ("accept-language", ""), ("accept-ranges", ""), ("accept", ""),
    ("access-control-allow-origin", ""), ("age", ""), ("allow", ""), ("authorization", ""),
    ("cache-control", ""), ("content-disposition", ""), ("content-encoding", ""), ("content-language", ""),
    ("content-length", ""), ("content-location", ""), ("content-range", ""), ("content-type", ""),
    ("cookie", ""), ("date", ""), ("etag", ""), ("expect", ""), ("expires", ""), ("from", ""), ("host", ""),
    ("if-match", ""), ("if-modified-since", ""), ("if-none-match", ""), ("if-range", ""),
    ("if-unmodified-since", ""), ("last-modified", ""), ("link", ""), ("location", ""), ("max-forwards", ""),
    ("proxy-authenticate", ""), ("proxy-authorization", ""), ("range", ""), ("referer", ""), ("refresh", ""),
    ("retry-after", ""), ("server", ""), ("set-cookie", ""), ("strict-transport-security", ""),
    ("transfer-encoding", ""), ("user-agent", ""), ("vary", ""), ("via", ""), ("www-authenticate", ""),
]
assert len(STATIC_TABLE) == 61

# RFC 9204 Appendix A QPACK static table (index 0..98).  The reference holds the same table in
# lib/common/token_table.h (h2o_qpack_static_table); tests/test_qpack.py checks every index against the
# reference's decoding of it.
QPACK_STATIC_TABLE = [
    (":authority", ""), (":path", "/"), ("age", "0"), ("content-disposition", ""), ("content-length", "0"),
    ("cookie", ""), ("date", ""), ("etag", ""), ("if-modified-since", ""), ("if-none-match", ""),
    ("last-modified", ""), ("link", ""), ("location", ""), ("referer", ""), ("set-cookie", ""),
    (":method", "CONNECT"), (":method", "DELETE"), (":method", "GET"), (":method", "HEAD"), (":method", "OPTIONS"),
    (":method", "POST"), (":method", "PUT"), (":scheme", "http"), (":scheme", "https"), (":status", "103"),
    (":status", "200"), (":status", "304"), (":status", "404"), (":status", "503"), ("accept", "*/*"),
    ("accept", "application/dns-message"), ("accept-encoding", "gzip, deflate, br"), ("accept-ranges", "bytes"),
    ("access-control-allow-headers", "cache-control"), ("access-control-allow-headers", "content-type"),
    ("access-control-allow-origin", "*"), ("cache-control", "max-age=0"), ("cache-control", "max-age=2592000"),
    ("cache-control", "max-age=604800"), ("cache-control", "no-cache"), ("cache-control", "no-store"),
    ("cache-control", "public, max-age=31536000"), ("content-encoding", "br"), ("content-encoding", "gzip"),
    ("content-type", "application/dns-message"), ("content-type", "application/javascript"),
    ("content-type", "application/json"), ("content-type", "application/x-www-form-urlencoded"),
    ("content-type", "image/gif"), ("content-type", "image/jpeg"), ("content-type", "image/png"),
    ("content-type", "text/css"), ("content-type", "text/html; charset=utf-8"), ("content-type", "text/plain"),
    ("content-type", "text/plain;charset=utf-8"), ("range", "bytes=0-"), ("strict-transport-security", "max-age=31536000"),
    ("strict-transport-security", "max-age=31536000; includesubdomains"),
    ("strict-transport-security", "max-age=31536000; includesubdomains; preload"), ("vary", "accept-encoding"),
    ("vary", "origin"), ("x-content-type-options", "nosniff"), ("x-xss-protection", "1; mode=block"),
    (":status", "100"), (":status", "204"), (":status", "206"), (":status", "302"), (":status", "400"),
    (":status", "403"), (":status", "421"), (":status", "425"), (":status", "500"), ("accept-language", ""),
    ("access-control-allow-credentials", "FALSE"), ("access-control-allow-credentials", "TRUE"),
    ("access-control-allow-headers", "*"), ("access-control-allow-methods", "get"),
    ("access-control-allow-methods", "get, post, options"), ("access-control-allow-methods", "options"),
    ("access-control-expose-headers", "content-length"), ("access-control-request-headers", "content-type"),
    ("access-control-request-method", "get"), ("access-control-request-method", "post"), ("alt-svc", "clear"),
    ("authorization", ""), ("content-security-policy", "script-src 'none'; object-src 'none'; base-uri 'none'"),
    ("early-data", "1"), ("expect-ct", ""), ("forwarded", ""), ("if-range", ""), ("origin", ""), ("purpose", "prefetch"),
    ("server", ""), ("timing-allow-origin", "*"), ("upgrade-insecure-requests", "1"), ("user-agent", ""),
    ("x-forwarded-for", ""), ("x-frame-options", "deny"), ("x-frame-options", "sameorigin"),
]
assert len(QPACK_STATIC_TABLE) == 99


def static_arrays(table=None):
    """-> (bytes of all names and values back to back, [name_off, name_len, value_off, value_len] per entry)"""
    blob, ent = bytearray(), []
    for n, v in (STATIC_TABLE if table is None else table):
        ent += [len(blob), len(n)]
        blob += n.encode()
        ent += [len(blob), len(v)]
        blob += v.encode()
    return bytes(blob), ent


def code_lengths():
    lens = [ord(c) - ord("A") + 5 for c in _RFC7541_LENGTHS]
    assert len(lens) == NSYM, len(lens)
    return lens


def canonical_codes(lens):
    """Canonical code assignment: (length, symbol) order."""
    order = sorted(range(NSYM), key=lambda s: (lens[s], s))
    codes = [0] * NSYM
    code = 0
    prev_len = lens[order[0]]
    for i, s in enumerate(order):
        if i:
            code = (code + 1) << (lens[s] - prev_len)
        codes[s] = code
        prev_len = lens[s]
    # the code must be complete (Kraft sum == 1) and the last code all ones (EOS = 30 ones)
    assert sum(2.0 ** -l for l in lens) == 1.0
    assert codes[EOS] == (1 << 30) - 1 and lens[EOS] == 30
    return codes, order


def build_tree(lens, codes):
    """Binary tree: internal nodes are dicts {0: child, 1: child}; leaves are ints (symbols)."""
    root = {}
    for s in range(NSYM):
        node = root
        for i in range(lens[s] - 1, -1, -1):
            b = (codes[s] >> i) & 1
            if i == 0:
                assert b not in node
                node[b] = s
            else:
                node = node.setdefault(b, {})
    return root


def number_internal(root):
    """Preorder numbering of internal nodes; accept = path is all ones and <= 7 bits
    (mkhufftbl.py:374-381)."""
    ids, accept, nodes = {}, {}, []

    def walk(node, path):
        if not isinstance(node, dict):
            return
        ids[id(node)] = len(nodes)
        nodes.append(node)
        accept[id(node)] = len(path) <= 7 and all(b == 1 for b in path)
        walk(node[0], path + [0])
        walk(node[1], path + [1])

    walk(root, [])
    assert len(nodes) == 256
    return ids, accept, nodes


def sym_flags(sym):
    f = 0
    if sym not in NAME_VALID:
        f |= F_INV_NAME
    if sym not in VALUE_VALID:
        f |= F_INV_VALUE
    if ord("A") <= sym <= ord("Z"):
        f |= F_UPPER
    return f


def nibble_fsm(root):
    """256 states x 16 nibbles -> packed u32 {next_state | flags << 8 | sym << 16}.

    One nibble step walks 4 bits from the state's node; completing a leaf emits its symbol (at most one
    per nibble since the shortest code is 5 bits) and restarts at the root; completing EOS fails.
    The entry is ACCEPTED when the walk ends on the root after a completed symbol or on an accepting
    node (mkhufftbl.py:386-458 semantics)."""
    ids, accept, nodes = number_internal(root)
    table = []
    for node in nodes:
        row = []
        for nib in range(16):
            cur, sym, fail = node, None, False
            for i in range(3, -1, -1):
                cur = cur[(nib >> i) & 1]
                if not isinstance(cur, dict):
                    if cur == EOS:
                        fail = True
                        break
                    assert sym is None
                    sym = cur
                    cur = root
            if fail:
                row.append(F_FAIL << 8)
                continue
            flags = 0
            if sym is not None:
                flags |= F_SYM | sym_flags(sym)
            if accept[id(cur)]:
                flags |= F_ACCEPTED
            row.append(ids[id(cur)] | flags << 8 | (sym or 0) << 16)
        table.append(row)
    return table


def decode_prefix(root, bits, nbits):
    """Decode one symbol from the top of a `nbits`-bit window; returns (sym, len) or None."""
    cur = root
    for i in range(nbits):
        cur = cur[(bits >> (nbits - 1 - i)) & 1]
        if not isinstance(cur, dict):
            return cur, i + 1
    return None


def window_lut(root):
    """GPU decode LUT indexed by the next LUT_BITS (13) bits of the stream.

    u32 entry: [7:0] sym1 | [11:8] L1 | [15:12] L12 = L1 + L2 (= L1 without a second symbol) |
               [23:16] sym2 | [24] sym1 name-invalid | [25] sym1 value-invalid | [26] sym2 name-invalid |
               [27] sym2 value-invalid | [29:28] symbols in the entry (0 LONG, 1, 2) | [30] HAS2 |
               [31] LONG (first code longer than the window).
    sym2 sits in bits 16..23 so the kernels store it with a byte store of the entry's high half
    (ds_write_b8_d16_hi), no shift.  LONG entries carry L1 = LUT_BITS + 1, the shortest code they can
    stand for, so "L1 fits in the bits left" tells the kernel whether a long code can still fit, and
    L12 = 0, so the unchecked bulk step consumes nothing for them without masking (the long-code path
    takes over).  HAS2 and LONG sit in the top bits so that a sign-bit AND with (L + c) yields the
    take/skip masks directly.
    EOS (30 bits) never fits a window, so LONG covers it."""
    lut = []
    W = LUT_BITS
    for w in range(1 << W):
        r1 = decode_prefix(root, w, W)
        if r1 is None:
            lut.append(1 << 31 | (W + 1) << 8)
            continue
        s1, l1 = r1
        e = s1 | l1 << 8 | l1 << 12 | 1 << 28
        if s1 not in NAME_VALID:
            e |= 1 << 24
        if s1 not in VALUE_VALID:
            e |= 1 << 25
        rest = W - l1
        if rest >= 5:
            r2 = decode_prefix(root, w & ((1 << rest) - 1), rest)
            if r2 is not None:
                s2, l2 = r2
                e = (e & ~(0xF << 12) & ~(3 << 28)) | s2 << 16 | (l1 + l2) << 12 | 2 << 28 | 1 << 30
                if s2 not in NAME_VALID:
                    e |= 1 << 26
                if s2 not in VALUE_VALID:
                    e |= 1 << 27
        lut.append(e)
    return lut


def long_tables(lens, codes, order):
    """Canonical decode for codes longer than the window: per distinct length L (ascending):
    lim1[L] = ((first[L] + count[L]) << (32 - L)) - 1 (left-justified inclusive limit),
    first[L], base[L] (index of first[L]'s symbol in `order`)."""
    distinct = sorted(set(lens))
    lim1, first, base, L_out = [], [], [], []
    for L in distinct:
        syms = [s for s in order if lens[s] == L]
        f = codes[syms[0]]
        assert [codes[s] for s in syms] == list(range(f, f + len(syms)))
        lim1.append(((f + len(syms)) << (32 - L)) - 1)
        first.append(f)
        base.append(order.index(syms[0]))
        L_out.append(L)
    assert lim1[-1] == 0xFFFFFFFF
    return L_out, lim1, first, base


def ones_tables(lens, codes):
    """Leading-ones decode: every code is k leading ones, then (k < 30) a zero, then at most m_k <= 5
    more bits that select the symbol (canonical structure of the RFC 7541 code).
    kinfo[k] = base_k | m_k << 16 for k = 0..30 (k >= 30 is EOS); entry[base_k + next m_k bits] =
    sym | len << 9 | name-invalid << 14 | value-invalid << 15.  Indices past a shorter code repeat it."""
    by_k = {}
    for s in range(NSYM):
        b = format(codes[s], "0%db" % lens[s])
        k = len(b) - len(b.lstrip("1"))
        by_k.setdefault(k, []).append(s)
    kinfo, entries = [], []
    for k in range(31):
        syms = by_k.get(k, [])
        m = max(lens[s] for s in syms) - (k + 1) if k < 30 else 0
        m = max(m, 0)
        base = len(entries)
        for v in range(1 << m):
            hit = None
            for s in syms:
                rest = lens[s] - (k + 1) if k < 30 else 0
                tail = codes[s] & ((1 << rest) - 1) if rest > 0 else 0
                if rest <= m and (v >> (m - rest)) == tail:
                    hit = s
            assert hit is not None, (k, v)
            e = hit | lens[hit] << 9
            if hit < 256 and hit not in NAME_VALID:
                e |= 1 << 14
            if hit < 256 and hit not in VALUE_VALID:
                e |= 1 << 15
            entries.append(e)
        kinfo.append(base | m << 16)
    return kinfo, entries


def bitmap(pred):
    words = [0] * 8
    for c in range(256):
        if pred(c):
            words[c >> 5] |= 1 << (c & 31)
    return words


def fmt_array(vals, per_line, fmt):
    lines = []
    for i in range(0, len(vals), per_line):
        lines.append("    " + ", ".join(fmt.format(v) for v in vals[i:i + per_line]) + ",")
    return "\n".join(lines)


HEADER_NOTE = """/* GENERATED by tools/gen_tables.py from the RFC 7541 Appendix B code lengths -- do not edit.
 * Semantics follow the reference's generator misc/mkhufftbl.py (accept rule :374-381, transitions
 * :386-407, flags :419-458) and lib/http2/hpack_huffman_table.h; layouts are this project's own. */
"""


def product_header(lens, codes, order, lut, longt):
    L_out, lim1, first, base = longt
    kinfo, kent = ones_tables(lens, codes)
    name_inv = bitmap(lambda c: c not in NAME_VALID)
    value_inv = bitmap(lambda c: c not in VALUE_VALID)
    out = [HEADER_NOTE, "#pragma once", "#include <stdint.h>", ""]
    out.append("#define HHUFF_LUT_BITS %d" % LUT_BITS)
    out.append("#define HHUFF_NUM_LENGTHS %d" % len(L_out))
    out.append("#define HHUFF_FIRST_LONG_IDX %d  /* index of the first code length > HHUFF_LUT_BITS */"
               % next(i for i, L in enumerate(L_out) if L > LUT_BITS))
    out.append("")
    out.append("/* decode window LUT, 2^%d x u32: see tools/gen_tables.py:window_lut for the bit layout */" % LUT_BITS)
    out.append("#define HHUFF_DEC_LUT_INIT { \\")
    out.append(fmt_array(lut, 8, "0x{:08x}u").replace("\n", " \\\n") + " \\\n}")
    out.append("")
    out.append("/* canonical long-code decode: distinct code lengths ascending, inclusive left-justified limits,")
    out.append(" * first code of each length, index of that code's symbol in HHUFF_SORTED_SYMS */")
    out.append("#define HHUFF_LEN_INIT { %s }" % ", ".join(str(v) for v in L_out))
    out.append("#define HHUFF_LIM1_INIT { %s }" % ", ".join("0x%08xu" % v for v in lim1))
    out.append("#define HHUFF_FIRST_INIT { %s }" % ", ".join("0x%xu" % v for v in first))
    out.append("#define HHUFF_BASE_INIT { %s }" % ", ".join(str(v) for v in base))
    out.append("/* symbols in canonical (length, symbol) order; 256 = EOS */")
    out.append("#define HHUFF_SORTED_SYMS_INIT { \\")
    out.append(fmt_array(order, 16, "{}").replace("\n", " \\\n") + " \\\n}")
    out.append("")
    out.append("/* leading-ones decode (any code length): k = leading ones of the 32-bit window (capped at 30),")
    out.append(" * kinfo[k] = base | m << 16; entry = HHUFF_ONES_ENT[base + the m bits after the first zero] =")
    out.append(" * sym | len << 9 | name-invalid << 14 | value-invalid << 15 (see tools/gen_tables.py:ones_tables) */")
    out.append("#define HHUFF_ONES_NENT %d" % len(kent))
    out.append("#define HHUFF_ONES_KINFO_INIT { %s }" % ", ".join("0x%05xu" % v for v in kinfo))
    out.append("#define HHUFF_ONES_ENT_INIT { \\")
    out.append(fmt_array(kent, 12, "0x{:04x}u").replace("\n", " \\\n") + " \\\n}")
    out.append("")
    out.append("/* encode table: code (right-aligned) and bit length per byte value; EOS is never encoded */")
    out.append("#define HHUFF_ENC_CODE_INIT { \\")
    out.append(fmt_array(codes[:256], 8, "0x{:08x}u").replace("\n", " \\\n") + " \\\n}")
    out.append("#define HHUFF_ENC_NBITS_INIT { \\")
    out.append(fmt_array(lens[:256], 32, "{}").replace("\n", " \\\n") + " \\\n}")
    out.append("")
    out.append("/* 256-bit maps of bytes invalid in header names / values (bit c of word c>>5) */")
    out.append("#define HHUFF_NAME_INVALID_INIT { %s }" % ", ".join("0x%08xu" % w for w in name_inv))
    out.append("#define HHUFF_VALUE_INVALID_INIT { %s }" % ", ".join("0x%08xu" % w for w in value_inv))
    out.append("")
    blob, ent = static_arrays()
    out.append("/* RFC 7541 Appendix A static table: names and values back to back, and per index 1..61")
    out.append(" * {name_off, name_len, value_off, value_len} into them */")
    out.append("#define HHUFF_STATIC_NBYTES %d" % len(blob))
    out.append("#define HHUFF_STATIC_BYTES_INIT { \\")
    out.append(fmt_array(list(blob), 24, "{}").replace("\n", " \\\n") + " \\\n}")
    out.append("#define HHUFF_STATIC_ENT_INIT { \\")
    out.append(fmt_array(ent, 16, "{}").replace("\n", " \\\n") + " \\\n}")
    out.append("")
    qblob, qent = static_arrays(QPACK_STATIC_TABLE)
    out.append("/* RFC 9204 Appendix A QPACK static table: names and values back to back, and per index 0..98")
    out.append(" * {name_off, name_len, value_off, value_len} into them */")
    out.append("#define HHUFF_QSTATIC_NBYTES %d" % len(qblob))
    out.append("#define HHUFF_QSTATIC_BYTES_INIT { \\")
    out.append(fmt_array(list(qblob), 24, "{}").replace("\n", " \\\n") + " \\\n}")
    out.append("#define HHUFF_QSTATIC_ENT_INIT { \\")
    out.append(fmt_array(qent, 16, "{}").replace("\n", " \\\n") + " \\\n}")
    out.append("")
    return "\n".join(out)


def oracle_header(lens, codes, fsm):
    out = [HEADER_NOTE.replace("this project's own.", "this project's own.\n * ORACLE TABLES: test infrastructure only."),
           "#pragma once", "#include <stdint.h>", ""]
    out.append("enum { ORC_ACCEPTED = %d, ORC_SYM = %d, ORC_FAIL = %d, ORC_INV_NAME = %d, ORC_INV_VALUE = %d, "
               "ORC_UPPER = %d };" % (F_ACCEPTED, F_SYM, F_FAIL, F_INV_NAME, F_INV_VALUE, F_UPPER))
    out.append("")
    out.append("/* {code, nbits} per symbol 0..256 (hpack_huffman_table.h:29-71 restated) */")
    out.append("static const uint32_t orc_sym_code[257] = {")
    out.append(fmt_array(codes, 8, "0x{:08x}u"))
    out.append("};")
    out.append("static const uint8_t orc_sym_nbits[257] = {")
    out.append(fmt_array(lens, 32, "{}"))
    out.append("};")
    out.append("")
    out.append("/* raw-literal validity: h2o_hpack_validate_header_name / _value tables (hpack.c:171-180, 200-209) */")
    out.append("static const uint8_t orc_name_valid[256] = {")
    out.append(fmt_array([1 if c in NAME_VALID else 0 for c in range(256)], 32, "{}"))
    out.append("};")
    out.append("static const uint8_t orc_value_valid[256] = {")
    out.append(fmt_array([1 if c in VALUE_VALID else 0 for c in range(256)], 32, "{}"))
    out.append("};")
    out.append("")
    out.append("/* nibble FSM: [state][nibble] = next_state | flags << 8 | sym << 16 (hpack_huffman_table.h:89+) */")
    out.append("static const uint32_t orc_fsm[256][16] = {")
    for row in fsm:
        out.append("    {" + ", ".join("0x%06x" % v for v in row) + "},")
    out.append("};")
    out.append("")
    out.append("/* RFC 7541 Appendix A static table, indices 1..61 (entry 0 unused) */")
    out.append("static const char *const orc_static_name[62] = {\"\",")
    out.append(",\n".join('    "%s"' % n for n, _ in STATIC_TABLE) + "};")
    out.append("static const char *const orc_static_value[62] = {\"\",")
    out.append(",\n".join('    "%s"' % v for _, v in STATIC_TABLE) + "};")
    out.append("")
    out.append("/* RFC 9204 Appendix A QPACK static table, indices 0..98 */")
    out.append("static const char *const orc_qpack_static_name[99] = {")
    out.append(",\n".join('    "%s"' % n for n, _ in QPACK_STATIC_TABLE) + "};")
    out.append("static const char *const orc_qpack_static_value[99] = {")
    out.append(",\n".join('    "%s"' % v for _, v in QPACK_STATIC_TABLE) + "};")
    out.append("")
    return "\n".join(out)


def python_module(lens, codes):
    return "\n".join([
        '"""GENERATED by tools/gen_tables.py from the RFC 7541 Appendix B code lengths -- do not edit.',
        "",
        "Host-side copies of the code table and the header-name / header-value validity sets.",
        '"""',
        "ENC_CODE = (%s)" % ", ".join(str(c) for c in codes[:256]),
        "ENC_NBITS = (%s)" % ", ".join(str(l) for l in lens[:256]),
        "STATIC_TABLE = %r" % (tuple((n.encode(), v.encode()) for n, v in STATIC_TABLE),),
        "QPACK_STATIC_TABLE = %r" % (tuple((n.encode(), v.encode()) for n, v in QPACK_STATIC_TABLE),),
        "EOS_CODE = %d" % codes[EOS],
        "EOS_NBITS = %d" % lens[EOS],
        "NAME_VALID = frozenset((%s))" % ", ".join(str(c) for c in sorted(NAME_VALID)),
        "VALUE_VALID = frozenset((%s))" % ", ".join(str(c) for c in sorted(VALUE_VALID)),
        "",
    ])


def generate():
    lens = code_lengths()
    codes, order = canonical_codes(lens)
    root = build_tree(lens, codes)
    fsm = nibble_fsm(root)
    lut = window_lut(root)
    longt = long_tables(lens, codes, order)
    return {
        os.path.join(ROOT, "h2o_amd", "csrc", "hhuff_tables.h"): product_header(lens, codes, order, lut, longt),
        os.path.join(ROOT, "oracle", "huff_tables.h"): oracle_header(lens, codes, fsm),
        os.path.join(ROOT, "h2o_amd", "tables.py"): python_module(lens, codes),
    }


def main():
    check = "--check" in sys.argv
    stale = False
    for path, text in generate().items():
        old = open(path).read() if os.path.exists(path) else None
        if old != text:
            stale = True
            if not check:
                with open(path, "w") as f:
                    f.write(text)
                print("wrote", os.path.relpath(path, ROOT))
    if check and stale:
        print("generated tables are stale; run tools/gen_tables.py")
        sys.exit(1)


if __name__ == "__main__":
    main()
