#!/usr/bin/env python3
"""Generate tests/golden/* with the REAL reference codec -- test infrastructure only.

Runs here, in the build container, where oracle/_ref/libh2oref.so is compiled from
/root/reference/lib/http2/hpack.c and lib/http3/qpack.c (oracle/Makefile).  The fixtures it writes are
data (inputs + the reference's outputs) and travel to the GPU box; the reference does not.

Fixture sets (numpy .npz, arrays only, no pickles):
  kat.npz          known answers from the reference's own tests (t/00unit/lib/http2/hpack.c:175-186,
                   :293-306, :474-513, :666-682; t/00unit/lib/http3/qpack.c:236) and SURVEY Appendix A
  corpus.npz       every Huffman-flagged literal string in fuzz/http2-corpus (HEADERS + CONTINUATION
                   blocks, our own HPACK walker), decoded by the reference; raw literals encoded by it
  random_<cfg>.npz seeded synthetic batches per benchmark configuration (h2o_amd/synth.py), encoded and
                   re-decoded by the reference, plus the plain bytes decoded as (mostly invalid) Huffman
  adversarial.npz  hand-built decode edge cases (padding, EOS, truncation, long codes, names/values) and encode
                   edge cases ('X'-only strings, the ceil(bits / 8) < len verdict's edge, long codes, every byte)
  framing.npz      HPACK h2o_hpack_encode_string and QPACK flatten_string (prefix 3/5/7) outputs
  resp.npz         response header blocks / sections as h2o's clients parse them (h2o_hpack_parse_response,
                   h2o_qpack_parse_response run by the reference itself): verdicts, records, fields
  blocks.npz       header blocks (f4): the fuzz corpus's connections, the unit test's request sequences,
                   a static-table sweep and synthetic connections (h2o_amd/hpack_synth.py), decoded by
                   h2o_hpack_decode_header field after field with a table per connection (4096 bytes);
  blocks_256.npz   the unit test's response blocks and synthetic connections with a 256-byte table
  literals.npz     string literals as they sit in header blocks: every literal of the fuzz corpus's
                   HPACK blocks plus hand-built edge cases (raw names/values to validate, bad and
                   truncated integers, invalid Huffman), and QPACK name literals (prefix 3/5) -- the
                   reference's decode_int / decode_huffman / validators / h2o_lookup_token composed as
                   decode_string and decode_header_{name,value}_literal call them (oracle/ref_shim.c)
  hpenc.npz        HTTP/2 response header blocks (f4 encode half): synthetic sessions of responses flattened by
                   the real h2o_hpack_flatten_response / _trailers, and of client requests by the real
                   h2o_hpack_flatten_request, with one encoder table per connection (oracle/ref_hpenc.c), the
                   restatement checked against them as they are written; sessions with invalid arguments and
                   short output regions
  qpenc.npz        HTTP/3 response HEADERS frames (f4, QPACK encode half): synthetic responses (datagram flow ids,
                   statuses outside the static table, dont_compress, names added without their token) flattened by
                   the real h2o_qpack_flatten_response as h2o's HTTP/3 server calls it (ref_shim.c ref_qpe_step),
                   and client requests (CONNECT-UDP datagram flow ids) by the real h2o_qpack_flatten_request

Usage:  python3 oracle/gen_golden.py            (rewrites tests/golden/)
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path[0] = ROOT  # import `oracle` as the package, not this directory

from h2o_amd import synth  # noqa: E402
from oracle import oracle as O  # noqa: E402

GOLDEN = os.path.join(ROOT, "tests", "golden")
REF_ROOT = "/root/reference"
PREFACE = b"PRI * HTTP/2.0\r\n\r\nSM\r\n\r\n"


def pack(strings):
    return synth.pack(list(strings))


# ------------------------------------------------------------------------------------------------
# reference runs
# ------------------------------------------------------------------------------------------------
def ref_decode_set(strings, is_name):
    """-> dict of arrays: inputs + reference verdicts (soft bits from a zero word and from 0x2/0x1 preset)."""
    r = O.ref()
    out_len, status, decoded = [], [], []
    soft_preset = []
    for s, nm in zip(strings, is_name):
        d, soft = r.decode(s, bool(nm))
        _, soft_p = r.decode(s, bool(nm), soft_in=0x2 if nm else 0x1)
        soft_preset.append(soft_p)
        if d is None:
            out_len.append(O.FAIL)
            status.append(O.STATUS_FAIL)
        else:
            out_len.append(len(d))
            status.append(soft)
            decoded.append(d)
    data, off = pack(strings)
    dec_data, dec_off = pack(decoded)
    return dict(dec_in=data, dec_in_off=off, is_name_bits=synth.bits_from_bools(is_name),
                dec_len=np.asarray(out_len, np.uint32), dec_status=np.asarray(status, np.uint8),
                dec_soft_preset=np.asarray(soft_preset, np.uint8), dec_out=dec_data, dec_out_off=dec_off)


def ref_encode_set(strings):
    r = O.ref()
    out_len, encoded = [], []
    for s in strings:
        e = r.encode(s)
        if e is None:
            out_len.append(O.FAIL)
        else:
            out_len.append(len(e))
            encoded.append(e)
    data, off = pack(strings)
    ed, eo = pack(encoded)
    return dict(enc_in=data, enc_in_off=off, enc_len=np.asarray(out_len, np.uint32), enc_out=ed, enc_out_off=eo)


# ------------------------------------------------------------------------------------------------
# fuzz corpus walker (HTTP/2 frames -> HPACK header blocks -> string literals)
# ------------------------------------------------------------------------------------------------
def _int(buf, p, prefix):
    """RFC 7541 5.1 prefix integer -> (value, new position) or (None, None)."""
    if p >= len(buf):
        return None, None
    mx = (1 << prefix) - 1
    v = buf[p] & mx
    p += 1
    if v < mx:
        return v, p
    shift = 0
    while p < len(buf) and shift <= 56:
        b = buf[p]
        p += 1
        v += (b & 127) << shift
        if not b & 128:
            return v, p
        shift += 7
    return None, None


def header_blocks(raw):
    b = raw[len(PREFACE):] if raw.startswith(PREFACE) else raw
    pos, blocks, cur = 0, [], None
    while pos + 9 <= len(b):
        L = int.from_bytes(b[pos:pos + 3], "big")
        typ, flags = b[pos + 3], b[pos + 4]
        pos += 9
        payload = b[pos:pos + L]
        pos += L
        if len(payload) < L:
            break
        if typ == 1:
            p = payload
            if flags & 0x8:
                if not p or p[0] >= len(p):
                    continue
                p = p[1:len(p) - p[0]]
            if flags & 0x20:
                p = p[5:]
            cur = bytearray(p)
            if flags & 0x4:
                blocks.append(bytes(cur))
                cur = None
        elif typ == 9 and cur is not None:
            cur += payload
            if flags & 0x4:
                blocks.append(bytes(cur))
                cur = None
    if cur:
        blocks.append(bytes(cur))
    return blocks


def block_strings(block):
    """-> list of (is_name, huffman_flag, bytes) for every string literal of an HPACK block"""
    out, p = [], 0

    def string(p):
        if p >= len(block):
            return None, None, None
        h = bool(block[p] & 0x80)
        n, p = _int(block, p, 7)
        if n is None or p + n > len(block):
            return None, None, None
        return h, block[p:p + n], p + n

    while p < len(block):
        c = block[p]
        if c & 0x80:
            _, p = _int(block, p, 7)
            if p is None:
                break
            continue
        if c & 0x40:
            idx, p = _int(block, p, 6)
        elif c & 0x20:
            _, p = _int(block, p, 5)
            if p is None:
                break
            continue
        else:
            idx, p = _int(block, p, 4)
        if p is None:
            break
        if idx == 0:
            h, s, p = string(p)
            if p is None:
                break
            out.append((True, h, s))
        h, s, p = string(p)
        if p is None:
            break
        out.append((False, h, s))
    return out


def corpus_strings():
    d = os.path.join(REF_ROOT, "fuzz", "http2-corpus")
    huff, raw = [], []
    for f in sorted(os.listdir(d)):
        with open(os.path.join(d, f), "rb") as fh:
            data = fh.read()
        for blk in header_blocks(data):
            for is_name, h, s in block_strings(blk):
                (huff if h else raw).append((is_name, bytes(s)))
    return huff, raw


# ------------------------------------------------------------------------------------------------
# fixture sets
# ------------------------------------------------------------------------------------------------
def huff_bits(s):
    """Huffman bytes of `s` by direct bit packing (valid even when not shorter than `s`)."""
    bits = "".join(format(synth.tables.ENC_CODE[c], "0%db" % synth.tables.ENC_NBITS[c]) for c in s)
    bits += "1" * (-len(bits) % 8)
    return int(bits, 2).to_bytes(len(bits) // 8, "big") if bits else b""


def kat_set():
    enc = huff_bits
    dec_cases = [
        (bytes.fromhex("f1e3c2e5f23a6ba0ab90f4ff"), 0),  # hpack test :175-186 -> www.example.com
        (bytes.fromhex("a8eb10649cbf"), 0),  # RFC 7541 C.4.2 "no-cache"
        (bytes.fromhex("25a849e95ba97d7f"), 1),  # C.4.3 "custom-key"
        (bytes.fromhex("25a849e95bb8e8b4bf"), 0),  # C.4.3 "custom-value"
        (bytes.fromhex("f2b543a4bf"), 1),  # hpack test :474-488 "x-name"
        (bytes.fromhex("49509f"), 0),  # hpack test :505-513 "test"
        (bytes.fromhex("5071ff"), 0),  # :666-682 " ab" (soft: leading SP)
        (bytes.fromhex("ffffea1c7f"), 0),  # "\tab" (soft: leading HT)
        (bytes.fromhex("1c6a7f"), 0),  # "ab " (soft: trailing SP)
        (b"", 0), (b"", 1),  # empty value ok / empty name soft
        (b"\xff", 0), (b"\x1f", 0), (b"\x1e", 0), (b"\x07\xff", 0), (b"\xff\xff\xff\xff", 0),
        (enc(b"Aeeeeeee"), 1), (enc(b":Aeeeeeee"), 1), (enc(b":Path"), 1), (enc(b"Content-Type"), 1),
        (enc(b"ae eeeee"), 1), (enc(b"ae eeeee"), 0), (enc(b"aeeeeeee\n"), 0), (enc(b"aeeeeeee\x7f"), 0),
        (enc(b"\taeeeeeee"), 0), (enc(b"aeeeeeee\t"), 0), (enc(b"aeeeeeee\x80"), 0), (enc(b"aeeeeeee\x80"), 1),
    ]
    d = ref_encode_set([b"www.example.com", b"", b"a", b"aa", b"A", b"\x00", b"aaa", b"ABCDEFGH", b"00000000",
                        b"no-cache", b"custom-key", b"custom-value", b"x-name", b"test", b" ab",
                        b"private", b"Mon, 21 Oct 2013 20:13:21 GMT", b"https://www.example.com"]
                       + [b"X" * k for k in range(1, 9)])
    d.update(ref_decode_set([s for s, _ in dec_cases], [n for _, n in dec_cases]))
    return d


def random_set(cfg, n, seed):
    b = synth.make_batch(cfg, n=n, seed=seed, adversarial_frac=0.05)
    plain = synth.unpack(b["data"], b["off"])
    d = ref_encode_set(plain)
    # decode inputs: every successful encoding (wire-like), then the plain bytes read as Huffman
    names = np.unpackbits(b["is_name_bits"].view(np.uint8), bitorder="little")[:n].astype(bool)
    encs = [r for r in synth.unpack(d["enc_out"], d["enc_out_off"])]
    enc_names = [nm for nm, L in zip(names, d["enc_len"]) if L != O.FAIL]
    dec_in = encs + plain
    dec_names = list(enc_names) + list(names)
    d.update(ref_decode_set(dec_in, dec_names))
    d["seed"] = np.asarray([seed], np.int64)
    return d


def adversarial_set(seed=7):
    rng = np.random.default_rng(seed)
    r = O.ref()
    cases = []
    # random byte strings
    for _ in range(3000):
        L = int(rng.integers(0, 48))
        cases.append(bytes(rng.integers(0, 256, L, dtype=np.uint8)))
    # valid encodings of varied plain strings, then mutated
    syms, p = synth.header_alphabet()
    for _ in range(1500):
        L = int(rng.integers(1, 40))
        s = bytes(rng.choice(syms, L, p=p)) if rng.random() < 0.7 else bytes(rng.integers(0, 256, L, dtype=np.uint8))
        e = r.encode(s)
        if e is None:
            continue
        cases.append(e)
        cases.append(e + b"\xff")  # padding > 7 bits
        cases.append(e[:-1])  # truncated
        b = bytearray(e)
        b[-1] ^= 1  # padding bit flipped
        cases.append(bytes(b))
        b = bytearray(e)
        b[int(rng.integers(0, len(b)))] ^= 1 << int(rng.integers(0, 8))  # random bit flip
        cases.append(bytes(b))
        k = int(rng.integers(0, len(e)))
        cases.append(e[:k] + b"\xff\xff\xff\xff" + e[k:])  # EOS-containing run of ones
    # strings of long codes only (control bytes, high bytes)
    for _ in range(300):
        L = int(rng.integers(1, 20))
        s = bytes(rng.choice(np.r_[0:32, 127:256], L).astype(np.uint8))
        cases.append(huff_bits(s))
    # EOS exactly at the end / after a symbol, with 0-7 bits of padding around it
    for pre in range(0, 8):
        bits = "0" * 5 * pre + "1" * 30
        bits += "1" * (-len(bits) % 8)
        cases.append(int(bits, 2).to_bytes(len(bits) // 8, "big"))
    is_name = rng.random(len(cases)) < 0.5
    return ref_decode_set(cases, is_name)


def adversarial_encode_strings(seed=8):
    """encode edge cases, verdicts from the compiled reference (h2o_hpack_encode_huffman, hpack.c:774-804):
    'X'-only strings, which never compress ('X' is an 8-bit code: t/40http3/test.pl:194 relies on it); strings
    at the verdict's edge (hpack.c:799-800: ceil(bits / 8) < len passes, == len fails), built from 5-bit and
    8-bit symbols so the total is 8n - 9 .. 8n - 1 bits; long-code-only strings (control bytes, 0x80+, up to 30-bit
    codes); every single byte; the empty string; all 256 bytes in a row; and random mixes"""
    rng = np.random.default_rng(seed)
    out = [b"", bytes(range(256)), bytes(range(255, -1, -1))]
    out += [b"X" * L for L in range(0, 300, 7)] + [b"X" * 4096]
    out += [bytes([b]) for b in range(256)]
    for n in range(2, 60):
        for k in range(0, 9):  # n - k symbols 'X' (8 bits) and k symbols 'a' (5 bits): 8n - 3k bits
            if k <= n:
                out.append(b"X" * (n - k) + b"a" * k)
                out.append(bytes(rng.permutation(list(b"X" * (n - k) + b"a" * k)).astype(np.uint8)))
    for _ in range(400):
        L = int(rng.integers(1, 64))
        out.append(bytes(rng.choice(np.r_[0:32, 127:256], L).astype(np.uint8)))
    syms, p = synth.header_alphabet()
    for _ in range(600):
        L = int(rng.integers(1, 200))
        a = rng.choice(syms, L, p=p).astype(np.uint8)
        bad = rng.random(L) < rng.choice([0.0, 0.05, 0.3, 1.0])
        a[bad] = rng.integers(0, 256, int(bad.sum()), dtype=np.uint8)
        out.append(bytes(a))
    return out


def framing_set(seed=11):
    rng = np.random.default_rng(seed)
    r = O.ref()
    strings = [b"", b"a", b"www.example.com", b"X" * 200, bytes(range(256))]
    syms, p = synth.header_alphabet()
    for _ in range(300):
        L = int(rng.choice([rng.integers(0, 30), rng.integers(100, 200), rng.integers(256, 768), rng.integers(1000, 3000)]))
        if rng.random() < 0.5:
            s = bytes(rng.choice(synth.COOKIE_CHARSET, L))
        else:
            s = bytes(rng.choice(syms, L, p=p))
        strings.append(s)
    prefix = rng.choice([3, 5, 7], len(strings)).astype(np.uint8)
    first = rng.integers(0, 256, len(strings), dtype=np.uint8)
    raw = rng.random(len(strings)) < 0.1
    hpack_out = [r.encode_string(s) for s in strings]
    qpack_out = [r.flatten_string(s, int(pb), int(fb), bool(rw)) for s, pb, fb, rw in zip(strings, prefix, first, raw)]
    data, off = pack(strings)
    hd, ho = pack(hpack_out)
    qd, qo = pack(qpack_out)
    # prefix-integer known answers (hpack.c:52-83 / :757-772)
    ints = [0, 1, 2, 30, 31, 32, 62, 63, 64, 126, 127, 128, 254, 255, 256, 1337, 4096, 16383, 16384, 2 ** 21,
            2 ** 28 - 1, 2 ** 31, 2 ** 40 + 5, 2 ** 62, 2 ** 63 - 1]
    int_out = []
    for pb in (3, 4, 5, 6, 7):
        for v in ints:
            int_out.append(r.encode_int(v, pb))
    iod, ioo = pack(int_out)
    return dict(fr_in=data, fr_in_off=off, fr_prefix=prefix, fr_first=first, fr_raw=raw.astype(np.uint8),
                hpack_out=hd, hpack_out_off=ho, qpack_out=qd, qpack_out_off=qo,
                int_values=np.asarray(ints, np.uint64), int_out=iod, int_out_off=ioo)


def block_literals(block):
    """-> list of (offset of the literal's first byte, is_name) for every string literal of a block"""
    out, p = [], 0
    while p < len(block):
        c = block[p]
        if c & 0x80:
            _, p = _int(block, p, 7)
            if p is None:
                break
            continue
        if c & 0x40:
            idx, p = _int(block, p, 6)
        elif c & 0x20:
            _, p = _int(block, p, 5)
            if p is None:
                break
            continue
        else:
            idx, p = _int(block, p, 4)
        if p is None:
            break
        for is_name in ((True, False) if idx == 0 else (False,)):
            if p >= len(block):
                return out
            out.append((p, is_name))
            n, q = _int(block, p, 7)
            if n is None or q + n > len(block):
                return out
            p = q + n
    return out


def _lit(first_hi, prefix, huff, payload, r=None):
    """literal bytes: first byte's bits above the H flag, H flag at bit `prefix`, prefix-int length"""
    head = bytes([(first_hi & ~((2 << prefix) - 1) & 0xFF) | ((1 << prefix) if huff else 0)])
    enc = O.ref().encode_int(len(payload), prefix, head[0])
    return enc + payload


def literals_set(seed=13):
    r = O.ref()
    rng = np.random.default_rng(seed)
    buf, offs, ends, names = bytearray(), [], [], []
    # (1) HPACK: the corpus's header blocks as they are
    d = os.path.join(REF_ROOT, "fuzz", "http2-corpus")
    for f in sorted(os.listdir(d)):
        with open(os.path.join(d, f), "rb") as fh:
            data = fh.read()
        for blk in header_blocks(data):
            base = len(buf)
            lits = block_literals(blk)
            if not lits:
                continue
            buf += blk
            for p, nm in lits:
                offs.append(base + p)
                ends.append(base + len(blk))
                names.append(nm)
    n_corpus = len(offs)
    # (2) HPACK edge cases, one block
    huf = lambda s: huff_bits(s)  # noqa: E731
    cases = [  # (is_name, literal bytes)
        (True, _lit(0, 7, False, b"Content-Type")), (True, _lit(0, 7, False, b"x y")), (True, _lit(0, 7, False, b"")),
        (True, _lit(0, 7, False, b":authority")), (True, _lit(0, 7, False, b":custom")),
        (True, _lit(0, 7, False, b"a B")), (True, _lit(0, 7, False, b"ab\x00c")), (True, _lit(0, 7, False, b"ok-name")),
        (True, _lit(0, 7, False, b"A b")), (True, _lit(0, 7, False, b"a\x01B c")), (True, _lit(0, 7, False, b"Zz")),
        (False, _lit(0, 7, False, b" lead")), (False, _lit(0, 7, False, b"trail\t")), (False, _lit(0, 7, False, b"")),
        (False, _lit(0, 7, False, b"\x01bad")), (False, _lit(0, 7, False, b"del\x7f")), (False, _lit(0, 7, False, b"fine")),
        (False, _lit(0, 7, False, bytes(range(0x80, 0x100)))),
        (True, _lit(0, 7, True, huf(b"UPPER"))), (True, _lit(0, 7, True, huf(b":upper-OK"))), (True, _lit(0, 7, True, b"")),
        (False, _lit(0, 7, True, huf(b" sp "))), (False, _lit(0, 7, True, b"\xff\xff\xff\xff")),
        (False, _lit(0, 7, True, huf(b"www.example.com")[:-1])), (False, _lit(0, 7, True, huf(b"A" * 300))),
        (False, bytes([0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0x01])),  # 9th octet continuation
        (False, bytes([0x7F, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0x7F])),  # > INT64_MAX? (value check)
        (False, bytes([0x05]) + b"abc"),  # length past the block end (TRUNCATED) -- last before the tail
    ]
    base = len(buf)
    blk = bytearray()
    for nm, b in cases[:-1]:
        offs.append(base + len(blk))
        names.append(nm)
        blk += b
    offs.append(base + len(blk))
    names.append(cases[-1][0])
    blk += cases[-1][1]
    buf += blk
    ends += [base + len(blk)] * len(cases)
    # truncated integer at the very end of a block, and an empty tail
    base = len(buf)
    buf += bytes([0x7F, 0x80])
    offs += [base, base + 2]
    ends += [base + 2, base + 2]
    names += [False, False]
    n_hpack = len(offs)
    # (3) QPACK name literals with prefix 3 and 5 (and values with 7): raw / Huffman, tokens
    syms, p = synth.header_alphabet()
    q_off = {3: [], 5: [], 7: []}
    q_end = {3: [], 5: [], 7: []}
    q_name = {3: [], 5: [], 7: []}
    qbuf = bytearray()
    pool = [b":path", b":status", b":custom", b"content-type", b"Accept", b"x-a b", b""]
    for i in range(1500):
        pb = int(rng.choice([3, 5, 7]))
        nm = pb != 7 or rng.random() < 0.3
        k = rng.random()
        if k < 0.3:
            s = pool[int(rng.integers(0, len(pool)))]
        else:
            s = bytes(rng.choice(syms, int(rng.integers(0, 40)), p=p))
        huff = rng.random() < 0.5
        lit = _lit(int(rng.integers(0, 256)), pb, huff, huf(s) if huff else s)
        q_off[pb].append(len(qbuf))
        qbuf += lit
        q_end[pb].append(len(qbuf))
        q_name[pb].append(nm)
    res = dict(lit_in=np.frombuffer(bytes(buf), np.uint8), lit_off=np.asarray(offs, np.uint32),
               lit_end=np.asarray(ends, np.uint32), lit_names=synth.bits_from_bools(np.asarray(names, bool)),
               n_corpus=np.asarray([n_corpus], np.uint32), q_in=np.frombuffer(bytes(qbuf), np.uint8))
    lit_in = res["lit_in"]
    out, ol, po, cons, st = r.literals_batch(lit_in, res["lit_off"], res["lit_end"], n_hpack, 7,
                                             is_name_bits=res["lit_names"])
    slots = (po.astype(np.uint64) * 8) // 5
    res.update(h_out_len=ol, h_pay_off=po, h_consumed=cons, h_status=st,
               h_out=np.frombuffer(b"".join(out[int(a):int(a) + int(L)].tobytes() for a, L in zip(slots, ol)
                                            if L != 0xFFFFFFFF), np.uint8))
    for pb in (3, 5, 7):
        qo, qe = np.asarray(q_off[pb], np.uint32), np.asarray(q_end[pb], np.uint32)
        qn = synth.bits_from_bools(np.asarray(q_name[pb], bool))
        out, ol, po, cons, st = r.literals_batch(res["q_in"], qo, qe, len(qo), pb, qpack=True, is_name_bits=qn)
        slots = (po.astype(np.uint64) * 8) // 5
        res.update({"q%d_off" % pb: qo, "q%d_end" % pb: qe, "q%d_names" % pb: qn, "q%d_out_len" % pb: ol,
                    "q%d_pay_off" % pb: po, "q%d_consumed" % pb: cons, "q%d_status" % pb: st,
                    "q%d_out" % pb: np.frombuffer(b"".join(out[int(a):int(a) + int(L)].tobytes()
                                                           for a, L in zip(slots, ol) if L != 0xFFFFFFFF), np.uint8)})
    return res


# ------------------------------------------------------------------------------------------------
# header blocks (f4): h2o_hpack_decode_header over whole blocks, one dynamic table per connection
# ------------------------------------------------------------------------------------------------
# request sequences of the reference's unit test (t/00unit/lib/http2/hpack.c:287-296: RFC 7541 C.3 / C.4)
UNIT_REQUESTS = [
    [b"\x82\x86\x84\x41\x0f\x77\x77\x77\x2e\x65\x78\x61\x6d\x70\x6c\x65\x2e\x63\x6f\x6d",
     b"\x82\x86\x84\xbe\x58\x08\x6e\x6f\x2d\x63\x61\x63\x68\x65",
     b"\x82\x87\x85\xbf\x40\x0a\x63\x75\x73\x74\x6f\x6d\x2d\x6b\x65\x79\x0c\x63\x75\x73\x74"
     b"\x6f\x6d\x2d\x76\x61\x6c\x75\x65"],
    [b"\x82\x86\x84\x41\x8c\xf1\xe3\xc2\xe5\xf2\x3a\x6b\xa0\xab\x90\xf4\xff",
     b"\x82\x86\x84\xbe\x58\x86\xa8\xeb\x10\x64\x9c\xbf",
     b"\x82\x87\x85\xbf\x40\x88\x25\xa8\x49\xe9\x5b\xa9\x7d\x7f\x89\x25\xa8\x49\xe9\x5b\xb8\xe8\xb4\xbf"],
]
# response blocks of the same test with a 256-byte table (:309-331, including the disabled vectors)
UNIT_RESPONSES_256 = [
    [b"\x08\x03\x33\x30\x32\x58\x85\xae\xc3\x77\x1a\x4b\x61\x96\xd0\x7a\xbe\x94\x10"
     b"\x54\xd4\x44\xa8\x20\x05\x95\x04\x0b\x81\x66\xe0\x82\xa6\x2d\x1b\xff\x6e\x91"
     b"\x9d\x29\xad\x17\x18\x63\xc7\x8f\x0b\x97\xc8\xe9\xae\x82\xae\x43\xd3",
     b"\x08\x03\x33\x30\x37\xc0\xbf\xbe"],
    [b"\x48\x03\x33\x30\x37\xc1\xc0\xbf",
     b"\x88\xc1\x61\x1d\x4d\x6f\x6e\x2c\x20\x32\x31\x20\x4f\x63\x74\x20\x32\x30\x31\x33\x20\x32\x30\x3a"
     b"\x31\x33\x3a\x32\x32\x20\x47\x4d\x54\xc0\x5a\x04\x67\x7a\x69\x70\x77\x38\x66\x6f\x6f\x3d\x41\x53"
     b"\x44\x4a\x4b\x48\x51\x4b\x42\x5a\x58\x4f\x51\x57\x45\x4f\x50\x49\x55\x41\x58\x51\x57\x45\x4f\x49"
     b"\x55\x3b\x20\x6d\x61\x78\x2d\x61\x67\x65\x3d\x33\x36\x30\x30\x3b\x20\x76\x65\x72\x73\x69\x6f\x6e\x3d\x31"],
]


def soft_code(bits):
    """what h2o_hpack_decode_header reports for a field's soft errors: its err_desc names the name
    error when there is one (hpack.c:427-431): 1 name, 2 value only, 0 none"""
    bits = np.asarray(bits)
    return np.where(bits & 1, 1, np.where(bits & 2, 2, 0)).astype(np.uint8)


def blocks_set(conns, table_size, requests=False):
    from h2o_amd import hpack_synth as HS

    b = HS.pack_connections(conns, table_size)
    r = O.ref().hpack_decode_blocks(b["data"], b["blk_off"], b["conn_first"], table_size)
    nb = len(b["blk_off"]) - 1
    names, values, soft = [], [], []
    for bi in range(nb):
        s = int(b["blk_off"][bi])
        for f in range(s, s + int(r["nfields"][bi])):
            names.append(r["arena"][r["name_off"][f]:r["name_off"][f] + r["name_len"][f]].tobytes())
            values.append(r["arena"][r["value_off"][f]:r["value_off"][f] + r["value_len"][f]].tobytes())
            soft.append(r["fflags"][f])
    nd, no = pack(names)
    vd, vo = pack(values)
    out = dict(data=b["data"], blk_off=b["blk_off"], conn_first=b["conn_first"],
               table_size=np.asarray([table_size], np.uint32), nfields=r["nfields"][:nb], bstatus=r["bstatus"][:nb],
               fld_name=nd, fld_name_off=no, fld_value=vd, fld_value_off=vo, fld_soft=np.asarray(soft, np.uint8))
    if requests:
        # h2o_hpack_parse_request over the same blocks (ref_hpack_parse_requests): its verdicts, the request
        # record of every block and each decoded field's flags (soft bits | HHUFF_FIELD_HEADER).  Its fields
        # are a prefix of the decode-only fields of the same block (the same decoder, stopped earlier), which
        # is checked here so the fixture need not repeat them.
        q = O.ref().hpack_decode_blocks(b["data"], b["blk_off"], b["conn_first"], table_size, requests=True)
        fl = []
        for bi in range(nb):
            s0, k = int(b["blk_off"][bi]), int(q["nfields"][bi])
            assert k <= int(r["nfields"][bi]) or int(r["bstatus"][bi]) != 0
            for f in range(s0, s0 + k):
                assert q["arena"][q["name_off"][f]:q["name_off"][f] + q["name_len"][f]].tobytes() == \
                    r["arena"][r["name_off"][f]:r["name_off"][f] + r["name_len"][f]].tobytes()
                assert q["arena"][q["value_off"][f]:q["value_off"][f] + q["value_len"][f]].tobytes() == \
                    r["arena"][r["value_off"][f]:r["value_off"][f] + r["value_len"][f]].tobytes()
                fl.append(q["fflags"][f])
        out.update(rq_nfields=q["nfields"][:nb], rq_bstatus=q["bstatus"][:nb],
                   rq_req=q["req"][:nb].view(np.uint32).reshape(nb, 12), rq_fflags=np.asarray(fl, np.uint8))
    return out


def blocks_sets():
    from h2o_amd import hpack_synth as HS

    d = os.path.join(REF_ROOT, "fuzz", "http2-corpus")
    corpus = []
    for fn in sorted(os.listdir(d)):
        blocks = header_blocks(open(os.path.join(d, fn), "rb").read())
        if blocks:
            corpus.append(blocks)
    static_sweep = [[b"".join(HS.encode_int(i, 7, 0x80) for i in range(1, 62))]]
    syn = HS.make_connections(2500, seed=21, adversarial_frac=0.25)
    syn_conns = [[syn["data"][syn["blk_off"][k]:syn["blk_off"][k + 1]].tobytes()
                  for k in range(syn["conn_first"][c], syn["conn_first"][c + 1])] for c in range(len(syn["conn_first"]) - 1)]
    s256 = HS.make_connections(400, seed=22, table_size=256, adversarial_frac=0.25)
    s256_conns = [[s256["data"][s256["blk_off"][k]:s256["blk_off"][k + 1]].tobytes()
                   for k in range(s256["conn_first"][c], s256["conn_first"][c + 1])]
                  for c in range(len(s256["conn_first"]) - 1)]
    rq = HS.make_connections(1500, seed=23, adversarial_frac=0.05, request_frac=0.12)
    rq_conns = [[rq["data"][rq["blk_off"][k]:rq["blk_off"][k + 1]].tobytes()
                 for k in range(rq["conn_first"][c], rq["conn_first"][c + 1])] for c in range(len(rq["conn_first"]) - 1)]
    out = {"blocks": blocks_set(UNIT_REQUESTS + static_sweep + corpus + syn_conns + rq_conns, 4096, requests=True),
           "blocks_256": blocks_set(UNIT_RESPONSES_256 + s256_conns, 256)}
    for k, v in out.items():
        print("%-12s connections %5d  blocks %6d  fields %7d  errors %d" % (
            k, len(v["conn_first"]) - 1, len(v["blk_off"]) - 1, int(v["nfields"].sum()), int((v["bstatus"] != 0).sum())))
    return out


QPACK_SESSIONS = [  # name, seed, connections, steps, header_table_size, max_blocked, adversarial fraction,
    # fraction of requests with one of h2o_hpack_parse_request's cases
    ("q4096", 61, 300, 4, 4096, 4, 0.3, 0.0),
    ("q256", 62, 150, 3, 256, 2, 0.3, 0.0),
    ("q0", 63, 100, 2, 0, 0, 0.2, 0.0),
    ("qreq", 64, 500, 3, 4096, 4, 0.05, 0.3),
]


def qpack_stream_ids(ns, step):
    """client-initiated bidirectional stream ids (multiples of 4), a quarter of them large enough that the
    Section Acknowledgment's 7-bit prefix integer takes 2 to 9 bytes"""
    k = np.arange(ns, dtype=np.uint64)
    big = np.uint64(1) << (np.uint64(7) * (k % np.uint64(9)) + np.uint64(4))
    sid = np.uint64(4) * (k + np.uint64(1000 * step)) + np.where(k % 4 == 3, big * np.uint64(4), np.uint64(0))
    return sid & np.uint64((1 << 62) - 4)


def qpack_edge_session():
    """hand-built connections (one step): empty inputs, truncated and bad instructions, the corner cases of
    Required Insert Count / Base, post-base references, pseudo-header token names, raw upper-case names"""
    from h2o_amd import qpack_synth as QS

    q, i = QS.qstring, QS.encode_int
    www = q(b"www.example.com")
    conns = [
        (b"", [b"", b"\x00", b"\x00\x00", b"\x00\x00\xd1", b"\x00\x80\xd1", b"\x00\x00\xff\x3f"]),
        # insert :authority=www.example.com (static name 0), then read it back (RFC 9204 B.2 shape)
        (i(0, 6, 0xC0) + www, [b"\x02\x00\x80", b"\x02\x80\x10", b"\x02\x81\x10", b"\x03\x00\x80",
                               b"\x02\x00\x81", b"\x00\x00\x80", b"\x02\x00\x40" + q(b"v")]),
        # literal-name inserts: token pseudo-header raw (soft dropped), odd chars (soft kept), upper case (fail)
        (q(b":path", 5, 0x40, True) + q(b"/a", 7, 0, True) + q(b"x y", 5, 0x40, True) + q(b"v", 7, 0),
         [b"\x03\x00\x80\x81", b"\x03\x00\x41" + q(b"\x01bad")]),
        (q(b"X-Upper", 5, 0x40, True) + q(b"v", 7, 0), [b"\x00\x00\xd1"]),
        # duplicate, capacity update to 0 (evicts all), capacity above the table size
        (i(0, 6, 0xC0) + www + i(0, 5, 0x00) + i(0, 5, 0x20), [b"\x03\x00\x80", b"\x00\x00\xd1"]),
        (i(5000, 5, 0x20), [b"\x00\x00\xd1"]),
        # truncated instruction (waits for more input), then a section blocked on it
        (i(0, 6, 0xC0) + www[:5], [b"\x02\x00\x80"]),
        # entry larger than the table; dynamic name reference past the table
        (q(b"x-big", 5, 0x40) + q(b"v" * 5000, 7, 0, True), []),
        (i(7, 6, 0x80) + q(b"v"), []),
        # literal lines: static name with Huffman / raw values, literal names Huffman / raw / empty
        (b"", [b"\x00\x00\x51" + q(b"/index.html"), b"\x00\x00\x5f\x00" + q(b" lead", 7, 0, True),
               b"\x00\x00" + q(b"custom-key", 3, 0x20) + q(b"custom-value"),
               b"\x00\x00" + q(b"", 3, 0x20, True) + q(b"v"), b"\x00\x00" + q(b":status", 3, 0x20, True) + q(b"200"),
               b"\x00\x00" + q(b"Upper", 3, 0x20, True) + q(b"v"), b"\x00\x00\x2f\xff\xff\xff\xff\xff\xff\xff\xff\xff\x7f"]),
        # blocked sections take the free slots in section order (num_blocked = index % 6, max_blocked 2):
        # connection 12 (num_blocked 0) parks two and fails the third, connection 13 (1) parks one, fails one
        (b"", []),
        (b"", []),
        (b"", [b"\x03\x00\x80", b"\x00\x00\xd1", b"\x03\x00\x80", b"\x04\x00\x80"]),
        (b"", [b"\x03\x00\x80", b"\x03\x00\x81"]),
    ]
    sec, sec_len, cf, enc = [], [], [0], []
    for e, ss in conns:
        sec += ss
        sec_len += [len(x) for x in ss]
        cf.append(len(sec_len))
        enc.append(e)
    sec_off = np.zeros(len(sec_len) + 1, np.uint64)
    sec_off[1:] = np.cumsum(sec_len)
    base = int(sec_off[-1])
    enc_off = base + np.concatenate([[0], np.cumsum([len(e) for e in enc])[:-1]]).astype(np.uint64)
    return [dict(data=np.frombuffer(b"".join(sec) + b"".join(enc), np.uint8).copy(), sec_off=sec_off.astype(np.uint32),
                 conn_first=np.asarray(cf, np.uint32), enc_off=enc_off.astype(np.uint32),
                 enc_len=np.asarray([len(e) for e in enc], np.uint32), header_table_size=4096)]


def qpack_set():
    """tests/golden/qpack.npz: QPACK decoder sessions run through the reference's own decoder (oracle/_ref,
    qpack.c included: h2o_qpack_decoder_handle_input, parse_decode_context, check_decode_context_blocked,
    decode_header); per session the step inputs and the reference's outputs"""
    from h2o_amd import qpack_synth as QS

    out = {}
    sessions = [(n, QS.make_session(nc, steps=st, seed=sd, header_table_size=h, adversarial_frac=adv,
                                    request_frac=rf), nc, h, mb)
                for n, sd, nc, st, h, mb, adv, rf in QPACK_SESSIONS]
    sessions.append(("qedge", qpack_edge_session(), 14, 4096, 2))
    for name, steps, nconn, hts, mb in sessions:
        sr = O.QpackSession(O.ref(), nconn, hts, mb)
        # the same session through h2o_qpack_parse_request (a second decoder: the encoder streams act alike)
        sq = O.QpackSession(O.ref(), nconn, hts, mb)
        nbl = (np.arange(nconn) % 6).astype(np.uint32)
        out[name + "_meta"] = np.asarray([nconn, hts, mb, len(steps)], np.uint32)
        out[name + "_num_blocked"] = nbl
        for k, st in enumerate(steps):
            ao = QS.arena_offsets(st["sec_off"], hts)
            r = sr.step(st["data"], st["enc_off"], st["enc_len"], st["sec_off"], st["conn_first"], ao, nbl)
            ns = len(st["sec_off"]) - 1
            names, values, soft = [], [], []
            for s_ in range(ns):
                o = int(st["sec_off"][s_])
                for f in range(o, o + int(r["nfields"][s_])):
                    names.append(r["arena"][r["name_off"][f]:r["name_off"][f] + r["name_len"][f]].tobytes())
                    values.append(r["arena"][r["value_off"][f]:r["value_off"][f] + r["value_len"][f]].tobytes())
                    soft.append(r["fflags"][f])
            nd, no = pack(names)
            vd, vo = pack(values)
            p = "%s_%d_" % (name, k)
            for key in ("data", "sec_off", "conn_first", "enc_off", "enc_len"):
                out[p + key] = st[key]
            out[p + "arena_off"] = ao
            for key in ("nfields", "sstatus", "req_insert_count"):
                out[p + key] = r[key][:ns]
            for key in ("enc_status", "enc_consumed", "insert_count"):
                out[p + key] = r[key][:nconn]
            out[p + "fld_name"], out[p + "fld_name_off"], out[p + "fld_value"], out[p + "fld_value_off"] = nd, no, vd, vo
            out[p + "fld_soft"] = np.asarray(soft, np.uint8)
            # h2o_qpack_parse_request: verdicts, request records, acks, the fields' flags (their names and
            # values are a prefix of the decode-only fields above, checked here)
            sid = qpack_stream_ids(ns, k)
            q = sq.step(st["data"], st["enc_off"], st["enc_len"], st["sec_off"], st["conn_first"], ao, nbl, stream_id=sid)
            fl = []
            for s_ in range(ns):
                o, kq = int(st["sec_off"][s_]), int(q["nfields"][s_])
                assert kq <= int(r["nfields"][s_]) or int(r["sstatus"][s_]) != 0
                for f in range(o, o + kq):
                    assert q["arena"][q["name_off"][f]:q["name_off"][f] + q["name_len"][f]].tobytes() == \
                        r["arena"][r["name_off"][f]:r["name_off"][f] + r["name_len"][f]].tobytes()
                    assert q["arena"][q["value_off"][f]:q["value_off"][f] + q["value_len"][f]].tobytes() == \
                        r["arena"][r["value_off"][f]:r["value_off"][f] + r["value_len"][f]].tobytes()
                    fl.append(q["fflags"][f])
            out[p + "rq_stream_id"] = sid
            out[p + "rq_nfields"] = q["nfields"][:ns]
            out[p + "rq_sstatus"] = q["sstatus"][:ns]
            out[p + "rq_req"] = q["req"][:ns].view(np.uint32).reshape(ns, 18)
            out[p + "rq_fflags"] = np.asarray(fl, np.uint8)
        sr.close()
        sq.close()
    return out


def _resp_fields(r, blk_off, nb, nfields):
    names, values, fl = [], [], []
    for bi in range(nb):
        s = int(blk_off[bi])
        for f in range(s, s + int(nfields[bi])):
            names.append(r["arena"][r["name_off"][f]:r["name_off"][f] + r["name_len"][f]].tobytes())
            values.append(r["arena"][r["value_off"][f]:r["value_off"][f] + r["value_len"][f]].tobytes())
            fl.append(r["fflags"][f])
    nd, no = pack(names)
    vd, vo = pack(values)
    return dict(fld_name=nd, fld_name_off=no, fld_value=vd, fld_value_off=vo, fflags=np.asarray(fl, np.uint8))


def resp_set():
    """tests/golden/resp.npz: response header blocks as h2o's clients parse them, through the reference's own
    functions (oracle/_ref): h2o_hpack_parse_response over HPACK blocks (ref_hpack_parse_responses: heads and
    trailers, lib/common/http2client.c:332 / :421) and h2o_qpack_parse_response over QPACK sections
    (ref_qpack_step_resp, lib/common/http3client.c:542, each section also checked against the real function).
    Per set: the inputs, every block's verdict, record and fields (names, values, flags)."""
    from h2o_amd import hpack_synth as HS
    from h2o_amd import qpack_synth as QS

    out = {}
    edge = [[b""], [b"\x88"], [b"\x08\x03200"], [b"\x08\x03" + b"2x0"], [b"\x0f\x1c\x03abc"],
            [b"\x88", b"\x0f\x1c\x03123"], [b"\x88\x88"], [b"\x82"], [b"\x88", b""]]
    edge_tr = [0, 0, 0, 0, 0, 0, 1, 0, 0, 0, 1]  # per block: the second block of two is trailers
    sets = []
    a = HS.make_response_connections(1500, seed=41, adversarial_frac=0.05, rule_frac=0.12)
    b = HS.make_response_connections(800, blocks_per_conn=(1, 1), seed=42, adversarial_frac=0.0, rule_frac=1.0,
                                     trailer_frac=0.25)
    e = HS.pack_connections(edge, 4096)
    e["trailers"] = np.asarray(edge_tr, np.uint8)
    c = HS.make_response_connections(300, seed=43, table_size=256, adversarial_frac=0.2, rule_frac=0.2)
    u = HS.pack_connections(UNIT_RESPONSES_256, 256)
    u["trailers"] = np.zeros(len(u["blk_off"]) - 1, np.uint8)

    def join(parts):
        conns, tr = [], []
        for s in parts:
            for ci in range(len(s["conn_first"]) - 1):
                ks = range(int(s["conn_first"][ci]), int(s["conn_first"][ci + 1]))
                conns.append([s["data"][s["blk_off"][k]:s["blk_off"][k + 1]].tobytes() for k in ks])
                tr += [int(s["trailers"][k]) for k in ks]
        return conns, np.asarray(tr, np.uint8)

    for name, parts, ts in (("h", [e, a, b], 4096), ("h256", [u, c], 256)):
        conns, tr = join(parts)
        pk = HS.pack_connections(conns, ts)
        nb = len(pk["blk_off"]) - 1
        r = O.ref().hpack_decode_blocks(pk["data"], pk["blk_off"], pk["conn_first"], ts, responses=True, trailers=tr)
        p = name + "_"
        out.update({p + "data": pk["data"], p + "blk_off": pk["blk_off"], p + "conn_first": pk["conn_first"],
                    p + "trailers": tr, p + "table_size": np.asarray([ts], np.uint32), p + "nfields": r["nfields"][:nb],
                    p + "bstatus": r["bstatus"][:nb], p + "res": r["res"][:nb].view(np.uint32).reshape(nb, 4)})
        out.update({p + k: v for k, v in _resp_fields(r, pk["blk_off"], nb, r["nfields"]).items()})
        print("resp %-5s connections %5d  blocks %6d  fields %7d  errors %d" % (
            name, len(pk["conn_first"]) - 1, nb, int(r["nfields"][:nb].sum()), int((r["bstatus"][:nb] != 0).sum())))
    # HTTP/3: a decoder session whose sections are response heads
    nconn, hts, mb = 400, 4096, 4
    steps = QS.make_session(nconn, steps=3, seed=44, header_table_size=hts, adversarial_frac=0.05, request_frac=0.35,
                            responses=True)
    sq = O.QpackSession(O.ref(), nconn, hts, mb)
    nbl = (np.arange(nconn) % 6).astype(np.uint32)
    out["q_meta"] = np.asarray([nconn, hts, mb, len(steps)], np.uint32)
    out["q_num_blocked"] = nbl
    for k, st in enumerate(steps):
        ao = QS.arena_offsets(st["sec_off"], hts)
        ns = len(st["sec_off"]) - 1
        sid = qpack_stream_ids(ns, k)
        q = sq.step(st["data"], st["enc_off"], st["enc_len"], st["sec_off"], st["conn_first"], ao, nbl, stream_id=sid,
                    responses=True)
        p = "q_%d_" % k
        for key in ("data", "sec_off", "conn_first", "enc_off", "enc_len"):
            out[p + key] = st[key]
        out[p + "arena_off"] = ao
        out[p + "stream_id"] = sid
        for key in ("nfields", "sstatus", "req_insert_count"):
            out[p + key] = q[key][:ns]
        for key in ("enc_status", "enc_consumed", "insert_count"):
            out[p + key] = q[key][:nconn]
        out[p + "res"] = q["res"][:ns].view(np.uint32).reshape(ns, 10)
        out.update({p + kk: v for kk, v in _resp_fields(q, st["sec_off"], ns, q["nfields"]).items()})
    sq.close()
    return out


HPENC_SESSIONS = [  # name, seed, connections, steps, knobs (h2o_amd.hpenc_synth.make_session), error mutations
    ("h4096", 301, 160, 3, dict(), False),
    ("hedge", 302, 120, 3, dict(small_table_frac=0.3, trailers_frac=0.1, big_frac=0.01, notoken_frac=0.1,
                                dont_compress_frac=0.15, frame_frac=0.3), False),
    ("herr", 303, 120, 2, dict(small_table_frac=0.1, big_frac=0.005, dont_compress_frac=0.05), True),
    # client requests (h2o_hpack_flatten_request, hpenc_synth.make_request_session)
    ("rq4096", 311, 160, 3, dict(requests=True), False),
    ("rqedge", 312, 120, 3, dict(requests=True, small_table_frac=0.3, big_frac=0.02, notoken_frac=0.1,
                                 dont_compress_frac=0.15, frame_frac=0.3), False),
    ("rqerr", 313, 120, 2, dict(requests=True, small_table_frac=0.1, big_frac=0.01, dont_compress_frac=0.05), True),
]


def hpenc_errors(rng, st):
    """invalid arguments and short output regions -> HHUFF_RES_EINVAL / _SPACE, and the connection's later
    responses HHUFF_RES_SKIPPED"""
    res, hdr = st["res"], st["hdr"]
    n = res.size
    regions = np.diff(st["out_off"].astype(np.int64))
    for r in rng.choice(n, max(1, n // 40), replace=False):
        regions[r] = int(rng.integers(0, 24))
    for r in rng.choice(n, max(1, n // 80), replace=False):
        if not res["flags"][r] & 12:  # not trailers or requests (a request's `status` counts its own fields)
            res["status"][r] = int(rng.choice([0, 99, 1000]))
    for r in rng.choice(n, max(1, n // 150), replace=False):
        res["max_frame_size"][r] = int(rng.choice([100, 16383, 1 << 24]))
    if hdr.size:
        for h in rng.choice(hdr.size, max(1, hdr.size // 400), replace=False):
            hdr["value_off"][h] = st["data"].size - int(rng.integers(0, 3))
            hdr["value_len"][h] = 5
    st["out_off"] = np.concatenate([[0], np.cumsum(regions)]).astype(np.uint64)


def hpenc_set():
    """HTTP/2 response header blocks (f4 encode half): sessions of synthetic responses flattened by the
    real h2o_hpack_flatten_response / _trailers, and of client requests by the real h2o_hpack_flatten_request
    (oracle/ref_hpenc.c), one encoder table per connection
    across the steps; per step the inputs and the reference's frames (compacted), lengths and statuses"""
    from h2o_amd import hpenc_synth as HE

    out = {}
    for name, seed, nconn, nsteps, knobs, errors in HPENC_SESSIONS:
        knobs = dict(knobs)
        make = HE.make_request_session if knobs.pop("requests", False) else HE.make_session
        steps = make(nconn, steps=nsteps, seed=seed, **knobs)
        rng = np.random.default_rng(seed + 7)
        sr, so = O.HpeSession(O.ref(), nconn), O.HpeSession(O.oracle(), nconn)
        out[name + "_meta"] = np.array([nconn, nsteps], np.uint32)
        for k, st in enumerate(steps):
            if errors:
                hpenc_errors(rng, st)
            args = (st["data"], st["hdr"], st["res"], st["conn_first"], st["out_off"], st["server_off"],
                    st["server_len"])
            r, q = sr.step(*args), so.step(*args)
            for key in ("out_len", "headers_size", "rstatus"):
                assert (r[key] == q[key]).all(), (name, k, key)
            frames = b"".join(r["out"][int(o):int(o) + int(L)].tobytes() for o, L in zip(st["out_off"], r["out_len"]))
            assert frames == b"".join(q["out"][int(o):int(o) + int(L)].tobytes()
                                      for o, L in zip(st["out_off"], q["out_len"])), (name, k)
            p = "%s_%d_" % (name, k)
            out.update({p + "data": st["data"], p + "hdr": st["hdr"].view(np.uint32).reshape(-1),
                        p + "res": st["res"].view(np.uint32).reshape(-1), p + "conn_first": st["conn_first"],
                        p + "server": np.array([st["server_off"], st["server_len"]], np.uint32),
                        p + "out_off": st["out_off"], p + "frames": np.frombuffer(frames, np.uint8),
                        p + "out_len": r["out_len"], p + "headers_size": r["headers_size"], p + "rstatus": r["rstatus"]})
        sr.close()
        so.close()
    return out


QPENC_SETS = [  # name, seed, connections, knobs (make_session), to_qpack knobs, error mutations
    ("q1", 401, 300, dict(), dict(), False),
    ("qedge", 402, 200, dict(big_frac=0.01, notoken_frac=0.1, dont_compress_frac=0.15),
     dict(dfid_frac=0.2, odd_status_frac=0.1), False),
    ("qerr", 403, 200, dict(big_frac=0.005), dict(dfid_frac=0.05), True),
    # client requests (h2o_qpack_flatten_request; hpenc_synth.make_request_session + to_qpack_requests)
    ("qrq", 411, 300, dict(requests=True, notoken_frac=0.05, dont_compress_frac=0.05), dict(dfid_frac=0.1), False),
    ("qrqerr", 412, 200, dict(requests=True, big_frac=0.01), dict(dfid_frac=0.05), True),
]


def qpenc_set():
    """HTTP/3 response HEADERS frames (f4, QPACK encode half): synthetic responses flattened by the real
    h2o_qpack_flatten_response as h2o's HTTP/3 server calls it (oracle/ref_shim.c ref_qpe_step), the restatement
    checked against them as they are written"""
    from h2o_amd import hpenc_synth as HE

    out = {}
    for name, seed, nconn, knobs, qknobs, errors in QPENC_SETS:
        knobs = dict(knobs)
        if knobs.pop("requests", False):
            q = HE.to_qpack_requests(HE.make_request_session(nconn, seed=seed, **knobs)[0], seed=seed, **qknobs)
        else:
            q = HE.to_qpack(HE.make_session(nconn, seed=seed, **knobs)[0], seed=seed, **qknobs)
        if errors:
            rng = np.random.default_rng(seed + 7)
            n = q["res"].size
            regions = np.diff(q["out_off"].astype(np.int64))
            for r in rng.choice(n, max(1, n // 40), replace=False):
                regions[r] = int(rng.integers(0, 24))
            q["out_off"] = np.concatenate([[0], np.cumsum(regions)]).astype(np.uint64)
            for h in rng.choice(q["hdr"].size, max(1, q["hdr"].size // 400), replace=False):
                q["hdr"]["value_off"][h] = q["data"].size - int(rng.integers(0, 3))
                q["hdr"]["value_len"][h] = 5
        args = (q["data"], q["hdr"], q["res"], q["out_off"], q["server_off"], q["server_len"])
        r, o = O.qpe_step(O.ref(), *args), O.qpe_step(O.oracle(), *args)
        for key in ("out_len", "header_len", "rstatus"):
            assert (r[key] == o[key]).all(), (name, key)
        frames = b"".join(r["out"][int(a):int(a) + int(L)].tobytes() for a, L in zip(q["out_off"], r["out_len"]))
        assert frames == b"".join(o["out"][int(a):int(a) + int(L)].tobytes() for a, L in zip(q["out_off"], o["out_len"]))
        p = name + "_"
        out.update({p + "data": q["data"], p + "hdr": q["hdr"].view(np.uint32).reshape(-1),
                    p + "res": q["res"].view(np.uint32).reshape(-1),
                    p + "server": np.array([q["server_off"], q["server_len"]], np.uint32), p + "out_off": q["out_off"],
                    p + "frames": np.frombuffer(frames, np.uint8), p + "out_len": r["out_len"][:q["res"].size],
                    p + "header_len": r["header_len"][:q["res"].size], p + "rstatus": r["rstatus"][:q["res"].size]})
    return out


def main():
    if "--only-resp" in sys.argv:
        np.savez_compressed(os.path.join(GOLDEN, "resp.npz"), **resp_set())
        return
    if "--only-qpenc" in sys.argv:
        np.savez_compressed(os.path.join(GOLDEN, "qpenc.npz"), **qpenc_set())
        return
    if "--only-adversarial-encode" in sys.argv:  # add the encode vectors to adversarial.npz, decode ones unchanged
        path = os.path.join(GOLDEN, "adversarial.npz")
        with np.load(path, allow_pickle=False) as z:
            arrays = {k: z[k] for k in z.files if not k.startswith("enc_")}
        arrays.update(ref_encode_set(adversarial_encode_strings()))
        np.savez_compressed(path, **arrays)
        print("adversarial: encode %d" % len(arrays["enc_len"]))
        return
    if "--only-hpenc" in sys.argv:
        np.savez_compressed(os.path.join(GOLDEN, "hpenc.npz"), **hpenc_set())
        return
    if "--only-qpack" in sys.argv:
        np.savez_compressed(os.path.join(GOLDEN, "qpack.npz"), **qpack_set())
        return
    if "--only-blocks" in sys.argv:
        for name, arrays in blocks_sets().items():
            np.savez_compressed(os.path.join(GOLDEN, name + ".npz"), **arrays)
        return
    if not O.ref_available():
        sys.exit("oracle/_ref/libh2oref.so missing: run `make -C oracle` where /root/reference exists")
    os.makedirs(GOLDEN, exist_ok=True)
    sets = {"kat": kat_set()}
    huff, raw = corpus_strings()
    c = ref_decode_set([s for _, s in huff], [nm for nm, _ in huff])
    c.update(ref_encode_set([s for _, s in raw]))
    sets["corpus"] = c
    for cfg, n, seed in (("c2", 3000, 101), ("c3", 1200, 102), ("c4", 3000, 103), ("c5", 300, 104)):
        sets["random_" + cfg] = random_set(cfg, n, seed)
    sets["adversarial"] = adversarial_set()
    sets["adversarial"].update(ref_encode_set(adversarial_encode_strings()))
    sets["framing"] = framing_set()
    sets["literals"] = literals_set()
    sets.update(blocks_sets())
    sets["qpack"] = qpack_set()
    sets["hpenc"] = hpenc_set()
    sets["qpenc"] = qpenc_set()
    sets["resp"] = resp_set()
    for name, arrays in sets.items():
        path = os.path.join(GOLDEN, name + ".npz")
        np.savez_compressed(path, **arrays)
        nd = len(arrays.get("dec_len", []))
        ne = len(arrays.get("enc_len", []))
        print("%-16s decode %6d  encode %6d  %8d bytes" % (name, nd, ne, os.path.getsize(path)))


if __name__ == "__main__":
    main()
