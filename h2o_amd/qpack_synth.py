"""Seeded synthetic QPACK connections for the f4 QPACK decoder (QPACK half).

An encoder model in the spirit of RFC 9204 encoders: each connection keeps a model of the decoder's
dynamic table with h2o's insert / evict rules (lib/http3/qpack.c:153-190, base_offset 1 so that h2o's
absolute index = RFC absolute index + 1) and emits, per step, encoder-stream instructions (insert with a
static or dynamic name reference, insert with a literal name, duplicate, set capacity) followed by
request field sections whose lines are indexed (static, dynamic, post-base) or literal (static / dynamic /
post-base name reference, literal name), every string Huffman-coded when that is strictly shorter.
Required Insert Count and Base are encoded as RFC 9204 4.5.1 prescribes (sometimes with a post-base
Base).  Encoder streams are cut at arbitrary bytes across steps: a step's buffer holds what the decoder
did not consume before plus the new bytes, as h2o's encoder-stream receive buffer does.  Some sections
reference inserts that arrive only in a later step (blocked).

Adversarial connections (a fraction) get one mutation: truncated / bit-flipped sections or encoder
bytes, references past the table, oversized capacities, entries larger than the table, upper-case raw
names, invalid characters (soft errors), bad Required Insert Count encodings.

Step layout (include/hhuff.h hhuff_qpack_decode): sections packed back to back first (`sec_off`
[nsec+1], `conn_first` [nconn+1]), then each connection's encoder bytes (`enc_off`, `enc_len`).
"""
import numpy as np

from . import tables
from .hpack_synth import _huffman, _vocab, _request, _request_rules, _response, _response_rules, encode_int

QSTATIC = tables.QPACK_STATIC_TABLE
ENTRY_OVERHEAD = 32


def qstring(s: bytes, prefix_bits=7, first=0, force_raw=False):
    """a QPACK string literal: H bit just above the prefix, Huffman when strictly shorter"""
    if s and not force_raw:
        h = _huffman(s)
        if len(h) < len(s):
            return encode_int(len(h), prefix_bits, first | (1 << prefix_bits)) + h
    return encode_int(len(s), prefix_bits, first) + s


class _QTable:
    """the decoder's dynamic table as h2o keeps it (qpack.c:153-190); entries by RFC absolute index"""

    def __init__(self, cap):
        self.e = []  # (abs, name, value), oldest first
        self.size, self.cap, self.inserts = 0, cap, 0

    def insert(self, name, value):
        add = len(name) + len(value) + ENTRY_OVERHEAD
        if add > self.cap:
            return False
        while self.e and self.size + add > self.cap:
            self._evict()
        self.e.append((self.inserts, name, value))
        self.size += add
        self.inserts += 1
        return True

    def _evict(self):
        _, n, v = self.e.pop(0)
        self.size -= len(n) + len(v) + ENTRY_OVERHEAD

    def set_cap(self, cap):
        self.cap = cap
        while self.e and self.size > self.cap:
            self._evict()

    def find(self, name, value):
        full = nm = None
        for a, n, v in reversed(self.e):
            if n == name:
                nm = a if nm is None else nm
                if v == value:
                    return a, a
        return full, nm


def _static_find(name, value):
    nm = None
    for i, (n, v) in enumerate(QSTATIC):
        if n == name:
            if v == value:
                return i, i
            nm = i if nm is None else nm
    return None, nm


def encode_section(rng, t: _QTable, fields, max_entries, live_limit=None):
    """one request field section against table t (all of t's inserts visible to the decoder)"""
    lines, refs = [], []
    for name, value in fields:
        sf, sn = _static_find(name, value)
        df, dn = t.find(name, value)
        raw = rng.random() < 0.1
        if sf is not None and rng.random() < 0.9:
            lines.append(("static", sf))
        elif df is not None and rng.random() < 0.9:
            lines.append(("dyn", df))
            refs.append(df)
        elif dn is not None and rng.random() < 0.5:
            lines.append(("dynname", dn, value, raw))
            refs.append(dn)
        elif sn is not None:
            lines.append(("staticname", sn, value, raw))
        else:
            lines.append(("literal", name, value, raw))
    ric = max(refs) + 1 if refs else 0
    base = ric
    if refs and rng.random() < 0.25:  # post-base references for the newest entries
        base = int(rng.integers(min(refs), ric + 1))
    out = bytearray()
    if ric == 0:
        out += b"\x00"
    else:
        out += encode_int(ric % (2 * max_entries) + 1, 8)
    out += encode_int(base - ric, 7, 0) if base >= ric else encode_int(ric - base - 1, 7, 0x80)
    for ln in lines:
        if ln[0] == "static":
            out += encode_int(ln[1], 6, 0xC0)
        elif ln[0] == "dyn":
            a = ln[1]
            out += encode_int(base - 1 - a, 6, 0x80) if a < base else encode_int(a - base, 4, 0x10)
        elif ln[0] == "dynname":
            a, value, raw = ln[1:]
            n_bit = 0x20 if rng.random() < 0.1 else 0
            out += encode_int(base - 1 - a, 4, 0x40 | n_bit) if a < base else encode_int(a - base, 3, (0x08 if n_bit else 0))
            out += qstring(value, 7, 0, raw)
        elif ln[0] == "staticname":
            i, value, raw = ln[1:]
            out += encode_int(i, 4, 0x50 | (0x20 if rng.random() < 0.1 else 0))
            out += qstring(value, 7, 0, raw)
        else:
            name, value, raw = ln[1:]
            out += qstring(name, 3, 0x20 | (0x10 if rng.random() < 0.1 else 0), raw)
            out += qstring(value, 7, 0, raw)
    return bytes(out)


def _encoder_instructions(rng, t: _QTable, fields, header_table_size):
    """insert some of a request's fields into t; -> list of instruction bytes"""
    ins = []
    if rng.random() < 0.05:
        cap = int(rng.integers(header_table_size // 2, header_table_size + 1))
        ins.append(encode_int(cap, 5, 0x20))
        t.set_cap(cap)
    for name, value in fields:
        if rng.random() < 0.5 or t.find(name, value)[0] is not None:
            if t.e and rng.random() < 0.05:  # duplicate the newest entries now and then
                a = t.e[-1][0]
                _, n, v = t.e[-1]
                if len(n) + len(v) + ENTRY_OVERHEAD <= t.cap:
                    ins.append(encode_int(t.inserts - 1 - a, 5, 0x00))
                    t.insert(n, v)
            continue
        if len(name) + len(value) + ENTRY_OVERHEAD > t.cap:
            continue
        raw = rng.random() < 0.1
        _, sn = _static_find(name, value)
        _, dn = t.find(name, value)
        if sn is not None and rng.random() < 0.8:
            b = encode_int(sn, 6, 0xC0) + qstring(value, 7, 0, raw)
        elif dn is not None and rng.random() < 0.8:
            b = encode_int(t.inserts - 1 - dn, 6, 0x80) + qstring(value, 7, 0, raw)
        else:
            b = qstring(name, 5, 0x40, raw) + qstring(value, 7, 0, raw)
        ins.append(b)
        t.insert(name, value)
    return ins


def _mutate_section(rng, sec, max_entries):
    s = bytearray(sec)
    kind = int(rng.integers(8))
    if kind == 0 and len(s) > 2:
        s = s[:int(rng.integers(1, len(s)))]
    elif kind == 1 and s:
        i = int(rng.integers(len(s)))
        s[i] ^= 1 << int(rng.integers(8))
    elif kind == 2:  # static index past the table
        s += encode_int(99 + int(rng.integers(50)), 6, 0xC0)
    elif kind == 3:  # upper-case raw literal name
        s += qstring(b"X-Upper", 3, 0x20, True) + qstring(b"v", 7, 0, True)
    elif kind == 4:  # soft errors
        bad = [(b"bad name", b"v"), (b"x-ok", b"a\x01b"), (b"x-ok", b" lead"), (b"x-ok", b"trail\t"), (b":path", b"/x"),
               (b":bogus", b"x"), (b"", b"empty")][int(rng.integers(7))]
        s += qstring(bad[0], 3, 0x20, rng.random() < 0.5) + qstring(bad[1], 7, 0, rng.random() < 0.5)
    elif kind == 5:  # dynamic reference past Base
        s += encode_int(int(rng.integers(0, 40)), 6, 0x80)
    elif kind == 6:  # bad Required Insert Count (larger than 2 * MaxEntries)
        s = bytearray(encode_int(2 * max_entries + 1 + int(rng.integers(10)), 8)) + s[1:]
    else:  # value length past the section
        s += encode_int(3, 4, 0x50) + encode_int(9, 7, 0) + b"ab"
    return bytes(s)


def _mutate_encoder(rng, ins, header_table_size):
    kind = int(rng.integers(6))
    if kind == 0 and ins:
        i = int(rng.integers(len(ins)))
        b = bytearray(ins[i])
        b[int(rng.integers(len(b)))] ^= 1 << int(rng.integers(8))
        ins[i] = bytes(b)
    elif kind == 1:
        ins.append(encode_int(header_table_size + 1 + int(rng.integers(100)), 5, 0x20))
    elif kind == 2:  # entry larger than the table
        ins.append(qstring(b"x-big", 5, 0x40, True) + qstring(b"v" * (header_table_size + 1), 7, 0, True))
    elif kind == 3:  # dynamic name reference / duplicate past the table
        ins.append(encode_int(500 + int(rng.integers(50)), 6, 0x80) + qstring(b"v", 7, 0))
    elif kind == 4:
        ins.append(encode_int(300 + int(rng.integers(50)), 5, 0x00))
    else:  # upper-case raw literal name
        ins.append(qstring(b"X-Upper", 5, 0x40, True) + qstring(b"v", 7, 0, True))


def make_session(nconn, steps=3, seed=0, header_table_size=4096, adversarial_frac=0.05, max_sections=(1, 4),
                 blocked_frac=0.05, request_frac=0.0, responses=False):
    """-> list over steps of dict(data, sec_off, conn_first, enc_off, enc_len) for one decoder session.
    request_frac: the fraction of requests given one of h2o_hpack_parse_request's cases (duplicate / late /
    unknown pseudo-headers, content-length, connection-specific fields, te, host, cache-digest,
    datagram-flow-id, the 100 / 1000 field limits, ...: hpack_synth._request_rules) -- what
    h2o_qpack_parse_request checks for HTTP/3 (qpack.c:848).  responses=True: the sections are response heads
    (what h2o's HTTP/3 client parses, h2o_qpack_parse_response), request_frac of them given one of
    h2o_hpack_parse_response's cases (hpack_synth._response_rules)"""
    rng = np.random.default_rng(seed)
    V = _vocab(rng)
    hosts = V[0]
    max_entries = max(1, header_table_size // 32)
    per_conn = []  # per connection: list over steps of (encoder bytes, [sections])
    for c in range(nconn):
        t = _QTable(header_table_size)
        host = hosts[int(rng.integers(len(hosts)))]
        adv = rng.random() < adversarial_frac
        adv_step = int(rng.integers(steps))
        stream, cuts, secs = b"", [], []
        bounds = [0]  # instruction boundaries in the stream
        for s in range(steps):
            ins, sections = [], []
            for _ in range(int(rng.integers(max_sections[0], max_sections[1] + 1))):
                if responses:
                    req = _response(rng, V)
                    if request_frac and rng.random() < request_frac:
                        req = _response_rules(rng, req, False)
                else:
                    req = _request(rng, V, host)
                    if request_frac and rng.random() < request_frac:
                        req = _request_rules(rng, req)
                ins += _encoder_instructions(rng, t, req, header_table_size)
                if header_table_size == 0 or rng.random() < 0.1:
                    sections.append(encode_section(rng, _QTable(0), req, max_entries))
                else:
                    sections.append(encode_section(rng, t, req, max_entries))
            if adv and s == adv_step:
                if rng.random() < 0.5 and sections:
                    k = int(rng.integers(len(sections)))
                    sections[k] = _mutate_section(rng, sections[k], max_entries)
                else:
                    _mutate_encoder(rng, ins, header_table_size)
            for b in ins:
                stream += b
                bounds.append(len(stream))
            cut = len(stream)
            if ins and s + 1 < steps and rng.random() < blocked_frac * 4:
                cut = int(rng.integers(bounds[-2], len(stream) + 1))  # last instruction arrives later (blocked)
            cuts.append(cut)
            secs.append(sections)
        cuts[-1] = len(stream)
        steps_c, done = [], 0
        for s in range(steps):
            chunk = stream[done:cuts[s]]
            steps_c.append((chunk, secs[s]))
            done = max(b for b in bounds if b <= cuts[s])  # what the decoder consumes (for a valid stream)
        per_conn.append(steps_c)
    out = []
    for s in range(steps):
        sec_bytes, sec_len, conn_first, enc = [], [], [0], []
        for c in range(nconn):
            chunk, sections = per_conn[c][s]
            sec_bytes += sections
            sec_len += [len(x) for x in sections]
            conn_first.append(len(sec_len))
            enc.append(chunk)
        sec_off = np.zeros(len(sec_len) + 1, np.uint64)
        sec_off[1:] = np.cumsum(sec_len)
        base = int(sec_off[-1])
        enc_off = np.zeros(nconn, np.uint64)
        enc_off[1:] = np.cumsum([len(e) for e in enc])[:-1] if nconn > 1 else []
        enc_off += base
        data = b"".join(sec_bytes) + b"".join(enc)
        out.append(dict(data=np.frombuffer(data, np.uint8).copy(), sec_off=sec_off.astype(np.uint32),
                        conn_first=np.asarray(conn_first, np.uint32), enc_off=enc_off.astype(np.uint32),
                        enc_len=np.asarray([len(e) for e in enc], np.uint32), header_table_size=header_table_size))
    return out


def arena_offsets(sec_off, header_table_size):
    """a generous arena slice per section: every field of an L-byte section is either a literal (<= 8/5 of
    its bytes) or a copy of a static (<= 76 bytes) or dynamic (<= table size) entry"""
    L = np.diff(np.asarray(sec_off, dtype=np.uint64))
    # dynamic entries of the synthetic sessions stay far below 8 KiB: a tighter bound keeps large-table
    # sessions' arenas under the 2^32 reach of the u32 field offsets (a slice too small is HHUFF_QPK_ARENA on
    # both sides of a comparison)
    ent = np.uint64(min(int(header_table_size), 8192))
    cap = (L * 8) // 5 + L * np.uint64(80) + (L // 2 + 1) * ent + np.uint64(16)
    out = np.zeros(L.size + 1, np.uint64)
    out[1:] = np.cumsum(cap)
    return out
