"""Seeded synthetic HPACK connections (header blocks) for the f4 block decoder.

An encoder model in the spirit of h2o's own (lib/http2/hpack.c:858-937 do_encode_header): fields found in
the static table or the model's dynamic table are indexed; others are literals with incremental indexing
(most), without indexing or never indexed, with an indexed name where the name is known, each string
Huffman-coded when that is strictly shorter (h2o_hpack_encode_string, hpack.c:816-837).  The model keeps
its own dynamic table with h2o's add / evict rules so that its dynamic indices are the ones a decoder
sees; blocks may open with table-size updates.  Requests draw from a vocabulary of realistic names and
values (pseudo-headers, user agents, cookies, paths), so later blocks of a connection hit the dynamic
table the way browser traffic does.

Adversarial connections (a fraction) then get one mutation: a truncated block, a flipped byte, an index
past the table, an oversized table-size update, an upper-case raw name, invalid characters in raw names
and values (soft errors), or a literal whose length runs past the block.

A batch: blocks packed back to back (`data`, `blk_off` [nblocks+1]) and `conn_first` [nconn+1]: the
include/hhuff.h hhuff_hpack_decode_blocks layout.
"""
import numpy as np

from . import tables

STATIC = tables.STATIC_TABLE  # ((name, value), ...) for indices 1..61
ENTRY_OVERHEAD = 32


def _huffman(s: bytes):
    bits, nb = 0, 0
    for c in s:
        bits = (bits << tables.ENC_NBITS[c]) | tables.ENC_CODE[c]
        nb += tables.ENC_NBITS[c]
    pad = (-nb) % 8
    bits = (bits << pad) | ((1 << pad) - 1)
    n = (nb + pad) // 8
    return bits.to_bytes(n, "big") if n else b""


def encode_int(value, prefix_bits, first=0):
    mx = (1 << prefix_bits) - 1
    if value < mx:
        return bytes([first | value])
    out = [first | mx]
    value -= mx
    while value >= 128:
        out.append(0x80 | (value & 127))
        value >>= 7
    out.append(value)
    return bytes(out)


def encode_string(s: bytes, force_raw=False):
    """h2o_hpack_encode_string: Huffman when strictly shorter, else raw (H bit 0)"""
    if s and not force_raw:
        h = _huffman(s)
        if len(h) < len(s):
            return encode_int(len(h), 7, 0x80) + h
    return encode_int(len(s), 7, 0) + s


class _Table:
    """dynamic table model with h2o's rules (hpack.c:263-317, :352-366)"""

    def __init__(self, cap):
        self.e, self.size, self.cap = [], 0, cap

    def add(self, name, value):
        add = len(name) + len(value) + ENTRY_OVERHEAD
        while self.e and self.size + add > self.cap:
            self.evict()
        if not self.e and add > self.cap:
            return
        self.e.insert(0, (name, value))
        self.size += add

    def evict(self):
        n, v = self.e.pop()
        self.size -= len(n) + len(v) + ENTRY_OVERHEAD

    def resize(self, cap):
        self.cap = cap
        while self.e and self.size > self.cap:
            self.evict()

    def find(self, name, value):
        """-> (full index or 0, name index or 0)"""
        full = name_i = 0
        for i, (n, v) in enumerate(STATIC):
            if n == name:
                name_i = name_i or i + 1
                if v == value:
                    return i + 1, name_i
        for i, (n, v) in enumerate(self.e):
            if n == name:
                name_i = name_i or 62 + i
                if v == value:
                    return 62 + i, name_i
        return full, name_i


def _vocab(rng):
    def word(k, alpha=b"abcdefghijklmnopqrstuvwxyz0123456789"):
        return bytes(rng.choice(np.frombuffer(alpha, np.uint8), size=k))

    hosts = [b"www.%s.com" % word(int(rng.integers(4, 12))) for _ in range(40)]
    paths = [b"/" + b"/".join(word(int(rng.integers(2, 10))) for _ in range(int(rng.integers(1, 5))))
             + (b"?" + word(int(rng.integers(3, 20))) if rng.random() < 0.4 else b"") for _ in range(400)]
    agents = [b"Mozilla/5.0 (X11; Linux x86_64) AppleWebKit/537.36 (KHTML, like Gecko) Chrome/%d.0.%d.%d Safari/537.36"
              % (int(rng.integers(90, 130)), int(rng.integers(1000, 9999)), int(rng.integers(10, 200)))
              for _ in range(8)]
    cookies = [b"; ".join(b"%s=%s" % (word(int(rng.integers(3, 8))), word(int(rng.integers(8, 40)),
                                                                         b"ABCDEFabcdef0123456789-_"))
                         for _ in range(int(rng.integers(1, 5)))) for _ in range(60)]
    accepts = [b"text/html,application/xhtml+xml,application/xml;q=0.9,*/*;q=0.8", b"*/*", b"application/json",
               b"image/avif,image/webp,*/*"]
    return hosts, paths, agents, cookies, accepts


def _request(rng, V, host):
    hosts, paths, agents, cookies, accepts = V
    f = [(b":method", b"GET" if rng.random() < 0.85 else b"POST"), (b":scheme", b"https"), (b":authority", host),
         (b":path", paths[int(rng.integers(len(paths)))]), (b"user-agent", agents[int(rng.integers(len(agents)))]),
         (b"accept", accepts[int(rng.integers(len(accepts)))]), (b"accept-encoding", b"gzip, deflate, br")]
    if rng.random() < 0.6:
        f.append((b"cookie", cookies[int(rng.integers(len(cookies)))]))
    if rng.random() < 0.3:
        f.append((b"x-request-id", b"%032x" % int(rng.integers(1 << 62))))
    if rng.random() < 0.2:
        f.append((b"referer", b"https://" + host + paths[int(rng.integers(len(paths)))]))
    return f


def _request_rules(rng, f):
    """one of h2o_hpack_parse_request's cases (hpack.c:502-637) applied to a request's field list"""
    kind = int(rng.integers(17))
    reg = [(b"x-h%d" % i, b"v%d" % i) for i in range(int(rng.integers(1, 4)))]
    if kind == 0:  # duplicate pseudo-header
        k = int(rng.integers(4))
        f.insert(k + 1, f[k])
    elif kind == 1:  # pseudo-header after a regular field
        f.append([(b":path", b"/late"), (b":method", b"GET"), (b":authority", b"x.example")][int(rng.integers(3))])
    elif kind == 2:  # empty :path
        f[3] = (b":path", b"")
    elif kind == 3:  # unknown / response pseudo-headers
        f.insert(int(rng.integers(4)), [(b":status", b"200"), (b":foo", b"bar"), (b":", b"x")][int(rng.integers(3))])
    elif kind == 4:  # :protocol once (extended CONNECT) or twice
        f.insert(1, (b":protocol", b"websocket"))
        if rng.random() < 0.5:
            f.insert(2, (b":protocol", b"websocket"))
    elif kind == 5:  # content-length, valid or not (h2o_strtosize)
        v = [b"0", b"123", b"9999999999999999999", b"10000000000000000000", b"", b"12a", b"-1", b" 5", b"1" * 20,
             b"007"][int(rng.integers(10))]
        f.append((b"content-length", v))
        if rng.random() < 0.2:
            f.append((b"content-length", b"42"))
    elif kind == 6:  # connection-specific fields
        f.append(([(b"connection", b"keep-alive"), (b"transfer-encoding", b"chunked"), (b"upgrade", b"h2c"),
                   (b"http2-settings", b"AAMAAABkAAQAAP__")][int(rng.integers(4))]))
    elif kind == 7:  # te
        f.append((b"te", [b"trailers", b"Trailers", b"TRAILERS", b"gzip", b"trailers, gzip"][int(rng.integers(5))]))
    elif kind == 8:  # host, with or without :authority
        if rng.random() < 0.5:
            del f[2]
        f.append((b"host", b"h.example"))
    elif kind == 9:  # expect, once or twice
        f.append((b"expect", b"100-continue"))
        if rng.random() < 0.4:
            f.append((b"expect", b"other"))
    elif kind == 10:  # datagram-flow-id (dropped for HTTP/2), cache-digest (listed)
        f.append([(b"datagram-flow-id", b"4"), (b"cache-digest", b"AfdA; complete")][int(rng.integers(2))])
    elif kind == 11:  # past H2O_MAX_HEADERS (100): the rest is dropped, the block ends soft
        f += [(b"x-n%d" % (i % 7), b"%d" % i) for i in range(int(rng.integers(95, 130)))]
    elif kind == 12:  # past H2O_HPACK_MAX_HEADERS_HARD_LIMIT (1000)
        f += [(b"accept-encoding", b"gzip, deflate")] * int(rng.integers(990, 1010))
    elif kind == 13:  # :scheme variants
        f[1] = (b":scheme", [b"http", b"masque", b"ftp", b"HTTPS", b""][int(rng.integers(5))])
    elif kind == 14:  # fields h2o lists even though other servers treat them as hop-by-hop
        f.append([(b"keep-alive", b"timeout=5"), (b"proxy-connection", b"keep-alive")][int(rng.integers(2))])
    elif kind == 15:  # regular fields between pseudo-headers, a CONNECT without :path
        f.insert(2, reg[0])
    else:  # only pseudo-headers / only regular fields
        f = f[:4] if rng.random() < 0.5 else f[4:]
    return f


def encode_block(rng, table, fields, max_cap, size_update=None):
    out = bytearray()
    if size_update is not None:
        out += encode_int(size_update, 5, 0x20)
        table.resize(size_update)
    for name, value in fields:
        full, name_i = table.find(name, value)
        if full and rng.random() < 0.95:
            out += encode_int(full, 7, 0x80)
            continue
        r = rng.random()
        raw = rng.random() < 0.1
        if r < 0.75:
            out += encode_int(name_i, 6, 0x40) if name_i else b"\x40" + encode_string(name, raw)
            out += encode_string(value, raw)
            table.add(name, value)
        else:
            first = 0x00 if r < 0.9 else 0x10
            out += encode_int(name_i, 4, first) if name_i else bytes([first]) + encode_string(name, raw)
            out += encode_string(value, raw)
    return bytes(out)


def _mutate(rng, blocks, max_cap):
    b = int(rng.integers(len(blocks)))
    blk = bytearray(blocks[b])
    kind = int(rng.integers(9))
    if kind == 0 and len(blk) > 1:  # truncated block
        blk = blk[:int(rng.integers(1, len(blk)))]
    elif kind == 1 and blk:  # flipped byte
        i = int(rng.integers(len(blk)))
        blk[i] ^= 1 << int(rng.integers(8))
    elif kind == 2:  # index past the table
        blk += encode_int(62 + 200 + int(rng.integers(100)), 7, 0x80)
    elif kind == 3:  # oversized table-size update
        blk = bytearray(encode_int(max_cap + 1 + int(rng.integers(1000)), 5, 0x20)) + blk
    elif kind == 4:  # upper-case raw name (PROTOCOL error)
        blk += b"\x00" + encode_string(b"X-Upper", True) + encode_string(b"v", True)
    elif kind == 5:  # soft errors: invalid name chars / value CTL / surrounding whitespace
        bad = [(b"bad name", b"v"), (b"x-ok", b"a\x01b"), (b"x-ok", b" leading"), (b"x-ok", b"trailing\t"),
               (b"", b"empty-name"), (b":pseudo", b"x")][int(rng.integers(6))]
        blk += b"\x00" + encode_string(bad[0], rng.random() < 0.5) + encode_string(bad[1], rng.random() < 0.5)
    elif kind == 6:  # literal length past the block
        blk += b"\x00" + encode_int(5, 7, 0) + b"abc"
    elif kind == 7:  # entry larger than the table, then indexed
        big = b"v" * (max_cap + 10)
        blk += b"\x40" + encode_string(b"x-big", True) + encode_string(big, True) + encode_int(62, 7, 0x80)
    else:  # trailing size update (the block then ends inside a field)
        blk += encode_int(max_cap // 2, 5, 0x20)
    blocks[b] = bytes(blk)


def make_connections(nconn, blocks_per_conn=(1, 8), seed=0, table_size=4096, adversarial_frac=0.05, request_frac=0.0):
    """-> dict(data u8[], blk_off u32[nb+1], conn_first u32[nconn+1], table_size); request_frac of the requests
    exercise one of h2o_hpack_parse_request's rules (_request_rules)"""
    rng = np.random.default_rng(seed)
    V = _vocab(rng)
    hosts = V[0]
    blocks, conn_first = [], [0]
    for c in range(nconn):
        table = _Table(table_size)
        host = hosts[int(rng.integers(len(hosts)))]
        nb = int(rng.integers(blocks_per_conn[0], blocks_per_conn[1] + 1))
        cb = []
        for k in range(nb):
            su = None
            if rng.random() < 0.05:
                su = int(rng.integers(0, table_size + 1))
            f = _request(rng, V, host)
            if request_frac and rng.random() < request_frac:
                f = _request_rules(rng, f)
            cb.append(encode_block(rng, table, f, table_size, su))
        if rng.random() < adversarial_frac:
            _mutate(rng, cb, table_size)
        blocks += cb
        conn_first.append(len(blocks))
    data, off = b"".join(blocks), np.zeros(len(blocks) + 1, np.uint64)
    off[1:] = np.cumsum([len(b) for b in blocks])
    return dict(data=np.frombuffer(data, np.uint8).copy(), blk_off=off.astype(np.uint32),
                conn_first=np.asarray(conn_first, np.uint32), table_size=table_size)


def pack_connections(conns, table_size=4096):
    """list of connections (each a list of block bytes) -> the batch layout"""
    blocks, conn_first = [], [0]
    for cb in conns:
        blocks += list(cb)
        conn_first.append(len(blocks))
    off = np.zeros(len(blocks) + 1, np.uint64)
    off[1:] = np.cumsum([len(b) for b in blocks])
    return dict(data=np.frombuffer(b"".join(blocks), np.uint8).copy(), blk_off=off.astype(np.uint32),
                conn_first=np.asarray(conn_first, np.uint32), table_size=table_size)


# ---- response header blocks (the client side: h2o_hpack_parse_response, lib/http2/hpack.c:642-750) ----
def _response(rng, V):
    """a server response head as a client receives it: :status first, then regular fields"""
    hosts, paths, agents, cookies, accepts = V
    st = [b"200", b"200", b"200", b"204", b"206", b"301", b"302", b"304", b"404", b"500", b"103"][int(rng.integers(11))]
    f = [(b":status", st), (b"content-type", [b"text/html; charset=utf-8", b"application/json", b"image/webp"]
                                              [int(rng.integers(3))]),
         (b"date", b"Sat, 17 Oct 2026 %02d:%02d:%02d GMT" % (int(rng.integers(24)), int(rng.integers(60)),
                                                              int(rng.integers(60)))),
         (b"server", b"h2o/2.3.0-dev")]
    if rng.random() < 0.6:
        f.append((b"cache-control", [b"max-age=3600", b"no-cache", b"private, max-age=0"][int(rng.integers(3))]))
    if rng.random() < 0.5:
        f.append((b"etag", b'"%016x"' % int(rng.integers(1 << 62))))
    if rng.random() < 0.3:
        f.append((b"set-cookie", cookies[int(rng.integers(len(cookies)))]))
    if rng.random() < 0.2:
        f.append((b"location", b"https://" + hosts[int(rng.integers(len(hosts)))] + paths[int(rng.integers(len(paths)))]))
    return f


def _trailers(rng):
    f = [(b"x-checksum", b"%08x" % int(rng.integers(1 << 31)))]
    if rng.random() < 0.5:
        f.append((b"grpc-status", b"%d" % int(rng.integers(17))))
    if rng.random() < 0.3:
        f.append((b"grpc-message", b"ok"))
    return f


def _response_rules(rng, f, trailers):
    """one of h2o_hpack_parse_response's cases applied to a head's (or trailers') field list"""
    kind = int(rng.integers(14))
    if kind == 0:  # :status variants (three digits, the first 1-9; PARSE_DIGIT keeps the digits before a bad one)
        v = [b"099", b"1000", b"20", b"2x0", b"20x", b"x00", b"999", b"100", b"", b"0200", b"2 0"][int(rng.integers(11))]
        if trailers:
            f.insert(0, (b":status", v))
        else:
            f[0] = (b":status", v)
    elif kind == 1:  # duplicate :status
        f.insert(1, (b":status", b"200"))
    elif kind == 2:  # missing :status: a regular field first, or no field at all
        f = f[1:] if not trailers else f
        if rng.random() < 0.2:
            f = []
    elif kind == 3:  # other pseudo-headers
        f.insert(int(rng.integers(len(f) + 1)), [(b":path", b"/"), (b":method", b"GET"), (b":foo", b"x"),
                                                 (b":authority", b"a.example")][int(rng.integers(4))])
    elif kind == 4:  # :status after a regular field
        f.append((b":status", b"200"))
    elif kind == 5:  # the passed-through special fields
        f.append([(b"content-length", b"123"), (b"content-length", b"abc"), (b"host", b"h.example"),
                  (b"cache-digest", b"AfdA; complete")][int(rng.integers(4))])
    elif kind == 6:  # the rejected ones
        f.append([(b"connection", b"close"), (b"transfer-encoding", b"chunked"), (b"upgrade", b"h2c"),
                  (b"http2-settings", b"AAMA"), (b"te", b"trailers"), (b"expect", b"100-continue")]
                 [int(rng.integers(6))])
    elif kind == 7:  # datagram-flow-id: not listed (stored for HTTP/3)
        f.insert(max(1, int(rng.integers(len(f) + 1))), (b"datagram-flow-id", b"4"))
    elif kind == 8:  # past H2O_MAX_HEADERS (100)
        f += [(b"x-n%d" % (i % 7), b"%d" % i) for i in range(int(rng.integers(95, 130)))]
    elif kind == 9:  # past the hard limit (1000)
        f += [(b"vary", b"accept-encoding")] * int(rng.integers(990, 1010))
    elif kind == 10:  # soft errors in values (the first one is kept in err_desc)
        f.append((b"x-bad", [b"a\x01b", b" lead", b"trail\t"][int(rng.integers(3))]))
    elif kind == 11:  # keep-alive / proxy-connection: listed
        f.append([(b"keep-alive", b"timeout=5"), (b"proxy-connection", b"keep-alive")][int(rng.integers(2))])
    else:  # only :status
        f = f[:1]
    return f


def make_response_connections(nconn, blocks_per_conn=(1, 8), seed=0, table_size=4096, adversarial_frac=0.05,
                              rule_frac=0.3, trailer_frac=0.2):
    """-> the make_connections layout plus trailers u8[nb] (nonzero: a trailers block, status == NULL);
    rule_frac of the blocks exercise one of h2o_hpack_parse_response's rules (_response_rules)"""
    rng = np.random.default_rng(seed)
    V = _vocab(rng)
    blocks, conn_first, trailers = [], [0], []
    for c in range(nconn):
        table = _Table(table_size)
        nb = int(rng.integers(blocks_per_conn[0], blocks_per_conn[1] + 1))
        cb, ct = [], []
        for k in range(nb):
            su = None
            if rng.random() < 0.05:
                su = int(rng.integers(0, table_size + 1))
            tr = rng.random() < trailer_frac
            f = _trailers(rng) if tr else _response(rng, V)
            if rng.random() < rule_frac:
                f = _response_rules(rng, f, tr)
            cb.append(encode_block(rng, table, f, table_size, su))
            ct.append(1 if tr else 0)
        if rng.random() < adversarial_frac:
            _mutate(rng, cb, table_size)
        blocks += cb
        trailers += ct
        conn_first.append(len(blocks))
    data, off = b"".join(blocks), np.zeros(len(blocks) + 1, np.uint64)
    off[1:] = np.cumsum([len(b) for b in blocks])
    return dict(data=np.frombuffer(data, np.uint8).copy(), blk_off=off.astype(np.uint32),
                conn_first=np.asarray(conn_first, np.uint32), table_size=table_size,
                trailers=np.asarray(trailers, np.uint8))
