"""Seeded synthetic HTTP/2 responses for the f4 encode side (h2o_hpack_flatten_response).

Connections of 1-8 responses each, as an h2o server sends them: a site profile per connection (content
types, caching and security headers, a server name) and per response a status (mostly 200, some 204 / 206
/ 301 / 304 / 404 and informational 103s), a date that moves every few responses, an etag and last-modified,
now and then set-cookie (some values under 20 bytes: sent never-indexed, hpack.c:892-903), a request id
that never repeats (a non-token name: a new-name literal every time), a content length, and rarely:
trailers (h2o_hpack_flatten_trailers), headers added without their token (h2o_add_header_by_str with
maybe_token 0), header dont_compress flags, a peer SETTINGS_HEADER_TABLE_SIZE below 4096 (a Dynamic Table
Size Update, evictions; a few connections change it between responses), responses longer than
max_frame_size (CONTINUATION frames), and a larger max_frame_size.

A batch (the include/hhuff.h hhuff_hpack_flatten_responses layout): `data` (every distinct string once),
`hdr` (HPE_HEADER_DTYPE records), `res` (HPE_RESPONSE_DTYPE), `conn_first` [nconn+1], `server_off`,
`server_len`, `out_off` [nres+1] (hhuff_hpack_response_bound per response, 16-byte aligned).
Several steps of one session continue the same connections (HHUFF_ENC_CONTINUE).
"""
import numpy as np

from .codec import HPE_HEADER_DTYPE, HPE_RESPONSE_DTYPE, QPE_RESPONSE_DTYPE, HDR_DONT_COMPRESS, HDR_TOKEN, \
    QRES_DATAGRAM, QRES_REQUEST, RES_END_STREAM, RES_REQUEST, RES_SERVER, RES_TRAILERS, hpack_response_bound, qpack_response_bound

SERVER = b"h2o/2.3.0-dev"
_CTYPES = [b"text/html; charset=utf-8", b"text/css", b"application/javascript", b"image/png", b"image/jpeg",
           b"image/webp", b"application/json", b"font/woff2", b"text/plain", b"image/svg+xml", b"video/mp4"]
_CACHE = [b"public, max-age=31536000, immutable", b"no-cache", b"no-store", b"private, max-age=0",
          b"max-age=3600", b"public, max-age=86400", b"must-revalidate, max-age=60"]
_STATUS = [200] * 70 + [304] * 8 + [204] * 3 + [206] * 3 + [404] * 4 + [301] * 3 + [302] * 2 + [500] + [503] + [103] * 2 + \
    [400, 401, 403, 429]
_DAYS = [b"Mon", b"Tue", b"Wed", b"Thu", b"Fri", b"Sat", b"Sun"]
_MONTHS = [b"Jan", b"Feb", b"Mar", b"Apr", b"May", b"Jun", b"Jul", b"Aug", b"Sep", b"Oct", b"Nov", b"Dec"]
_HEX = np.frombuffer(b"0123456789abcdef", np.uint8)
_B64 = np.frombuffer(b"ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789-_", np.uint8)


def _date(t):
    d, s = divmod(int(t), 86400)
    return b"%s, %02d %s 2026 %02d:%02d:%02d GMT" % (_DAYS[d % 7], 1 + d % 28, _MONTHS[(d // 28) % 12], s // 3600,
                                                      s // 60 % 60, s % 60)


def _rand(rng, alphabet, n):
    return alphabet[rng.integers(0, alphabet.size, n)].tobytes()


class _Batch:
    def __init__(self):
        self.pool = {}
        self.chunks = []
        self.size = 0
        self.hdr = []
        self.res = []

    def s(self, b):
        off = self.pool.get(b)
        if off is None:
            off = self.size
            self.pool[b] = off
            self.chunks.append(b)
            self.size += len(b)
        return off

    def header(self, name, value, flags):
        self.hdr.append((self.s(name), len(name), self.s(value), len(value), flags))


def _site(rng):
    sec = []
    if rng.random() < 0.6:
        sec.append((b"strict-transport-security", b"max-age=63072000; includeSubDomains; preload"))
    if rng.random() < 0.5:
        sec.append((b"x-content-type-options", b"nosniff"))
    if rng.random() < 0.4:
        sec.append((b"x-frame-options", [b"DENY", b"SAMEORIGIN"][int(rng.integers(0, 2))]))
    if rng.random() < 0.3:
        sec.append((b"alt-svc", b'h3=":443"; ma=86400'))
    if rng.random() < 0.2:
        sec.append((b"access-control-allow-origin", b"*"))
    if rng.random() < 0.15:
        sec.append((b"content-security-policy", b"default-src 'self'; img-src * data:; script-src 'self' "
                    b"https://cdn.example.net; style-src 'self' 'unsafe-inline'"))
    return dict(ctypes=[_CTYPES[i] for i in rng.choice(len(_CTYPES), 4, replace=False)],
                cache=[_CACHE[i] for i in rng.choice(len(_CACHE), 2, replace=False)], sec=sec,
                vary=rng.random() < 0.7, t=int(rng.integers(0, 10 ** 7)))


# token names used below (lib/common/token_table.h); everything else is added by string
_TOKENS = {b"date", b"content-type", b"cache-control", b"etag", b"last-modified", b"vary", b"set-cookie", b"age",
           b"accept-ranges", b"content-encoding", b"location", b"link", b"expires", b"strict-transport-security",
           b"x-content-type-options", b"x-frame-options", b"alt-svc", b"access-control-allow-origin",
           b"content-security-policy", b"server", b"content-length", b"te", b"x-xss-protection", b"content-range",
           b"retry-after", b"cookie"}


def _response(rng, site, B, k, big_frac):
    st = _STATUS[int(rng.integers(0, len(_STATUS)))]
    hs = []
    if st == 103:
        hs.append((b"link", b"</style.css>; rel=preload; as=style"))
        return st, hs, None, False
    site["t"] += int(rng.integers(0, 3))
    hs.append((b"date", _date(site["t"])))
    if st in (200, 206, 304):
        hs.append((b"content-type", site["ctypes"][int(rng.integers(0, 4))]))
        hs.append((b"cache-control", site["cache"][int(rng.integers(0, 2))]))
        hs.append((b"etag", b'"' + _rand(rng, _HEX, int(rng.integers(8, 33))) + b'"'))
        hs.append((b"last-modified", _date(site["t"] - int(rng.integers(0, 10 ** 6)))))
        if site["vary"]:
            hs.append((b"vary", b"accept-encoding"))
        if rng.random() < 0.5:
            hs.append((b"content-encoding", [b"gzip", b"br"][int(rng.integers(0, 2))]))
        hs.append((b"accept-ranges", b"bytes"))
        if st == 206:
            hs.append((b"content-range", b"bytes 0-%d/%d" % (int(rng.integers(1, 99999)), int(rng.integers(10 ** 5, 10 ** 7)))))
        if rng.random() < 0.3:
            hs.append((b"age", b"%d" % int(rng.integers(0, 5000))))
    elif st in (301, 302):
        hs.append((b"location", b"https://www.example.com/" + _rand(rng, _B64, int(rng.integers(4, 40)))))
    elif st == 503 or st == 429:
        hs.append((b"retry-after", b"%d" % int(rng.integers(1, 120))))
    hs += site["sec"]
    if rng.random() < 0.2:
        v = _rand(rng, _B64, int(rng.integers(4, 12))) if rng.random() < 0.3 else _rand(rng, _B64, int(rng.integers(20, 90)))
        hs.append((b"set-cookie", b"sid=" + v + (b"; Path=/; Secure; HttpOnly" if len(v) > 12 else b"")))
    hs.append((b"x-request-id", _rand(rng, _HEX, 32)))
    if rng.random() < 0.1:
        hs.append((b"server-timing", b"cdn-cache; desc=%s, edge; dur=%d" % ([b"HIT", b"MISS"][int(rng.integers(0, 2))],
                                                                           int(rng.integers(1, 300)))))
    if rng.random() < big_frac:  # longer than max_frame_size: CONTINUATION frames
        for _ in range(int(rng.integers(1, 4))):
            hs.append((b"link", b", ".join(b"</a/%s.js>; rel=preload; as=script" % _rand(rng, _B64, 12)
                                             for _ in range(int(rng.integers(300, 700))))))
    cl = int(rng.integers(0, 1 << 22)) if st not in (204, 304) and rng.random() < 0.85 else None
    end = st in (204, 304) or rng.random() < 0.05
    return st, hs, cl, end


def make_session(nconn, steps=1, resp_per_conn=(1, 8), seed=0, small_table_frac=0.05, trailers_frac=0.02,
                 big_frac=0.001, notoken_frac=0.01, dont_compress_frac=0.01, frame_frac=0.05):
    """-> list of `steps` batches over the same nconn connections (a connection's responses continue in the
    next step: call with HHUFF_ENC_CONTINUE)"""
    rng = np.random.default_rng(seed)
    sites = [_site(rng) for _ in range(nconn)]
    caps = [4096 if rng.random() >= small_table_frac else int(rng.choice([0, 64, 256, 1024, 2048])) for _ in range(nconn)]
    mfs = [16384 if rng.random() >= frame_frac else int(rng.choice([1 << 15, 1 << 20, (1 << 24) - 1])) for _ in range(nconn)]
    sids = [1] * nconn
    out = []
    for _ in range(steps):
        B = _Batch()
        server_off = B.s(SERVER)
        conn_first = [0]
        for c in range(nconn):
            for k in range(int(rng.integers(resp_per_conn[0], resp_per_conn[1] + 1))):
                if rng.random() < 0.02:  # the peer changes SETTINGS_HEADER_TABLE_SIZE
                    caps[c] = int(rng.choice([0, 128, 512, 1024, 4096, 65536]))
                trailers = rng.random() < trailers_frac
                if trailers:
                    st, hs, cl, end = 0, [(b"server-timing", b"total; dur=%d" % int(rng.integers(1, 999))),
                                          (b"x-checksum", _rand(rng, _HEX, 16))], None, True
                else:
                    st, hs, cl, end = _response(rng, sites[c], B, k, big_frac)
                first = len(B.hdr)
                for name, value in hs:
                    f = HDR_TOKEN if name in _TOKENS and rng.random() >= notoken_frac else 0
                    if rng.random() < dont_compress_frac:
                        f |= HDR_DONT_COMPRESS
                    B.header(name, value, f)
                fl = (RES_END_STREAM if end else 0) | (RES_TRAILERS if trailers else 0) | \
                    (RES_SERVER if st != 103 and not trailers else 0)
                B.res.append((np.uint64(0xFFFFFFFFFFFFFFFF) if cl is None else cl, sids[c], st, first, len(B.hdr) - first,
                              caps[c], mfs[c], fl, 0))
                if not trailers:
                    sids[c] += 2
            conn_first.append(len(B.res))
        hdr = np.array(B.hdr, dtype=HPE_HEADER_DTYPE) if B.hdr else np.zeros(0, HPE_HEADER_DTYPE)
        res = np.array(B.res, dtype=HPE_RESPONSE_DTYPE)
        data = np.frombuffer(b"".join(B.chunks), np.uint8).copy()
        out.append(dict(data=data, hdr=hdr, res=res, conn_first=np.array(conn_first, np.uint32), server_off=server_off,
                        server_len=len(SERVER), out_off=out_offsets(hdr, res, len(SERVER))))
    return out


# ---- the client side: h2o_hpack_flatten_request (lib/http2/hpack.c:1044-1096) as lib/common/http2client.c:1140
# calls it for a proxied request ----
_REQ_TOKENS = {b"user-agent", b"accept", b"accept-language", b"accept-encoding", b"cookie", b"content-type",
               b"content-length", b"referer", b"x-forwarded-for", b"via", b"authorization", b"if-none-match",
               b"if-modified-since", b"origin", b"range", b"cache-control", b"priority", b"forwarded", b"te"}
_METHODS = [b"GET"] * 75 + [b"POST"] * 10 + [b"HEAD"] * 4 + [b"PUT"] * 3 + [b"DELETE"] * 2 + [b"OPTIONS"] * 2 + \
    [b"PATCH"] + [b"CONNECT"] * 2 + [b"XCONNECT"]  # XCONNECT: an RFC 9220 extended CONNECT (:protocol)
_UAS = [b"Mozilla/5.0 (X11; Linux x86_64) AppleWebKit/537.36 (KHTML, like Gecko) Chrome/126.0 Safari/537.36",
        b"curl/8.5.0", b"h2o/2.3.0-dev", b"Mozilla/5.0 (Macintosh; Intel Mac OS X 14_5) Gecko/20100101 Firefox/127.0"]
_ACCEPTS = [b"*/*", b"text/html,application/xhtml+xml,application/xml;q=0.9,*/*;q=0.8", b"application/json",
            b"image/avif,image/webp,*/*"]
_AES = [b"gzip, deflate"] * 5 + [b"gzip, deflate, br"] * 3 + [b"br", b"identity"]


def _client(rng):
    host = b"%s.example.%s" % (_rand(rng, _B64[26:52], int(rng.integers(3, 10))), [b"com", b"net", b"org"][int(rng.integers(0, 3))])
    if rng.random() < 0.2:
        host += b":%d" % int(rng.integers(1024, 65536))
    return dict(host=host, ua=_UAS[int(rng.integers(0, len(_UAS)))], lang=[b"en-US,en;q=0.9", b"ja,en;q=0.5", b"de-DE"][
        int(rng.integers(0, 3))], ae=_AES[int(rng.integers(0, len(_AES)))] if rng.random() < 0.9 else None,
        cookie=b"sid=" + _rand(rng, _B64, int(rng.integers(8, 40))) if rng.random() < 0.4 else None,
        scheme=b"https" if rng.random() < 0.88 else b"http" if rng.random() < 0.85 else [b"masque", b"ftp", b""][
            int(rng.integers(0, 3))], xff=b"192.0.2.%d" % int(rng.integers(1, 255)))


def _request(rng, cl, big_frac):
    """-> (own fields, headers, end_stream): flatten_request's own fields in its order, then the headers"""
    m = _METHODS[int(rng.integers(0, len(_METHODS)))]
    extended = m == b"XCONNECT"
    if extended:
        m = b"CONNECT"
    own = [(b":method", m)]
    old_style = m == b"CONNECT" and not extended
    if not old_style:
        own.append((b":scheme", cl["scheme"]))
    own.append((b":authority", cl["host"] if not old_style else b"proxy.example.net:443"))
    if not old_style:
        u = rng.random()
        path = b"/" if u < 0.1 else b"/index.html" if u < 0.15 else b"/chat" if extended else \
            b"/%s/%s" % (_rand(rng, _B64[26:52], int(rng.integers(2, 8))), _rand(rng, _B64, int(rng.integers(1, 40))))
        if rng.random() < 0.3 and not extended:
            path += b"?q=" + _rand(rng, _B64, int(rng.integers(1, 30)))
        own.append((b":path", path))
    if extended:
        own.append((b":protocol", [b"websocket", b"connect-udp", b""][int(rng.integers(0, 3))]))
    body = m in (b"POST", b"PUT", b"PATCH")
    if body and rng.random() < 0.3:  # send_own_expect (http2client.c:1135-1136)
        own.append((b"expect", b"100-continue"))
    hs = [(b"user-agent", cl["ua"]), (b"accept", _ACCEPTS[int(rng.integers(0, len(_ACCEPTS)))])]
    if cl["ae"] is not None:
        hs.append((b"accept-encoding", cl["ae"]))
    hs.append((b"accept-language", cl["lang"]))
    if cl["cookie"] is not None:
        hs.append((b"cookie", cl["cookie"]))
    if rng.random() < 0.3:
        hs.append((b"referer", b"https://%s/%s" % (cl["host"], _rand(rng, _B64, int(rng.integers(1, 20))))))
    if rng.random() < 0.1:
        hs.append((b"if-none-match", b'"' + _rand(rng, _HEX, 16) + b'"'))
    if body:
        hs.append((b"content-type", [b"application/json", b"application/x-www-form-urlencoded"][int(rng.integers(0, 2))]))
        hs.append((b"content-length", b"%d" % int(rng.integers(0, 1 << 20))))
    if rng.random() < 0.05:
        hs.append((b"authorization", b"Bearer " + _rand(rng, _B64, int(rng.integers(5, 60)))))
    hs.append((b"x-forwarded-for", cl["xff"]))
    hs.append((b"via", b"2 h2o"))
    hs.append((b"x-request-id", _rand(rng, _HEX, 32)))
    if rng.random() < 0.05:  # accept-encoding "gzip, deflate" a second time, then some other value
        hs.append((b"accept-encoding", b"gzip, deflate"))
    if rng.random() < big_frac:  # longer than max_frame_size: CONTINUATION frames
        hs.append((b"cookie", b"; ".join(b"k%d=%s" % (j, _rand(rng, _B64, 24)) for j in range(int(rng.integers(600, 1500))))))
    end = not body and m != b"CONNECT"
    return own, hs, end


def make_request_session(nconn, steps=1, req_per_conn=(1, 8), seed=0, small_table_frac=0.05, big_frac=0.002,
                         notoken_frac=0.01, dont_compress_frac=0.01, frame_frac=0.05):
    """Client requests (HHUFF_RES_REQUEST records: `status` = the number of own fields), one encoder table per
    upstream connection; same batch layout as make_session"""
    rng = np.random.default_rng(seed)
    clients = [_client(rng) for _ in range(nconn)]
    caps = [4096 if rng.random() >= small_table_frac else int(rng.choice([0, 64, 256, 1024, 2048])) for _ in range(nconn)]
    mfs = [16384 if rng.random() >= frame_frac else int(rng.choice([1 << 15, 1 << 20, (1 << 24) - 1])) for _ in range(nconn)]
    sids = [1] * nconn
    out = []
    for _ in range(steps):
        B = _Batch()
        server_off = B.s(SERVER)
        conn_first = [0]
        for c in range(nconn):
            for _k in range(int(rng.integers(req_per_conn[0], req_per_conn[1] + 1))):
                if rng.random() < 0.02:
                    caps[c] = int(rng.choice([0, 128, 512, 1024, 4096, 65536]))
                own, hs, end = _request(rng, clients[c], big_frac)
                first = len(B.hdr)
                for name, value in own:
                    B.header(name, value, HDR_TOKEN)
                for name, value in hs:
                    f = HDR_TOKEN if name in _REQ_TOKENS and rng.random() >= notoken_frac else 0
                    if rng.random() < dont_compress_frac:
                        f |= HDR_DONT_COMPRESS
                    B.header(name, value, f)
                fl = RES_REQUEST | (RES_END_STREAM if end else 0) | (RES_SERVER if rng.random() < 0.05 else 0)
                B.res.append((np.uint64(0xFFFFFFFFFFFFFFFF) if rng.random() < 0.9 else int(rng.integers(0, 1 << 30)),
                              sids[c], len(own), first, len(B.hdr) - first, caps[c], mfs[c], fl, 0))
                sids[c] += 2
            conn_first.append(len(B.res))
        hdr = np.array(B.hdr, dtype=HPE_HEADER_DTYPE) if B.hdr else np.zeros(0, HPE_HEADER_DTYPE)
        res = np.array(B.res, dtype=HPE_RESPONSE_DTYPE)
        data = np.frombuffer(b"".join(B.chunks), np.uint8).copy()
        out.append(dict(data=data, hdr=hdr, res=res, conn_first=np.array(conn_first, np.uint32), server_off=server_off,
                        server_len=len(SERVER), out_off=out_offsets(hdr, res, len(SERVER))))
    return out


def out_offsets(hdr, res, server_len):
    """[nres + 1] u64 region starts: hhuff_hpack_response_bound per response, 16-byte aligned"""
    nv = (hdr["name_len"].astype(np.int64) + hdr["value_len"]) if hdr.size else np.zeros(0, np.int64)
    csum = np.concatenate([[0], np.cumsum(nv)])
    first = res["hdr_first"].astype(np.int64)
    nh = res["nhdr"].astype(np.int64)
    nvb = csum[first + nh] - csum[first]
    sl = np.where(res["flags"] & RES_SERVER, server_len, 0)
    b = hpack_response_bound(nvb, nh, sl, res["max_frame_size"].astype(np.int64))
    b = (b + 15) // 16 * 16
    return np.concatenate([[0], np.cumsum(b)]).astype(np.uint64)


def build_batch(conns, server=SERVER):
    """An explicit batch: conns = [[response, ...] per connection], response = dict(status=, headers=[(name,
    value, flags)], content_length=None, flags=RES_*, header_table_size=4096, max_frame_size=16384,
    stream_id=1)"""
    B = _Batch()
    server_off = B.s(server)
    conn_first = [0]
    for rs in conns:
        for r in rs:
            first = len(B.hdr)
            for name, value, f in r.get("headers", []):
                B.header(name, value, f)
            cl = r.get("content_length")
            B.res.append((np.uint64(0xFFFFFFFFFFFFFFFF) if cl is None else cl, r.get("stream_id", 1), r.get("status", 200),
                          first, len(B.hdr) - first, r.get("header_table_size", 4096), r.get("max_frame_size", 16384),
                          r.get("flags", 0), 0))
        conn_first.append(len(B.res))
    hdr = np.array(B.hdr, dtype=HPE_HEADER_DTYPE) if B.hdr else np.zeros(0, HPE_HEADER_DTYPE)
    res = np.array(B.res, dtype=HPE_RESPONSE_DTYPE) if B.res else np.zeros(0, HPE_RESPONSE_DTYPE)
    data = np.frombuffer(b"".join(B.chunks), np.uint8).copy()
    return dict(data=data, hdr=hdr, res=res, conn_first=np.array(conn_first, np.uint32), server_off=server_off,
                server_len=len(server), out_off=out_offsets(hdr, res, len(server)))


def tile(b, k):
    """k copies of batch b's connections (independent connections with the same responses; the strings are
    shared): a large batch without generating every connection"""
    nres, nhdr = b["res"].size, b["hdr"].size
    res = np.tile(b["res"], k)
    hdr = np.tile(b["hdr"], k)
    res["hdr_first"] += np.repeat(np.arange(k, dtype=np.uint32) * nhdr, nres)
    cf = b["conn_first"].astype(np.int64)
    conn_first = np.concatenate([cf[:-1] + j * nres for j in range(k)] + [[k * nres]]).astype(np.uint32)
    return dict(data=b["data"], hdr=hdr, res=res, conn_first=conn_first, server_off=b["server_off"],
                server_len=b["server_len"], out_off=out_offsets(hdr, res, b["server_len"]))


def to_qpack(b, seed=0, dfid_frac=0.02, odd_status_frac=0.01):
    """The same responses as HTTP/3 responses (include/hhuff.h hhuff_qpack_response_t; trailers dropped --
    h2o's HTTP/3 server sends them through the same flatten), a few with a datagram flow id or a status outside
    the HTTP status range: -> dict data, hdr, res, server_off, server_len, out_off"""
    rng = np.random.default_rng(seed)
    keep = (b["res"]["flags"] & RES_TRAILERS) == 0
    src = b["res"][keep]
    res = np.zeros(src.size, QPE_RESPONSE_DTYPE)
    for k in ("content_length", "status", "hdr_first", "nhdr"):
        res[k] = src[k]
    res["flags"] = src["flags"] & RES_SERVER
    data = b["data"]
    extra = []
    dfid = rng.random(src.size) < dfid_frac
    for r in np.flatnonzero(dfid):
        v = b"%d" % int(rng.integers(0, 1 << 40))
        res["dfid_off"][r] = data.size + sum(len(e) for e in extra)
        res["dfid_len"][r] = len(v)
        extra.append(v)
    res["flags"][dfid] |= QRES_DATAGRAM
    odd = rng.random(src.size) < odd_status_frac
    res["status"][odd] = rng.choice([0, 7, 99, 599, 1000, 65535, 65536 + 200], int(odd.sum()))
    if extra:
        data = np.concatenate([data, np.frombuffer(b"".join(extra), np.uint8)])
    return dict(data=data, hdr=b["hdr"], res=res, server_off=b["server_off"], server_len=b["server_len"],
                out_off=qpack_out_offsets(b["hdr"], res, b["server_len"]))


def to_qpack_requests(b, seed=0, dfid_frac=0.05):
    """make_request_session's requests as HTTP/3 requests (h2o_qpack_flatten_request, lib/http3/qpack.c:1312-1350,
    as lib/common/http3client.c:792 calls it): HHUFF_QRES_REQUEST records with the same own fields, minus the
    HTTP/2 client's own "expect" (h2o_qpack_flatten_request has no send_own_expect: it stays as a header), and a
    datagram flow id on some (CONNECT-UDP, http3client.c:781-785) -> dict data, hdr, res, server_off, server_len,
    out_off"""
    rng = np.random.default_rng(seed)
    src, hdr, data = b["res"], b["hdr"], b["data"]
    res = np.zeros(src.size, QPE_RESPONSE_DTYPE)
    for k in ("content_length", "status", "hdr_first", "nhdr"):
        res[k] = src[k]
    last = src["hdr_first"].astype(np.int64) + src["status"].astype(np.int64) - 1
    has_own = src["status"] > 0
    nl = np.where(has_own, hdr["name_len"][np.maximum(last, 0)], 0)
    vo = hdr["name_off"][np.maximum(last, 0)].astype(np.int64)
    expect = has_own & (nl == 6) & np.array([data[o:o + 6].tobytes() == b"expect" for o in vo], bool)
    res["status"][expect] -= 1
    res["flags"] = QRES_REQUEST | (src["flags"] & RES_SERVER)  # server: ignored for requests
    extra = []
    dfid = rng.random(src.size) < dfid_frac
    for r in np.flatnonzero(dfid):
        v = b"%d" % int(rng.integers(0, 1 << 40))
        res["dfid_off"][r] = data.size + sum(len(e) for e in extra)
        res["dfid_len"][r] = len(v)
        extra.append(v)
    res["flags"][dfid] |= QRES_DATAGRAM
    if extra:
        data = np.concatenate([data, np.frombuffer(b"".join(extra), np.uint8)])
    return dict(data=data, hdr=hdr, res=res, server_off=b["server_off"], server_len=b["server_len"],
                out_off=qpack_out_offsets(hdr, res, b["server_len"]))


def qpack_out_offsets(hdr, res, server_len):
    nv = (hdr["name_len"].astype(np.int64) + hdr["value_len"]) if hdr.size else np.zeros(0, np.int64)
    csum = np.concatenate([[0], np.cumsum(nv)])
    first = res["hdr_first"].astype(np.int64)
    nh = res["nhdr"].astype(np.int64)
    sl = np.where(res["flags"] & RES_SERVER, server_len, 0)
    b = qpack_response_bound(csum[first + nh] - csum[first], nh, sl, res["dfid_len"].astype(np.int64))
    b = (b + 15) // 16 * 16
    return np.concatenate([[0], np.cumsum(b)]).astype(np.uint64)
