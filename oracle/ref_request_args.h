/*
 * ORACLE -- TEST INFRASTRUCTURE ONLY.  The reference harnesses' (ref_hpenc.c, ref_shim.c) reading of a request
 * record of include/hhuff.h back into the arguments of h2o_hpack_flatten_request (lib/http2/hpack.c:1044-1096)
 * and h2o_qpack_flatten_request (lib/http3/qpack.c:1312-1350).
 */
#ifndef REF_REQUEST_ARGS_H
#define REF_REQUEST_ARGS_H
#include <stdint.h>
#include <string.h>

#include "h2o/memory.h"
#include "h2o/url.h"

typedef struct {
    h2o_iovec_t method, protocol;
    h2o_url_t url;
    h2o_url_scheme_t custom;
    int expect;
} ref_req_t;

static inline int is_name(const uint8_t *in, const uint32_t *H, const char *lit)
{
    return h2o_memis((const char *)in + H[0], H[1], lit, strlen(lit));
}

/* h2o_hpack_flatten_request's arguments from a request's own fields hdr[hfirst .. + nown): :method, :scheme and
 * :authority and :path (scheme and path absent for an old-style CONNECT: method CONNECT without :protocol),
 * :protocol if any, expect: 100-continue if any -- in that order, token names without dont_compress.  0, or -1
 * when the fields are not that (a caller error).  expect_ok = 0 for HTTP/3 (h2o_qpack_flatten_request has no
 * send_own_expect). */
static inline int ref_req_args(const uint8_t *in, const uint32_t *hdr, uint32_t hfirst, uint32_t nown, int expect_ok,
                               ref_req_t *a)
{
    memset(a, 0, sizeof(*a));
    const uint32_t *H = hdr + 5 * (size_t)hfirst;
    int has_protocol = 0;
    for (uint32_t i = 0; i < nown; ++i) {
        if (H[5 * i + 4] != 2u)
            return -1;
        has_protocol |= is_name(in, H + 5 * i, ":protocol");
    }
    uint32_t i = 0;
    if (i == nown || !is_name(in, H, ":method"))
        return -1;
    a->method = h2o_iovec_init(in + H[2], H[3]);
    int old_style_connect = h2o_memis(a->method.base, a->method.len, H2O_STRLIT("CONNECT")) && !has_protocol;
    ++i;
    a->url.scheme = &H2O_URL_SCHEME_HTTPS;
    if (!old_style_connect) {
        const uint32_t *S = H + 5 * i;
        if (i == nown || !is_name(in, S, ":scheme"))
            return -1;
        h2o_iovec_t v = h2o_iovec_init(in + S[2], S[3]);
        if (h2o_memis(v.base, v.len, H2O_STRLIT("https"))) {
            a->url.scheme = &H2O_URL_SCHEME_HTTPS;
        } else if (h2o_memis(v.base, v.len, H2O_STRLIT("http"))) {
            a->url.scheme = &H2O_URL_SCHEME_HTTP;
        } else {
            a->custom.name = v;
            a->url.scheme = &a->custom;
        }
        ++i;
    }
    if (i == nown || !is_name(in, H + 5 * i, ":authority"))
        return -1;
    a->url.authority = h2o_iovec_init(in + H[5 * i + 2], H[5 * i + 3]);
    ++i;
    if (!old_style_connect) {
        if (i == nown || !is_name(in, H + 5 * i, ":path"))
            return -1;
        a->url.path = h2o_iovec_init(in + H[5 * i + 2], H[5 * i + 3]);
        ++i;
    }
    a->protocol = h2o_iovec_init(NULL, 0);
    if (i < nown && is_name(in, H + 5 * i, ":protocol")) {
        a->protocol = h2o_iovec_init(in + H[5 * i + 2], H[5 * i + 3]);
        if (a->protocol.base == NULL)
            a->protocol.base = (char *)in; /* present, even when empty */
        ++i;
    }
    if (expect_ok && i < nown && is_name(in, H + 5 * i, "expect")) {
        if (!h2o_memis((const char *)in + H[5 * i + 2], H[5 * i + 3], H2O_STRLIT("100-continue")))
            return -1;
        a->expect = 1;
        ++i;
    }
    return i == nown ? 0 : -1;
}

#endif
