/*
 * ORACLE -- TEST INFRASTRUCTURE ONLY.  Response-encoder harness around the REAL reference, compiled from
 * the sources where they lie (oracle/Makefile; nothing is copied):
 *   lib/http2/hpack.c   h2o_hpack_flatten_response :1137-1177, h2o_hpack_flatten_trailers :1179-1196
 *                       (do_encode_header :858-937 and the encoder's dynamic table under them)
 *   lib/http2/frame.c   h2o_http2_encode_frame_header (the HEADERS / CONTINUATION frame headers)
 *   lib/common/memory.c h2o_buffer_t, the output buffer flatten_* reserve into
 *   lib/common/token.c  h2o_lookup_token (token names are passed as the token's own h2o_iovec_t, as h2o's
 *                       response headers carry them), h2o__tokens, h2o_hpack_static_table
 * One h2o_hpack_header_table_t per connection, hpack_capacity 4096 as lib/http2/connection.c:1847 sets
 * conn->_output_header_table; a step flattens every connection's responses in order, as
 * lib/http2/stream.c:311-314 (final responses, server_name given) / :404-406 (informational, no server
 * name) and lib/http2/connection.c:1580-1582 (trailers) call them, into the caller's output slots -- the
 * contract of include/hhuff.h hhuff_hpack_flatten_responses.  Request records (flag 8) go through the real
 * h2o_hpack_flatten_request (:1044-1096) as lib/common/http2client.c:1140 calls it: their own fields (the first
 * `status` headers) are turned back into its arguments -- method, the url's scheme object (H2O_URL_SCHEME_HTTPS /
 * _HTTP for "https" / "http", so h2o's pointer comparison sees them), authority and path, protocol, and
 * send_own_expect for a trailing "expect: 100-continue".
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "h2o/hpack.h"
#include "h2o/http2_common.h"
#include "h2o/memory.h"
#include "h2o/token.h"
#include "h2o/url.h"
#include "ref_request_args.h"

#define REF_API __attribute__((visibility("default")))

typedef struct {
    uint32_t nconn;
    h2o_hpack_header_table_t *t;
    int *failed;
} ref_hpe_session_t;

static h2o_buffer_prototype_t hpe_proto = {{4096}, NULL};

REF_API void *ref_hpe_open(uint32_t nconn)
{
    ref_hpe_session_t *s = calloc(1, sizeof(*s));
    s->nconn = nconn;
    s->t = calloc(nconn ? nconn : 1, sizeof(*s->t));
    s->failed = calloc(nconn ? nconn : 1, sizeof(int));
    for (uint32_t c = 0; c < nconn; ++c)
        s->t[c].hpack_capacity = H2O_HTTP2_SETTINGS_DEFAULT.header_table_size; /* connection.c:1847 */
    return s;
}

REF_API void ref_hpe_close(void *h)
{
    ref_hpe_session_t *s = h;
    for (uint32_t c = 0; c < s->nconn; ++c)
        h2o_hpack_dispose_header_table(&s->t[c]);
    free(s->t);
    free(s->failed);
    free(s);
}

/* the HEADERS (+ CONTINUATION) frames' payload bytes */
static size_t frames_payload(const uint8_t *p, size_t size)
{
    size_t off = 0, sum = 0;
    while (off + 9 <= size) {
        size_t len = (size_t)p[off] << 16 | (size_t)p[off + 1] << 8 | p[off + 2];
        sum += len;
        off += 9 + len;
    }
    return sum;
}

/* Returns 0, or the number of headers flagged HHUFF_HDR_TOKEN whose name is not an h2o token (a caller
 * error: nothing is flattened then). */
REF_API int ref_hpe_step(void *h, const uint8_t *in, uint64_t in_size, const uint32_t *hdr, const uint32_t *res,
                         const uint32_t *conn_first, uint32_t server_off, uint32_t server_len, uint8_t *out,
                         const uint64_t *out_off, uint32_t *out_len, uint32_t *headers_size, int32_t *rstatus)
{
    ref_hpe_session_t *s = h;
    uint32_t nres = conn_first[s->nconn];
    int bad_tokens = 0;
    for (uint32_t r = 0; r < nres; ++r) {
        const uint32_t *R = res + 10 * (size_t)r;
        for (uint32_t i = 0; i < R[5]; ++i) {
            const uint32_t *H = hdr + 5 * (size_t)(R[4] + i);
            if ((H[4] & 2u) && h2o_lookup_token((const char *)in + H[0], H[1]) == NULL)
                ++bad_tokens;
        }
        /* a request's own fields must be flatten_request's arguments (a string past in_size is refused later) */
        int in_bounds = 1;
        for (uint32_t i = 0; i < R[5]; ++i) {
            const uint32_t *H = hdr + 5 * (size_t)(R[4] + i);
            in_bounds &= (uint64_t)H[0] + H[1] <= in_size && (uint64_t)H[2] + H[3] <= in_size;
        }
        ref_req_t a;
        if ((R[8] & 8u) && !(R[8] & 4u) && in_bounds && (R[3] > R[5] || ref_req_args(in, hdr, R[4], R[3], 1, &a) != 0))
            ++bad_tokens;
    }
    if (bad_tokens)
        return bad_tokens;
    h2o_iovec_t server_name = h2o_iovec_init(in + server_off, server_len);
    for (uint32_t c = 0; c < s->nconn; ++c) {
        h2o_hpack_header_table_t *t = &s->t[c];
        for (uint32_t r = conn_first[c]; r < conn_first[c + 1]; ++r) {
            const uint32_t *R = res + 10 * (size_t)r;
            uint64_t content_length;
            memcpy(&content_length, R, 8);
            uint32_t sid = R[2], status = R[3], hfirst = R[4], nh = R[5], cap = R[6], mfs = R[7], fl = R[8];
            int trailers = (fl & 4u) != 0, request = (fl & 8u) && !trailers;
            out_len[r] = 0;
            headers_size[r] = 0;
            if (s->failed[c]) {
                rstatus[r] = -301;
                continue;
            }
            int bad = (!trailers && !request && (status < 100 || status > 999)) || mfs < 16384 || mfs > 0xffffff ||
                      ((fl & 2u) && !trailers && !request && (uint64_t)server_off + server_len > in_size);
            h2o_iovec_t *names = calloc(nh ? nh : 1, sizeof(h2o_iovec_t));
            h2o_header_t *headers = calloc(nh ? nh : 1, sizeof(h2o_header_t));
            for (uint32_t i = 0; i < nh; ++i) {
                const uint32_t *H = hdr + 5 * (size_t)(hfirst + i);
                if ((uint64_t)H[0] + H[1] > in_size || (uint64_t)H[2] + H[3] > in_size) {
                    bad = 1;
                    break;
                }
                const h2o_token_t *tok = (H[4] & 2u) ? h2o_lookup_token((const char *)in + H[0], H[1]) : NULL;
                names[i] = h2o_iovec_init(in + H[0], H[1]);
                headers[i].name = tok != NULL ? (h2o_iovec_t *)&tok->buf : &names[i];
                headers[i].value = h2o_iovec_init(in + H[2], H[3]);
                headers[i].flags.dont_compress = (H[4] & 1u) != 0;
            }
            if (bad) {
                rstatus[r] = -303;
                s->failed[c] = 1;
                free(names);
                free(headers);
                continue;
            }
            h2o_buffer_t *buf;
            h2o_buffer_init(&buf, &hpe_proto);
            size_t hs = 0;
            if (trailers) {
                h2o_hpack_flatten_trailers(&buf, t, cap, sid, mfs, headers, nh);
                hs = frames_payload((const uint8_t *)buf->bytes, buf->size);
            } else if (request) {
                ref_req_t a;
                ref_req_args(in, hdr, hfirst, status, 1, &a);
                h2o_hpack_flatten_request(&buf, t, cap, sid, mfs, a.method, &a.url, a.protocol, headers + status, nh - status,
                                          fl & 1u, a.expect);
                hs = frames_payload((const uint8_t *)buf->bytes, buf->size);
            } else {
                hs = h2o_hpack_flatten_response(&buf, t, cap, sid, mfs, (int)status, headers, nh,
                                                (fl & 2u) ? &server_name : NULL,
                                                content_length == UINT64_MAX ? SIZE_MAX : (size_t)content_length, fl & 1u);
            }
            if (buf->size > out_off[r + 1] - out_off[r]) {
                rstatus[r] = -300;
                s->failed[c] = 1;
            } else {
                memcpy(out + out_off[r], buf->bytes, buf->size);
                out_len[r] = (uint32_t)buf->size;
                headers_size[r] = (uint32_t)hs;
                rstatus[r] = 0;
            }
            h2o_buffer_dispose(&buf);
            free(names);
            free(headers);
        }
    }
    return 0;
}

/* The token facts the restatement and the GPU path rely on (lib/common/token_table.h): every token's
 * http2_static_table_name_index is the first static-table entry with its name (0 when none has it), and
 * dont_compress is set exactly for cookie and set-cookie.  Returns the number of tokens that disagree. */
REF_API int ref_hpe_token_check(void)
{
    int bad = 0;
    for (size_t i = 0; i < h2o__num_tokens; ++i) {
        const h2o_token_t *tok = &h2o__tokens[i];
        int first = 0;
        for (int k = 0; k < 61; ++k) {
            const h2o_iovec_t *n = &h2o_hpack_static_table[k].name->buf;
            if (n->len == tok->buf.len && memcmp(n->base, tok->buf.base, n->len) == 0) {
                first = k + 1;
                break;
            }
        }
        int dc = h2o_memis(tok->buf.base, tok->buf.len, H2O_STRLIT("cookie")) ||
                 h2o_memis(tok->buf.base, tok->buf.len, H2O_STRLIT("set-cookie"));
        bad += tok->flags.http2_static_table_name_index != first || tok->flags.dont_compress != dc;
    }
    return bad;
}
