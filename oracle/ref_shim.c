/*
 * ORACLE -- TEST INFRASTRUCTURE ONLY.  Binds the REAL reference codec, compiled from the sources
 * where they lie under /root/reference (nothing is copied), into oracle/_ref/libh2oref.so:
 *   lib/http2/hpack.c   h2o_hpack_decode_huffman :117, h2o_hpack_encode_huffman :774,
 *                       h2o_hpack_encode_string :816, h2o_hpack_decode_int :52
 *   lib/http3/qpack.c   static flatten_string :1042 (reached by including the .c, as the reference's
 *                       own unit test does at t/00unit/lib/http3/qpack.c:24)
 *   lib/common/token.c  h2o_lookup_token (QPACK raw names, qpack.c:585)
 * ref_decode_literal below is harness glue: it strings the reference's own public pieces together in
 * the order decode_string (hpack.c:223-261) and decode_header_{name,value}_literal (qpack.c:559-629)
 * call them, minus the memory pool those static functions allocate from.
 * Used in the build container to produce tests/golden/* and to pin the restatement; the built
 * oracle/_ref/libh2oref.so is git-ignored but travels to the GPU box with the tree (like libhhuff.so),
 * where bench.py times it as the CPU baseline (cpu_baseline.kind "reference") and the drop-in tests
 * run h2o's own callers through it.  Built only where /root/reference exists.
 */
#include "lib/http3/qpack.c"
#include "ref_request_args.h"

#define REF_API __attribute__((visibility("default")))

static size_t ref_dec(char *dst, unsigned *soft, const uint8_t *src, size_t len, int is_name)
{
    const char *err_desc = NULL;
    return h2o_hpack_decode_huffman(dst, soft, src, len, is_name, &err_desc);
}

static size_t ref_flat(uint8_t *dst, const uint8_t *s, size_t len, unsigned prefix_bits, int raw)
{
    h2o_byte_vector_t v = {dst, 0, len + 1 + H2O_HPACK_ENCODE_INT_MAX_LENGTH};
    flatten_string(&v, (const char *)s, len, prefix_bits, raw);
    return v.size;
}

REF_API size_t ref_decode_huffman(char *dst, unsigned *soft, const uint8_t *src, size_t len, int is_name)
{
    return ref_dec(dst, soft, src, len, is_name);
}
REF_API size_t ref_encode_huffman(uint8_t *dst, const uint8_t *src, size_t len)
{
    return h2o_hpack_encode_huffman(dst, src, len);
}
REF_API size_t ref_encode_string(uint8_t *dst, const uint8_t *s, size_t len)
{
    return h2o_hpack_encode_string(dst, (const char *)s, len);
}
REF_API size_t ref_flatten_string(uint8_t *dst, const uint8_t *s, size_t len, unsigned prefix_bits, int raw)
{
    return ref_flat(dst, s, len, prefix_bits, raw);
}
REF_API int64_t ref_decode_int(const uint8_t **src, const uint8_t *end, unsigned prefix_bits)
{
    return h2o_hpack_decode_int(src, end, prefix_bits);
}
REF_API uint8_t *ref_encode_int(uint8_t *dst, int64_t v, unsigned prefix_bits)
{
    return h2o_hpack_encode_int(dst, v, prefix_bits);
}

static int ref_lit(const uint8_t *lit, const uint8_t *end, unsigned prefix_bits, int is_name, int qpack, uint8_t *out,
                   uint64_t lit_pos, uint32_t *hdr, uint32_t *consumed, uint32_t *out_len, unsigned *soft)
{
    const char *err_desc = NULL;
    const uint8_t *p = lit;
    *hdr = 0, *consumed = 0, *out_len = 0xFFFFFFFFu;
    if (p >= end)
        return 1; /* INCOMPLETE */
    int huff = (*p >> prefix_bits) & 1;
    int64_t len = h2o_hpack_decode_int(&p, end, prefix_bits);
    if (len == H2O_HTTP2_ERROR_INCOMPLETE)
        return 1;
    if (len < 0)
        return 2; /* BAD_INT */
    if (len > end - p)
        return 3; /* TRUNCATED */
    if (len > (int64_t)((1u << 29) - 1))
        return 6; /* TOO_LONG: the HIP path's per-string limit */
    *hdr = (uint32_t)(p - lit);
    char *dst = (char *)out + ((lit_pos + *hdr) * 8u) / 5u;
    if (huff) {
        size_t r = h2o_hpack_decode_huffman(dst, soft, p, (size_t)len, is_name, &err_desc);
        if (r == SIZE_MAX)
            return 4; /* HUFFMAN */
        *out_len = (uint32_t)r;
    } else {
        if (is_name) {
            int skip = qpack ? h2o_lookup_token((const char *)p, (size_t)len) != NULL : (len != 0 && *p == ':');
            if (!skip && !h2o_hpack_validate_header_name(soft, (const char *)p, (size_t)len, &err_desc))
                return 5; /* UPPERCASE */
        } else {
            h2o_hpack_validate_header_value(soft, (const char *)p, (size_t)len);
        }
        memcpy(dst, p, (size_t)len);
        *out_len = (uint32_t)len;
    }
    *consumed = *hdr + (uint32_t)len;
    return 0;
}

#define ORC_CODEC_LITERAL ref_lit
#define ORC_CODEC_DECODE ref_dec
#define ORC_CODEC_ENCODE h2o_hpack_encode_huffman
#define ORC_CODEC_FLATTEN ref_flat
#define ORC_BATCH_PREFIX ref
#define ORC_BATCH_API REF_API
#include "batch_driver.h"

/* ---- QPACK decoder (QPACK half) around the reference's own functions ----
 * One h2o_qpack_decoder_t per connection (h2o_qpack_create_decoder :240).  A step feeds each connection's
 * encoder-stream bytes to h2o_qpack_decoder_handle_input (:420-485), then decodes each of its field
 * sections the way h2o_qpack_parse_request does (:830-858): parse_decode_context, check_decode_context_blocked,
 * then decode_header (:652-752) field after field -- the loop h2o_hpack_parse_request runs over the section
 * (lib/http2/hpack.c:513-527) without its pseudo-header bookkeeping -- copying every name and value into the
 * caller's arena (the output contract of include/hhuff.h hhuff_qpack_decode). */
#define REF_QPK_ARENA (-300)
#define REF_QPK_SKIPPED (-301)
#define REF_QPK_BLOCKED (-302)

typedef struct {
    uint32_t nconn;
    h2o_qpack_decoder_t **d;
    int *failed;
} ref_qpk_session_t;

REF_API void *ref_qpack_open(uint32_t nconn, uint32_t header_table_size, uint64_t max_blocked)
{
    ref_qpk_session_t *s = calloc(1, sizeof(*s));
    s->nconn = nconn;
    s->d = calloc(nconn ? nconn : 1, sizeof(*s->d));
    s->failed = calloc(nconn ? nconn : 1, sizeof(int));
    for (uint32_t c = 0; c < nconn; ++c)
        s->d[c] = h2o_qpack_create_decoder(header_table_size, max_blocked);
    return s;
}

REF_API void ref_qpack_close(void *h)
{
    ref_qpk_session_t *s = h;
    for (uint32_t c = 0; c < s->nconn; ++c)
        h2o_qpack_destroy_decoder(s->d[c]);
    free(s->d);
    free(s->failed);
    free(s);
}

REF_API int ref_qpack_step(void *h, const uint8_t *in, const uint32_t *enc_off, const uint32_t *enc_len,
                           const uint32_t *sec_off, const uint32_t *conn_first, const uint32_t *num_blocked, uint8_t *arena,
                           const uint64_t *arena_off, uint32_t *name_off, uint32_t *name_len, uint32_t *value_off,
                           uint32_t *value_len, uint8_t *fflags, uint32_t *nfields, int32_t *sstatus,
                           uint64_t *req_insert_count, int32_t *enc_status, uint32_t *enc_consumed, uint64_t *insert_count)
{
    ref_qpk_session_t *s = h;
    for (uint32_t c = 0; c < s->nconn; ++c) {
        h2o_qpack_decoder_t *q = s->d[c];
        enc_status[c] = 0;
        enc_consumed[c] = 0;
        insert_count[c] = 0;
        if (s->failed[c]) {
            enc_status[c] = REF_QPK_SKIPPED;
        } else if (enc_len[c]) {
            const uint8_t *src = in + enc_off[c], *end = src + enc_len[c];
            const char *err_desc = NULL;
            int r = h2o_qpack_decoder_handle_input(q, &insert_count[c], &src, end, &err_desc);
            enc_consumed[c] = (uint32_t)(src - (in + enc_off[c]));
            enc_status[c] = r;
            s->failed[c] = r != 0;
        }
        uint64_t nb = num_blocked ? num_blocked[c] : 0; /* +1 per parked stream (lib/http3/server.c:1553) */
        for (uint32_t k = conn_first[c]; k < conn_first[c + 1]; ++k) {
            nfields[k] = 0;
            req_insert_count[k] = 0;
            if (s->failed[c]) {
                sstatus[k] = REF_QPK_SKIPPED;
                continue;
            }
            const uint8_t *src = in + sec_off[k], *end = in + sec_off[k + 1];
            struct st_h2o_qpack_decode_header_ctx_t ctx;
            h2o_qpack_section_stats_t stats = {0};
            uint64_t blocked_ref = 0;
            int st = parse_decode_context(q, &ctx, &src, end);
            if (st == 0) {
                req_insert_count[k] = (uint64_t)ctx.req_insert_count;
                st = check_decode_context_blocked(q, &ctx, nb, &blocked_ref);
                if (st == 0 && blocked_ref != 0) {
                    st = REF_QPK_BLOCKED;
                    ++nb;
                }
            }
            ctx.stats = &stats;
            h2o_mem_pool_t pool;
            h2o_mem_init_pool(&pool);
            uint64_t cur = arena_off[k], aend = arena_off[k + 1] < (1ull << 32) ? arena_off[k + 1] : (1ull << 32);
            uint32_t nf = 0, slot = sec_off[k];
            while (st == 0 && src != end) {
                h2o_iovec_t *name, value;
                const char *err_desc = NULL;
                int ret = decode_header(&pool, &ctx, &name, &value, &src, end, &err_desc);
                if (ret != 0 && ret != H2O_HTTP2_ERROR_INVALID_HEADER_CHAR) {
                    st = ret;
                    break;
                }
                if (cur + name->len + value.len > aend) {
                    st = REF_QPK_ARENA;
                    break;
                }
                memcpy(arena + cur, name->base, name->len);
                name_off[slot + nf] = (uint32_t)cur;
                name_len[slot + nf] = (uint32_t)name->len;
                cur += name->len;
                memcpy(arena + cur, value.base, value.len);
                value_off[slot + nf] = (uint32_t)cur;
                value_len[slot + nf] = (uint32_t)value.len;
                cur += value.len;
                fflags[slot + nf] = ret == 0 ? 0 : (err_desc == h2o_hpack_soft_err_found_invalid_char_in_header_name ? 1 : 2);
                ++nf;
            }
            h2o_mem_clear_pool(&pool);
            nfields[k] = nf;
            sstatus[k] = st;
        }
    }
    return 0;
}

/* ---- h2o_qpack_parse_request (qpack.c:830-858) as h2o's HTTP/3 server calls it ----
 * lib/http3/server.c:1540-1545: no cache digests, a datagram-flow-id out-parameter, the connection's
 * num_qpack_blocked.  Per section the request record (include/hhuff.h hhuff_qpack_request_t, 18 u32
 * words) is produced by h2o_qpack_parse_request's own steps -- parse_decode_context,
 * check_decode_context_blocked, h2o_hpack_parse_request over decode_header (through a wrapper that copies
 * each field to the arena and, from the out-parameters' changes between calls, learns which field each
 * one took and which went to the header list), normalize_error_code, send_header_ack -- and every section
 * is ALSO run through the real h2o_qpack_parse_request on the same decoder, whose return value, header
 * acknowledgment, content length, pseudo-header map, header count, err_desc, scheme and out-parameter
 * bytes must agree (the count of disagreeing sections is the return value). */
#define Q3_OUTS 7 /* method, (scheme), authority, path, protocol, expect, datagram_flow_id */
typedef struct {
    struct st_h2o_qpack_decode_header_ctx_t *dctx;
    uint8_t *arena;
    uint64_t cur, aend;
    uint32_t *name_off, *name_len, *value_off, *value_len, slot, nf;
    uint8_t *fflags;
    h2o_iovec_t *out[Q3_OUTS];
    const h2o_url_scheme_t **scheme;
    h2o_headers_t *headers;
    h2o_iovec_t snap[Q3_OUTS];
    const h2o_url_scheme_t *scheme_snap;
    size_t hsize_snap;
    int32_t taken[Q3_OUTS];
    int hard, arena_full;
} q3_ctx_t;

static void q3_settle(q3_ctx_t *x)
{
    if (x->nf == 0)
        return;
    int32_t k = (int32_t)x->nf - 1;
    if (x->headers->size > x->hsize_snap)
        x->fflags[x->slot + k] |= 4;
    for (int i = 0; i < Q3_OUTS; ++i) {
        if (i == 1) {
            if (*x->scheme != x->scheme_snap)
                x->taken[1] = k;
            continue;
        }
        if (x->out[i]->base != x->snap[i].base || x->out[i]->len != x->snap[i].len)
            x->taken[i] = k;
    }
}

static void q3_snapshot(q3_ctx_t *x)
{
    for (int i = 0; i < Q3_OUTS; ++i)
        if (i != 1)
            x->snap[i] = *x->out[i];
    x->scheme_snap = *x->scheme;
    x->hsize_snap = x->headers->size;
}

static int q3_decode_cb(h2o_mem_pool_t *pool, void *ctx, h2o_iovec_t **name, h2o_iovec_t *value, const uint8_t **src,
                        const uint8_t *src_end, const char **err_desc)
{
    q3_ctx_t *x = ctx;
    q3_settle(x);
    q3_snapshot(x);
    int ret = decode_header(pool, x->dctx, name, value, src, src_end, err_desc);
    if (ret != 0 && ret != H2O_HTTP2_ERROR_INVALID_HEADER_CHAR) {
        x->hard = 1;
        return ret;
    }
    if (x->cur + (*name)->len + value->len > x->aend) {
        x->arena_full = 1;
        *err_desc = NULL;
        return REF_QPK_ARENA;
    }
    uint32_t f = x->slot + x->nf;
    memcpy(x->arena + x->cur, (*name)->base, (*name)->len);
    x->name_off[f] = (uint32_t)x->cur;
    x->name_len[f] = (uint32_t)(*name)->len;
    x->cur += (*name)->len;
    memcpy(x->arena + x->cur, value->base, value->len);
    x->value_off[f] = (uint32_t)x->cur;
    x->value_len[f] = (uint32_t)value->len;
    x->cur += value->len;
    x->fflags[f] = ret == 0 ? 0 : (*err_desc == h2o_hpack_soft_err_found_invalid_char_in_header_name ? 1 : 2);
    ++x->nf;
    return ret;
}

static uint32_t q3_err_code(const char *e)
{
    if (e == NULL)
        return 0;
    if (e == h2o_hpack_soft_err_found_invalid_char_in_header_name)
        return 1;
    if (e == h2o_hpack_soft_err_found_invalid_char_in_header_value)
        return 2;
    if (e == h2o_hpack_err_headers_too_long)
        return 3;
    if (e == h2o_hpack_err_invalid_pseudo_header)
        return 4;
    if (e == h2o_hpack_err_invalid_content_length_header)
        return 5;
    if (e == h2o_hpack_err_unexpected_connection_specific_header)
        return 6;
    if (e == h2o_hpack_err_found_upper_case_in_header_name)
        return 7;
    if (e == h2o_hpack_err_missing_mandatory_pseudo_header)
        return 9;
    return 99;
}

static int q3_iov_eq(h2o_iovec_t a, h2o_iovec_t b)
{
    return a.len == b.len && (a.len == 0 || memcmp(a.base, b.base, a.len) == 0);
}

REF_API int ref_qpack_step_req(void *h, const uint8_t *in, const uint32_t *enc_off, const uint32_t *enc_len,
                               const uint32_t *sec_off, const uint32_t *conn_first, const uint32_t *num_blocked,
                               uint8_t *arena, const uint64_t *arena_off, uint32_t *name_off, uint32_t *name_len,
                               uint32_t *value_off, uint32_t *value_len, uint8_t *fflags, uint32_t *nfields,
                               int32_t *sstatus, uint64_t *req_insert_count, int32_t *enc_status, uint32_t *enc_consumed,
                               uint64_t *insert_count, const uint64_t *stream_id, uint32_t *req)
{
    ref_qpk_session_t *s = h;
    int mismatches = 0;
    for (uint32_t c = 0; c < s->nconn; ++c) {
        h2o_qpack_decoder_t *q = s->d[c];
        enc_status[c] = 0;
        enc_consumed[c] = 0;
        insert_count[c] = 0;
        if (s->failed[c]) {
            enc_status[c] = REF_QPK_SKIPPED;
        } else if (enc_len[c]) {
            const uint8_t *src = in + enc_off[c], *end = src + enc_len[c];
            const char *err_desc = NULL;
            int r = h2o_qpack_decoder_handle_input(q, &insert_count[c], &src, end, &err_desc);
            enc_consumed[c] = (uint32_t)(src - (in + enc_off[c]));
            enc_status[c] = r;
            s->failed[c] = r != 0;
        }
        uint64_t nb = num_blocked ? num_blocked[c] : 0; /* +1 per parked stream (lib/http3/server.c:1553) */
        for (uint32_t k = conn_first[c]; k < conn_first[c + 1]; ++k) {
            uint32_t *w = req + 18 * (size_t)k;
            nfields[k] = 0;
            req_insert_count[k] = 0;
            h2o_iovec_t method = {NULL, 0}, authority = {NULL, 0}, path = {NULL, 0}, protocol = {NULL, 0}, expect = {NULL, 0},
                        dfid = {NULL, 0};
            const h2o_url_scheme_t *scheme = NULL;
            h2o_headers_t headers = {NULL, 0, 0};
            int exists_map = 0;
            size_t content_length = SIZE_MAX, outbufsize = 0;
            uint8_t outbuf[16] = {0};
            const char *err_desc = NULL;
            q3_ctx_t x;
            memset(&x, 0, sizeof(x));
            for (int i = 0; i < Q3_OUTS; ++i)
                x.taken[i] = -1;
            int st;
            h2o_mem_pool_t pool;
            h2o_mem_init_pool(&pool);
            const uint8_t *src0 = in + sec_off[k], *end = in + sec_off[k + 1];
            if (s->failed[c]) {
                st = REF_QPK_SKIPPED;
            } else {
                /* h2o_qpack_parse_request's own steps */
                const uint8_t *src = src0;
                struct st_h2o_qpack_decode_header_ctx_t ctx;
                h2o_qpack_section_stats_t stats = {0};
                uint64_t blocked_ref = 0;
                st = parse_decode_context(q, &ctx, &src, end);
                if (st == 0) {
                    req_insert_count[k] = (uint64_t)ctx.req_insert_count;
                    st = check_decode_context_blocked(q, &ctx, nb, &blocked_ref);
                }
                int blocked = st == 0 && blocked_ref != 0;
                if (st == 0 && !blocked) {
                    ctx.stats = &stats;
                    x.dctx = &ctx, x.arena = arena, x.cur = arena_off[k];
                    x.aend = arena_off[k + 1] < (1ull << 32) ? arena_off[k + 1] : (1ull << 32);
                    x.name_off = name_off, x.name_len = name_len, x.value_off = value_off, x.value_len = value_len;
                    x.fflags = fflags, x.slot = sec_off[k];
                    x.out[0] = &method, x.out[1] = &method, x.out[2] = &authority, x.out[3] = &path;
                    x.out[4] = &protocol, x.out[5] = &expect, x.out[6] = &dfid;
                    x.scheme = &scheme, x.headers = &headers;
                    st = h2o_hpack_parse_request(&pool, q3_decode_cb, &x, &method, &scheme, &authority, &path, &protocol,
                                                 &headers, &exists_map, &content_length, &expect, NULL, &dfid, src,
                                                 end - src, &err_desc);
                    q3_settle(&x);
                    if (x.arena_full)
                        st = REF_QPK_ARENA;
                    else if (st != 0 && st != H2O_HTTP2_ERROR_INVALID_HEADER_CHAR)
                        st = normalize_error_code(st);
                    else
                        outbufsize = send_header_ack(q, &ctx, outbuf, (int64_t)stream_id[k]);
                }
                /* the real function, on the same decoder and the same blocked count */
                h2o_iovec_t m2 = {NULL, 0}, a2 = {NULL, 0}, p2 = {NULL, 0}, pr2 = {NULL, 0}, e2 = {NULL, 0}, d2 = {NULL, 0};
                const h2o_url_scheme_t *sc2 = NULL;
                h2o_headers_t hd2 = {NULL, 0, 0};
                int map2 = 0;
                size_t cl2 = SIZE_MAX, obs2 = 0;
                uint8_t ob2[16] = {0};
                uint64_t bref2 = 0;
                h2o_qpack_section_stats_t st2 = {0};
                const char *ed2 = NULL;
                h2o_mem_pool_t pool2;
                h2o_mem_init_pool(&pool2);
                int ret2 = h2o_qpack_parse_request(&pool2, q, (int64_t)stream_id[k], &m2, &sc2, &a2, &p2, &pr2, &hd2, &map2,
                                                   &cl2, &e2, NULL, &d2, nb, &bref2, &st2, ob2, &obs2, src0, end - src0, &ed2);
                if (!x.arena_full) {
                    int ok = (blocked ? (ret2 == 0 && bref2 != 0) : (ret2 == st && bref2 == 0)) && obs2 == outbufsize &&
                             memcmp(ob2, outbuf, 16) == 0 && cl2 == content_length && map2 == exists_map &&
                             hd2.size == headers.size && ed2 == err_desc && sc2 == scheme && q3_iov_eq(m2, method) &&
                             q3_iov_eq(a2, authority) && q3_iov_eq(p2, path) && q3_iov_eq(pr2, protocol) &&
                             q3_iov_eq(e2, expect) && q3_iov_eq(d2, dfid);
                    mismatches += !ok;
                }
                h2o_mem_clear_pool(&pool2);
                if (blocked) {
                    st = REF_QPK_BLOCKED;
                    ++nb;
                }
            }
            h2o_mem_clear_pool(&pool);
            nfields[k] = x.nf;
            sstatus[k] = st;
            uint64_t cl = content_length;
            memcpy(w, &cl, 8);
            memcpy(w + 2, x.taken, 24);
            w[8] = (uint32_t)exists_map;
            w[9] = (uint32_t)headers.size;
            w[10] = x.hard ? 8u /* HHUFF_HERR_DECODE */ : q3_err_code(err_desc);
            w[11] = scheme == NULL ? 0 : scheme == &H2O_URL_SCHEME_HTTP ? 1 : scheme == &H2O_URL_SCHEME_HTTPS ? 2 : 3;
            w[12] = (uint32_t)x.taken[6];
            w[13] = (uint32_t)outbufsize;
            memcpy(w + 14, outbuf, 16);
        }
    }
    return mismatches;
}

/* ---- h2o_qpack_parse_response (qpack.c:860-882) as h2o's HTTP/3 client calls it ----
 * lib/common/http3client.c:542-544: a status and a datagram-flow-id out-parameter.  Per section the record
 * (include/hhuff.h hhuff_qpack_response_head_t, 10 u32 words) is produced by h2o_qpack_parse_response's own
 * steps through the copying decode_cb wrapper (it learns which fields went to the header list and which one
 * took the datagram flow id), and every section is ALSO run through the real h2o_qpack_parse_response on the
 * same decoder (with a blocked_ref: the sessions' decoders may permit blocked sections, where the client's
 * permits none); return value, status, header count, err_desc, datagram flow id and acknowledgment must agree
 * (the count of disagreeing sections is the return value). */
REF_API int ref_qpack_step_resp(void *h, const uint8_t *in, const uint32_t *enc_off, const uint32_t *enc_len,
                                const uint32_t *sec_off, const uint32_t *conn_first, const uint32_t *num_blocked,
                                uint8_t *arena, const uint64_t *arena_off, uint32_t *name_off, uint32_t *name_len,
                                uint32_t *value_off, uint32_t *value_len, uint8_t *fflags, uint32_t *nfields,
                                int32_t *sstatus, uint64_t *req_insert_count, int32_t *enc_status, uint32_t *enc_consumed,
                                uint64_t *insert_count, const uint64_t *stream_id, uint32_t *res)
{
    ref_qpk_session_t *s = h;
    int mismatches = 0;
    for (uint32_t c = 0; c < s->nconn; ++c) {
        h2o_qpack_decoder_t *q = s->d[c];
        enc_status[c] = 0;
        enc_consumed[c] = 0;
        insert_count[c] = 0;
        if (s->failed[c]) {
            enc_status[c] = REF_QPK_SKIPPED;
        } else if (enc_len[c]) {
            const uint8_t *src = in + enc_off[c], *end = src + enc_len[c];
            const char *err_desc = NULL;
            int r = h2o_qpack_decoder_handle_input(q, &insert_count[c], &src, end, &err_desc);
            enc_consumed[c] = (uint32_t)(src - (in + enc_off[c]));
            enc_status[c] = r;
            s->failed[c] = r != 0;
        }
        uint64_t nb = num_blocked ? num_blocked[c] : 0;
        for (uint32_t k = conn_first[c]; k < conn_first[c + 1]; ++k) {
            uint32_t *w = res + 10 * (size_t)k;
            nfields[k] = 0;
            req_insert_count[k] = 0;
            int status = 0;
            h2o_iovec_t unused = {NULL, 0}, dfid = {NULL, 0};
            h2o_headers_t headers = {NULL, 0, 0};
            size_t outbufsize = 0;
            uint8_t outbuf[16] = {0};
            const char *err_desc = NULL;
            q3_ctx_t x;
            memset(&x, 0, sizeof(x));
            for (int i = 0; i < Q3_OUTS; ++i)
                x.taken[i] = -1, x.out[i] = &unused;
            x.out[6] = &dfid;
            x.scheme = (const h2o_url_scheme_t **)&x.scheme_snap; /* unchanging: q3_settle sees no scheme */
            int st;
            h2o_mem_pool_t pool;
            h2o_mem_init_pool(&pool);
            const uint8_t *src0 = in + sec_off[k], *end = in + sec_off[k + 1];
            if (s->failed[c]) {
                st = REF_QPK_SKIPPED;
            } else {
                const uint8_t *src = src0;
                struct st_h2o_qpack_decode_header_ctx_t ctx;
                h2o_qpack_section_stats_t stats = {0};
                uint64_t blocked_ref = 0;
                st = parse_decode_context(q, &ctx, &src, end);
                if (st == 0) {
                    req_insert_count[k] = (uint64_t)ctx.req_insert_count;
                    st = check_decode_context_blocked(q, &ctx, nb, &blocked_ref);
                }
                int blocked = st == 0 && blocked_ref != 0;
                if (st == 0 && !blocked) {
                    ctx.stats = &stats;
                    x.dctx = &ctx, x.arena = arena, x.cur = arena_off[k];
                    x.aend = arena_off[k + 1] < (1ull << 32) ? arena_off[k + 1] : (1ull << 32);
                    x.name_off = name_off, x.name_len = name_len, x.value_off = value_off, x.value_len = value_len;
                    x.fflags = fflags, x.slot = sec_off[k];
                    x.headers = &headers;
                    st = h2o_hpack_parse_response(&pool, q3_decode_cb, &x, &status, &headers, &dfid, src, end - src,
                                                  &err_desc);
                    q3_settle(&x);
                    if (x.arena_full)
                        st = REF_QPK_ARENA;
                    else if (st != 0)
                        st = normalize_error_code(st);
                    else
                        outbufsize = send_header_ack(q, &ctx, outbuf, (int64_t)stream_id[k]);
                }
                /* the real function, on the same decoder and the same blocked count */
                int status2 = 0;
                h2o_iovec_t d2 = {NULL, 0};
                h2o_headers_t hd2 = {NULL, 0, 0};
                size_t obs2 = 0;
                uint8_t ob2[16] = {0};
                uint64_t bref2 = 0;
                h2o_qpack_section_stats_t st2 = {0};
                const char *ed2 = NULL;
                h2o_mem_pool_t pool2;
                h2o_mem_init_pool(&pool2);
                int ret2 = h2o_qpack_parse_response(&pool2, q, (int64_t)stream_id[k], &status2, &hd2, &d2, nb, &bref2, &st2,
                                                    ob2, &obs2, src0, end - src0, &ed2);
                if (!x.arena_full) {
                    int ok = (blocked ? (ret2 == 0 && bref2 != 0) : (ret2 == st && bref2 == 0)) && obs2 == outbufsize &&
                             memcmp(ob2, outbuf, 16) == 0 && status2 == status && hd2.size == headers.size &&
                             ed2 == err_desc && q3_iov_eq(d2, dfid);
                    mismatches += !ok;
                }
                h2o_mem_clear_pool(&pool2);
                if (blocked) {
                    st = REF_QPK_BLOCKED;
                    ++nb;
                }
            }
            h2o_mem_clear_pool(&pool);
            nfields[k] = x.nf;
            sstatus[k] = st;
            w[0] = (uint32_t)status;
            w[1] = (uint32_t)headers.size;
            w[2] = x.hard ? 8u /* HHUFF_HERR_DECODE */ : q3_err_code(err_desc);
            w[3] = (uint32_t)x.taken[6];
            w[4] = (uint32_t)outbufsize;
            w[5] = 0;
            memcpy(w + 6, outbuf, 16);
        }
    }
    return mismatches;
}

/* ---- h2o_qpack_flatten_response (qpack.c:1352-1399) as h2o's HTTP/3 server calls it ----
 * lib/http3/server.c:1680-1683: the connection's encoder, no encoder-stream buffer (so nothing is ever inserted
 * into the encoder's table), the globalconf server name, the response's content length and datagram flow id.
 * One response after another into the caller's output slots: the include/hhuff.h hhuff_qpack_flatten_responses
 * contract (res = hhuff_qpack_response_t, 8 u32 words; hdr = hhuff_hpack_header_t, 5 words). */
/* Request records (flag 16) go through the real h2o_qpack_flatten_request (:1312-1350) as lib/common/http3client.c:792
 * calls it, their own fields turned back into its arguments (ref_request_args.h). */
REF_API int ref_qpe_step(const uint8_t *in, uint64_t in_size, const uint32_t *hdr, const uint32_t *res, uint32_t nres,
                         uint32_t server_off, uint32_t server_len, uint8_t *out, const uint64_t *out_off, uint32_t *out_len,
                         uint32_t *header_len, int32_t *rstatus)
{
    h2o_qpack_encoder_t *enc = h2o_qpack_create_encoder(4096, 100);
    h2o_iovec_t server_name = h2o_iovec_init(in + server_off, server_len);
    int bad_tokens = 0;
    for (uint32_t r = 0; r < nres; ++r) {
        const uint32_t *R = res + 8 * (size_t)r;
        uint64_t content_length;
        memcpy(&content_length, R, 8);
        uint32_t status = R[2], hfirst = R[3], nh = R[4], fl = R[5], doff = R[6], dlen = R[7];
        int request = (fl & 16u) != 0;
        int server = !request && (fl & 2u) && server_len != 0, dfid = (fl & 8u) != 0;
        out_len[r] = header_len[r] = 0;
        int bad = (server && (uint64_t)server_off + server_len > in_size) || (dfid && (uint64_t)doff + dlen > in_size);
        h2o_iovec_t *names = calloc(nh ? nh : 1, sizeof(h2o_iovec_t));
        h2o_header_t *headers = calloc(nh ? nh : 1, sizeof(h2o_header_t));
        for (uint32_t i = 0; i < nh && !bad; ++i) {
            const uint32_t *H = hdr + 5 * (size_t)(hfirst + i);
            if ((uint64_t)H[0] + H[1] > in_size || (uint64_t)H[2] + H[3] > in_size) {
                bad = 1;
                break;
            }
            const h2o_token_t *tok = (H[4] & 2u) ? h2o_lookup_token((const char *)in + H[0], H[1]) : NULL;
            bad_tokens += (H[4] & 2u) && tok == NULL;
            names[i] = h2o_iovec_init(in + H[0], H[1]);
            headers[i].name = tok != NULL ? (h2o_iovec_t *)&tok->buf : &names[i];
            headers[i].value = h2o_iovec_init(in + H[2], H[3]);
            headers[i].flags.dont_compress = (H[4] & 1u) != 0;
        }
        if (bad) {
            rstatus[r] = -303;
        } else {
            h2o_mem_pool_t pool;
            h2o_mem_init_pool(&pool);
            h2o_qpack_section_stats_t stats = {0};
            size_t shl = 0;
            h2o_iovec_t dv = dfid ? h2o_iovec_init(in + doff, dlen) : h2o_iovec_init(NULL, 0);
            if (dfid && dv.base == NULL)
                dv.base = (char *)"";
            h2o_iovec_t f;
            ref_req_t a;
            if (request && (status > nh || ref_req_args(in, hdr, hfirst, status, 0, &a) != 0)) {
                ++bad_tokens; /* not flatten_request's arguments: a caller error */
                f = h2o_iovec_init(NULL, 0);
            } else if (request) {
                f = h2o_qpack_flatten_request(enc, &pool, 4 * (int64_t)r, NULL, a.method, a.url.scheme, a.url.authority,
                                              a.url.path, a.protocol, headers + status, nh - status, dv, &stats);
                unsigned t = (uint8_t)f.base[1] >> 6;
                uint64_t v = t == 0 ? 1 : t == 1 ? 2 : t == 2 ? 4 : 8;
                shl = f.len - 1 - v; /* the field section: the frame minus its type and length (finalize_flatten) */
            } else {
                f = h2o_qpack_flatten_response(enc, &pool, 4 * (int64_t)r, NULL, (int)status, headers, nh,
                                               server ? &server_name : NULL,
                                               content_length == UINT64_MAX ? SIZE_MAX : (size_t)content_length, dv,
                                               &stats, &shl);
            }
            if (f.len > out_off[r + 1] - out_off[r]) {
                rstatus[r] = -300;
            } else {
                memcpy(out + out_off[r], f.base, f.len);
                out_len[r] = (uint32_t)f.len;
                header_len[r] = (uint32_t)shl;
                rstatus[r] = 0;
            }
            h2o_mem_clear_pool(&pool);
        }
        free(names);
        free(headers);
    }
    h2o_qpack_destroy_encoder(enc);
    return bad_tokens;
}

/* The rule the restatement and the GPU path use for h2o_qpack_lookup_static[token] (lib/common/token_table.h):
 * the h2o_qpack_static_table entry with the token's name and the same value (is_exact), else the first entry
 * with the name, else -1.  Checked for every token against every static value plus two others; returns the
 * number of disagreements. */
REF_API int ref_qpe_lookup_check(void)
{
    int bad = 0;
    for (size_t t = 0; t < h2o__num_tokens; ++t) {
        const h2o_token_t *tok = &h2o__tokens[t];
        for (int v = -2; v < 99; ++v) {
            h2o_iovec_t value = v == -2 ? h2o_iovec_init(H2O_STRLIT("")) : v == -1 ? h2o_iovec_init(H2O_STRLIT("zz-other"))
                                                                                   : h2o_qpack_static_table[v].value;
            int exact = -1, want_exact = 0;
            int32_t got = h2o_qpack_lookup_static[t](value, &exact), want = -1;
            for (int32_t i = 0; i < 99; ++i) {
                if (h2o_qpack_static_table[i].name != tok)
                    continue;
                if (want < 0)
                    want = i;
                if (h2o_memis(h2o_qpack_static_table[i].value.base, h2o_qpack_static_table[i].value.len, value.base, value.len)) {
                    want = i;
                    want_exact = 1;
                    break;
                }
            }
            bad += got != want || (got >= 0 && exact != want_exact);
        }
    }
    return bad;
}
