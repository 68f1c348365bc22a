/*
 * ORACLE -- TEST INFRASTRUCTURE ONLY.  Header-block harness around the REAL reference decoder, compiled
 * from the sources where they lie (oracle/Makefile; nothing is copied):
 *   lib/http2/hpack.c   h2o_hpack_decode_header :319-435 (dynamic table :263-317)
 *   lib/common/memory.c the h2o_mem_pool_t / shared-buffer allocator it decodes into
 *   lib/common/token.c  h2o_lookup_token, h2o_hpack_static_table
 * ref_hpack_decode_blocks loops h2o_hpack_decode_header over every block the way
 * h2o_hpack_parse_request does (hpack.c:513-527), one h2o_hpack_header_table_t per connection with
 * hpack_capacity = hpack_max_capacity = table_size (as lib/http2/connection.c:1844 sets it), and copies
 * each decoded name and value into the caller's arena -- the output contract of
 * include/hhuff.h hhuff_hpack_decode_blocks.
 * ref_hpack_parse_requests runs h2o_hpack_parse_request (hpack.c:502-637) itself over every block, with
 * the arguments h2o's HTTP/2 server passes (lib/http2/connection.c:626-629: a cache-digest receiver --
 * lib/http2/cache_digests.c, so lib/common/url.c's scheme objects and OpenSSL's SHA-256 are linked -- and
 * no datagram flow id), and records what it produced in the include/hhuff.h hhuff_request_t layout; a
 * decode_cb wrapper around h2o_hpack_decode_header copies each field to the arena and, from the
 * out-parameters' changes between calls, learns which field each one took and which fields went to the
 * header list.
 * ref_hpack_parse_responses runs h2o_hpack_parse_response (hpack.c:642-750) over every block as h2o's HTTP/2
 * client calls it (lib/common/http2client.c:332 with a status out-parameter, :421 with status == NULL for
 * trailers; no datagram flow id) through the same wrapper, and records the include/hhuff.h hhuff_response_t.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "h2o/cache_digests.h"
#include "h2o/hpack.h"
#include "h2o/url.h"
#include "h2o/http2_common.h"
#include "h2o/memory.h"

#define REF_API __attribute__((visibility("default")))
#define REF_BLK_ARENA (-300)
#define REF_BLK_SKIPPED (-301)

REF_API int ref_hpack_decode_blocks(const uint8_t *in, const uint32_t *blk_off, const uint32_t *conn_first, uint32_t nconn,
                                    uint32_t table_size, uint8_t *arena, const uint64_t *arena_off, uint32_t *name_off,
                                    uint32_t *name_len, uint32_t *value_off, uint32_t *value_len, uint8_t *fflags,
                                    uint32_t *nfields, int32_t *bstatus, int nthreads)
{
    (void)nthreads;
    for (uint32_t c = 0; c < nconn; ++c) {
        h2o_hpack_header_table_t table;
        memset(&table, 0, sizeof(table));
        table.hpack_capacity = table.hpack_max_capacity = table_size;
        int failed = 0;
        for (uint32_t b = conn_first[c]; b < conn_first[c + 1]; ++b) {
            nfields[b] = 0;
            if (failed) {
                bstatus[b] = REF_BLK_SKIPPED;
                continue;
            }
            h2o_mem_pool_t pool;
            h2o_mem_init_pool(&pool);
            const uint8_t *src = in + blk_off[b], *end = in + blk_off[b + 1];
            uint64_t cur = arena_off[b], aend = arena_off[b + 1] < (1ull << 32) ? arena_off[b + 1] : (1ull << 32);
            uint32_t nf = 0, slot = blk_off[b];
            int st = 0;
            while (src != end) {
                h2o_iovec_t *name, value;
                const char *err_desc = NULL;
                int ret = h2o_hpack_decode_header(&pool, &table, &name, &value, &src, end, &err_desc);
                if (ret != 0 && ret != H2O_HTTP2_ERROR_INVALID_HEADER_CHAR) {
                    st = ret;
                    break;
                }
                if (cur + name->len + value.len > aend) {
                    st = REF_BLK_ARENA;
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
                /* the field's soft errors are what decode_header reports as INVALID_HEADER_CHAR
                 * (hpack.c:427-431); which bit is recovered from err_desc */
                fflags[slot + nf] = ret == 0 ? 0 : (err_desc == h2o_hpack_soft_err_found_invalid_char_in_header_name ? 1 : 2);
                ++nf;
            }
            h2o_mem_clear_pool(&pool);
            nfields[b] = nf;
            bstatus[b] = st;
            failed = st != 0;
        }
        h2o_hpack_dispose_header_table(&table);
    }
    return 0;
}

/* ---- h2o_hpack_parse_request ---- */
typedef struct {
    h2o_hpack_header_table_t *table;
    uint8_t *arena;
    uint64_t cur, aend;
    uint32_t *name_off, *name_len, *value_off, *value_len, slot, nf;
    uint8_t *fflags;
    /* parse_request's out-parameters, and what they held before the previous field */
    h2o_iovec_t *out[6]; /* method, (scheme), authority, path, protocol, expect */
    const h2o_url_scheme_t **scheme;
    h2o_headers_t *headers;
    h2o_iovec_t snap[6];
    const h2o_url_scheme_t *scheme_snap;
    size_t hsize_snap;
    int32_t taken[6];
} rq_ctx_t;

/* attribute the out-parameter changes since the last call to field nf - 1 */
static void rq_settle(rq_ctx_t *x)
{
    if (x->nf == 0)
        return;
    int32_t k = (int32_t)x->nf - 1;
    if (x->headers->size > x->hsize_snap)
        x->fflags[x->slot + k] |= 4;
    for (int i = 0; i < 6; ++i) {
        if (i == 1) {
            if (*x->scheme != x->scheme_snap)
                x->taken[1] = k;
            continue;
        }
        if (x->out[i]->base != x->snap[i].base || x->out[i]->len != x->snap[i].len)
            x->taken[i] = k;
    }
}

static void rq_snapshot(rq_ctx_t *x)
{
    for (int i = 0; i < 6; ++i)
        if (i != 1)
            x->snap[i] = *x->out[i];
    x->scheme_snap = *x->scheme;
    x->hsize_snap = x->headers->size;
}

static int rq_decode_cb(h2o_mem_pool_t *pool, void *ctx, h2o_iovec_t **name, h2o_iovec_t *value, const uint8_t **src,
                        const uint8_t *src_end, const char **err_desc)
{
    rq_ctx_t *x = ctx;
    rq_settle(x);
    rq_snapshot(x);
    int ret = h2o_hpack_decode_header(pool, x->table, name, value, src, src_end, err_desc);
    if (ret != 0 && ret != H2O_HTTP2_ERROR_INVALID_HEADER_CHAR)
        return ret;
    if (x->cur + (*name)->len + value->len > x->aend) {
        *err_desc = NULL; /* a hard error for parse_request, with no description */
        return REF_BLK_ARENA;
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

static uint32_t rq_err_code(const char *e)
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

REF_API int ref_hpack_parse_requests(const uint8_t *in, const uint32_t *blk_off, const uint32_t *conn_first, uint32_t nconn,
                                     uint32_t table_size, uint8_t *arena, const uint64_t *arena_off, uint32_t *name_off,
                                     uint32_t *name_len, uint32_t *value_off, uint32_t *value_len, uint8_t *fflags,
                                     uint32_t *nfields, int32_t *bstatus, uint32_t *req, int nthreads)
{
    (void)nthreads;
    for (uint32_t c = 0; c < nconn; ++c) {
        h2o_hpack_header_table_t table;
        memset(&table, 0, sizeof(table));
        table.hpack_capacity = table.hpack_max_capacity = table_size;
        int failed = 0;
        for (uint32_t b = conn_first[c]; b < conn_first[c + 1]; ++b) {
            uint32_t *w = req + 12 * (size_t)b;
            nfields[b] = 0;
            h2o_iovec_t method = {NULL, 0}, authority = {NULL, 0}, path = {NULL, 0}, protocol = {NULL, 0}, expect = {NULL, 0};
            const h2o_url_scheme_t *scheme = NULL;
            h2o_headers_t headers = {NULL, 0, 0};
            int exists_map = 0;
            size_t content_length = SIZE_MAX;
            const char *err_desc = NULL;
            rq_ctx_t x;
            memset(&x, 0, sizeof(x));
            for (int i = 0; i < 6; ++i)
                x.taken[i] = -1;
            if (!failed) {
                h2o_mem_pool_t pool;
                h2o_mem_init_pool(&pool);
                h2o_cache_digests_t *digests = NULL;
                x.table = &table, x.arena = arena, x.cur = arena_off[b];
                x.aend = arena_off[b + 1] < (1ull << 32) ? arena_off[b + 1] : (1ull << 32);
                x.name_off = name_off, x.name_len = name_len, x.value_off = value_off, x.value_len = value_len;
                x.fflags = fflags, x.slot = blk_off[b];
                x.out[0] = &method, x.out[2] = &authority, x.out[3] = &path, x.out[4] = &protocol, x.out[5] = &expect;
                x.out[1] = &method; /* unused slot (the scheme is a pointer) */
                x.scheme = &scheme, x.headers = &headers;
                int ret = h2o_hpack_parse_request(&pool, rq_decode_cb, &x, &method, &scheme, &authority, &path, &protocol,
                                                  &headers, &exists_map, &content_length, &expect, &digests, NULL,
                                                  in + blk_off[b], blk_off[b + 1] - blk_off[b], &err_desc);
                rq_settle(&x);
                if (digests != NULL)
                    h2o_cache_digests_destroy(digests);
                h2o_mem_clear_pool(&pool);
                nfields[b] = x.nf;
                bstatus[b] = ret;
                failed = ret != 0 && ret != H2O_HTTP2_ERROR_INVALID_HEADER_CHAR;
            } else {
                bstatus[b] = REF_BLK_SKIPPED;
            }
            uint64_t cl = content_length;
            memcpy(w, &cl, 8);
            memcpy(w + 2, x.taken, 24);
            w[8] = (uint32_t)exists_map;
            w[9] = (uint32_t)headers.size;
            w[10] = rq_err_code(err_desc);
            w[11] = scheme == NULL ? 0 : scheme == &H2O_URL_SCHEME_HTTP ? 1 : scheme == &H2O_URL_SCHEME_HTTPS ? 2 : 3;
        }
        h2o_hpack_dispose_header_table(&table);
    }
    return 0;
}

/* ---- h2o_hpack_parse_response ---- */
REF_API int ref_hpack_parse_responses(const uint8_t *in, const uint32_t *blk_off, const uint32_t *conn_first, uint32_t nconn,
                                      uint32_t table_size, const uint8_t *trailers, uint8_t *arena, const uint64_t *arena_off,
                                      uint32_t *name_off, uint32_t *name_len, uint32_t *value_off, uint32_t *value_len,
                                      uint8_t *fflags, uint32_t *nfields, int32_t *bstatus, uint32_t *res, int nthreads)
{
    (void)nthreads;
    for (uint32_t c = 0; c < nconn; ++c) {
        h2o_hpack_header_table_t table;
        memset(&table, 0, sizeof(table));
        table.hpack_capacity = table.hpack_max_capacity = table_size;
        int failed = 0;
        for (uint32_t b = conn_first[c]; b < conn_first[c + 1]; ++b) {
            uint32_t *w = res + 4 * (size_t)b;
            nfields[b] = 0;
            int status = 0;
            h2o_headers_t headers = {NULL, 0, 0};
            h2o_iovec_t unused = {NULL, 0};
            const char *err_desc = NULL;
            rq_ctx_t x;
            memset(&x, 0, sizeof(x));
            for (int i = 0; i < 6; ++i)
                x.taken[i] = -1, x.out[i] = &unused;
            x.scheme = (const h2o_url_scheme_t **)&x.scheme_snap; /* unchanging: rq_settle sees no scheme */
            if (!failed) {
                h2o_mem_pool_t pool;
                h2o_mem_init_pool(&pool);
                x.table = &table, x.arena = arena, x.cur = arena_off[b];
                x.aend = arena_off[b + 1] < (1ull << 32) ? arena_off[b + 1] : (1ull << 32);
                x.name_off = name_off, x.name_len = name_len, x.value_off = value_off, x.value_len = value_len;
                x.fflags = fflags, x.slot = blk_off[b];
                x.headers = &headers;
                int is_trailers = trailers != NULL && trailers[b] != 0;
                int ret = h2o_hpack_parse_response(&pool, rq_decode_cb, &x, is_trailers ? NULL : &status, &headers, NULL,
                                                   in + blk_off[b], blk_off[b + 1] - blk_off[b], &err_desc);
                rq_settle(&x);
                h2o_mem_clear_pool(&pool);
                nfields[b] = x.nf;
                bstatus[b] = ret;
                failed = ret != 0 && ret != H2O_HTTP2_ERROR_INVALID_HEADER_CHAR;
            } else {
                bstatus[b] = REF_BLK_SKIPPED;
            }
            w[0] = (uint32_t)status;
            w[1] = (uint32_t)headers.size;
            w[2] = rq_err_code(err_desc);
            w[3] = (uint32_t)-1; /* no datagram flow id out-parameter (http2client.c:332) */
        }
        h2o_hpack_dispose_header_table(&table);
    }
    return 0;
}
