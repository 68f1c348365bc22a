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
