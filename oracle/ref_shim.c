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
 * Used here (in the build container) to produce tests/golden/* and to pin the restatement.  It is
 * never needed on the GPU box.
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
