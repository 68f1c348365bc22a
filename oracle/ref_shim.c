/*
 * ORACLE -- TEST INFRASTRUCTURE ONLY.  Binds the REAL reference codec, compiled from the sources
 * where they lie under /root/reference (nothing is copied), into oracle/_ref/libh2oref.so:
 *   lib/http2/hpack.c   h2o_hpack_decode_huffman :117, h2o_hpack_encode_huffman :774,
 *                       h2o_hpack_encode_string :816, h2o_hpack_decode_int :52
 *   lib/http3/qpack.c   static flatten_string :1042 (reached by including the .c, as the reference's
 *                       own unit test does at t/00unit/lib/http3/qpack.c:24)
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

#define ORC_CODEC_DECODE ref_dec
#define ORC_CODEC_ENCODE h2o_hpack_encode_huffman
#define ORC_CODEC_FLATTEN ref_flat
#define ORC_BATCH_PREFIX ref
#define ORC_BATCH_API REF_API
#include "batch_driver.h"
