/* ORACLE -- TEST INFRASTRUCTURE ONLY (see huff_oracle.c).  Batch drivers use the array contract of
 * include/hhuff.h so tests can compare the HIP path and the oracle element by element. */
#pragma once
#include <stddef.h>
#include <stdint.h>

#define ORC_SOFT_NAME 0x1u  /* H2O_HPACK_SOFT_ERROR_BIT_INVALID_NAME, include/h2o/hpack.h:50 */
#define ORC_SOFT_VALUE 0x2u /* H2O_HPACK_SOFT_ERROR_BIT_INVALID_VALUE, include/h2o/hpack.h:51 */
#define ORC_INT_INCOMPLETE (-255) /* H2O_HTTP2_ERROR_INCOMPLETE, include/h2o/http2_common.h:57 */
#define ORC_INT_COMPRESSION (-9) /* H2O_HTTP2_ERROR_COMPRESSION, include/h2o/http2_common.h:49 */
#define ORC_FAIL_LEN 0xFFFFFFFFu
#define ORC_STATUS_FAIL 0x80u

size_t orc_decode_huffman(char *dst, unsigned *soft_errors, const uint8_t *src, size_t len, int is_name);
size_t orc_encode_huffman(uint8_t *dst, const uint8_t *src, size_t len);
uint8_t *orc_encode_int(uint8_t *dst, int64_t value, unsigned prefix_bits);
int64_t orc_decode_int(const uint8_t **src, const uint8_t *src_end, unsigned prefix_bits);
size_t orc_encode_string(uint8_t *dst, const uint8_t *s, size_t len);
size_t orc_flatten_string(uint8_t *dst, const uint8_t *s, size_t len, unsigned prefix_bits, int dont_compress);

int orc_decode_batch(const uint8_t *in, const uint32_t *in_off, const uint32_t *in_len, uint32_t n,
                     const uint32_t *is_name_bits, uint8_t *out, const uint32_t *out_off, uint32_t *out_len,
                     uint8_t *status, int nthreads);
int orc_encode_batch(const uint8_t *in, const uint32_t *in_off, const uint32_t *in_len, uint32_t n, uint8_t *out,
                     const uint32_t *out_off, uint32_t *out_len, uint8_t *status, int nthreads);
int orc_flatten_batch(const uint8_t *in, const uint32_t *in_off, const uint32_t *in_len, uint32_t n,
                      const uint8_t *first_bytes, unsigned prefix_bits, const uint32_t *raw_bits, uint8_t *out,
                      const uint32_t *out_off, uint32_t *out_len, int nthreads);
