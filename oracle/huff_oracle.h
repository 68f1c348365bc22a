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
#define ORC_MAX_STR ((1u << 29) - 1) /* per-string limit of the HIP path (include/hhuff.h) */
/* string-literal verdicts (include/hhuff.h HHUFF_LIT_*) */
#define ORC_LIT_INCOMPLETE 1
#define ORC_LIT_BAD_INT 2
#define ORC_LIT_TRUNCATED 3
#define ORC_LIT_HUFFMAN 4
#define ORC_LIT_UPPERCASE 5
#define ORC_LIT_TOO_LONG 6
#define ORC_STATUS_FAIL 0x80u
/* header blocks (f4): h2o return codes (include/h2o/http2_common.h:41, :49, :55) and the batch's own */
#define ORC_ERR_PROTOCOL (-1)
#define ORC_ERR_COMPRESSION (-9)
#define ORC_ERR_INVALID_CHAR (-254)
#define ORC_BLK_ARENA (-300)   /* HHUFF_BLK_ARENA: the block's arena slice is too small */
#define ORC_BLK_SKIPPED (-301) /* HHUFF_BLK_SKIPPED: an earlier block of the connection failed */
/* QPACK decoder (f4, QPACK half): h2o's codes (include/h2o/http3_common.h:73, :77) and the batch's own */
#define ORC_QPK_DECOMPRESSION_FAILED 0x30200 /* H2O_HTTP3_ERROR_QPACK_DECOMPRESSION_FAILED (app code 0x200) */
#define ORC_QPK_INCOMPLETE (-1)              /* H2O_HTTP3_ERROR_INCOMPLETE */
#define ORC_QPK_BLOCKED (-302) /* HHUFF_QPK_BLOCKED: Required Insert Count not reached (*blocked_ref != 0) */

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
int orc_decode_literal(const uint8_t *lit, const uint8_t *end, unsigned prefix_bits, int is_name, int qpack,
                       uint8_t *out, uint64_t lit_pos, uint32_t *hdr, uint32_t *consumed, uint32_t *out_len,
                       unsigned *soft);
int orc_literals_batch(const uint8_t *in, const uint32_t *lit_off, const uint32_t *lit_end, uint32_t n,
                       unsigned prefix_bits, unsigned flags, const uint32_t *is_name_bits, uint8_t *out,
                       uint32_t *out_len, uint32_t *pay_off, uint32_t *consumed, uint8_t *status, int nthreads);

/* raw-literal validators (h2o_hpack_validate_header_name / _value, hpack.c:163-221) */
int orc_validate_header_name(unsigned *soft, const uint8_t *s, size_t len);
void orc_validate_header_value(unsigned *soft, const uint8_t *s, size_t len);
int orc_is_qpack_token(const uint8_t *s, size_t len);
void *orc_qpack_open(uint32_t nconn, uint32_t header_table_size, uint64_t max_blocked);
void orc_qpack_close(void *h);
int orc_qpack_step(void *h, const uint8_t *in, const uint32_t *enc_off, const uint32_t *enc_len, const uint32_t *sec_off,
                   const uint32_t *conn_first, const uint32_t *num_blocked, uint8_t *arena, const uint64_t *arena_off,
                   uint32_t *name_off, uint32_t *name_len, uint32_t *value_off, uint32_t *value_len, uint8_t *fflags,
                   uint32_t *nfields, int32_t *sstatus, uint64_t *req_insert_count, int32_t *enc_status,
                   uint32_t *enc_consumed, uint64_t *insert_count);
int orc_hpack_decode_blocks(const uint8_t *in, const uint32_t *blk_off, const uint32_t *conn_first, uint32_t nconn,
                            uint32_t table_size, uint8_t *arena, const uint64_t *arena_off, uint32_t *name_off,
                            uint32_t *name_len, uint32_t *value_off, uint32_t *value_len, uint8_t *fflags,
                            uint32_t *nfields, int32_t *bstatus, int nthreads);
/* the same with h2o_hpack_parse_request's rules (hpack.c:502-637); req: 12 u32 words per block
 * (include/hhuff.h hhuff_request_t) */
int orc_hpack_parse_requests(const uint8_t *in, const uint32_t *blk_off, const uint32_t *conn_first, uint32_t nconn,
                             uint32_t table_size, uint8_t *arena, const uint64_t *arena_off, uint32_t *name_off,
                             uint32_t *name_len, uint32_t *value_off, uint32_t *value_len, uint8_t *fflags,
                             uint32_t *nfields, int32_t *bstatus, uint32_t *req, int nthreads);
