/*
 * ORACLE -- TEST INFRASTRUCTURE ONLY.  Never linked into, loaded by, or called from the product
 * (h2o_amd/).  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may use it.
 *
 * A clean-room CPU restatement of h2o's HPACK Huffman hot path, same algorithm class as the reference:
 *   - decode: 4-bit nibble FSM over a 256-state x 16 table, two dependent lookups per input byte
 *             (lib/http2/hpack.c:85-99 huffdecode4, :117-156 h2o_hpack_decode_huffman)
 *   - encode: 64-bit accumulator with 40 bits of headroom, byte emit with a dst_end check
 *             (lib/http2/hpack.c:774-804 h2o_hpack_encode_huffman)
 *   - framing: prefix integers (hpack.c:52-83 decode_int, :752-772 encode_int), HPACK string literal
 *             (hpack.c:806-837 encode_as_is / h2o_hpack_encode_string), QPACK string literal
 *             (lib/http3/qpack.c:1036-1066 flatten_int / flatten_string)
 * Tables come from tools/gen_tables.py (oracle/huff_tables.h).
 *
 * Parity pinning: tests/test_oracle_golden.py checks this file against golden vectors that the compiled
 * reference (oracle/_ref, built from /root/reference/lib/http2/hpack.c by oracle/Makefile) produced,
 * committed under tests/golden/ together with oracle/gen_golden.py.
 */
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "huff_tables.h"
#include "huff_oracle.h"

/* hpack.c:85-99 -- one nibble step */
static inline char *orc_nibble(char *dst, uint8_t nib, uint8_t *state, int *maybe_eos, uint8_t *seen)
{
    uint32_t e = orc_fsm[*state][nib];
    uint8_t flags = (uint8_t)(e >> 8);
    if (flags & ORC_FAIL)
        return NULL;
    if (flags & ORC_SYM) {
        *dst++ = (char)(e >> 16);
        /* only the two INVALID bits are accumulated; ORC_UPPER never is (hpack.c:93) */
        *seen |= flags & (ORC_INV_NAME | ORC_INV_VALUE);
    }
    *state = (uint8_t)e;
    *maybe_eos = (flags & ORC_ACCEPTED) != 0;
    return dst;
}

/* hpack.c:110-115 */
static inline int orc_value_ws_ok(const char *s, size_t len)
{
    return !(len != 0 && (s[0] == 0x20 || s[0] == 0x09 || s[len - 1] == 0x20 || s[len - 1] == 0x09));
}

/* hpack.c:117-156 */
size_t orc_decode_huffman(char *dst0, unsigned *soft_errors, const uint8_t *src, size_t len, int is_name)
{
    char *dst = dst0;
    uint8_t state = 0, seen = 0;
    int maybe_eos = 1;
    for (const uint8_t *end = src + len; src < end; ++src) {
        if ((dst = orc_nibble(dst, *src >> 4, &state, &maybe_eos, &seen)) == NULL)
            return SIZE_MAX;
        if ((dst = orc_nibble(dst, *src & 15, &state, &maybe_eos, &seen)) == NULL)
            return SIZE_MAX;
    }
    if (!maybe_eos)
        return SIZE_MAX;
    size_t n = (size_t)(dst - dst0);
    if (is_name) {
        /* empty name -> soft; ':'-prefixed names skip validation; the upper-case hard error at
         * hpack.c:142-144 is unreachable because the UPPER flag is never accumulated */
        if (n == 0 || ((seen & ORC_INV_NAME) && dst0[0] != ':'))
            *soft_errors |= ORC_SOFT_NAME;
    } else {
        if ((seen & ORC_INV_VALUE) || !orc_value_ws_ok(dst0, n))
            *soft_errors |= ORC_SOFT_VALUE;
    }
    return n;
}

/* hpack.c:774-804 */
size_t orc_encode_huffman(uint8_t *dst0, const uint8_t *src, size_t len)
{
    uint8_t *dst = dst0, *dst_end = dst0 + len;
    uint64_t acc = 0;
    int room = 40; /* free bit positions below bit 40 */
    for (const uint8_t *end = src + len; src != end; ++src) {
        unsigned nb = orc_sym_nbits[*src];
        acc |= (uint64_t)orc_sym_code[*src] << (room - (int)nb);
        room -= (int)nb;
        while (room <= 32) {
            *dst++ = (uint8_t)(acc >> 32);
            acc <<= 8;
            room += 8;
            if (dst == dst_end)
                return SIZE_MAX;
        }
    }
    if (room != 40) {
        acc |= ((uint64_t)1 << room) - 1; /* pad with the EOS prefix (all ones) */
        *dst++ = (uint8_t)(acc >> 32);
    }
    if (dst == dst_end)
        return SIZE_MAX;
    return (size_t)(dst - dst0);
}

/* hpack.c:752-772 */
uint8_t *orc_encode_int(uint8_t *dst, int64_t value, unsigned prefix_bits)
{
    int64_t pmax = ((int64_t)1 << prefix_bits) - 1;
    if (value < pmax) {
        *dst++ |= (uint8_t)value;
        return dst;
    }
    value -= pmax;
    *dst++ |= (uint8_t)pmax;
    for (; value >= 128; value >>= 7)
        *dst++ = (uint8_t)(0x80 | value);
    *dst++ = (uint8_t)value;
    return dst;
}

/* hpack.c:52-83; returns ORC_INT_INCOMPLETE / ORC_INT_COMPRESSION on error */
int64_t orc_decode_int(const uint8_t **src, const uint8_t *src_end, unsigned prefix_bits)
{
    uint8_t pmax = (uint8_t)((1u << prefix_bits) - 1);
    if (*src >= src_end)
        return ORC_INT_INCOMPLETE;
    uint64_t v = *(*src)++ & pmax;
    if (v != pmax)
        return (int64_t)v;
    unsigned shift;
    for (shift = 0; shift < 56; shift += 7) {
        if (*src == src_end)
            return ORC_INT_INCOMPLETE;
        v += (uint64_t)(**src & 127) << shift;
        if ((*(*src)++ & 128) == 0)
            return (int64_t)v;
    }
    if (*src == src_end)
        return ORC_INT_INCOMPLETE;
    if (**src & 128)
        return ORC_INT_COMPRESSION;
    v += (uint64_t)(*(*src)++ & 127) << shift;
    if (v > (uint64_t)INT64_MAX)
        return ORC_INT_COMPRESSION;
    return (int64_t)v;
}

/* hpack.c:806-837: Huffman if it is strictly shorter, else raw; dst capacity len + 1 + 10 */
size_t orc_encode_string(uint8_t *dst, const uint8_t *s, size_t len)
{
    if (len != 0) {
        size_t hl = orc_encode_huffman(dst + 1, s, len);
        if (hl != SIZE_MAX) {
            if (hl < 127) {
                dst[0] = (uint8_t)(0x80 | hl);
                return 1 + hl;
            }
            uint8_t head[16];
            head[0] = 0x80;
            size_t head_len = (size_t)(orc_encode_int(head, (int64_t)hl, 7) - head);
            memmove(dst + head_len, dst + 1, hl);
            memcpy(dst, head, head_len);
            return head_len + hl;
        }
    }
    uint8_t *p = dst;
    *p = 0;
    p = orc_encode_int(p, (int64_t)len, 7);
    memcpy(p, s, len);
    return (size_t)(p - dst) + len;
}

/* qpack.c:1042-1066: `dst[0]` holds the caller's first byte whose bits above the H bit are kept */
size_t orc_flatten_string(uint8_t *dst, const uint8_t *s, size_t len, unsigned prefix_bits, int dont_compress)
{
    size_t hl;
    if (dont_compress || (hl = orc_encode_huffman(dst + 1, s, len)) == SIZE_MAX) {
        dst[0] &= (uint8_t)~((2u << prefix_bits) - 1);
        uint8_t *p = orc_encode_int(dst, (int64_t)len, prefix_bits);
        memcpy(p, s, len);
        return (size_t)(p - dst) + len;
    }
    uint8_t head[16], *p = head;
    *p = dst[0] & (uint8_t)~((1u << prefix_bits) - 1);
    *p |= (uint8_t)(1u << prefix_bits);
    p = orc_encode_int(p, (int64_t)hl, prefix_bits);
    size_t head_len = (size_t)(p - head);
    if (head_len == 1) {
        dst[0] = head[0];
    } else {
        memmove(dst + head_len, dst + 1, hl);
        memcpy(dst, head, head_len);
    }
    return head_len + hl;
}

/* ---- string literals (decode_string hpack.c:223-261; QPACK qpack.c:559-629 without the pool) ---- */

/* h2o_hpack_validate_header_name (hpack.c:163-193): 0 = upper-case letter (hard error) */
static int orc_validate_name(unsigned *soft, const uint8_t *s, size_t len)
{
    if (len == 0) {
        *soft |= ORC_SOFT_NAME;
        return 1;
    }
    for (; len != 0; ++s, --len) {
        if (!orc_name_valid[*s]) {
            if ((unsigned)(*s - 'A') < 26u)
                return 0;
            *soft |= ORC_SOFT_NAME;
        }
    }
    return 1;
}

/* h2o_hpack_validate_header_value (hpack.c:195-221) */
static void orc_validate_value(unsigned *soft, const uint8_t *s, size_t len)
{
    int bad = !orc_value_ws_ok((const char *)s, len);
    for (size_t i = 0; !bad && i < len; ++i)
        bad = !orc_value_valid[s[i]];
    if (bad)
        *soft |= ORC_SOFT_VALUE;
}

int orc_validate_header_name(unsigned *soft, const uint8_t *s, size_t len) { return orc_validate_name(soft, s, len); }
void orc_validate_header_value(unsigned *soft, const uint8_t *s, size_t len) { orc_validate_value(soft, s, len); }

/* QPACK raw names skip validation when h2o_lookup_token finds them (qpack.c:585); the only tokens
 * the validator would flag are the pseudo-header names (lib/common/token_table.h) */
static int orc_is_pseudo_token(const uint8_t *s, size_t len)
{
    static const char *const tok[] = {":authority", ":method", ":path", ":protocol", ":scheme", ":status"};
    for (size_t k = 0; k < sizeof(tok) / sizeof(tok[0]); ++k)
        if (strlen(tok[k]) == len && memcmp(tok[k], s, len) == 0)
            return 1;
    return 0;
}

int orc_is_qpack_token(const uint8_t *s, size_t len) { return orc_is_pseudo_token(s, len); }

int orc_decode_literal(const uint8_t *lit, const uint8_t *end, unsigned prefix_bits, int is_name, int qpack,
                       uint8_t *out, uint64_t lit_pos, uint32_t *hdr, uint32_t *consumed, uint32_t *out_len,
                       unsigned *soft)
{
    const uint8_t *p = lit;
    *hdr = 0;
    *consumed = 0;
    *out_len = ORC_FAIL_LEN;
    if (p >= end)
        return ORC_LIT_INCOMPLETE;
    int huff = (*p >> prefix_bits) & 1;
    int64_t len = orc_decode_int(&p, end, prefix_bits);
    if (len == ORC_INT_INCOMPLETE)
        return ORC_LIT_INCOMPLETE;
    if (len < 0)
        return ORC_LIT_BAD_INT;
    if (len > end - p)
        return ORC_LIT_TRUNCATED;
    if (len > (int64_t)ORC_MAX_STR)
        return ORC_LIT_TOO_LONG;
    *hdr = (uint32_t)(p - lit);
    uint8_t *dst = out + ((lit_pos + *hdr) * 8u) / 5u;
    if (huff) {
        size_t r = orc_decode_huffman((char *)dst, soft, p, (size_t)len, is_name);
        if (r == SIZE_MAX)
            return ORC_LIT_HUFFMAN;
        *out_len = (uint32_t)r;
    } else {
        if (is_name) {
            int skip = qpack ? orc_is_pseudo_token(p, (size_t)len) : (len != 0 && p[0] == ':');
            if (!skip && !orc_validate_name(soft, p, (size_t)len))
                return ORC_LIT_UPPERCASE;
        } else {
            orc_validate_value(soft, p, (size_t)len);
        }
        memcpy(dst, p, (size_t)len);
        *out_len = (uint32_t)len;
    }
    *consumed = *hdr + (uint32_t)len;
    return 0;
}

/* ---- batch drivers (same array contract as include/hhuff.h) ---------------------------------- */

#define ORC_CODEC_DECODE orc_decode_huffman
#define ORC_CODEC_ENCODE orc_encode_huffman
#define ORC_CODEC_FLATTEN orc_flatten_string
#define ORC_CODEC_LITERAL orc_decode_literal
#define ORC_BATCH_PREFIX orc
#include "batch_driver.h"
