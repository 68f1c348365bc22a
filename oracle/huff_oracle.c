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

/* ---- batch drivers (same array contract as include/hhuff.h) ---------------------------------- */

#define ORC_CODEC_DECODE orc_decode_huffman
#define ORC_CODEC_ENCODE orc_encode_huffman
#define ORC_CODEC_FLATTEN orc_flatten_string
#define ORC_BATCH_PREFIX orc
#include "batch_driver.h"
