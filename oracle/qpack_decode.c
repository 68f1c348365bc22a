/*
 * ORACLE -- TEST INFRASTRUCTURE ONLY.  Clean-room CPU restatement of h2o's QPACK decoder (SURVEY.md 8
 * f4, QPACK half): the encoder-stream instructions of h2o_qpack_decoder_handle_input
 * (lib/http3/qpack.c:420-485) building one dynamic table per connection (header_table_insert :166-190,
 * header_table_evict :153-164, the insert helpers :266-418), then field sections decoded the way
 * h2o_qpack_parse_request reads them (:830-858): parse_decode_context (:754-799),
 * check_decode_context_blocked (:801-820) and decode_header (:652-752) field after field.
 * Output contract: include/hhuff.h hhuff_qpack_decode.  A session keeps every connection's table
 * between steps, as the GPU path keeps it in scratch with HHUFF_QPK_CONTINUE.
 */
#include <stdlib.h>
#include <string.h>

#include "huff_oracle.h"
#include "huff_tables.h"
#include "orc_request.h"

#define QPK_ENTRY_OVERHEAD 32u                /* HEADER_ENTRY_SIZE_OFFSET, qpack.c:32 */
#define QPK_STATIC_COUNT 99u                  /* h2o_qpack_static_table[99], include/h2o/token_table.h:114 */
#define QPK_QUICINT_MAX 4611686018427387903LL /* PTLS_QUICINT_MAX */

typedef struct {
    uint8_t *name, *value;
    uint32_t nlen, vlen;
    unsigned soft;
} qpk_entry_t;

typedef struct {
    qpk_entry_t *e; /* live entries, oldest first: e[k] has absolute index base_offset + k */
    uint64_t num, cap_entries;
    int64_t base_offset; /* absolute index of the oldest entry; starts at 1 (qpack.c:143) */
    uint64_t num_bytes, max_size;
    uint32_t header_table_size, max_entries;
    uint64_t total_inserts;
    int failed;
} qpk_conn_t;

typedef struct {
    uint32_t nconn;
    uint64_t max_blocked;
    qpk_conn_t *c;
} qpk_session_t;

static void qpk_evict(qpk_conn_t *t, uint64_t delta) /* header_table_evict (qpack.c:153-164) */
{
    uint64_t k = 0;
    while (k < t->num && t->num_bytes + delta > t->max_size) {
        qpk_entry_t *x = &t->e[k++];
        t->num_bytes -= (uint64_t)x->nlen + x->vlen + QPK_ENTRY_OVERHEAD;
        free(x->name);
        free(x->value);
        ++t->base_offset;
    }
    if (k) {
        memmove(t->e, t->e + k, (t->num - k) * sizeof(qpk_entry_t));
        t->num -= k;
    }
}

/* decoder_insert + header_table_insert (qpack.c:266-271, :166-190): takes ownership of name / value */
static void qpk_insert(qpk_conn_t *t, uint8_t *name, uint32_t nlen, uint8_t *value, uint32_t vlen, unsigned soft)
{
    qpk_evict(t, (uint64_t)nlen + vlen + QPK_ENTRY_OVERHEAD);
    if (t->num == t->cap_entries) {
        uint64_t nc = t->cap_entries ? 2 * t->cap_entries : 16;
        t->e = (qpk_entry_t *)realloc(t->e, nc * sizeof(qpk_entry_t));
        t->cap_entries = nc;
    }
    qpk_entry_t *x = &t->e[t->num++];
    x->name = name, x->value = value, x->nlen = nlen, x->vlen = vlen, x->soft = soft;
    t->num_bytes += (uint64_t)nlen + vlen + QPK_ENTRY_OVERHEAD;
    ++t->total_inserts;
}

static int64_t qpk_table_total(const qpk_conn_t *t) { return t->base_offset + (int64_t)t->num; } /* :321-324 */

static const qpk_entry_t *qpk_resolve_abs(const qpk_conn_t *t, int64_t index) /* resolve_dynamic_abs :201-213 */
{
    if (index < t->base_offset || index - t->base_offset >= (int64_t)t->num)
        return NULL;
    return &t->e[index - t->base_offset];
}

static uint8_t *dup_bytes(const uint8_t *s, size_t n)
{
    uint8_t *p = (uint8_t *)malloc(n + 1);
    memcpy(p, s, n);
    return p;
}

/* decode_value (qpack.c:222-238) into a fresh buffer; SIZE_MAX on a Huffman failure */
static size_t qpk_decode_value(uint8_t **out, unsigned *soft, int huff, const uint8_t *src, size_t len)
{
    uint8_t *buf = (uint8_t *)malloc(len * 2 + 1);
    size_t r;
    if (huff) {
        r = orc_decode_huffman((char *)buf, soft, src, len, 0);
    } else {
        orc_validate_header_value(soft, src, len);
        memcpy(buf, src, len);
        r = len;
    }
    if (r == SIZE_MAX) {
        free(buf);
        return SIZE_MAX;
    }
    *out = buf;
    return r;
}

/* decode_value_and_insert (qpack.c:273-287) */
static int qpk_value_and_insert(qpk_conn_t *t, uint8_t *name, uint32_t nlen, unsigned soft, int vhuff, const uint8_t *v,
                                size_t vlen)
{
    uint8_t *value;
    size_t r = qpk_decode_value(&value, &soft, vhuff, v, vlen);
    if (r == SIZE_MAX) {
        free(name);
        return ORC_QPK_DECOMPRESSION_FAILED;
    }
    if ((uint64_t)nlen + r + QPK_ENTRY_OVERHEAD > t->max_size) { /* header exceeds table size */
        free(name);
        free(value);
        return ORC_QPK_DECOMPRESSION_FAILED;
    }
    qpk_insert(t, name, nlen, value, (uint32_t)r, soft);
    return 0;
}

/* decode_int (qpack.c:215-220): 0, ORC_QPK_INCOMPLETE or ORC_QPK_DECOMPRESSION_FAILED */
static int qpk_int(int64_t *v, const uint8_t **src, const uint8_t *end, unsigned prefix_bits)
{
    if ((*v = orc_decode_int(src, end, prefix_bits)) < 0)
        return *v == ORC_INT_INCOMPLETE ? ORC_QPK_INCOMPLETE : ORC_QPK_DECOMPRESSION_FAILED;
    return 0;
}

/* h2o_qpack_decoder_handle_input (qpack.c:420-485): returns the error; *consumed = how far the caller's
 * *src advanced (past every instruction the loop finished, failed ones included, :476); *insert_count
 * as the reference reports it */
static int qpk_handle_input(qpk_conn_t *t, const uint8_t *in, const uint8_t *end, uint32_t *consumed,
                            uint64_t *insert_count)
{
    const uint8_t *src = in, *done = in;
    uint64_t old_total = t->total_inserts;
    int ret = 0;
    *insert_count = 0;
    while (src != end && ret == 0) {
        switch (*src >> 5) {
        default: { /* insert with name reference (:430-444) */
            int64_t name_index, value_len;
            int name_is_static = (*src & 0x40) != 0;
            if ((ret = qpk_int(&name_index, &src, end, 6)) != 0)
                goto Exit;
            if (src == end)
                goto Exit;
            int vhuff = (*src & 0x80) != 0;
            if ((ret = qpk_int(&value_len, &src, end, 7)) != 0)
                goto Exit;
            if (!(value_len <= end - src))
                goto Exit;
            if (name_is_static) { /* insert_token_header (:289-300): soft starts at 0 */
                if ((uint64_t)name_index >= QPK_STATIC_COUNT) {
                    ret = ORC_QPK_DECOMPRESSION_FAILED;
                } else {
                    const char *n = orc_qpack_static_name[name_index];
                    ret = qpk_value_and_insert(t, dup_bytes((const uint8_t *)n, strlen(n)), (uint32_t)strlen(n), 0,
                                               vhuff, src, (size_t)value_len);
                }
            } else { /* insert_with_name_reference, dynamic (:335-348) */
                int64_t base_index = qpk_table_total(t) - 1;
                const qpk_entry_t *ref;
                if (name_index > base_index || (ref = qpk_resolve_abs(t, base_index - name_index)) == NULL) {
                    ret = ORC_QPK_DECOMPRESSION_FAILED;
                } else {
                    /* token names carry no name bit; literal names keep theirs (:343-347) */
                    ret = qpk_value_and_insert(t, dup_bytes(ref->name, ref->nlen), ref->nlen, ref->soft & ORC_SOFT_NAME,
                                               vhuff, src, (size_t)value_len);
                }
            }
            src += value_len;
        } break;
        case 2:
        case 3: { /* insert without name reference (:446-462) */
            int64_t name_len, value_len;
            int nhuff = (*src & 0x20) != 0;
            if ((ret = qpk_int(&name_len, &src, end, 5)) != 0)
                goto Exit;
            if (!(name_len < end - src))
                goto Exit;
            const uint8_t *qn = src;
            src += name_len;
            int vhuff = (*src & 0x80) != 0;
            if ((ret = qpk_int(&value_len, &src, end, 7)) != 0)
                goto Exit;
            if (!(value_len <= end - src))
                goto Exit;
            /* insert_without_name_reference (:352-393) */
            unsigned soft = 0;
            uint8_t *name;
            size_t nl;
            if (nhuff) {
                name = (uint8_t *)malloc((size_t)name_len * 2 + 1);
                nl = orc_decode_huffman((char *)name, &soft, qn, (size_t)name_len, 1);
                if (nl == SIZE_MAX) {
                    free(name);
                    ret = ORC_QPK_DECOMPRESSION_FAILED;
                    goto Next;
                }
            } else {
                if (!orc_validate_header_name(&soft, qn, (size_t)name_len)) {
                    ret = ORC_QPK_DECOMPRESSION_FAILED;
                    goto Next;
                }
                name = dup_bytes(qn, (size_t)name_len);
                nl = (size_t)name_len;
            }
            /* a name h2o_lookup_token knows goes in as a token header with soft bits 0 (:383-384); the only
             * tokens that can carry soft bits here are the raw pseudo-header names */
            if (orc_is_qpack_token(name, nl))
                soft = 0;
            ret = qpk_value_and_insert(t, name, (uint32_t)nl, soft, vhuff, src, (size_t)value_len);
        Next:
            src += value_len;
        } break;
        case 0: { /* duplicate (:463-468, :395-406) */
            int64_t index;
            if ((ret = qpk_int(&index, &src, end, 5)) != 0)
                goto Exit;
            if (index >= (int64_t)t->num) {
                ret = ORC_QPK_DECOMPRESSION_FAILED;
            } else {
                const qpk_entry_t *x = &t->e[t->num - 1 - (uint64_t)index];
                uint8_t *n = dup_bytes(x->name, x->nlen), *v = dup_bytes(x->value, x->vlen);
                qpk_insert(t, n, x->nlen, v, x->vlen, x->soft);
            }
        } break;
        case 1: { /* dynamic table size update (:469-474, :408-418) */
            int64_t max_size;
            if ((ret = qpk_int(&max_size, &src, end, 5)) != 0)
                goto Exit;
            if (max_size > (int64_t)t->header_table_size) {
                ret = ORC_QPK_DECOMPRESSION_FAILED;
            } else {
                t->max_size = (uint64_t)max_size;
                qpk_evict(t, 0);
            }
        } break;
        }
        done = src;
    }
Exit:
    if (ret == ORC_QPK_INCOMPLETE)
        ret = 0;
    if (ret == 0 && old_total != t->total_inserts)
        *insert_count = t->total_inserts;
    *consumed = (uint32_t)(done - in);
    return ret;
}

/* ---- field sections ---- */

typedef struct {
    const qpk_conn_t *t;
    int64_t req_insert_count, base_index;
} qpk_ctx_t;

typedef struct {
    uint8_t *arena;
    uint64_t cur, end;
} qpk_arena_t;

static int qpk_copy(qpk_arena_t *A, const uint8_t *s, uint32_t n, uint32_t *off)
{
    if (A->cur + n > A->end)
        return ORC_BLK_ARENA;
    memcpy(A->arena + A->cur, s, n);
    *off = (uint32_t)A->cur;
    A->cur += n;
    return 0;
}

/* parse_decode_context (qpack.c:754-799) */
static int qpk_parse_context(const qpk_conn_t *t, qpk_ctx_t *ctx, const uint8_t **src, const uint8_t *end)
{
    int64_t ric, delta;
    ctx->t = t;
    if (qpk_int(&ric, src, end, 8) != 0)
        return ORC_QPK_DECOMPRESSION_FAILED;
    if (ric > 0) {
        if (t->max_entries == 0)
            return ORC_QPK_DECOMPRESSION_FAILED;
        const uint32_t full_range = 2 * t->max_entries;
        uint64_t max_value = t->total_inserts + t->max_entries;
        uint64_t rounded = max_value / full_range * full_range;
        ric = (int64_t)((uint64_t)ric + rounded - 1); /* int64 += uint64: wraps as the reference's does */
        if ((uint64_t)ric > max_value) {
            if (ric <= (int64_t)full_range)
                return ORC_QPK_DECOMPRESSION_FAILED;
            ric -= full_range;
        }
        if (ric == 0)
            return ORC_QPK_DECOMPRESSION_FAILED;
        if (ric > QPK_QUICINT_MAX)
            return ORC_QPK_DECOMPRESSION_FAILED;
    }
    ctx->req_insert_count = ric;
    if (*src >= end)
        return ORC_QPK_DECOMPRESSION_FAILED;
    int sign = (**src & 0x80) != 0;
    if (qpk_int(&delta, src, end, 7) != 0)
        return ORC_QPK_DECOMPRESSION_FAILED;
    if (delta > QPK_QUICINT_MAX)
        return ORC_QPK_DECOMPRESSION_FAILED;
    ctx->base_index = sign == 0 ? ric + delta : ric - delta - 1;
    if (ctx->base_index < 0)
        return ORC_QPK_DECOMPRESSION_FAILED;
    return 0;
}

/* resolve_dynamic / resolve_dynamic_postbase (qpack.c:523-557) */
static const qpk_entry_t *qpk_dyn(const qpk_ctx_t *ctx, const uint8_t **src, const uint8_t *end, unsigned prefix,
                                  int postbase)
{
    int64_t off, index;
    if (qpk_int(&off, src, end, prefix) != 0)
        return NULL;
    if (postbase) {
        if (off > INT64_MAX - ctx->base_index - 1)
            return NULL;
        index = ctx->base_index + off + 1;
    } else {
        if (off >= ctx->base_index)
            return NULL;
        index = ctx->base_index - off;
    }
    if (ctx->req_insert_count < index)
        return NULL;
    return qpk_resolve_abs(ctx->t, index);
}

static int qpk_static(int64_t *index, const uint8_t **src, const uint8_t *end, unsigned prefix) /* resolve_static :506-521 */
{
    if (qpk_int(index, src, end, prefix) != 0 || (uint64_t)*index >= QPK_STATIC_COUNT)
        return -1;
    return 0;
}

/* decode_header_value_literal (qpack.c:603-629) into the arena */
static int qpk_value_literal(qpk_arena_t *A, unsigned *soft, const uint8_t **src, const uint8_t *end, uint32_t *off,
                             uint32_t *len)
{
    int64_t n;
    if (!(*src < end))
        return ORC_QPK_DECOMPRESSION_FAILED;
    int huff = (**src & 0x80) != 0;
    if (qpk_int(&n, src, end, 7) != 0)
        return ORC_QPK_DECOMPRESSION_FAILED;
    if (end - *src < n)
        return ORC_QPK_DECOMPRESSION_FAILED;
    if (huff) {
        if (A->cur + ((uint64_t)n * 8u) / 5u > A->end)
            return ORC_BLK_ARENA;
        size_t r = orc_decode_huffman((char *)A->arena + A->cur, soft, *src, (size_t)n, 0);
        if (r == SIZE_MAX)
            return ORC_QPK_DECOMPRESSION_FAILED;
        *len = (uint32_t)r;
    } else {
        orc_validate_header_value(soft, *src, (size_t)n);
        if (A->cur + (uint64_t)n > A->end)
            return ORC_BLK_ARENA;
        memcpy(A->arena + A->cur, *src, (size_t)n);
        *len = (uint32_t)n;
    }
    *off = (uint32_t)A->cur;
    A->cur += *len;
    *src += n;
    return 0;
}

/* decode_header_name_literal (qpack.c:559-601), prefix 3 */
static int qpk_name_literal(qpk_arena_t *A, unsigned *soft, const uint8_t **src, const uint8_t *end, uint32_t *off,
                            uint32_t *len)
{
    int64_t n;
    int huff = (**src >> 3) & 1;
    if (qpk_int(&n, src, end, 3) != 0)
        return ORC_QPK_DECOMPRESSION_FAILED;
    if (end - *src < n)
        return ORC_QPK_DECOMPRESSION_FAILED;
    if (huff) {
        if (A->cur + ((uint64_t)n * 8u) / 5u > A->end)
            return ORC_BLK_ARENA;
        size_t r = orc_decode_huffman((char *)A->arena + A->cur, soft, *src, (size_t)n, 1);
        if (r == SIZE_MAX)
            return ORC_QPK_DECOMPRESSION_FAILED;
        *len = (uint32_t)r;
    } else {
        /* tokens are returned as they are; anything else is validated (:583-588) */
        if (!orc_is_qpack_token(*src, (size_t)n) && !orc_validate_header_name(soft, *src, (size_t)n))
            return ORC_QPK_DECOMPRESSION_FAILED;
        if (A->cur + (uint64_t)n > A->end)
            return ORC_BLK_ARENA;
        memcpy(A->arena + A->cur, *src, (size_t)n);
        *len = (uint32_t)n;
    }
    *off = (uint32_t)A->cur;
    A->cur += *len;
    *src += n;
    return 0;
}

static int qpk_static_name(qpk_arena_t *A, int64_t si, uint32_t *noff, uint32_t *nlen)
{
    *nlen = (uint32_t)strlen(orc_qpack_static_name[si]);
    return qpk_copy(A, (const uint8_t *)orc_qpack_static_name[si], *nlen, noff);
}

/* decode_header (qpack.c:652-752): 0 / ORC_ERR_INVALID_CHAR = a field was produced */
static int qpk_field(const qpk_ctx_t *ctx, const uint8_t **src, const uint8_t *end, qpk_arena_t *A, uint32_t *noff,
                     uint32_t *nlen, uint32_t *voff, uint32_t *vlen, unsigned *soft_out)
{
    unsigned soft = 0;
    int64_t si;
    const qpk_entry_t *e;
    int r;
    const unsigned kind = **src >> 4;
    switch (kind) {
    case 12:
    case 13:
    case 14:
    case 15: /* indexed field line, static (:659-669) */
        if (qpk_static(&si, src, end, 6) != 0)
            return ORC_QPK_DECOMPRESSION_FAILED;
        if ((r = qpk_static_name(A, si, noff, nlen)) != 0)
            return r;
        *vlen = (uint32_t)strlen(orc_qpack_static_value[si]);
        if ((r = qpk_copy(A, (const uint8_t *)orc_qpack_static_value[si], *vlen, voff)) != 0)
            return r;
        break;
    case 8:
    case 9:
    case 10:
    case 11: /* indexed field line, dynamic (:670-682) */
    case 1:  /* indexed field line, post-base (:713-722) */
        if ((e = qpk_dyn(ctx, src, end, kind == 1 ? 4 : 6, kind == 1)) == NULL)
            return ORC_QPK_DECOMPRESSION_FAILED;
        if ((r = qpk_copy(A, e->name, e->nlen, noff)) != 0 || (r = qpk_copy(A, e->value, e->vlen, voff)) != 0)
            return r;
        *nlen = e->nlen;
        *vlen = e->vlen;
        soft = e->soft;
        break;
    case 5:
    case 7: /* literal, static name reference (:683-692) */
        if (qpk_static(&si, src, end, 4) != 0)
            return ORC_QPK_DECOMPRESSION_FAILED;
        if ((r = qpk_static_name(A, si, noff, nlen)) != 0)
            return r;
        if ((r = qpk_value_literal(A, &soft, src, end, voff, vlen)) != 0)
            return r;
        break;
    case 4:
    case 6: /* literal, dynamic name reference (:693-704) */
    case 0: /* literal, post-base name reference (:723-733) */
        if ((e = qpk_dyn(ctx, src, end, kind == 0 ? 3 : 4, kind == 0)) == NULL)
            return ORC_QPK_DECOMPRESSION_FAILED;
        if ((r = qpk_copy(A, e->name, e->nlen, noff)) != 0)
            return r;
        *nlen = e->nlen;
        soft = e->soft & ORC_SOFT_NAME;
        if ((r = qpk_value_literal(A, &soft, src, end, voff, vlen)) != 0)
            return r;
        break;
    default: /* 2, 3: literal without name reference (:705-712) */
        if ((r = qpk_name_literal(A, &soft, src, end, noff, nlen)) != 0)
            return r;
        if ((r = qpk_value_literal(A, &soft, src, end, voff, vlen)) != 0)
            return r;
        break;
    }
    *soft_out = soft;
    return soft ? ORC_ERR_INVALID_CHAR : 0;
}

/* ---- session API (ctypes) ---- */

void *orc_qpack_open(uint32_t nconn, uint32_t header_table_size, uint64_t max_blocked)
{
    qpk_session_t *s = (qpk_session_t *)calloc(1, sizeof(*s));
    s->nconn = nconn;
    s->max_blocked = max_blocked;
    s->c = (qpk_conn_t *)calloc(nconn ? nconn : 1, sizeof(qpk_conn_t));
    for (uint32_t c = 0; c < nconn; ++c) { /* h2o_qpack_create_decoder (qpack.c:240-252) */
        s->c[c].base_offset = 1;
        s->c[c].max_size = header_table_size;
        s->c[c].header_table_size = header_table_size;
        s->c[c].max_entries = header_table_size / 32;
    }
    return s;
}

void orc_qpack_close(void *h)
{
    qpk_session_t *s = (qpk_session_t *)h;
    for (uint32_t c = 0; c < s->nconn; ++c) {
        qpk_conn_t *t = &s->c[c];
        for (uint64_t k = 0; k < t->num; ++k) {
            free(t->e[k].name);
            free(t->e[k].value);
        }
        free(t->e);
    }
    free(s->c);
    free(s);
}

/* send_header_ack (qpack.c:642-649): 0x80 | stream_id as a 7-bit prefix integer (h2o_hpack_encode_int) */
static uint32_t qpk_header_ack(uint64_t stream_id, uint8_t *out)
{
    out[0] = 0x80;
    return (uint32_t)(orc_encode_int(out, (int64_t)stream_id, 7) - out);
}

/* One step for every connection c: its encoder-stream bytes in[enc_off[c], + enc_len[c]), then its field
 * sections conn_first[c] .. conn_first[c+1]-1 (section k = in[sec_off[k], sec_off[k+1])) against the table
 * as the encoder stream left it; num_blocked[c] (NULL = 0) is the caller's count of the connection's
 * blocked streams (h2o's conn->num_qpack_blocked, lib/http3/server.c:1544).  With req != NULL every section
 * goes through h2o_qpack_parse_request (qpack.c:830-858): h2o_hpack_parse_request's rules with the HTTP/3
 * arguments, normalize_error_code, send_header_ack; req = 18 u32 words per section: the hhuff_request_t
 * words, datagram_flow_id, ack_len, ack[16].  With res != NULL every section goes through
 * h2o_qpack_parse_response (qpack.c:860-882) as h2o's HTTP/3 client calls it (lib/common/http3client.c:542):
 * h2o_hpack_parse_response's rules on a response head with a datagram-flow-id out-parameter, the same
 * normalisation, and the acknowledgment only after a clean parse; res = 10 u32 words per section
 * (include/hhuff.h hhuff_qpack_response_head_t: status, nheaders, err, dfid, ack_len, 0, ack[16]). */
static int qpk_step(qpk_session_t *s, const uint8_t *in, const uint32_t *enc_off, const uint32_t *enc_len,
                    const uint32_t *sec_off, const uint32_t *conn_first, const uint32_t *num_blocked, uint8_t *arena,
                    const uint64_t *arena_off, uint32_t *name_off, uint32_t *name_len, uint32_t *value_off,
                    uint32_t *value_len, uint8_t *fflags, uint32_t *nfields, int32_t *sstatus, uint64_t *req_insert_count,
                    int32_t *enc_status, uint32_t *enc_consumed, uint64_t *insert_count, const uint64_t *stream_id,
                    uint32_t *req, uint32_t *res)
{
    for (uint32_t c = 0; c < s->nconn; ++c) {
        qpk_conn_t *t = &s->c[c];
        enc_status[c] = 0;
        enc_consumed[c] = 0;
        insert_count[c] = 0;
        if (t->failed) {
            enc_status[c] = ORC_BLK_SKIPPED;
        } else if (enc_len[c]) {
            int r = qpk_handle_input(t, in + enc_off[c], in + enc_off[c] + enc_len[c], &enc_consumed[c], &insert_count[c]);
            enc_status[c] = r;
            t->failed = r != 0;
        }
        /* h2o raises conn->num_qpack_blocked for every stream it parks (lib/http3/server.c:1553), so each
         * blocked section of this step counts against max_blocked for the sections after it */
        uint64_t nb = num_blocked ? num_blocked[c] : 0;
        for (uint32_t k = conn_first[c]; k < conn_first[c + 1]; ++k) {
            nfields[k] = 0;
            req_insert_count[k] = 0;
            orc_req_t rq;
            orc_resp_t rs;
            orc_rq_init(&rq);
            orc_rs_init(&rs, 0);
            int st = 0;
            qpk_ctx_t ctx = {t, 0, 0};
            uint32_t nf = 0;
            if (t->failed) {
                st = ORC_BLK_SKIPPED;
            } else {
                const uint8_t *p = in + sec_off[k], *end = in + sec_off[k + 1];
                st = qpk_parse_context(t, &ctx, &p, end);
                if (st == 0) {
                    req_insert_count[k] = (uint64_t)ctx.req_insert_count;
                    /* check_decode_context_blocked (:801-820) */
                    if (!(ctx.req_insert_count < qpk_table_total(t))) {
                        st = nb >= s->max_blocked ? ORC_QPK_DECOMPRESSION_FAILED : ORC_QPK_BLOCKED;
                        nb += st == ORC_QPK_BLOCKED;
                    }
                }
                uint32_t slot = sec_off[k];
                qpk_arena_t A = {arena, arena_off[k], arena_off[k + 1] < (1ull << 32) ? arena_off[k + 1] : (1ull << 32)};
                if (res && st == 0 && p == end) { /* no :status (hpack.c:652-655), normalised (:877-878) */
                    rs.err = 9;
                    st = ORC_QPK_DECOMPRESSION_FAILED;
                }
                while (st == 0 && p != end) {
                    uint32_t no = 0, nl = 0, vo = 0, vl = 0;
                    unsigned soft = 0;
                    int rc = qpk_field(&ctx, &p, end, &A, &no, &nl, &vo, &vl, &soft);
                    if (rc != 0 && rc != ORC_ERR_INVALID_CHAR) {
                        st = rc;
                        rq.err = rc == ORC_BLK_ARENA ? 0 : 8; /* HHUFF_HERR_DECODE: decode_header's own error */
                        rs.err = rq.err;
                        break;
                    }
                    int header = 0, rr = 0;
                    if (req)
                        rr = orc_rq_field(&rq, arena + no, nl, arena + vo, vl, soft, (int32_t)nf, &header, 1);
                    if (res)
                        rr = orc_rs_field(&rs, arena + no, nl, arena + vo, vl, soft, (int32_t)nf, &header, 1);
                    name_off[slot + nf] = no;
                    name_len[slot + nf] = nl;
                    value_off[slot + nf] = vo;
                    value_len[slot + nf] = vl;
                    fflags[slot + nf] = (uint8_t)(soft | (header ? 4u : 0u));
                    ++nf;
                    if (rr != 0) { /* normalize_error_code (:822-828) */
                        st = ORC_QPK_DECOMPRESSION_FAILED;
                        break;
                    }
                }
                if (req && st == 0 && rq.err != 0)
                    st = ORC_ERR_INVALID_CHAR; /* hpack.c:636-637 */
                if (res && st == 0 && rs.err != 0)
                    st = ORC_ERR_INVALID_CHAR; /* hpack.c:745-747 */
            }
            nfields[k] = nf;
            sstatus[k] = st;
            if (req) {
                uint32_t *w = req + 18 * (size_t)k;
                orc_rq_store(w, &rq);
                w[12] = (uint32_t)rq.dfid;
                uint8_t ack[16] = {0};
                w[13] = (st == 0 || st == ORC_ERR_INVALID_CHAR) && ctx.req_insert_count != 0
                            ? qpk_header_ack(stream_id[k], ack) : 0;
                memcpy(w + 14, ack, 16);
            }
            if (res) {
                uint32_t *w = res + 10 * (size_t)k;
                orc_rs_store(w, &rs);
                uint8_t ack[16] = {0};
                w[4] = st == 0 && ctx.req_insert_count != 0 ? qpk_header_ack(stream_id[k], ack) : 0;
                w[5] = 0;
                memcpy(w + 6, ack, 16);
            }
        }
    }
    return 0;
}

int orc_qpack_step(void *h, const uint8_t *in, const uint32_t *enc_off, const uint32_t *enc_len, const uint32_t *sec_off,
                   const uint32_t *conn_first, const uint32_t *num_blocked, uint8_t *arena, const uint64_t *arena_off,
                   uint32_t *name_off, uint32_t *name_len, uint32_t *value_off, uint32_t *value_len, uint8_t *fflags,
                   uint32_t *nfields, int32_t *sstatus, uint64_t *req_insert_count, int32_t *enc_status,
                   uint32_t *enc_consumed, uint64_t *insert_count)
{
    return qpk_step((qpk_session_t *)h, in, enc_off, enc_len, sec_off, conn_first, num_blocked, arena, arena_off, name_off,
                    name_len, value_off, value_len, fflags, nfields, sstatus, req_insert_count, enc_status, enc_consumed,
                    insert_count, NULL, NULL, NULL);
}

int orc_qpack_step_req(void *h, const uint8_t *in, const uint32_t *enc_off, const uint32_t *enc_len,
                       const uint32_t *sec_off, const uint32_t *conn_first, const uint32_t *num_blocked, uint8_t *arena,
                       const uint64_t *arena_off, uint32_t *name_off, uint32_t *name_len, uint32_t *value_off,
                       uint32_t *value_len, uint8_t *fflags, uint32_t *nfields, int32_t *sstatus,
                       uint64_t *req_insert_count, int32_t *enc_status, uint32_t *enc_consumed, uint64_t *insert_count,
                       const uint64_t *stream_id, uint32_t *req)
{
    return qpk_step((qpk_session_t *)h, in, enc_off, enc_len, sec_off, conn_first, num_blocked, arena, arena_off, name_off,
                    name_len, value_off, value_len, fflags, nfields, sstatus, req_insert_count, enc_status, enc_consumed,
                    insert_count, stream_id, req, NULL);
}

int orc_qpack_step_resp(void *h, const uint8_t *in, const uint32_t *enc_off, const uint32_t *enc_len,
                        const uint32_t *sec_off, const uint32_t *conn_first, const uint32_t *num_blocked, uint8_t *arena,
                        const uint64_t *arena_off, uint32_t *name_off, uint32_t *name_len, uint32_t *value_off,
                        uint32_t *value_len, uint8_t *fflags, uint32_t *nfields, int32_t *sstatus,
                        uint64_t *req_insert_count, int32_t *enc_status, uint32_t *enc_consumed, uint64_t *insert_count,
                        const uint64_t *stream_id, uint32_t *res)
{
    return qpk_step((qpk_session_t *)h, in, enc_off, enc_len, sec_off, conn_first, num_blocked, arena, arena_off, name_off,
                    name_len, value_off, value_len, fflags, nfields, sstatus, req_insert_count, enc_status, enc_consumed,
                    insert_count, stream_id, NULL, res);
}
