/*
 * ORACLE -- TEST INFRASTRUCTURE ONLY.  Clean-room CPU restatement of HPACK header-block decoding
 * (SURVEY.md 8 f4): h2o_hpack_decode_header (lib/http2/hpack.c:319-435) applied field after field over
 * each header block the way h2o_hpack_parse_request loops over it (hpack.c:513-527), with one dynamic
 * table per connection (header_table_add :277-317, header_table_evict_one :263-275, size updates
 * :352-366).  Strings go through decode_string's semantics (hpack.c:223-261), restated in
 * huff_oracle.c.  Output contract: include/hhuff.h hhuff_hpack_decode_blocks.
 */
#include <pthread.h>
#include <stdlib.h>
#include <string.h>
#include <strings.h>

#include "huff_oracle.h"
#include "huff_tables.h"
#include "orc_request.h"

#define ENTRY_OVERHEAD 32u /* HEADER_TABLE_ENTRY_SIZE_OFFSET, hpack.c:30 */
#define STATIC_COUNT 61u   /* HEADER_TABLE_OFFSET - 1, hpack.c:27 */

typedef struct {
    uint8_t *name, *value;
    uint32_t nlen, vlen;
    unsigned soft;
} orc_entry_t;

typedef struct {
    orc_entry_t *e; /* e[0] is the newest entry (dynamic index 62) */
    uint32_t num, cap_entries;
    uint64_t size, capacity, max_capacity;
} orc_table_t;

static void tbl_evict_one(orc_table_t *t)
{
    orc_entry_t *x = &t->e[--t->num];
    t->size -= (uint64_t)x->nlen + x->vlen + ENTRY_OVERHEAD;
    free(x->name);
    free(x->value);
    memset(x, 0, sizeof(*x));
}

/* header_table_add with max_num_entries = SIZE_MAX (hpack.c:413) */
static void tbl_add(orc_table_t *t, const uint8_t *name, uint32_t nlen, const uint8_t *value, uint32_t vlen,
                    unsigned soft)
{
    uint64_t add = (uint64_t)nlen + vlen + ENTRY_OVERHEAD;
    while (t->num != 0 && t->size + add > t->capacity)
        tbl_evict_one(t);
    if (t->num == 0 && add > t->capacity)
        return; /* does not fit an empty table: not added */
    if (t->num == t->cap_entries) {
        uint32_t nc = t->cap_entries ? 2 * t->cap_entries : 16;
        t->e = (orc_entry_t *)realloc(t->e, nc * sizeof(orc_entry_t));
        t->cap_entries = nc;
    }
    memmove(t->e + 1, t->e, t->num * sizeof(orc_entry_t));
    orc_entry_t *x = &t->e[0];
    x->name = (uint8_t *)malloc(nlen + 1);
    x->value = (uint8_t *)malloc(vlen + 1);
    memcpy(x->name, name, nlen);
    memcpy(x->value, value, vlen);
    x->nlen = nlen;
    x->vlen = vlen;
    x->soft = soft;
    t->size += add;
    ++t->num;
}

static void tbl_free(orc_table_t *t)
{
    while (t->num)
        tbl_evict_one(t);
    free(t->e);
}

typedef struct {
    uint8_t *arena;
    uint64_t cur, end;
} orc_arena_t;

enum { STR_OK = 0, STR_FAIL = 1, STR_UPPER = 2, STR_ARENA = 3 };

/* decode_string (hpack.c:223-261) into the arena; *off / *len the decoded bytes */
static int orc_block_string(const uint8_t **src, const uint8_t *end, int is_name, unsigned *soft, orc_arena_t *A,
                            uint32_t *off, uint32_t *len)
{
    if (*src >= end)
        return STR_FAIL;
    int huff = (**src & 0x80) != 0;
    int64_t n = orc_decode_int(src, end, 7);
    if (n < 0 || n > end - *src)
        return STR_FAIL;
    if (huff) {
        if (A->cur + ((uint64_t)n * 8u) / 5u > A->end)
            return STR_ARENA;
        size_t r = orc_decode_huffman((char *)A->arena + A->cur, soft, *src, (size_t)n, is_name);
        if (r == SIZE_MAX)
            return STR_FAIL;
        *len = (uint32_t)r;
    } else {
        if (is_name) {
            if ((n == 0 || **src != ':') && !orc_validate_header_name(soft, *src, (size_t)n))
                return STR_UPPER;
        } else {
            orc_validate_header_value(soft, *src, (size_t)n);
        }
        if (A->cur + (uint64_t)n > A->end)
            return STR_ARENA;
        memcpy(A->arena + A->cur, *src, (size_t)n);
        *len = (uint32_t)n;
    }
    *off = (uint32_t)A->cur;
    A->cur += *len;
    *src += n;
    return STR_OK;
}

static int orc_block_copy(orc_arena_t *A, const uint8_t *s, uint32_t n, uint32_t *off)
{
    if (A->cur + n > A->end)
        return STR_ARENA;
    memcpy(A->arena + A->cur, s, n);
    *off = (uint32_t)A->cur;
    A->cur += n;
    return STR_OK;
}

/* one field (h2o_hpack_decode_header, hpack.c:319-435): 0 / ORC_ERR_INVALID_CHAR = a field was
 * produced; otherwise a hard error (ORC_ERR_COMPRESSION / ORC_ERR_PROTOCOL / ORC_BLK_ARENA) */
static int orc_block_field(orc_table_t *t, const uint8_t **src, const uint8_t *end, orc_arena_t *A, uint32_t *noff,
                           uint32_t *nlen, uint32_t *voff, uint32_t *vlen, unsigned *soft_out)
{
    int64_t index = 0;
    int value_indexed = 0, do_index = 0;
    for (;;) {
        if (*src >= end)
            return ORC_ERR_COMPRESSION;
        uint8_t b = **src;
        if (b >= 128) { /* indexed */
            if ((index = orc_decode_int(src, end, 7)) <= 0)
                return ORC_ERR_COMPRESSION;
            value_indexed = 1;
        } else if (b >= 64) { /* literal with incremental indexing */
            if (b == 64)
                ++*src;
            else if ((index = orc_decode_int(src, end, 6)) <= 0)
                return ORC_ERR_COMPRESSION;
            do_index = 1;
        } else if (b < 32) { /* literal without indexing / never indexed */
            if ((b & 0xf) == 0)
                ++*src;
            else if ((index = orc_decode_int(src, end, 4)) <= 0)
                return ORC_ERR_COMPRESSION;
        } else { /* dynamic table size update */
            int64_t cap = orc_decode_int(src, end, 5);
            if (cap < 0 || (uint64_t)cap > t->max_capacity)
                return ORC_ERR_COMPRESSION;
            t->capacity = (uint64_t)cap;
            while (t->num != 0 && t->size > t->capacity)
                tbl_evict_one(t);
            continue;
        }
        break;
    }
    unsigned soft = 0;
    int r;
    const orc_entry_t *ent = NULL;
    if (index > 0) {
        if ((uint64_t)index <= STATIC_COUNT) {
            const char *n = orc_static_name[index];
            if ((r = orc_block_copy(A, (const uint8_t *)n, (uint32_t)strlen(n), noff)) != STR_OK)
                return ORC_BLK_ARENA;
            *nlen = (uint32_t)strlen(n);
            if (value_indexed) {
                const char *v = orc_static_value[index];
                if ((r = orc_block_copy(A, (const uint8_t *)v, (uint32_t)strlen(v), voff)) != STR_OK)
                    return ORC_BLK_ARENA;
                *vlen = (uint32_t)strlen(v);
            }
        } else if ((uint64_t)index - STATIC_COUNT - 1 < t->num) {
            ent = &t->e[index - STATIC_COUNT - 1];
            soft = ent->soft;
            if (orc_block_copy(A, ent->name, ent->nlen, noff) != STR_OK)
                return ORC_BLK_ARENA;
            *nlen = ent->nlen;
            if (value_indexed) {
                if (orc_block_copy(A, ent->value, ent->vlen, voff) != STR_OK)
                    return ORC_BLK_ARENA;
                *vlen = ent->vlen;
            }
        } else {
            return ORC_ERR_COMPRESSION;
        }
    } else {
        r = orc_block_string(src, end, 1, &soft, A, noff, nlen);
        if (r == STR_ARENA)
            return ORC_BLK_ARENA;
        if (r != STR_OK)
            return r == STR_UPPER ? ORC_ERR_PROTOCOL : ORC_ERR_COMPRESSION;
    }
    if (!value_indexed) {
        soft &= ~ORC_SOFT_VALUE;
        r = orc_block_string(src, end, 0, &soft, A, voff, vlen);
        if (r == STR_ARENA)
            return ORC_BLK_ARENA;
        if (r != STR_OK)
            return ORC_ERR_COMPRESSION;
    }
    if (do_index)
        tbl_add(t, A->arena + *noff, *nlen, A->arena + *voff, *vlen, soft);
    *soft_out = soft;
    return soft ? ORC_ERR_INVALID_CHAR : 0;
}

/* ---- h2o_hpack_parse_request (hpack.c:502-637) as h2o's HTTP/2 server calls it (connection.c:626-629) ----
 * The request record is include/hhuff.h hhuff_request_t, 12 u32 words: [0..1] content_length, [2..7]
 * method, scheme, authority, path, protocol, expect (field index or -1), [8] exists map, [9] nheaders,
 * [10] err (HHUFF_HERR_*), [11] scheme kind. */
enum {
    RQ_REGULAR, RQ_AUTHORITY, RQ_METHOD, RQ_PATH, RQ_PROTOCOL, RQ_SCHEME, RQ_CONTENT_LENGTH, RQ_EXPECT, RQ_HOST, RQ_TE,
    RQ_CACHE_DIGEST, RQ_DATAGRAM_FLOW_ID, RQ_REJECT
};
/* the tokens parse_request tells apart: the pseudo-header tokens and the is_hpack_special ones
 * (lib/common/token_table.h, 5th flag) */
static const struct {
    const char *name;
    int kind;
} rq_tokens[] = {{":authority", RQ_AUTHORITY}, {":method", RQ_METHOD}, {":path", RQ_PATH}, {":protocol", RQ_PROTOCOL},
                 {":scheme", RQ_SCHEME}, {"cache-digest", RQ_CACHE_DIGEST}, {"connection", RQ_REJECT},
                 {"content-length", RQ_CONTENT_LENGTH}, {"datagram-flow-id", RQ_DATAGRAM_FLOW_ID},
                 {"expect", RQ_EXPECT}, {"host", RQ_HOST}, {"http2-settings", RQ_REJECT}, {"te", RQ_TE},
                 {"transfer-encoding", RQ_REJECT}, {"upgrade", RQ_REJECT}};

static int rq_kind(const uint8_t *s, uint32_t n)
{
    for (size_t i = 0; i < sizeof(rq_tokens) / sizeof(rq_tokens[0]); ++i)
        if (strlen(rq_tokens[i].name) == n && memcmp(rq_tokens[i].name, s, n) == 0)
            return rq_tokens[i].kind;
    return RQ_REGULAR;
}

/* h2o_strtosize (lib/common/string.c:86-113) */
static uint64_t rq_strtosize(const uint8_t *s, uint32_t n)
{
    uint64_t v = 0, m = 1;
    if (n == 0)
        return UINT64_MAX;
    for (uint32_t i = n; i-- > 0;) {
        if (s[i] < '0' || s[i] > '9')
            return UINT64_MAX;
        v += (uint64_t)(s[i] - '0') * m;
        if (i == 0)
            break;
        m *= 10;
        if (m == 10000000000000000000ull)
            return UINT64_MAX;
    }
    return v;
}

void orc_rq_init(orc_req_t *r)
{
    memset(r, 0, sizeof(*r));
    r->content_length = UINT64_MAX;
    for (int i = 0; i < 6; ++i)
        r->slot[i] = -1;
    r->dfid = -1;
    r->pseudo_ok = 1;
}

void orc_rq_store(uint32_t *w, const orc_req_t *r)
{
    memcpy(w, &r->content_length, 8);
    memcpy(w + 2, r->slot, 24);
    w[8] = r->map, w[9] = r->nheaders, w[10] = r->err, w[11] = r->scheme_kind;
}

/* field k decoded with soft bits `soft`: 0, or the hard error; *header = h2o_add_header took it.  h3: the
 * arguments of h2o's HTTP/3 server (lib/http3/server.c:1540-1545): digests == NULL (a cache-digest field is
 * rejected, hpack.c:606-617) and a datagram-flow-id out-parameter (the field is stored, :610-613) */
int orc_rq_field(orc_req_t *r, const uint8_t *name, uint32_t nl, const uint8_t *value, uint32_t vl, unsigned soft,
                 int32_t k, int *header, int h3)
{
    enum { M = 0, S = 1, A = 2, P = 3, PR = 4, E = 5 };
    *header = 0;
    if (soft && r->err == 0)
        r->err = (soft & ORC_SOFT_NAME) ? 1 : 2;
    if (++r->ndecoded > 1000) { /* H2O_HPACK_MAX_HEADERS_HARD_LIMIT */
        r->err = 3;
        return ORC_ERR_COMPRESSION;
    }
    int kind = rq_kind(name, nl);
    if (nl > 0 && name[0] == ':') {
        if (!r->pseudo_ok) {
            r->err = 4;
            return ORC_ERR_PROTOCOL;
        }
        int which, bit;
        switch (kind) {
        case RQ_AUTHORITY: which = A, bit = 8; break;
        case RQ_METHOD: which = M, bit = 1; break;
        case RQ_PATH: which = P, bit = 4; break;
        case RQ_SCHEME: which = S, bit = 2; break;
        case RQ_PROTOCOL:
            if (r->slot[PR] >= 0)
                return ORC_ERR_PROTOCOL; /* no err_desc */
            r->slot[PR] = k, r->map |= 16;
            return 0;
        default:
            return ORC_ERR_PROTOCOL; /* unknown pseudo-header: no err_desc */
        }
        if (r->slot[which] >= 0 || (which == P && vl == 0)) {
            r->err = 4;
            return ORC_ERR_PROTOCOL;
        }
        r->slot[which] = k, r->map |= (uint32_t)bit;
        if (which == S)
            r->scheme_kind = (vl == 5 && memcmp(value, "https", 5) == 0) ? 2 : (vl == 6 && memcmp(value, "masque", 6) == 0) ? 3 : 1;
        return 0;
    }
    r->pseudo_ok = 0;
    switch (kind) {
    case RQ_CONTENT_LENGTH:
        if ((r->content_length = rq_strtosize(value, vl)) == UINT64_MAX) {
            r->err = 5;
            return ORC_ERR_PROTOCOL;
        }
        return 0;
    case RQ_EXPECT:
        r->slot[E] = k;
        return 0;
    case RQ_HOST:
        if (r->slot[A] < 0)
            r->slot[A] = k;
        return 0;
    case RQ_DATAGRAM_FLOW_ID:
        if (h3)
            r->dfid = k;
        return 0;
    case RQ_CACHE_DIGEST:
        if (h3) {
            r->err = 6;
            return ORC_ERR_PROTOCOL;
        }
        break;
    case RQ_TE:
        if (vl == 8 && strncasecmp((const char *)value, "trailers", 8) == 0)
            break;
        r->err = 6;
        return ORC_ERR_PROTOCOL;
    case RQ_REJECT:
        r->err = 6;
        return ORC_ERR_PROTOCOL;
    default:
        break;
    }
    if (r->nheaders < 100) { /* H2O_MAX_HEADERS */
        ++r->nheaders;
        *header = 1;
    } else if (r->err == 0) {
        r->err = 3;
    }
    return 0;
}

void orc_rs_init(orc_resp_t *r, int trailers)
{
    memset(r, 0, sizeof(*r));
    r->dfid = -1;
    r->trailers = trailers;
}

void orc_rs_store(uint32_t *w, const orc_resp_t *r)
{
    w[0] = (uint32_t)r->status, w[1] = r->nheaders, w[2] = r->err, w[3] = (uint32_t)r->dfid;
}

/* h2o_hpack_parse_response (hpack.c:642-750) for field k: 0 or the hard error; *header = listed.  h3: a
 * datagram-flow-id out-parameter (lib/common/http3client.c:542); HTTP/2's client passes NULL (http2client.c:332) */
int orc_rs_field(orc_resp_t *r, const uint8_t *name, uint32_t nl, const uint8_t *value, uint32_t vl, unsigned soft,
                 int32_t k, int *header, int h3)
{
    *header = 0;
    if (soft && r->err == 0)
        r->err = (soft & ORC_SOFT_NAME) ? 1 : 2;
    if (++r->ndecoded > 1000) { /* :668-671 */
        r->err = 3;
        return ORC_ERR_COMPRESSION;
    }
    if (nl > 0 && name[0] == ':') { /* :672-704 */
        if (r->trailers || !(nl == 7 && memcmp(name, ":status", 7) == 0) || r->status != 0 || vl != 3) {
            r->err = 4;
            return ORC_ERR_PROTOCOL;
        }
        static const int mul[3] = {100, 10, 1};
        for (int i = 0; i < 3; ++i) { /* PARSE_DIGIT: each digit is added before the next is looked at */
            if (value[i] < '0' + (i == 0 ? 1 : 0) || value[i] > '9') {
                r->err = 4;
                return ORC_ERR_PROTOCOL;
            }
            r->status += (value[i] - '0') * mul[i];
        }
        return 0;
    }
    if (!r->trailers && r->status == 0) { /* :706-709 */
        r->err = 9;
        return ORC_ERR_PROTOCOL;
    }
    switch (rq_kind(name, nl)) { /* the is_hpack_special tokens, :712-725 */
    case RQ_CONTENT_LENGTH:
    case RQ_CACHE_DIGEST:
    case RQ_HOST:
        break;
    case RQ_DATAGRAM_FLOW_ID:
        if (h3)
            r->dfid = k;
        return 0;
    case RQ_EXPECT:
    case RQ_TE:
    case RQ_REJECT:
        r->err = 6;
        return ORC_ERR_PROTOCOL;
    default:
        break;
    }
    if (r->nheaders < 100) {
        ++r->nheaders;
        *header = 1;
    } else if (r->err == 0) {
        r->err = 3;
    }
    return 0;
}

typedef struct {
    const uint8_t *in;
    const uint32_t *blk_off, *conn_first;
    uint32_t c_begin, c_end, table_size;
    uint8_t *arena;
    const uint64_t *arena_off;
    uint32_t *name_off, *name_len, *value_off, *value_len, *nfields;
    uint8_t *fflags;
    int32_t *bstatus;
    uint32_t *req; /* request mode: 12 words per block, else NULL */
    uint32_t *res; /* response mode: 4 words per block, else NULL */
    const uint8_t *trailers; /* response mode: nonzero = a trailers block (NULL: none) */
} orc_blk_job_t;

static void orc_hpack_connection(const orc_blk_job_t *j, uint32_t c)
{
    orc_table_t t = {NULL, 0, 0, 0, j->table_size, j->table_size};
    int failed = 0;
    for (uint32_t b = j->conn_first[c]; b < j->conn_first[c + 1]; ++b) {
        orc_req_t rq;
        orc_resp_t rs;
        orc_rq_init(&rq);
        orc_rs_init(&rs, j->trailers != NULL && j->trailers[b] != 0);
        j->nfields[b] = 0;
        if (failed) {
            j->bstatus[b] = ORC_BLK_SKIPPED;
            if (j->req)
                orc_rq_store(j->req + 12 * (size_t)b, &rq);
            if (j->res)
                orc_rs_store(j->res + 4 * (size_t)b, &rs);
            continue;
        }
        const uint8_t *p = j->in + j->blk_off[b], *end = j->in + j->blk_off[b + 1];
        /* field offsets are u32: arena bytes at or past 2^32 are out of reach (include/hhuff.h) */
        orc_arena_t A = {j->arena, j->arena_off[b], j->arena_off[b + 1] < (1ull << 32) ? j->arena_off[b + 1] : (1ull << 32)};
        uint32_t nf = 0, slot = j->blk_off[b];
        int st = 0;
        if (j->res && p == end) { /* a head needs :status (hpack.c:652-655); empty trailers: decode_header (:328-329) */
            if (!rs.trailers)
                rs.err = 9;
            st = rs.trailers ? ORC_ERR_COMPRESSION : ORC_ERR_PROTOCOL;
        }
        while (st == 0 && p != end) {
            uint32_t no = 0, nl = 0, vo = 0, vl = 0;
            unsigned soft = 0;
            int rc = orc_block_field(&t, &p, end, &A, &no, &nl, &vo, &vl, &soft);
            if (rc != 0 && rc != ORC_ERR_INVALID_CHAR) {
                st = rc;
                rq.err = rc == ORC_ERR_PROTOCOL ? 7 : 0; /* *err_desc = decode_err (hpack.c:523-525, :663-665) */
                rs.err = rq.err;
                break;
            }
            int header = 0, rr = 0;
            if (j->req)
                rr = orc_rq_field(&rq, j->arena + no, nl, j->arena + vo, vl, soft, (int32_t)nf, &header, 0);
            if (j->res)
                rr = orc_rs_field(&rs, j->arena + no, nl, j->arena + vo, vl, soft, (int32_t)nf, &header, 0);
            j->name_off[slot + nf] = no;
            j->name_len[slot + nf] = nl;
            j->value_off[slot + nf] = vo;
            j->value_len[slot + nf] = vl;
            j->fflags[slot + nf] = (uint8_t)(soft | (header ? 4u : 0u));
            ++nf;
            if (rr != 0) {
                st = rr;
                break;
            }
        }
        if (j->req) {
            if (st == 0 && rq.err != 0)
                st = ORC_ERR_INVALID_CHAR; /* hpack.c:636-637 */
            orc_rq_store(j->req + 12 * (size_t)b, &rq);
        }
        if (j->res) {
            if (st == 0 && rs.err != 0)
                st = ORC_ERR_INVALID_CHAR; /* hpack.c:745-747 */
            orc_rs_store(j->res + 4 * (size_t)b, &rs);
        }
        j->nfields[b] = nf;
        j->bstatus[b] = st;
        failed = st != 0 && st != ORC_ERR_INVALID_CHAR;
    }
    tbl_free(&t);
}

static void *orc_blk_worker(void *arg)
{
    const orc_blk_job_t *j = (const orc_blk_job_t *)arg;
    for (uint32_t c = j->c_begin; c < j->c_end; ++c)
        orc_hpack_connection(j, c);
    return NULL;
}

static int orc_hpack_blocks(const uint8_t *in, const uint32_t *blk_off, const uint32_t *conn_first, uint32_t nconn,
                            uint32_t table_size, uint8_t *arena, const uint64_t *arena_off, uint32_t *name_off,
                            uint32_t *name_len, uint32_t *value_off, uint32_t *value_len, uint8_t *fflags,
                            uint32_t *nfields, int32_t *bstatus, uint32_t *req, uint32_t *res, const uint8_t *trailers,
                            int nthreads)
{
    if (nthreads < 1)
        nthreads = 1;
    if ((uint32_t)nthreads > nconn)
        nthreads = nconn ? (int)nconn : 1;
    orc_blk_job_t *jobs = (orc_blk_job_t *)calloc((size_t)nthreads, sizeof(*jobs));
    pthread_t *th = (pthread_t *)calloc((size_t)nthreads, sizeof(*th));
    if (!jobs || !th) {
        free(jobs);
        free(th);
        return -1;
    }
    for (int k = 0; k < nthreads; ++k) {
        orc_blk_job_t *j = &jobs[k];
        j->in = in, j->blk_off = blk_off, j->conn_first = conn_first, j->table_size = table_size;
        j->arena = arena, j->arena_off = arena_off, j->name_off = name_off, j->name_len = name_len;
        j->value_off = value_off, j->value_len = value_len, j->fflags = fflags, j->nfields = nfields;
        j->bstatus = bstatus, j->req = req, j->res = res, j->trailers = trailers;
        j->c_begin = (uint32_t)(((uint64_t)nconn * k) / nthreads);
        j->c_end = (uint32_t)(((uint64_t)nconn * (k + 1)) / nthreads);
    }
    for (int k = 1; k < nthreads; ++k)
        pthread_create(&th[k], NULL, orc_blk_worker, &jobs[k]);
    orc_blk_worker(&jobs[0]);
    for (int k = 1; k < nthreads; ++k)
        pthread_join(th[k], NULL);
    free(jobs);
    free(th);
    return 0;
}

int orc_hpack_decode_blocks(const uint8_t *in, const uint32_t *blk_off, const uint32_t *conn_first, uint32_t nconn,
                            uint32_t table_size, uint8_t *arena, const uint64_t *arena_off, uint32_t *name_off,
                            uint32_t *name_len, uint32_t *value_off, uint32_t *value_len, uint8_t *fflags,
                            uint32_t *nfields, int32_t *bstatus, int nthreads)
{
    return orc_hpack_blocks(in, blk_off, conn_first, nconn, table_size, arena, arena_off, name_off, name_len, value_off,
                            value_len, fflags, nfields, bstatus, NULL, NULL, NULL, nthreads);
}

int orc_hpack_parse_requests(const uint8_t *in, const uint32_t *blk_off, const uint32_t *conn_first, uint32_t nconn,
                             uint32_t table_size, uint8_t *arena, const uint64_t *arena_off, uint32_t *name_off,
                             uint32_t *name_len, uint32_t *value_off, uint32_t *value_len, uint8_t *fflags,
                             uint32_t *nfields, int32_t *bstatus, uint32_t *req, int nthreads)
{
    return orc_hpack_blocks(in, blk_off, conn_first, nconn, table_size, arena, arena_off, name_off, name_len, value_off,
                            value_len, fflags, nfields, bstatus, req, NULL, NULL, nthreads);
}

int orc_hpack_parse_responses(const uint8_t *in, const uint32_t *blk_off, const uint32_t *conn_first, uint32_t nconn,
                              uint32_t table_size, const uint8_t *trailers, uint8_t *arena, const uint64_t *arena_off,
                              uint32_t *name_off, uint32_t *name_len, uint32_t *value_off, uint32_t *value_len,
                              uint8_t *fflags, uint32_t *nfields, int32_t *bstatus, uint32_t *res, int nthreads)
{
    return orc_hpack_blocks(in, blk_off, conn_first, nconn, table_size, arena, arena_off, name_off, name_len, value_off,
                            value_len, fflags, nfields, bstatus, NULL, res, trailers, nthreads);
}
