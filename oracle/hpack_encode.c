/*
 * ORACLE -- TEST INFRASTRUCTURE ONLY.  Clean-room CPU restatement of h2o's HTTP/2 response encoder
 * (encode half), the contract of include/hhuff.h hhuff_hpack_flatten_responses:
 *   lib/http2/hpack.c  header_table_evict_one :263-275, header_table_add :277-317 (called with at most 32
 *                      entries, :921), encode_status :437-466, encode_content_length :468-485,
 *                      h2o_hpack_encode_int :757-772, encode_as_is :806-814, h2o_hpack_encode_string
 *                      :816-837 (Huffman through orc_encode_huffman, huff_oracle.c), header_table_adjust_size
 *                      :839-856, do_encode_header :858-937, encode_header :939-942, encode_header_token
 *                      :944-948, encode_method / encode_scheme / encode_path :950-985, fixup_frame_headers
 *                      :1012-1042, h2o_hpack_flatten_request :1044-1096 (the client side, called by
 *                      lib/common/http2client.c:1140), h2o_hpack_flatten_response :1137-1177,
 *                      h2o_hpack_flatten_trailers :1179-1196
 *   lib/http2/frame.c  h2o_http2_encode_frame_header :68-79
 *   lib/http2/connection.c:1847  a connection's encoder table starts with hpack_capacity 4096
 *   lib/common/token_table.h     the token flags do_encode_header reads: http2_static_table_name_index (the
 *                      first static-table entry with the token's name, 0 for tokens outside the static table)
 *                      and dont_compress (set for cookie and set-cookie only)
 * h2o compares a token name with a table entry's name by pointer (:870-872) and any other name by bytes
 * (:873-877); a name is a token exactly when its bytes are a token's, so an entry remembers whether it was
 * added under a token and a token name matches only such entries with equal bytes.
 * Pinned by oracle/ref_hpenc.c, which runs the real h2o_hpack_flatten_response / _trailers over the same
 * responses (tests/test_hpenc.py, tests/golden/hpenc.npz).
 */
#include <stdlib.h>
#include <string.h>

#include "huff_oracle.h"
#include "huff_tables.h"

#define ENTRY_OVERHEAD 32u    /* HEADER_TABLE_ENTRY_SIZE_OFFSET, hpack.c:30 */
#define TABLE_OFFSET 62u      /* HEADER_TABLE_OFFSET, hpack.c:29 */
#define MAX_ENTRIES 32u       /* header_table_add(..., 32), hpack.c:921 */
#define INITIAL_CAPACITY 4096 /* connection.c:1847 */

typedef struct {
    uint8_t *name, *value;
    uint32_t nlen, vlen;
    int token;
} hpe_entry_t;

typedef struct {
    hpe_entry_t e[MAX_ENTRIES]; /* e[0] is the newest (index 62) */
    uint32_t num;
    uint64_t size, capacity;
    int failed;
} hpe_table_t;

typedef struct {
    uint32_t nconn;
    hpe_table_t *t;
} hpe_session_t;

static void hpe_evict_one(hpe_table_t *t) /* hpack.c:263-275 */
{
    hpe_entry_t *x = &t->e[--t->num];
    t->size -= x->nlen + x->vlen + ENTRY_OVERHEAD;
    free(x->name);
    free(x->value);
    memset(x, 0, sizeof(*x));
}

/* header_table_add (hpack.c:277-317) with max_num_entries 32, then the copies of :922-933 */
static void hpe_add(hpe_table_t *t, const uint8_t *n, uint32_t nl, const uint8_t *v, uint32_t vl, int token)
{
    uint64_t add = (uint64_t)nl + vl + ENTRY_OVERHEAD;
    while (t->num != 0 && t->size + add > t->capacity)
        hpe_evict_one(t);
    while (MAX_ENTRIES <= t->num)
        hpe_evict_one(t);
    if (t->num == 0 && add > t->capacity)
        return;
    t->size += add;
    memmove(&t->e[1], &t->e[0], t->num * sizeof(hpe_entry_t));
    hpe_entry_t *x = &t->e[0];
    x->name = malloc(nl + 1);
    x->value = malloc(vl + 1);
    memcpy(x->name, n, nl);
    memcpy(x->value, v, vl);
    x->nlen = nl, x->vlen = vl, x->token = token;
    ++t->num;
}

static uint8_t *hpe_int(uint8_t *dst, uint8_t first, uint64_t v, unsigned prefix_bits)
{
    *dst = first;
    return orc_encode_int(dst, (int64_t)v, prefix_bits);
}

static uint8_t *hpe_as_is(uint8_t *dst, const uint8_t *s, uint32_t len) /* encode_as_is, hpack.c:806-814 */
{
    dst = hpe_int(dst, 0, len, 7);
    memcpy(dst, s, len);
    return dst + len;
}

/* lib/common/token_table.h: the static index of a token is that of the first static entry with its name */
static unsigned hpe_static_name_index(const uint8_t *n, uint32_t nl)
{
    for (unsigned i = 1; i < TABLE_OFFSET; ++i)
        if (strlen(orc_static_name[i]) == nl && memcmp(orc_static_name[i], n, nl) == 0)
            return i;
    return 0;
}

static int hpe_token_dont_compress(const uint8_t *n, uint32_t nl)
{
    return (nl == 6 && memcmp(n, "cookie", 6) == 0) || (nl == 10 && memcmp(n, "set-cookie", 10) == 0);
}

static int bytes_eq(const uint8_t *a, uint32_t al, const uint8_t *b, uint32_t bl)
{
    return al == bl && (al == 0 || memcmp(a, b, al) == 0);
}

/* do_encode_header (hpack.c:858-937) */
static uint8_t *hpe_encode_header(hpe_table_t *t, uint8_t *dst, const uint8_t *n, uint32_t nl, int token, const uint8_t *v,
                                  uint32_t vl, int dont_compress)
{
    unsigned name_index = token ? hpe_static_name_index(n, nl) : 0;
    for (uint32_t k = 0; k < t->num; ++k) { /* newest first (:864-890) */
        const hpe_entry_t *x = &t->e[k];
        if (token) {
            if (!x->token || !bytes_eq(n, nl, x->name, x->nlen))
                continue;
        } else {
            if (!bytes_eq(n, nl, x->name, x->nlen))
                continue;
            if (name_index == 0)
                name_index = k + TABLE_OFFSET;
        }
        if (!bytes_eq(v, vl, x->value, x->vlen))
            continue;
        return hpe_int(dst, 0x80, k + TABLE_OFFSET, 7); /* indexed (:881-884) */
    }
    if (!dont_compress && token)
        dont_compress = hpe_token_dont_compress(n, nl);
    if (dont_compress)
        dont_compress = vl < 20;
    if (name_index != 0) {
        dst = dont_compress ? hpe_int(dst, 0x10, name_index, 4) : hpe_int(dst, 0x40, name_index, 6);
    } else {
        *dst++ = 0x40;
        dst += orc_encode_string(dst, n, nl);
    }
    if (dont_compress) {
        dst = hpe_as_is(dst, v, vl);
    } else {
        dst += orc_encode_string(dst, v, vl);
        hpe_add(t, n, nl, v, vl, token);
    }
    return dst;
}

/* The one-byte static references h2o_hpack_flatten_request writes without looking at the table: encode_method
 * (:950-961), encode_scheme (:963-974; h2o compares the scheme object, whose name is "https" / "http" exactly
 * for H2O_URL_SCHEME_HTTPS / _HTTP), encode_path (:976-985) for its own fields, and accept-encoding
 * "gzip, deflate" among the headers (:1083-1086).  0 = none. */
static uint8_t hpe_request_fast(const uint8_t *n, uint32_t nl, const uint8_t *v, uint32_t vl, int own)
{
#define HPE_IS(p, l, lit) ((l) == sizeof(lit) - 1 && memcmp((p), (lit), sizeof(lit) - 1) == 0)
    if (!own)
        return HPE_IS(n, nl, "accept-encoding") && HPE_IS(v, vl, "gzip, deflate") ? 0x90 : 0;
    if (HPE_IS(n, nl, ":method"))
        return HPE_IS(v, vl, "GET") ? 0x82 : HPE_IS(v, vl, "POST") ? 0x83 : 0;
    if (HPE_IS(n, nl, ":scheme"))
        return HPE_IS(v, vl, "https") ? 0x87 : HPE_IS(v, vl, "http") ? 0x86 : 0;
    if (HPE_IS(n, nl, ":path"))
        return HPE_IS(v, vl, "/") ? 0x84 : HPE_IS(v, vl, "/index.html") ? 0x85 : 0;
    return 0;
#undef HPE_IS
}

static uint8_t *hpe_frame_header(uint8_t *dst, uint32_t len, uint8_t type, uint8_t flags, uint32_t sid) /* frame.c:68-79 */
{
    dst[0] = (uint8_t)(len >> 16), dst[1] = (uint8_t)(len >> 8), dst[2] = (uint8_t)len;
    dst[3] = type, dst[4] = flags;
    dst[5] = (uint8_t)(sid >> 24), dst[6] = (uint8_t)(sid >> 16), dst[7] = (uint8_t)(sid >> 8), dst[8] = (uint8_t)sid;
    return dst + 9;
}

/* fixup_frame_headers (hpack.c:1012-1042) on a buffer holding [9 reserved][payload]; returns the total */
static uint64_t hpe_frames(uint8_t *buf, uint64_t payload, uint8_t type, uint32_t sid, uint32_t max_frame, uint8_t flags)
{
    if (payload <= max_frame) {
        hpe_frame_header(buf, (uint32_t)payload, type, 0x4 | flags, sid);
        return 9 + payload;
    }
    hpe_frame_header(buf, max_frame, type, flags, sid);
    uint64_t size = 9 + payload, off = 9 + (uint64_t)max_frame;
    for (;;) {
        uint64_t left = size - off;
        memmove(buf + off + 9, buf + off, left);
        size += 9;
        if (left <= max_frame) {
            hpe_frame_header(buf + off, (uint32_t)left, 0x9, 0x4, sid);
            break;
        }
        hpe_frame_header(buf + off, max_frame, 0x9, 0, sid);
        off += 9 + (uint64_t)max_frame;
    }
    return size;
}

uint64_t orc_hpe_frames_size(uint64_t payload, uint32_t max_frame)
{
    return 9 + payload + (payload > max_frame ? 9 * ((payload - 1) / max_frame) : 0);
}

void *orc_hpe_open(uint32_t nconn)
{
    hpe_session_t *s = calloc(1, sizeof(*s));
    s->nconn = nconn;
    s->t = calloc(nconn ? nconn : 1, sizeof(hpe_table_t));
    for (uint32_t c = 0; c < nconn; ++c)
        s->t[c].capacity = INITIAL_CAPACITY;
    return s;
}

void orc_hpe_close(void *h)
{
    hpe_session_t *s = h;
    for (uint32_t c = 0; c < s->nconn; ++c)
        while (s->t[c].num)
            hpe_evict_one(&s->t[c]);
    free(s->t);
    free(s);
}

/* one step: the responses conn_first[c] .. conn_first[c+1]-1 of every connection, in order (the
 * include/hhuff.h hhuff_hpack_flatten_responses contract; res = hhuff_hpack_response_t records, hdr =
 * hhuff_hpack_header_t records) */
int orc_hpe_step(void *h, const uint8_t *in, uint64_t in_size, const uint32_t *hdr, const uint32_t *res,
                 const uint32_t *conn_first, uint32_t server_off, uint32_t server_len, uint8_t *out,
                 const uint64_t *out_off, uint32_t *out_len, uint32_t *headers_size, int32_t *rstatus)
{
    hpe_session_t *s = h;
    uint8_t *tmp = NULL;
    size_t tmp_cap = 0;
    for (uint32_t c = 0; c < s->nconn; ++c) {
        hpe_table_t *t = &s->t[c];
        for (uint32_t r = conn_first[c]; r < conn_first[c + 1]; ++r) {
            const uint32_t *R = res + 10 * (size_t)r;
            uint64_t content_length;
            memcpy(&content_length, R, 8);
            uint32_t sid = R[2], status = R[3], hfirst = R[4], nh = R[5], cap = R[6], mfs = R[7], fl = R[8];
            out_len[r] = 0;
            headers_size[r] = 0;
            if (t->failed) {
                rstatus[r] = -301; /* HHUFF_RES_SKIPPED */
                continue;
            }
            /* a request (h2o_hpack_flatten_request): no :status, server or content-length; `status` = the number of
             * leading headers that are its own fields (method, scheme, authority, path, protocol, expect) */
            int trailers = (fl & 4u) != 0, request = (fl & 8u) && !trailers, head = !trailers && !request, bad = 0;
            if ((head && (status < 100 || status > 999)) || (request && status > nh) || mfs < 16384 || mfs > 0xffffff)
                bad = 1; /* encode_status asserts (:441); SETTINGS_MAX_FRAME_SIZE bounds (RFC 9113 6.5.2) */
            if ((fl & 2u) && head && (uint64_t)server_off + server_len > in_size)
                bad = 1;
            size_t need = 9 + 5 + 5 + 5 + server_len + 32;
            for (uint32_t i = 0; i < nh; ++i) {
                const uint32_t *H = hdr + 5 * (size_t)(hfirst + i);
                if ((uint64_t)H[0] + H[1] > in_size || (uint64_t)H[2] + H[3] > in_size)
                    bad = 1;
                need += (size_t)H[1] + H[3] + 21;
            }
            if (bad) {
                rstatus[r] = -303; /* HHUFF_RES_EINVAL */
                t->failed = 1;
                continue;
            }
            need += 9 * (need / 16384 + 1);
            if (need > tmp_cap) {
                free(tmp);
                tmp_cap = need * 2;
                tmp = malloc(tmp_cap);
            }
            uint8_t *dst = tmp + 9;
            if (cap < t->capacity) { /* header_table_adjust_size (:839-856) */
                t->capacity = cap;
                while (t->num != 0 && t->size > t->capacity)
                    hpe_evict_one(t);
                dst = hpe_int(dst, 0x20, t->capacity, 5);
            }
            if (head) {
                switch (status) { /* encode_status (:437-466) */
                case 200: *dst++ = 0x88; break;
                case 204: *dst++ = 0x89; break;
                case 206: *dst++ = 0x8a; break;
                case 304: *dst++ = 0x8b; break;
                case 400: *dst++ = 0x8c; break;
                case 404: *dst++ = 0x8d; break;
                case 500: *dst++ = 0x8e; break;
                default:
                    *dst++ = 8, *dst++ = 3;
                    *dst++ = (uint8_t)('0' + status / 100), *dst++ = (uint8_t)('0' + status / 10 % 10);
                    *dst++ = (uint8_t)('0' + status % 10);
                }
                if ((fl & 2u) && server_len != 0) /* :1159-1163, the server token (static index 54) */
                    dst = hpe_encode_header(t, dst, (const uint8_t *)"server", 6, 1, in + server_off, server_len, 0);
            }
            for (uint32_t i = 0; i < nh; ++i) {
                const uint32_t *H = hdr + 5 * (size_t)(hfirst + i);
                uint8_t fast = request && (H[4] & 2u) ? hpe_request_fast(in + H[0], H[1], in + H[2], H[3], i < status) : 0;
                if (fast)
                    *dst++ = fast;
                else
                    dst = hpe_encode_header(t, dst, in + H[0], H[1], (H[4] & 2u) != 0, in + H[2], H[3], (H[4] & 1u) != 0);
            }
            if (head && content_length != UINT64_MAX) { /* encode_content_length (:468-485) */
                char d[24];
                int l = 0;
                uint64_t v = content_length;
                do
                    d[l++] = (char)('0' + v % 10);
                while ((v /= 10) != 0);
                *dst++ = 0x0f, *dst++ = 0x0d, *dst++ = (uint8_t)l;
                while (l)
                    *dst++ = (uint8_t)d[--l];
            }
            uint64_t payload = (uint64_t)(dst - (tmp + 9));
            uint64_t total = orc_hpe_frames_size(payload, mfs);
            if (total > out_off[r + 1] - out_off[r]) {
                rstatus[r] = -300; /* HHUFF_RES_SPACE */
                t->failed = 1;
                continue;
            }
            uint8_t flags = (trailers || (fl & 1u)) ? 0x1 : 0; /* END_STREAM (:1094-1095, :1174-1175, :1195) */
            uint64_t got = hpe_frames(tmp, payload, 0x1, sid, mfs, flags);
            (void)got;
            memcpy(out + out_off[r], tmp, total);
            out_len[r] = (uint32_t)total;
            headers_size[r] = (uint32_t)payload;
            rstatus[r] = 0;
        }
    }
    free(tmp);
    return 0;
}
