/*
 * ORACLE -- TEST INFRASTRUCTURE ONLY.  Clean-room CPU restatement of h2o's HTTP/3 response encoder (SURVEY.md 8
 * f4, QPACK encode half), the contract of include/hhuff.h hhuff_qpack_flatten_responses:
 *   lib/http3/qpack.c  h2o_qpack_flatten_response :1352-1399 as h2o's HTTP/3 server calls it
 *                      (lib/http3/server.c:1680-1683: no encoder-stream buffer), h2o_qpack_flatten_request
 *                      :1312-1350 as h2o's HTTP/3 client calls it (lib/common/http3client.c:792, no encoder-stream
 *                      buffer either; its own fields are token fields of the request's header list, and its
 *                      flatten_static_indexed 22 / 23 for the http / https scheme objects equals the generic
 *                      lookup's exact match), prepare_flatten :1247-1263,
 *                      flatten_static_indexed :1086-1094, flatten_static_nameref :1114-1120,
 *                      flatten_without_nameref :1138-1146, do_flatten_header :1148-1213, flatten_header
 *                      :1215-1228, flatten_known_header_with_static_lookup :1230-1238, finalize_flatten
 *                      :1265-1310, flatten_int / flatten_string :1036-1066
 *   lib/common/token_table.h  h2o_qpack_lookup_static (:1606), the generated per-token lookups: an entry of
 *                      h2o_qpack_static_table with the token's name and the same value (exact), else the first
 *                      entry with the name, else -1
 * With no encoder-stream buffer the encoder never inserts into its dynamic table (:1175-1176), so the table
 * stays empty, lookup_dynamic finds nothing, the largest reference stays 0 and the section prefix is 00 00:
 * a response's bytes depend on that response alone.
 * Pinned by oracle/ref_shim.c ref_qpe_step (the real h2o_qpack_flatten_response) and ref_qpe_lookup_check
 * (the lookup rule against every generated function), tests/test_qpenc.py, tests/golden/qpenc.npz.
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "huff_oracle.h"
#include "huff_tables.h"

#define QSTATIC 99

/* the lookup rule of the generated h2o_qpack_lookup_* functions (lib/common/token_table.h) */
int32_t orc_qpe_static_lookup(const uint8_t *n, uint32_t nl, const uint8_t *v, uint32_t vl, int *is_exact)
{
    int32_t first = -1;
    for (int32_t i = 0; i < QSTATIC; ++i) {
        const char *sn = orc_qpack_static_name[i], *sv = orc_qpack_static_value[i];
        if (strlen(sn) != nl || memcmp(sn, n, nl) != 0)
            continue;
        if (first < 0)
            first = i;
        if (strlen(sv) == vl && memcmp(sv, v, vl) == 0) {
            *is_exact = 1;
            return i;
        }
    }
    *is_exact = 0;
    return first;
}

static uint8_t *qpe_int(uint8_t *dst, uint8_t first, uint64_t v, unsigned prefix_bits)
{
    *dst = first;
    return orc_encode_int(dst, (int64_t)v, prefix_bits);
}

/* flatten_string (:1042-1066) with the first byte's bits above the H bit given */
static uint8_t *qpe_string(uint8_t *dst, uint8_t first, const uint8_t *s, uint32_t len, unsigned prefix_bits, int dc)
{
    *dst = first;
    return dst + orc_flatten_string(dst, s, len, prefix_bits, dc);
}

/* do_flatten_header (:1148-1213) without a dynamic table */
static uint8_t *qpe_field(uint8_t *dst, int32_t static_index, int is_exact, const uint8_t *n, uint32_t nl, const uint8_t *v,
                          uint32_t vl, int dc)
{
    if (static_index >= 0 && is_exact)
        return qpe_int(dst, 0xc0, (uint64_t)static_index, 6); /* flatten_static_indexed */
    if (static_index >= 0) {                                   /* flatten_static_nameref */
        dst = qpe_int(dst, 0x50 | (dc ? 0x20 : 0), (uint64_t)static_index, 4);
        return qpe_string(dst, 0, v, vl, 7, dc);
    }
    dst = qpe_string(dst, 0x20 | (dc ? 0x10 : 0), n, nl, 3, 0); /* flatten_without_nameref */
    return qpe_string(dst, 0, v, vl, 7, dc);
}

static uint32_t qpe_varint_len(uint64_t v) /* quicly_encodev_capacity */
{
    return v <= 63 ? 1 : v <= 16383 ? 2 : v <= 1073741823 ? 4 : 8;
}

static uint8_t *qpe_varint(uint8_t *p, uint64_t v) /* quicly_encodev */
{
    uint32_t l = qpe_varint_len(v);
    static const uint8_t tag[9] = {0, 0x00, 0x40, 0, 0x80, 0, 0, 0, 0xc0};
    for (uint32_t k = 0; k < l; ++k)
        p[k] = (uint8_t)(v >> (8 * (l - 1 - k)));
    p[0] |= tag[l];
    return p + l;
}

static uint32_t qpe_status_index(uint32_t s) /* INDEXED_STATUS (:1362-1377) */
{
    switch (s) {
    case 103: return 24;
    case 200: return 25;
    case 304: return 26;
    case 404: return 27;
    case 503: return 28;
    case 100: return 63;
    case 204: return 64;
    case 206: return 65;
    case 302: return 66;
    case 400: return 67;
    case 403: return 68;
    case 421: return 69;
    case 425: return 70;
    case 500: return 71;
    default: return 0;
    }
}

/* res = hhuff_qpack_response_t records (8 u32 words), hdr = hhuff_hpack_header_t records (5 u32 words) */
int orc_qpe_step(const uint8_t *in, uint64_t in_size, const uint32_t *hdr, const uint32_t *res, uint32_t nres,
                 uint32_t server_off, uint32_t server_len, uint8_t *out, const uint64_t *out_off, uint32_t *out_len,
                 uint32_t *header_len, int32_t *rstatus)
{
    uint8_t *tmp = NULL;
    size_t tmp_cap = 0;
    for (uint32_t r = 0; r < nres; ++r) {
        const uint32_t *R = res + 8 * (size_t)r;
        uint64_t content_length;
        memcpy(&content_length, R, 8);
        uint32_t status = R[2], hfirst = R[3], nh = R[4], fl = R[5], doff = R[6], dlen = R[7];
        int request = (fl & 16u) != 0; /* flatten_request: no :status, server or content-length */
        int server = !request && (fl & 2u) && server_len != 0, dfid = (fl & 8u) != 0;
        out_len[r] = header_len[r] = 0;
        int bad = (server && (uint64_t)server_off + server_len > in_size) || (dfid && (uint64_t)doff + dlen > in_size);
        size_t need = 64 + server_len + dlen;
        for (uint32_t i = 0; i < nh; ++i) {
            const uint32_t *H = hdr + 5 * (size_t)(hfirst + i);
            bad |= (uint64_t)H[0] + H[1] > in_size || (uint64_t)H[2] + H[3] > in_size;
            need += (size_t)H[1] + H[3] + 24;
        }
        if (bad) {
            rstatus[r] = -303; /* HHUFF_RES_EINVAL */
            continue;
        }
        if (need > tmp_cap) {
            free(tmp);
            tmp_cap = 2 * need;
            tmp = malloc(tmp_cap);
        }
        uint8_t *p = tmp;
        *p++ = 0, *p++ = 0; /* Required Insert Count 0, Delta Base 0 (finalize_flatten :1290-1301) */
        uint32_t si = qpe_status_index(status);
        if (request) {
        } else if (si) {
            p = qpe_int(p, 0xc0, si, 6);
        } else { /* :1379-1383: "%u" of (uint16_t)status against :status (24) */
            char d[8];
            int l = sprintf(d, "%u", (unsigned)(uint16_t)status);
            p = qpe_field(p, 24, 0, NULL, 0, (const uint8_t *)d, (uint32_t)l, 0);
        }
        if (server) /* :1387-1389, the server entry 92 */
            p = qpe_field(p, 92, 0, NULL, 0, in + server_off, server_len, 0);
        if (!request && content_length != UINT64_MAX) { /* :1391-1399 */
            if (content_length == 0) {
                p = qpe_int(p, 0xc0, 4, 6);
            } else {
                char d[24];
                int l = sprintf(d, "%llu", (unsigned long long)content_length);
                p = qpe_field(p, 4, 0, NULL, 0, (const uint8_t *)d, (uint32_t)l, 0);
            }
        }
        for (uint32_t i = 0; i < nh; ++i) { /* flatten_header (:1215-1228) */
            const uint32_t *H = hdr + 5 * (size_t)(hfirst + i);
            int exact = 0;
            int32_t sidx = (H[4] & 2u) ? orc_qpe_static_lookup(in + H[0], H[1], in + H[2], H[3], &exact) : -1;
            p = qpe_field(p, sidx, exact, in + H[0], H[1], in + H[2], H[3], (H[4] & 1u) != 0);
        }
        if (dfid) { /* datagram-flow-id: no static entry (h2o_qpack_lookup_datagram_flow_id) */
            int exact = 0;
            int32_t sidx = orc_qpe_static_lookup((const uint8_t *)"datagram-flow-id", 16, in + doff, dlen, &exact);
            p = qpe_field(p, sidx, exact, (const uint8_t *)"datagram-flow-id", 16, in + doff, dlen, 0);
        }
        uint64_t body = (uint64_t)(p - tmp);
        uint64_t total = 1 + qpe_varint_len(body) + body;
        if (total > out_off[r + 1] - out_off[r]) {
            rstatus[r] = -300; /* HHUFF_RES_SPACE */
            continue;
        }
        uint8_t *o = out + out_off[r];
        *o++ = 0x01; /* H2O_HTTP3_FRAME_TYPE_HEADERS */
        o = qpe_varint(o, body);
        memcpy(o, tmp, body);
        out_len[r] = (uint32_t)total;
        header_len[r] = (uint32_t)body;
        rstatus[r] = 0;
    }
    free(tmp);
    return 0;
}
