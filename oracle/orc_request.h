/*
 * ORACLE -- TEST INFRASTRUCTURE ONLY.  h2o_hpack_parse_request's rules (lib/http2/hpack.c:502-637) and
 * h2o_hpack_parse_response's (:642-750) as the restatement applies them field after field:
 * oracle/hpack_block.c (HTTP/2, lib/http2/connection.c:626-629, lib/common/http2client.c:332, :421) and
 * oracle/qpack_decode.c (HTTP/3, through h2o_qpack_parse_request / _response, lib/http3/qpack.c:848, :876).
 * The response record is include/hhuff.h hhuff_response_t, 4 words: status, nheaders, err, datagram flow id.
 * The request record is include/hhuff.h hhuff_request_t, 12 u32 words: [0..1] content_length, [2..7]
 * method, scheme, authority, path, protocol, expect (field index or -1), [8] exists map, [9] nheaders,
 * [10] err (HHUFF_HERR_*), [11] scheme kind.
 */
#pragma once
#include <stdint.h>

typedef struct {
    uint64_t content_length;
    int32_t slot[6]; /* method, scheme, authority, path, protocol, expect */
    int32_t dfid;    /* datagram-flow-id (HTTP/3) */
    uint32_t map, nheaders, err, scheme_kind, ndecoded;
    int pseudo_ok;
} orc_req_t;

void orc_rq_init(orc_req_t *r);
void orc_rq_store(uint32_t *w, const orc_req_t *r);
int orc_rq_field(orc_req_t *r, const uint8_t *name, uint32_t nl, const uint8_t *value, uint32_t vl, unsigned soft,
                 int32_t k, int *header, int h3);

typedef struct {
    int32_t status, dfid;
    uint32_t nheaders, err, ndecoded;
    int trailers;
} orc_resp_t;

void orc_rs_init(orc_resp_t *r, int trailers);
void orc_rs_store(uint32_t *w, const orc_resp_t *r);
int orc_rs_field(orc_resp_t *r, const uint8_t *name, uint32_t nl, const uint8_t *value, uint32_t vl, unsigned soft,
                 int32_t k, int *header, int h3);
