// h2o_hpack_parse_request's rules (lib/http2/hpack.c:502-637) and h2o_hpack_parse_response's
// (:642-750) on the GPU, shared by the HPACK block walk (hhuff_blocks.hip, as lib/http2/connection.c:626-629
// and lib/common/http2client.c:332, :421 call them) and the QPACK sections (hhuff_qpack.hip, as
// h2o_qpack_parse_request / h2o_qpack_parse_response call them for HTTP/3, lib/http3/qpack.c:848, :876).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "hhuff.h"

namespace hhuff {
namespace {
constexpr int32_t kReqErrProtocol = -1;     // H2O_HTTP2_ERROR_PROTOCOL (http2_common.h:41)
constexpr int32_t kReqErrCompression = -9;  // H2O_HTTP2_ERROR_COMPRESSION (:49)

// ---------------------------------------------------------------------------------------------------
// h2o_hpack_parse_request's rules (hpack.c:502-637), applied to each field right after it is decoded.
// h2o compares name POINTERS with its tokens; a name is a token exactly when its bytes are a token's
// (static-table names are tokens, literal names are interned through h2o_lookup_token, hpack.c:398-400,
// dynamic entries keep what they were given), so the classes below compare bytes.
// ---------------------------------------------------------------------------------------------------
enum : uint32_t {
    kNRegular = 0,     // anything h2o_add_header takes as it is
    kNAuthority,       // H2O_TOKEN_AUTHORITY
    kNMethod,          // H2O_TOKEN_METHOD
    kNPath,            // H2O_TOKEN_PATH
    kNProtocol,        // H2O_TOKEN_PROTOCOL
    kNScheme,          // H2O_TOKEN_SCHEME
    kNStatus,          // H2O_TOKEN_STATUS (an unknown pseudo-header to the request rules)
    kNPseudoOther,     // ':' + anything else
    kNContentLength,   // the is_hpack_special tokens (lib/common/token_table.h, 5th flag)
    kNExpect,
    kNHost,
    kNTe,
    kNCacheDigest,
    kNDatagramFlowId,
    kNConnSpecific,    // connection, http2-settings, transfer-encoding, upgrade
};

__device__ __forceinline__ bool bytes_eq(const uint8_t* s, const char* lit, uint32_t n) {
    for (uint32_t i = 0; i < n; ++i)
        if (s[i] != (uint8_t)lit[i]) return false;
    return true;
}

__device__ uint32_t req_name_class(const uint8_t* s, uint32_t n) {
    if (n != 0 && s[0] == ':') {
        switch (n) {
            case 5: return bytes_eq(s, ":path", 5) ? kNPath : kNPseudoOther;
            case 7:
                return bytes_eq(s, ":method", 7)   ? kNMethod
                       : bytes_eq(s, ":scheme", 7) ? kNScheme
                       : bytes_eq(s, ":status", 7) ? kNStatus
                                                   : kNPseudoOther;
            case 9: return bytes_eq(s, ":protocol", 9) ? kNProtocol : kNPseudoOther;
            case 10: return bytes_eq(s, ":authority", 10) ? kNAuthority : kNPseudoOther;
            default: return kNPseudoOther;
        }
    }
    switch (n) {
        case 2: return bytes_eq(s, "te", 2) ? kNTe : kNRegular;
        case 4: return bytes_eq(s, "host", 4) ? kNHost : kNRegular;
        case 6: return bytes_eq(s, "expect", 6) ? kNExpect : kNRegular;
        case 7: return bytes_eq(s, "upgrade", 7) ? kNConnSpecific : kNRegular;
        case 10: return bytes_eq(s, "connection", 10) ? kNConnSpecific : kNRegular;
        case 12: return bytes_eq(s, "cache-digest", 12) ? kNCacheDigest : kNRegular;
        case 14:
            return bytes_eq(s, "content-length", 14) ? kNContentLength
                   : bytes_eq(s, "http2-settings", 14) ? kNConnSpecific
                                                        : kNRegular;
        case 16: return bytes_eq(s, "datagram-flow-id", 16) ? kNDatagramFlowId : kNRegular;
        case 17: return bytes_eq(s, "transfer-encoding", 17) ? kNConnSpecific : kNRegular;
        default: return kNRegular;
    }
}

// h2o_strtosize (lib/common/string.c:86-113): at most 19 decimal digits, nothing else; ~0 on failure
__device__ uint64_t req_strtosize(const uint8_t* s, uint32_t n) {
    if (n == 0 || n > 19) return ~0ull;
    uint64_t v = 0;
    for (uint32_t i = 0; i < n; ++i) {
        const uint32_t d = (uint32_t)s[i] - '0';
        if (d > 9u) return ~0ull;
        v = v * 10u + d;
    }
    return v;
}

struct ReqState {  // one block's h2o_hpack_parse_request locals and out-parameters
    uint64_t content_length;
    int32_t method, scheme, authority, path, protocol, expect, dfid;
    uint32_t map, nheaders, err, scheme_kind, ndecoded;
    bool pseudo_ok;  // pseudo_header_exists_map != NULL: no regular field yet
    __device__ void reset() {
        content_length = ~0ull;
        method = scheme = authority = path = protocol = expect = dfid = -1;
        map = nheaders = err = scheme_kind = ndecoded = 0;
        pseudo_ok = true;
    }
};

constexpr uint32_t kMaxHeadersHard = 1000;  // H2O_HPACK_MAX_HEADERS_HARD_LIMIT (include/h2o/hpack.h:36)
constexpr uint32_t kMaxHeaders = 100;       // H2O_MAX_HEADERS (include/h2o/header.h:37)

// one decoded field k of the block (hpack.c:515-635); returns 0 or the hard error; sets *header when
// h2o_add_header takes the field.  H3: the arguments h2o's HTTP/3 server passes through
// h2o_qpack_parse_request (lib/http3/server.c:1540-1545): no cache-digest receiver (digests == NULL, so a
// cache-digest field is rejected with the other special fields, hpack.c:606-617) and a datagram flow id
// out-parameter (the field's value is stored, hpack.c:610-613).
template <bool H3 = false>
__device__ int32_t req_field(ReqState& r, uint32_t cls, const uint8_t* value, uint32_t vl, uint32_t soft, int32_t k,
                             bool& header) {
    header = false;
    if (soft != 0 && r.err == HHUFF_HERR_NONE) r.err = (soft & 1u) ? HHUFF_HERR_SOFT_NAME : HHUFF_HERR_SOFT_VALUE;
    if (++r.ndecoded > kMaxHeadersHard) {
        r.err = HHUFF_HERR_HEADERS_TOO_LONG;
        return kReqErrCompression;
    }
    if (cls >= kNAuthority && cls <= kNPseudoOther) {  // a pseudo-header name (first byte a colon)
        if (!r.pseudo_ok) {
            r.err = HHUFF_HERR_INVALID_PSEUDO;
            return kReqErrProtocol;
        }
        switch (cls) {
            case kNAuthority:
                if (r.authority >= 0) break;
                r.authority = k;
                r.map |= 8u;
                return 0;
            case kNMethod:
                if (r.method >= 0) break;
                r.method = k;
                r.map |= 1u;
                return 0;
            case kNProtocol:  // a duplicate is rejected without an err_desc (:546-548)
                if (r.protocol >= 0) return kReqErrProtocol;
                r.protocol = k;
                r.map |= 16u;
                return 0;
            case kNPath:
                if (r.path >= 0 || vl == 0) break;
                r.path = k;
                r.map |= 4u;
                return 0;
            case kNScheme:
                if (r.scheme >= 0) break;
                r.scheme = k;
                r.scheme_kind = (vl == 5 && bytes_eq(value, "https", 5)) ? 2u : (vl == 6 && bytes_eq(value, "masque", 6)) ? 3u : 1u;
                r.map |= 2u;
                return 0;
            default:  // unknown pseudo-header: rejected without an err_desc (:579-581)
                return kReqErrProtocol;
        }
        r.err = HHUFF_HERR_INVALID_PSEUDO;
        return kReqErrProtocol;
    }
    r.pseudo_ok = false;
    switch (cls) {
        case kNContentLength:
            if ((r.content_length = req_strtosize(value, vl)) == ~0ull) {
                r.err = HHUFF_HERR_CONTENT_LENGTH;
                return kReqErrProtocol;
            }
            return 0;
        case kNExpect:
            r.expect = k;
            return 0;
        case kNHost:
            if (r.authority < 0) r.authority = k;
            return 0;
        case kNDatagramFlowId:  // HTTP/2: datagram_flow_id == NULL (connection.c:629); HTTP/3: stored
            if (H3) r.dfid = k;
            return 0;
        case kNTe: {  // h2o_lcstris(value, "trailers")
            bool trailers = vl == 8;
            for (uint32_t i = 0; trailers && i < 8; ++i) {
                uint32_t c = value[i];
                c = (c - 'A' < 26u) ? c + 32u : c;
                trailers = c == (uint8_t)"trailers"[i];
            }
            if (!trailers) {
                r.err = HHUFF_HERR_CONNECTION_SPECIFIC;
                return kReqErrProtocol;
            }
            break;
        }
        case kNCacheDigest:  // HTTP/2: digests != NULL (connection.c:629): loaded, then listed
            if (H3) {  // HTTP/3: digests == NULL: "rest of the header fields that are marked as special"
                r.err = HHUFF_HERR_CONNECTION_SPECIFIC;
                return kReqErrProtocol;
            }
            break;
        case kNConnSpecific:
            r.err = HHUFF_HERR_CONNECTION_SPECIFIC;
            return kReqErrProtocol;
        default:
            break;
    }
    if (r.nheaders < kMaxHeaders) {
        ++r.nheaders;
        header = true;
    } else if (r.err == HHUFF_HERR_NONE) {
        r.err = HHUFF_HERR_HEADERS_TOO_LONG;
    }
    return 0;
}

// ---------------------------------------------------------------------------------------------------
// h2o_hpack_parse_response's rules (hpack.c:642-750): a response head (status != NULL) or trailers
// (status == NULL, http2client.c:421).  H3: the datagram flow id out-parameter h2o's HTTP/3 client passes
// (lib/common/http3client.c:542); HTTP/2 passes NULL (http2client.c:332).
// ---------------------------------------------------------------------------------------------------
struct RespState {
    int32_t status, dfid;
    uint32_t nheaders, err, ndecoded;
    bool trailers;
    __device__ void reset(bool tr) {
        status = 0;
        dfid = -1;
        nheaders = err = ndecoded = 0;
        trailers = tr;
    }
};

template <bool H3 = false>
__device__ int32_t resp_field(RespState& r, uint32_t cls, const uint8_t* value, uint32_t vl, uint32_t soft, int32_t k,
                              bool& header) {
    header = false;
    if (soft != 0 && r.err == HHUFF_HERR_NONE) r.err = (soft & 1u) ? HHUFF_HERR_SOFT_NAME : HHUFF_HERR_SOFT_VALUE;
    if (++r.ndecoded > kMaxHeadersHard) {  // :668-671
        r.err = HHUFF_HERR_HEADERS_TOO_LONG;
        return kReqErrCompression;
    }
    if (cls >= kNAuthority && cls <= kNPseudoOther) {  // name->base[0] == ':' (:672-704)
        if (r.trailers || cls != kNStatus || r.status != 0 || vl != 3) {
            r.err = HHUFF_HERR_INVALID_PSEUDO;
            return kReqErrProtocol;
        }
        // PARSE_DIGIT(100, 1), (10, 0), (1, 0): a digit is added to *status before the next one is checked
        const uint32_t mul[3] = {100u, 10u, 1u};
        for (uint32_t i = 0; i < 3; ++i) {
            const uint32_t d = (uint32_t)value[i] - '0';
            if (d > 9u || (i == 0 && d == 0u)) {
                r.err = HHUFF_HERR_INVALID_PSEUDO;
                return kReqErrProtocol;
            }
            r.status += (int32_t)(d * mul[i]);
        }
        return 0;
    }
    if (!r.trailers && r.status == 0) {  // :706-709
        r.err = HHUFF_HERR_MISSING_PSEUDO;
        return kReqErrProtocol;
    }
    switch (cls) {  // the is_hpack_special tokens (:712-725)
        case kNContentLength:
        case kNCacheDigest:
        case kNHost:
            break;  // passed through
        case kNDatagramFlowId:
            if (H3) r.dfid = k;
            return 0;  // goto Next: not listed
        case kNExpect:
        case kNTe:
        case kNConnSpecific:
            r.err = HHUFF_HERR_CONNECTION_SPECIFIC;
            return kReqErrProtocol;
        default:
            break;
    }
    if (r.nheaders < kMaxHeaders) {  // :726-738
        ++r.nheaders;
        header = true;
    } else if (r.err == HHUFF_HERR_NONE) {
        r.err = HHUFF_HERR_HEADERS_TOO_LONG;
    }
    return 0;
}

__device__ __forceinline__ void resp_store(hhuff_response_t* out, const RespState& r) {
    out->status = r.status;
    out->nheaders = r.nheaders;
    out->err = r.err;
    out->datagram_flow_id = r.dfid;
}

__device__ __forceinline__ void req_store(hhuff_request_t* out, const ReqState& r) {
    out->content_length = r.content_length;
    out->method = r.method;
    out->scheme = r.scheme;
    out->authority = r.authority;
    out->path = r.path;
    out->protocol = r.protocol;
    out->expect = r.expect;
    out->exists_map = r.map;
    out->nheaders = r.nheaders;
    out->err = r.err;
    out->scheme_kind = r.scheme_kind;
}

}  // namespace
}  // namespace hhuff
