// HPACK header blocks on the GPU: h2o_hpack_decode_header (lib/http2/hpack.c:319-435)
// applied field after field over each block, the way h2o_hpack_parse_request loops over a block
// (hpack.c:513-527), with one dynamic table per connection (header_table_add :277-317, eviction
// :263-275, size updates :352-366).
//
// Decomposition: a header block cannot be split -- every field may change the connection's dynamic
// table, which the next field may read -- so the parallel axis is the connection: one lane per
// connection walks its blocks in order (h2o serves thousands of connections per node; a batch is one
// event-loop tick's worth of them).  The dynamic table lives in per-connection scratch in HBM: a byte
// ring of table_size bytes (live entries never exceed it: each entry costs its bytes + 32 of the
// capacity) and an entry ring of table_size / 32 + 1 {byte offset, name length, value length, soft
// bits} records, newest first as in h2o.  Huffman literals decode with the same decode_core as the
// string kernels (window LUT in LDS, per workgroup); raw literals validate with the reference's rules.
// Every decoded name and value is written to the caller's arena; indexed fields copy the table entry.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "hhuff_device.h"
#include "hhuff.h"
#include "hhuff_launch.h"

namespace hhuff {
namespace {
__device__ const uint32_t b_dec_lut[1u << HHUFF_LUT_BITS] = HHUFF_DEC_LUT_INIT;
__device__ const uint32_t b_kinfo[31] = HHUFF_ONES_KINFO_INIT;
__device__ const uint32_t b_ones[HHUFF_ONES_NENT] = HHUFF_ONES_ENT_INIT;
__device__ const uint32_t b_name_invalid[8] = HHUFF_NAME_INVALID_INIT;
__device__ const uint32_t b_value_invalid[8] = HHUFF_VALUE_INVALID_INIT;
__device__ const uint8_t b_static_bytes[HHUFF_STATIC_NBYTES] = HHUFF_STATIC_BYTES_INIT;
__device__ const uint16_t b_static_ent[61 * 4] = HHUFF_STATIC_ENT_INIT;

constexpr int32_t kErrProtocol = -1;        // H2O_HTTP2_ERROR_PROTOCOL (http2_common.h:41)
constexpr int32_t kErrCompression = -9;     // H2O_HTTP2_ERROR_COMPRESSION (:49)
constexpr int32_t kErrInvalidChar = -254;   // H2O_HTTP2_ERROR_INVALID_HEADER_CHAR (:55)
constexpr int32_t kBlkArena = HHUFF_BLK_ARENA;
constexpr int32_t kBlkSkipped = HHUFF_BLK_SKIPPED;
constexpr uint32_t kEntryOverhead = 32;  // HEADER_TABLE_ENTRY_SIZE_OFFSET (hpack.c:30)
constexpr int64_t kIntIncomplete = -255, kIntBad = -9;
}  // namespace

// Phase timing (profile builds only, -DHHUFF_PROFILE; tools/prof_blocks.py): per lane, the shader cycles
// between the begin and end marks of each phase while the lane was in it, summed over lanes.
#ifdef HHUFF_PROFILE
__device__ unsigned long long g_bprof[8];
struct BProf {
    uint64_t a[8];
};
#define BP_T() __builtin_readcyclecounter()
#define BP_ADD(bp, k, t0) ((bp).a[k] += BP_T() - (t0))
#else
struct BProf {};
#define BP_T() 0ull
#define BP_ADD(bp, k, t0) ((void)(t0))
#endif

struct BlkArgs {
    const uint8_t* in;
    uint64_t in_size;
    const uint32_t* blk_off;
    const uint32_t* conn_first;
    uint32_t nconn, table_size;
    uint8_t* arena;
    const uint64_t* arena_off;
    uint32_t *name_off, *name_len, *value_off, *value_len;
    uint8_t* fflags;
    uint32_t* nfields;
    int32_t* bstatus;
    uint8_t* scratch;
    uint64_t conn_scratch;  // bytes of scratch per connection
    uint32_t flags;         // HHUFF_BLK_CONTINUE: start from the tables the previous call left in scratch
    hhuff_request_t* req;   // request mode (hhuff_hpack_parse_requests): h2o_hpack_parse_request per block
};

// per-connection scratch: [TableState 32 B][byte ring, table_size rounded to 16][entry ring]
struct TableState {
    uint32_t start, num, whead, failed;
    uint64_t size, cap;
};

constexpr uint32_t kBlkThreads = 256;

// The lane's reads of its block.  (Staging each lane's block through a private LDS window was tried and
// measured slower -- 6.4 ms against 4.5 ms for 65536 connections: the restage's 16-byte loads wait behind
// the wave's outstanding arena stores, and the time goes to divergence, not to input latency; DESIGN.md.)
struct Win {
    const uint8_t* in;
    uint64_t in_size;
    __device__ __forceinline__ uint32_t byte(uint64_t a) const { return in[a]; }
    __device__ __forceinline__ uint32_t word(uint64_t a) const { return GlobalSource{in, in_size}.word((uint32_t)a); }
};

struct WinSource {  // decode_core's source interface over a Win
    const Win* w;
    __device__ __forceinline__ uint32_t word(uint32_t a) const { return w->word(a); }
};

// h2o_hpack_decode_int (hpack.c:52-83) at position p, bounded by end
__device__ int64_t blk_decode_int(const Win& in, uint64_t& p, uint64_t end, uint32_t prefix_bits) {
    if (p >= end) return kIntIncomplete;
    const uint64_t pmax = (1u << prefix_bits) - 1u;
    uint64_t v = in.byte(p++) & pmax;
    if (v != pmax) return (int64_t)v;
    uint32_t shift = 0;
    for (; shift < 56; shift += 7) {
        if (p == end) return kIntIncomplete;
        const uint32_t b = in.byte(p++);
        v += (uint64_t)(b & 127u) << shift;
        if (!(b & 128u)) return (int64_t)v;
    }
    if (p == end) return kIntIncomplete;
    if (in.byte(p) & 128u) return kIntBad;
    v += (uint64_t)(in.byte(p++) & 127u) << shift;
    if (v > 0x7FFFFFFFFFFFFFFFull) return kIntBad;
    return (int64_t)v;
}

// Byte copies in batches of 16: the 16 loads issue back to back and one wait covers them, instead of a
// load-to-store round trip per byte (a lane's strings sit at unrelated addresses, so nothing coalesces).
template <typename Src, typename Dst>
__device__ __forceinline__ void copy16(Src src, Dst dst, uint32_t n) {
    for (uint32_t i = 0; i < n; i += 16) {
        uint8_t t[16];
#pragma unroll
        for (uint32_t k = 0; k < 16; ++k)
            if (i + k < n) t[k] = src(i + k);
#pragma unroll
        for (uint32_t k = 0; k < 16; ++k)
            if (i + k < n) dst(i + k, t[k]);
    }
}

struct DynTable {  // one connection's dynamic table (newest entry = dynamic index 62)
    uint8_t* ring;   // R bytes
    uint4* ent;      // E records {byte offset, name length, value length, soft bits}
    uint32_t R, E, start, num, whead;
    uint64_t size, cap, maxcap;
    __device__ __forceinline__ uint4 get(uint32_t k) const {
        uint32_t i = start + k;
        return ent[i >= E ? i - E : i];
    }
    __device__ __forceinline__ void evict_one() {
        --num;
        const uint4 e = get(num);
        size -= (uint64_t)e.y + e.z + kEntryOverhead;
    }
    __device__ __forceinline__ uint32_t wrap(uint32_t a) const { return a >= R ? a - R : a; }  // a < 2R
    __device__ __forceinline__ void put(const uint8_t* src, uint32_t n) {
        uint8_t* rg = ring;
        const uint32_t h = whead, RR = R;
        copy16([&](uint32_t i) { return src[i]; },
               [&](uint32_t i, uint8_t v) { rg[h + i >= RR ? h + i - RR : h + i] = v; }, n);
        whead = wrap(whead + n);
    }
    __device__ __forceinline__ void copy_out(uint32_t off, uint32_t n, uint8_t* dst) const {
        const uint8_t* rg = ring;
        const uint32_t RR = R;
        copy16([&](uint32_t i) { return rg[off + i >= RR ? off + i - RR : off + i]; },
               [&](uint32_t i, uint8_t v) { dst[i] = v; }, n);
    }
    __device__ void add(const uint8_t* name, uint32_t nlen, const uint8_t* value, uint32_t vlen, uint32_t soft) {
        const uint64_t add = (uint64_t)nlen + vlen + kEntryOverhead;
        while (num != 0 && size + add > cap) evict_one();
        if (num == 0 && add > cap) return;  // does not fit an empty table: not added (hpack.c:285-289)
        const uint32_t b0 = whead;
        put(name, nlen);
        put(value, vlen);
        start = start == 0 ? E - 1 : start - 1;
        ent[start] = make_uint4(b0, nlen, vlen, soft);
        size += add;
        ++num;
    }
};

enum : int { kStrOk = 0, kStrFail = 1, kStrUpper = 2, kStrArena = 3 };

// decode_string (hpack.c:223-261) at in[p] into arena[cur..aend)
__device__ int blk_string(const BlkArgs& A, const Win& W, uint64_t& p, uint64_t end, bool is_name, uint32_t& soft,
                          uint64_t& cur, uint64_t aend, uint32_t& off, uint32_t& len, const DecTables& T) {
    if (p >= end) return kStrFail;
    const bool huff = (W.byte(p) & 0x80u) != 0;
    const int64_t n = blk_decode_int(W, p, end, 7);
    if (n < 0 || (uint64_t)n > end - p) return kStrFail;
    if (huff) {
        if (cur + ((uint64_t)n * 8u) / 5u > aend) return kStrArena;
        if ((uint64_t)n > kMaxStrLen) return kStrFail;
        RegSink sink;
        sink.init(A.arena + cur);
        // decode with first / last byte tracking (soft bits need them, hpack.c:136-152)
        struct SinkFL {
            RegSink s;
            uint32_t first, last;
            __device__ __forceinline__ void put1(uint32_t b) {
                first = s.cnt == 0 ? (b & 0xFFu) : first;
                last = b & 0xFFu;
                s.put1(b);
            }
            __device__ __forceinline__ void put12(uint32_t syms, bool two) {
                first = s.cnt == 0 ? (syms & 0xFFu) : first;
                last = (two ? (syms >> 8) : syms) & 0xFFu;
                s.put12(syms, two);
            }
            __device__ __forceinline__ uint32_t count() const { return s.count(); }
        } fl{sink, 0u, 0u};
        const DecResult r = decode_core(WinSource{&W}, (uint32_t)p, (uint32_t)n, fl, T);
        if (!r.ok) return kStrFail;
        fl.s.finish();
        soft |= soft_bits(is_name, r.len, r.flags, fl.first, fl.last);
        len = r.len;
    } else {
        const uint8_t* src = A.in + p;
        if (cur + (uint64_t)n > aend) {  // the validators' verdicts come first (an upper-case name is PROTOCOL)
            if (is_name && (n == 0 || src[0] != ':')) {
                for (int64_t i = 0; i < n; ++i) {
                    const uint32_t c = src[i];
                    if (c - 'A' < 26u) return kStrUpper;
                }
            }
            return kStrArena;
        }
        // one pass: 16 bytes in, validated (h2o_hpack_validate_header_name / _value, hpack.c:163-221), out
        const bool check_name = is_name && (n == 0 || src[0] != ':');
        bool bad = is_name ? (n == 0 && check_name) : false, upper = false;
        uint8_t* dst = A.arena + cur;
        const uint32_t nn = (uint32_t)n;
        copy16([&](uint32_t i) { return src[i]; },
               [&](uint32_t i, uint8_t v) {
                   const uint32_t c = v;
                   if (is_name) {
                       if (check_name && ((b_name_invalid[c >> 5] >> (c & 31)) & 1u)) {
                           if (c - 'A' < 26u)
                               upper = true;
                           else
                               bad = true;
                       }
                   } else {
                       bad |= ((b_value_invalid[c >> 5] >> (c & 31)) & 1u) != 0;
                   }
                   dst[i] = v;
               },
               nn);
        if (upper) return kStrUpper;
        if (!is_name && n != 0) {  // whole-value rule (hpack.c:110-115): no surrounding whitespace
            const uint32_t a = src[0], z = src[n - 1];
            bad |= a == ' ' || a == '\t' || z == ' ' || z == '\t';
        }
        if (bad) soft |= is_name ? 0x1u : 0x2u;
        len = (uint32_t)n;
    }
    off = (uint32_t)cur;
    cur += len;
    p += (uint64_t)n;
    return kStrOk;
}

// one field (h2o_hpack_decode_header): 0 / kErrInvalidChar = a field was produced
__device__ int32_t blk_field(const BlkArgs& A, const Win& W, DynTable& t, uint64_t& p, uint64_t end, uint64_t& cur, uint64_t aend,
                             uint32_t& noff, uint32_t& nlen, uint32_t& voff, uint32_t& vlen, uint32_t& soft_out,
                             const DecTables& T, const uint8_t* SB, const uint16_t* SE, BProf& bp) {
    uint64_t t0 = BP_T();
    int64_t index = 0;
    bool value_indexed = false, do_index = false;
    for (;;) {
        if (p >= end) return kErrCompression;
        const uint32_t b = W.byte(p);
        if (b >= 128) {  // indexed header field
            if ((index = blk_decode_int(W, p, end, 7)) <= 0) return kErrCompression;
            value_indexed = true;
        } else if (b >= 64) {  // literal with incremental indexing
            if (b == 64)
                ++p;
            else if ((index = blk_decode_int(W, p, end, 6)) <= 0)
                return kErrCompression;
            do_index = true;
        } else if (b < 32) {  // literal without indexing / never indexed
            if ((b & 0xFu) == 0)
                ++p;
            else if ((index = blk_decode_int(W, p, end, 4)) <= 0)
                return kErrCompression;
        } else {  // dynamic table size update
            const int64_t c = blk_decode_int(W, p, end, 5);
            if (c < 0 || (uint64_t)c > t.maxcap) return kErrCompression;
            t.cap = (uint64_t)c;
            while (t.num != 0 && t.size > t.cap) t.evict_one();
            continue;
        }
        break;
    }
    uint32_t soft = 0;
    BP_ADD(bp, 0, t0);
    t0 = BP_T();
    if (index > 0) {
        if (index <= 61) {
            const uint32_t k = 4u * (uint32_t)(index - 1);
            const uint32_t no = SE[k], nl = SE[k + 1];
            if (cur + nl > aend) return kBlkArena;
            uint8_t* dn = A.arena + cur;
            copy16([&](uint32_t i) { return SB[no + i]; }, [&](uint32_t i, uint8_t v) { dn[i] = v; }, nl);
            noff = (uint32_t)cur;
            nlen = nl;
            cur += nl;
            if (value_indexed) {
                const uint32_t vo = SE[k + 2], vl = SE[k + 3];
                if (cur + vl > aend) return kBlkArena;
                uint8_t* dv = A.arena + cur;
                copy16([&](uint32_t i) { return SB[vo + i]; }, [&](uint32_t i, uint8_t v) { dv[i] = v; }, vl);
                voff = (uint32_t)cur;
                vlen = vl;
                cur += vl;
            }
        } else if ((uint64_t)(index - 62) < t.num) {
            const uint4 e = t.get((uint32_t)(index - 62));
            soft = e.w;
            if (cur + e.y > aend) return kBlkArena;
            t.copy_out(e.x, e.y, A.arena + cur);
            noff = (uint32_t)cur;
            nlen = e.y;
            cur += e.y;
            if (value_indexed) {
                if (cur + e.z > aend) return kBlkArena;
                uint32_t vo = e.x + e.y;
                if (vo >= t.R) vo -= t.R;
                t.copy_out(vo, e.z, A.arena + cur);
                voff = (uint32_t)cur;
                vlen = e.z;
                cur += e.z;
            }
        } else {
            return kErrCompression;
        }
        BP_ADD(bp, index <= 61 ? 1 : 2, t0);
    } else {
        const int r = blk_string(A, W, p, end, true, soft, cur, aend, noff, nlen, T);
        if (r == kStrArena) return kBlkArena;
        if (r != kStrOk) return r == kStrUpper ? kErrProtocol : kErrCompression;
        BP_ADD(bp, 3, t0);
    }
    t0 = BP_T();
    if (!value_indexed) {
        soft &= ~0x2u;
        const int r = blk_string(A, W, p, end, false, soft, cur, aend, voff, vlen, T);
        if (r == kStrArena) return kBlkArena;
        if (r != kStrOk) return kErrCompression;
        BP_ADD(bp, 4, t0);
    }
    t0 = BP_T();
    if (do_index) t.add(A.arena + noff, nlen, A.arena + voff, vlen, soft);
    BP_ADD(bp, 5, t0);
    soft_out = soft;
    return soft ? kErrInvalidChar : 0;
}

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
    kNPseudoOther,     // ':' + anything else (:status included)
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
            case 7: return bytes_eq(s, ":method", 7) ? kNMethod : bytes_eq(s, ":scheme", 7) ? kNScheme : kNPseudoOther;
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
    int32_t method, scheme, authority, path, protocol, expect;
    uint32_t map, nheaders, err, scheme_kind, ndecoded;
    bool pseudo_ok;  // pseudo_header_exists_map != NULL: no regular field yet
    __device__ void reset() {
        content_length = ~0ull;
        method = scheme = authority = path = protocol = expect = -1;
        map = nheaders = err = scheme_kind = ndecoded = 0;
        pseudo_ok = true;
    }
};

constexpr uint32_t kMaxHeadersHard = 1000;  // H2O_HPACK_MAX_HEADERS_HARD_LIMIT (include/h2o/hpack.h:36)
constexpr uint32_t kMaxHeaders = 100;       // H2O_MAX_HEADERS (include/h2o/header.h:37)

// one decoded field k of the block (hpack.c:515-635); returns 0 or the hard error; sets *header when
// h2o_add_header takes the field
__device__ int32_t req_field(ReqState& r, const uint8_t* name, uint32_t nl, const uint8_t* value, uint32_t vl,
                             uint32_t soft, int32_t k, bool& header) {
    header = false;
    if (soft != 0 && r.err == HHUFF_HERR_NONE) r.err = (soft & 1u) ? HHUFF_HERR_SOFT_NAME : HHUFF_HERR_SOFT_VALUE;
    if (++r.ndecoded > kMaxHeadersHard) {
        r.err = HHUFF_HERR_HEADERS_TOO_LONG;
        return kErrCompression;
    }
    const uint32_t cls = req_name_class(name, nl);
    if (nl != 0 && name[0] == ':') {
        if (!r.pseudo_ok) {
            r.err = HHUFF_HERR_INVALID_PSEUDO;
            return kErrProtocol;
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
                if (r.protocol >= 0) return kErrProtocol;
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
                return kErrProtocol;
        }
        r.err = HHUFF_HERR_INVALID_PSEUDO;
        return kErrProtocol;
    }
    r.pseudo_ok = false;
    switch (cls) {
        case kNContentLength:
            if ((r.content_length = req_strtosize(value, vl)) == ~0ull) {
                r.err = HHUFF_HERR_CONTENT_LENGTH;
                return kErrProtocol;
            }
            return 0;
        case kNExpect:
            r.expect = k;
            return 0;
        case kNHost:
            if (r.authority < 0) r.authority = k;
            return 0;
        case kNDatagramFlowId:  // datagram_flow_id == NULL for HTTP/2 (connection.c:629)
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
                return kErrProtocol;
            }
            break;
        }
        case kNCacheDigest:  // digests != NULL for HTTP/2 (connection.c:629): loaded, then listed
            break;
        case kNConnSpecific:
            r.err = HHUFF_HERR_CONNECTION_SPECIFIC;
            return kErrProtocol;
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

template <bool REQ>
__global__ __launch_bounds__(kBlkThreads) void hpack_blocks_kernel(BlkArgs A) {
    __shared__ __attribute__((aligned(16))) uint32_t s_lut[1u << HHUFF_LUT_BITS];
    __shared__ uint32_t s_kinfo[32];
    __shared__ uint32_t s_ones[HHUFF_ONES_NENT];
    __shared__ uint8_t s_static[HHUFF_STATIC_NBYTES];  // the static table (RFC 7541 Appendix A) for indexed copies
    __shared__ uint16_t s_sent[61 * 4];
    for (uint32_t k = threadIdx.x; k < HHUFF_STATIC_NBYTES; k += blockDim.x) s_static[k] = b_static_bytes[k];
    for (uint32_t k = threadIdx.x; k < 61 * 4; k += blockDim.x) s_sent[k] = b_static_ent[k];
    for (uint32_t k = threadIdx.x; k < (1u << HHUFF_LUT_BITS) / 4; k += blockDim.x)
        reinterpret_cast<uint4*>(s_lut)[k] = reinterpret_cast<const uint4*>(b_dec_lut)[k];
    for (uint32_t k = threadIdx.x; k < HHUFF_ONES_NENT; k += blockDim.x) s_ones[k] = b_ones[k];
    if (threadIdx.x < 31) s_kinfo[threadIdx.x] = b_kinfo[threadIdx.x];
    __syncthreads();
    DecTables T;  // assigned, not brace-initialised: a constant aggregate of LDS addresses cannot be a static initializer
    T.lut = s_lut;
    T.kinfo = s_kinfo;
    T.ones = s_ones;
    const uint32_t R = A.table_size, E = A.table_size / kEntryOverhead + 1;
    for (uint64_t c = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; c < A.nconn; c += (uint64_t)gridDim.x * blockDim.x) {
        uint8_t* scr = A.scratch + c * A.conn_scratch;
        TableState* ts = reinterpret_cast<TableState*>(scr);
        uint8_t* ring = scr + sizeof(TableState);
        DynTable t{ring, reinterpret_cast<uint4*>(ring + ((R + 15u) & ~15u)), R, E, 0u, 0u, 0u, 0u, A.table_size,
                   A.table_size};
        const Win W{A.in, A.in_size};
        BProf bp{};
        bool failed = false;
        if (A.flags & HHUFF_BLK_CONTINUE) {
            const TableState s0 = *ts;
            t.start = s0.start;
            t.num = s0.num;
            t.whead = s0.whead;
            t.size = s0.size;
            t.cap = s0.cap;
            failed = s0.failed != 0;
        }
        for (uint32_t b = A.conn_first[c]; b < A.conn_first[c + 1]; ++b) {
            A.nfields[b] = 0;
            ReqState rq;
            if (REQ) rq.reset();
            if (failed) {
                A.bstatus[b] = kBlkSkipped;
                if (REQ) req_store(A.req + b, rq);
                continue;
            }
            const uint64_t tb = BP_T();
            uint64_t p = A.blk_off[b];
            const uint64_t end = A.blk_off[b + 1];
            uint64_t cur = A.arena_off[b];
            const uint64_t aend = min(A.arena_off[b + 1], kArenaLimit);  // field offsets are u32
            const uint32_t slot = A.blk_off[b];
            uint32_t nf = 0;
            int32_t st = 0;
            while (p != end) {
                uint32_t no = 0, nl = 0, vo = 0, vl = 0, soft = 0;
                const int32_t rc = blk_field(A, W, t, p, end, cur, aend, no, nl, vo, vl, soft, T, s_static, s_sent, bp);
                if (rc != 0 && rc != kErrInvalidChar) {
                    st = rc;
                    // h2o_hpack_parse_request: *err_desc = decode_err (:523-525) -- only the upper-case name
                    // error carries one
                    if (REQ) rq.err = rc == kErrProtocol ? HHUFF_HERR_UPPER_CASE_NAME : HHUFF_HERR_NONE;
                    break;
                }
                bool header = false;
                int32_t rr = 0;
                const uint64_t tr = BP_T();
                if (REQ) rr = req_field(rq, A.arena + no, nl, A.arena + vo, vl, soft, (int32_t)nf, header);
                BP_ADD(bp, 6, tr);
                A.name_off[slot + nf] = no;
                A.name_len[slot + nf] = nl;
                A.value_off[slot + nf] = vo;
                A.value_len[slot + nf] = vl;
                A.fflags[slot + nf] = (uint8_t)(soft | (header ? HHUFF_FIELD_HEADER : 0u));
                ++nf;
                if (rr != 0) {
                    st = rr;
                    break;
                }
            }
            if (REQ) {
                if (st == 0 && rq.err != HHUFF_HERR_NONE) st = kErrInvalidChar;  // :636-637
                req_store(A.req + b, rq);
            }
            A.nfields[b] = nf;
            A.bstatus[b] = st;
            failed = st != 0 && st != kErrInvalidChar;
            BP_ADD(bp, 7, tb);
        }
#ifdef HHUFF_PROFILE
        for (int k = 0; k < 8; ++k) atomicAdd(&g_bprof[k], (unsigned long long)bp.a[k]);
#endif
        *ts = TableState{t.start, t.num, t.whead, failed ? 1u : 0u, t.size, t.cap};
    }
}

#ifdef HHUFF_PROFILE
hipError_t read_bprof(unsigned long long* out8, bool reset) {
    hipError_t e = hipMemcpyFromSymbol(out8, HIP_SYMBOL(g_bprof), sizeof(g_bprof));
    if (e == hipSuccess && reset) {
        unsigned long long z[8] = {};
        e = hipMemcpyToSymbol(HIP_SYMBOL(g_bprof), z, sizeof(z));
    }
    return e;
}
#endif

uint64_t hpack_conn_scratch(uint32_t table_size) {
    const uint64_t R = ((uint64_t)table_size + 15u) & ~15ull;
    return sizeof(TableState) + R + 16ull * (table_size / kEntryOverhead + 1u);
}

hipError_t launch_hpack_blocks(const uint8_t* in, uint64_t in_size, const uint32_t* blk_off, const uint32_t* conn_first,
                               uint32_t nconn, uint32_t table_size, uint8_t* arena, const uint64_t* arena_off,
                               uint32_t* name_off, uint32_t* name_len, uint32_t* value_off, uint32_t* value_len,
                               uint8_t* fflags, uint32_t* nfields, int32_t* bstatus, hhuff_request_t* req,
                               uint8_t* scratch, uint32_t flags, hipStream_t stream) {
    if (nconn == 0) return hipSuccess;
    BlkArgs A{in, in_size, blk_off, conn_first, nconn, table_size, arena, arena_off, name_off, name_len, value_off,
              value_len, fflags, nfields, bstatus, scratch, hpack_conn_scratch(table_size), flags, req};
    const uint32_t blocks = min((nconn + kBlkThreads - 1u) / kBlkThreads, 65535u);
    if (req)
        hipLaunchKernelGGL(hpack_blocks_kernel<true>, dim3(blocks), dim3(kBlkThreads), 0, stream, A);
    else
        hipLaunchKernelGGL(hpack_blocks_kernel<false>, dim3(blocks), dim3(kBlkThreads), 0, stream, A);
    return hipGetLastError();
}

}  // namespace hhuff
