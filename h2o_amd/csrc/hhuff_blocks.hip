// HPACK header blocks on the GPU: h2o_hpack_decode_header (lib/http2/hpack.c:319-435)
// applied field after field over each block, the way h2o_hpack_parse_request loops over a block
// (hpack.c:513-527), with one dynamic table per connection (header_table_add :277-317, eviction
// :263-275, size updates :352-366), and optionally h2o_hpack_parse_request's own rules (:502-637).
//
// A header block cannot be split -- every field may change the dynamic table the next one reads -- so the
// table work is sequential per connection.  What is not sequential is moved out of that walk:
//   1. literal pre-pass (blk_mark_kernel .. blk_list_kernel): a block's representation is readable without
//      its table (index values and literal lengths are explicit), so one lane per block finds every string
//      literal, and the literal kernels (launch_literals_dev) decode them all, balanced across connections;
//   2. the walk (hpack_walk_kernel, one lane per connection) does only the bookkeeping: representation,
//      table lookups and inserts, arena offsets, verdicts.  A field's name and value are *references* to
//      where their bytes already are -- a decoded literal, the static table, the connection's ring, or
//      (literals decoded in place) the arena -- and a table entry is such a pair of references;
//   3. the copy pass (blk_copy_kernel, 64 blocks per wave) moves every field's bytes into the
//      arena, and the table pass (blk_table_kernel, one wave per connection) writes each connection's live
//      entries into its other ring, so the next call (HHUFF_BLK_CONTINUE) finds them there.
// The walk stores little and waits on few loads; the byte traffic runs in the parallel passes.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "hhuff_device.h"
#include "hhuff.h"
#include "hhuff_launch.h"
#include "hhuff_request.h"

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
constexpr uint32_t kLitHuffmanV = 4, kLitUpperV = 5;  // HHUFF_LIT_HUFFMAN / _UPPERCASE verdicts
constexpr uint32_t kClsUnknown = 0xFFFFu;  // a table entry's name class not computed yet
}  // namespace

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
    // pre-decoded literals: bit p of lit_bits marks a string literal starting at input byte p, word_pre[w]
    // counts the marks before word w, and literal r (in position order) has the results of the literal
    // kernels: lit_len, lit_pay, lit_cons, lit_st, bytes at lit_out + floor(8 lit_pay[r] / 5).  NULL
    // lit_bits: every literal is decoded in place.
    const uint32_t* lit_bits;
    const uint32_t* word_pre;
    const uint32_t* lit_len;
    const uint32_t* lit_pay;
    const uint32_t* lit_cons;
    const uint8_t* lit_st;
    const uint8_t* lit_out;
    // per field slot: the byte sources of its name and value (read by the copy pass)
    uint64_t* fsrc_n;
    uint64_t* fsrc_v;
    hhuff_response_t* res;   // response mode (hhuff_hpack_parse_responses): h2o_hpack_parse_response per block
    const uint8_t* trailers;  // response mode: per block, nonzero = trailers (status == NULL); NULL = none
};
constexpr int kWalkPlain = 0, kWalkReq = 1, kWalkResp = 2;  // hpack_walk_kernel modes

// Byte sources: kind in the top three bits, offset below.  All stay valid until the call's passes have run.
constexpr uint64_t kSrcLit = 0;              // lit_out offset (a pre-decoded Huffman literal)
constexpr uint64_t kSrcStatic = 1ull << 61;  // static-table bytes (RFC 7541 Appendix A)
constexpr uint64_t kSrcScr = 2ull << 61;     // scratch offset (a connection's ring: bytes of earlier calls)
constexpr uint64_t kSrcArena = 3ull << 61;   // arena offset (a literal decoded in place)
constexpr uint64_t kSrcIn = 4ull << 61;      // input offset (a raw literal's payload, where it lies)
constexpr uint64_t kSrcOff = (1ull << 61) - 1;

__device__ __forceinline__ const uint8_t* src_ptr(const BlkArgs& A, uint64_t s) {
    const uint64_t o = s & kSrcOff;
    switch (s >> 61) {
        case 0: return A.lit_out + o;
        case 1: return b_static_bytes + o;
        case 2: return A.scratch + o;
        case 3: return A.arena + o;
        default: return A.in + o;
    }
}

// per-connection scratch: [TableState 32 B][Entry x E][ring 0][ring 1] (rings: table_size rounded to 16)
struct TableState {
    uint32_t start, num, ring, failed;  // ring: which ring holds the entries' bytes between calls
    uint64_t size, cap;
};
struct Entry {  // one dynamic-table entry: references to its name and value bytes
    uint64_t nsrc, vsrc;
    uint32_t nl, vl;
    uint16_t soft, cls;  // soft-error bits (hpack.c:419-421), name class for the request rules
    uint32_t pad;
};
static_assert(sizeof(TableState) == 32 && sizeof(Entry) == 32, "scratch records");

__device__ __host__ __forceinline__ uint32_t tbl_entries(uint32_t table_size) { return table_size / kEntryOverhead + 1; }
__device__ __host__ __forceinline__ uint64_t tbl_ring(uint32_t table_size) { return ((uint64_t)table_size + 15u) & ~15ull; }

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
struct DynTable {  // one connection's dynamic table (newest entry = dynamic index 62)
    Entry* ent;
    uint32_t E, start, num;
    uint64_t size, cap, maxcap;
    __device__ __forceinline__ uint32_t slot(uint32_t k) const {
        const uint32_t i = start + k;
        return i >= E ? i - E : i;
    }
    __device__ __forceinline__ Entry get(uint32_t k) const { return ent[slot(k)]; }
    __device__ __forceinline__ void evict_one() {
        --num;
        const uint2 l = *reinterpret_cast<const uint2*>(&ent[slot(num)].nl);
        size -= (uint64_t)l.x + l.y + kEntryOverhead;
    }
    __device__ void add(const Entry& e) {
        const uint64_t add = (uint64_t)e.nl + e.vl + kEntryOverhead;
        while (num != 0 && size + add > cap) evict_one();
        if (num == 0 && add > cap) return;  // does not fit an empty table: not added (hpack.c:285-289)
        start = start == 0 ? E - 1 : start - 1;
        ent[start] = e;
        size += add;
        ++num;
    }
};

enum : int { kStrOk = 0, kStrFail = 1, kStrUpper = 2, kStrArena = 3 };

// h2o_hpack_parse_request's rules: hhuff_request.h (shared with the QPACK sections, qpack.c:848)

// decode_string (hpack.c:223-261) at position p: the string's arena place [off, off + len) and the source of
// its bytes (a pre-decoded literal; or, decoded in place, the arena itself)
__device__ int blk_string(const BlkArgs& A, const Win& W, uint64_t& p, uint64_t end, bool is_name, uint32_t& soft,
                          uint64_t& cur, uint64_t aend, uint32_t& off, uint32_t& len, uint64_t& src, const DecTables& T) {
    if (p >= end) return kStrFail;
    if (A.lit_bits) {  // decoded already (hhuff_decode_literals over every literal the parse pass found)
        const uint32_t w = A.lit_bits[p >> 5], m = 1u << (p & 31);
        const uint32_t r = A.word_pre[p >> 5] + (uint32_t)__builtin_popcount(w & (m - 1u));
        const uint32_t st = (w & m) ? A.lit_st[r] : 0xFFu;
        const uint32_t verdict = (st >> 2) & 7u;
        if ((w & m) && (verdict == 0 || verdict == kLitHuffmanV || verdict == kLitUpperV)) {
            const uint32_t ln = A.lit_len[r];
            const bool huff = (W.byte(p) & 0x80u) != 0;
            uint64_t q = p;
            const uint64_t n = (uint64_t)blk_decode_int(W, q, end, 7);  // fits: the parse pass checked it
            // decode_string's order: Huffman -- arena room, then the decoder's verdict; raw -- the name
            // validator's verdict, then arena room
            if (huff) {
                if (cur + (n * 8u) / 5u > aend) return kStrArena;
                if (verdict != 0) return kStrFail;
            } else {
                if (verdict == kLitUpperV) return kStrUpper;
                if (cur + n > aend) return kStrArena;
            }
            src = huff ? kSrcLit | ((q * 8u) / 5u) : kSrcIn | q;  // raw payloads are not copied by the pre-pass
            soft |= st & 3u;
            len = ln;
            off = (uint32_t)cur;
            cur += ln;
            p = q + n;
            return kStrOk;
        }
        // unmarked, or another verdict (a payload past the library's length limit): decode in place below
    }
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
        const uint8_t* rsrc = A.in + p;
        if (cur + (uint64_t)n > aend) {  // the validators' verdicts come first (an upper-case name is PROTOCOL)
            if (is_name && (n == 0 || rsrc[0] != ':')) {
                for (int64_t i = 0; i < n; ++i) {
                    const uint32_t c = rsrc[i];
                    if (c - 'A' < 26u) return kStrUpper;
                }
            }
            return kStrArena;
        }
        // one pass: 16 bytes in, validated (h2o_hpack_validate_header_name / _value, hpack.c:163-221), out
        const bool check_name = is_name && (n == 0 || rsrc[0] != ':');
        bool bad = is_name ? (n == 0 && check_name) : false, upper = false;
        uint8_t* dst = A.arena + cur;
        const uint32_t nn = (uint32_t)n;
        copy16([&](uint32_t i) { return rsrc[i]; },
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
            const uint32_t a = rsrc[0], z = rsrc[n - 1];
            bad |= a == ' ' || a == '\t' || z == ' ' || z == '\t';
        }
        if (bad) soft |= is_name ? 0x1u : 0x2u;
        len = (uint32_t)n;
    }
    off = (uint32_t)cur;
    src = kSrcArena | cur;
    cur += len;
    p += (uint64_t)n;
    return kStrOk;
}


// one field (h2o_hpack_decode_header, hpack.c:319-435): 0 / kErrInvalidChar = a field was produced.  F gets
// its arena places and byte sources; no bytes move here.
struct FieldDesc {
    uint32_t noff, nl, voff, vl, soft, cls;
    uint64_t nsrc, vsrc;
};

__device__ int32_t blk_field(const BlkArgs& A, const Win& W, DynTable& t, uint64_t& p, uint64_t end, uint64_t& cur,
                             uint64_t aend, FieldDesc& F, const DecTables& T, const uint16_t* SE, const uint16_t* scls,
                             bool want_cls) {
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
    uint32_t soft = 0, cls = kClsUnknown;
    if (index > 0) {
        if (index <= 61) {
            const uint32_t k = 4u * (uint32_t)(index - 1);
            const uint32_t no = SE[k], nl = SE[k + 1];
            if (cur + nl > aend) return kBlkArena;
            F.nsrc = kSrcStatic | no;
            F.nl = nl;
            F.noff = (uint32_t)cur;
            cur += nl;
            cls = scls[index - 1];
            if (value_indexed) {
                const uint32_t vo = SE[k + 2], vl = SE[k + 3];
                if (cur + vl > aend) return kBlkArena;
                F.vsrc = kSrcStatic | vo;
                F.vl = vl;
                F.voff = (uint32_t)cur;
                cur += vl;
            }
        } else if ((uint64_t)(index - 62) < t.num) {
            const Entry e = t.get((uint32_t)(index - 62));
            soft = e.soft;
            if (cur + e.nl > aend) return kBlkArena;
            F.nsrc = e.nsrc;
            F.nl = e.nl;
            F.noff = (uint32_t)cur;
            cur += e.nl;
            cls = e.cls;
            if (value_indexed) {
                if (cur + e.vl > aend) return kBlkArena;
                F.vsrc = e.vsrc;
                F.vl = e.vl;
                F.voff = (uint32_t)cur;
                cur += e.vl;
            }
        } else {
            return kErrCompression;
        }
    } else {
        const int r = blk_string(A, W, p, end, true, soft, cur, aend, F.noff, F.nl, F.nsrc, T);
        if (r == kStrArena) return kBlkArena;
        if (r != kStrOk) return r == kStrUpper ? kErrProtocol : kErrCompression;
    }
    if (!value_indexed) {
        soft &= ~0x2u;
        const int r = blk_string(A, W, p, end, false, soft, cur, aend, F.voff, F.vl, F.vsrc, T);
        if (r == kStrArena) return kBlkArena;
        if (r != kStrOk) return kErrCompression;
    }
    if (want_cls && cls == kClsUnknown) cls = req_name_class(src_ptr(A, F.nsrc), F.nl);
    if (do_index) t.add(Entry{F.nsrc, F.vsrc, F.nl, F.vl, (uint16_t)soft, (uint16_t)cls, 0u});
    F.soft = soft;
    F.cls = cls;
    return soft ? kErrInvalidChar : 0;
}

template <int MODE>
__global__ __launch_bounds__(kBlkThreads) void hpack_walk_kernel(BlkArgs A) {
    constexpr bool REQ = MODE == kWalkReq, RESP = MODE == kWalkResp;
    __shared__ __attribute__((aligned(16))) uint32_t s_lut[1u << HHUFF_LUT_BITS];  // literals decoded in place
    __shared__ uint32_t s_kinfo[32];
    __shared__ uint32_t s_ones[HHUFF_ONES_NENT];
    __shared__ uint16_t s_sent[61 * 4];
    __shared__ uint16_t s_scls[61];  // the static names' classes for the request rules
    for (uint32_t k = threadIdx.x; k < 61 * 4; k += blockDim.x) s_sent[k] = b_static_ent[k];
    for (uint32_t k = threadIdx.x; k < (1u << HHUFF_LUT_BITS) / 4; k += blockDim.x)
        reinterpret_cast<uint4*>(s_lut)[k] = reinterpret_cast<const uint4*>(b_dec_lut)[k];
    for (uint32_t k = threadIdx.x; k < HHUFF_ONES_NENT; k += blockDim.x) s_ones[k] = b_ones[k];
    if (threadIdx.x < 31) s_kinfo[threadIdx.x] = b_kinfo[threadIdx.x];
    if (threadIdx.x < 61)
        s_scls[threadIdx.x] = (uint16_t)req_name_class(b_static_bytes + b_static_ent[4 * threadIdx.x],
                                                       b_static_ent[4 * threadIdx.x + 1]);
    __syncthreads();
    DecTables T;  // assigned, not brace-initialised: a constant aggregate of LDS addresses cannot be a static initializer
    T.lut = s_lut;
    T.kinfo = s_kinfo;
    T.ones = s_ones;
    const uint32_t E = tbl_entries(A.table_size);
    const Win W{A.in, A.in_size};
    for (uint64_t c = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; c < A.nconn; c += (uint64_t)gridDim.x * blockDim.x) {
        uint8_t* scr = A.scratch + c * A.conn_scratch;
        TableState* ts = reinterpret_cast<TableState*>(scr);
        DynTable t{reinterpret_cast<Entry*>(scr + sizeof(TableState)), E, 0u, 0u, 0ull, A.table_size, A.table_size};
        TableState s0{0u, 0u, 0u, 0u, 0ull, A.table_size};
        if (A.flags & HHUFF_BLK_CONTINUE) s0 = *ts;
        t.start = s0.start;
        t.num = s0.num;
        t.size = s0.size;
        t.cap = s0.cap;
        bool failed = s0.failed != 0;
        for (uint32_t b = A.conn_first[c]; b < A.conn_first[c + 1]; ++b) {
            ReqState rq;
            RespState rs;
            if (REQ) rq.reset();
            if (RESP) rs.reset(A.trailers != nullptr && A.trailers[b] != 0);
            if (failed) {
                A.nfields[b] = 0;
                A.bstatus[b] = kBlkSkipped;
                if (REQ) req_store(A.req + b, rq);
                if (RESP) resp_store(A.res + b, rs);
                continue;
            }
            uint64_t p = A.blk_off[b];
            const uint64_t end = A.blk_off[b + 1];
            uint64_t cur = A.arena_off[b];
            const uint64_t aend = min(A.arena_off[b + 1], kArenaLimit);  // field offsets are u32
            const uint32_t slot = A.blk_off[b];
            uint32_t nf = 0;
            int32_t st = 0;
            // h2o_hpack_parse_response: a head must hold :status (:652-655); it loops do-while, so an empty
            // trailers block meets decode_header's end-of-input check (hpack.c:328-329)
            if (RESP && p == end) {
                if (!rs.trailers) rs.err = HHUFF_HERR_MISSING_PSEUDO;
                st = rs.trailers ? kErrCompression : kErrProtocol;
            }
            while (st == 0 && p != end) {
                FieldDesc F{0u, 0u, 0u, 0u, 0u, 0u, 0ull, 0ull};
                const int32_t rc = blk_field(A, W, t, p, end, cur, aend, F, T, s_sent, s_scls, MODE != kWalkPlain);
                if (rc != 0 && rc != kErrInvalidChar) {
                    st = rc;
                    // h2o_hpack_parse_request / _response: *err_desc = decode_err (:523-525, :663-665) -- only
                    // the upper-case name error carries one
                    if (REQ) rq.err = rc == kErrProtocol ? HHUFF_HERR_UPPER_CASE_NAME : HHUFF_HERR_NONE;
                    if (RESP) rs.err = rc == kErrProtocol ? HHUFF_HERR_UPPER_CASE_NAME : HHUFF_HERR_NONE;
                    break;
                }
                bool header = false;
                int32_t rr = 0;
                if (REQ) rr = req_field(rq, F.cls, src_ptr(A, F.vsrc), F.vl, F.soft, (int32_t)nf, header);
                if (RESP) rr = resp_field(rs, F.cls, src_ptr(A, F.vsrc), F.vl, F.soft, (int32_t)nf, header);
                const uint32_t f = slot + nf;
                A.name_off[f] = F.noff;
                A.name_len[f] = F.nl;
                A.value_off[f] = F.voff;
                A.value_len[f] = F.vl;
                A.fflags[f] = (uint8_t)(F.soft | (header ? HHUFF_FIELD_HEADER : 0u));
                A.fsrc_n[f] = F.nsrc;
                A.fsrc_v[f] = F.vsrc;
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
            if (RESP) {
                if (st == 0 && rs.err != HHUFF_HERR_NONE) st = kErrInvalidChar;  // :745-747
                resp_store(A.res + b, rs);
            }
            A.nfields[b] = nf;
            A.bstatus[b] = st;
            failed = st != 0 && st != kErrInvalidChar;
        }
        *ts = TableState{t.start, t.num, s0.ring, failed ? 1u : 0u, t.size, t.cap};
    }
}

// Copy pass: 64 blocks per wave (wave_copy_fields), their fields' name / value bytes into the arena
// (literals decoded in place already sit there).
__global__ __launch_bounds__(256) void blk_copy_kernel(BlkArgs A) {
    const int lane = threadIdx.x & 63;
    const uint32_t nblk = A.conn_first[A.nconn];
    const uint32_t nw = gridDim.x * 4u;
    for (uint32_t b0 = (blockIdx.x * 4u + (threadIdx.x >> 6)) * 64u; b0 < nblk; b0 += nw * 64u) {
        const uint32_t b = b0 + (uint32_t)lane;
        const uint32_t s0 = b < nblk ? A.blk_off[b] : 0u, nf = b < nblk ? A.nfields[b] : 0u;
        wave_copy_fields(s0, nf, lane, [&](uint32_t f, bool val, const uint8_t*& src, uint8_t*& dst, uint32_t& len) {
            const uint32_t off = val ? A.value_off[f] : A.name_off[f];
            const uint64_t fs = val ? A.fsrc_v[f] : A.fsrc_n[f];
            src = src_ptr(A, fs);
            dst = A.arena + off;
            len = fs == (kSrcArena | off) ? 0u : (val ? A.value_len[f] : A.name_len[f]);
        });
    }
}

// Table pass: one wave per connection writes its live entries' bytes, newest first, into the ring the
// entries do not use now, and points the entries there: the next call (HHUFF_BLK_CONTINUE) reads only
// scratch.  Live bytes never exceed table_size (each entry costs its bytes + 32 of the capacity).
__global__ __launch_bounds__(256) void blk_table_kernel(BlkArgs A) {
    const int lane = threadIdx.x & 63;
    const uint64_t c = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    if (c >= A.nconn) return;
    const uint32_t E = tbl_entries(A.table_size);
    const uint64_t base = c * A.conn_scratch;
    TableState* ts = reinterpret_cast<TableState*>(A.scratch + base);
    Entry* ent = reinterpret_cast<Entry*>(A.scratch + base + sizeof(TableState));
    const TableState s = *ts;
    const uint32_t nring = s.ring ^ 1u;
    const uint64_t rbase = base + sizeof(TableState) + (uint64_t)E * sizeof(Entry) + nring * tbl_ring(A.table_size);
    uint32_t carry = 0;
    for (uint32_t k0 = 0; k0 < s.num; k0 += 64) {
        const uint32_t k = k0 + (uint32_t)lane;
        const bool live = k < s.num;
        uint32_t i = s.start + k;
        i = i >= E ? i - E : i;
        Entry e{};
        if (live) e = ent[i];
        const uint32_t sz = live ? e.nl + e.vl : 0u;
        const uint32_t dst = carry + wave_excl_scan(sz, lane);
        carry += (uint32_t)__builtin_amdgcn_readlane((int)(dst - carry + sz), 63);
        uint8_t* d = A.scratch + rbase + dst;
        wave_copy64(src_ptr(A, e.nsrc), d, live ? e.nl : 0u, lane);
        wave_copy64(src_ptr(A, e.vsrc), d + e.nl, live ? e.vl : 0u, lane);
        if (live) {
            ent[i].nsrc = kSrcScr | (rbase + dst);
            ent[i].vsrc = kSrcScr | (rbase + dst + e.nl);
        }
    }
    if (lane == 0) ts->ring = nring;
}

// ---------------------------------------------------------------------------------------------------
// Literal pre-pass.  The representation of a block is readable without its connection's table: index
// values and literal lengths are explicit (hpack.c:336-366, 223-236), so one lane per block can find every
// string literal a decoder of that block could reach.  Those are decoded together by the literal kernels
// (balanced across all connections, launch_literals_dev), and the per-connection walk then copies results
// instead of running a Huffman decoder per lane -- one lane per connection otherwise steps through 64
// connections' literals in lock step, each field costing the wave its slowest lane's literal.  The walk
// marks may include literals past a table-dependent error (an index beyond the table): decoded, unused.
// ---------------------------------------------------------------------------------------------------
constexpr uint32_t kMarkThreads = 256, kChunkWords = 1024;  // list pass: 1024 bitmap words per block

// literal at p (H flag + 7-bit-prefix length, then the payload) inside [p, end): mark it, step over it
__device__ __forceinline__ bool mark_literal(const Win& W, uint64_t& p, uint64_t end, bool is_name,
                                             uint32_t* __restrict__ lit_bits, uint32_t* __restrict__ name_bits) {
    if (p >= end) return false;
    uint64_t q = p;
    const int64_t n = blk_decode_int(W, q, end, 7);
    if (n < 0 || (uint64_t)n > end - q) return false;
    atomicOr(lit_bits + (p >> 5), 1u << (p & 31));
    if (is_name) atomicOr(name_bits + (p >> 5), 1u << (p & 31));
    p = q + (uint64_t)n;
    return true;
}

__global__ __launch_bounds__(kMarkThreads) void blk_mark_kernel(const uint8_t* __restrict__ in, uint64_t in_size,
                                                               const uint32_t* __restrict__ blk_off,
                                                               const uint32_t* __restrict__ conn_first, uint32_t nconn,
                                                               uint32_t* __restrict__ lit_bits,
                                                               uint32_t* __restrict__ name_bits) {
    const uint32_t nblk = conn_first[nconn];
    const Win W{in, in_size};
    for (uint32_t b = blockIdx.x * kMarkThreads + threadIdx.x; b < nblk; b += gridDim.x * kMarkThreads) {
        uint64_t p = blk_off[b];
        const uint64_t end = blk_off[b + 1];
        while (p < end) {  // the representation switch of blk_field / h2o_hpack_decode_header
            const uint32_t c = W.byte(p);
            bool name_lit = false;
            if (c >= 128) {
                if (blk_decode_int(W, p, end, 7) <= 0) break;
                continue;  // indexed: no literal
            } else if (c >= 64) {
                if (c == 64) {
                    ++p;
                    name_lit = true;
                } else if (blk_decode_int(W, p, end, 6) <= 0) {
                    break;
                }
            } else if (c < 32) {
                if ((c & 0xFu) == 0) {
                    ++p;
                    name_lit = true;
                } else if (blk_decode_int(W, p, end, 4) <= 0) {
                    break;
                }
            } else {
                if (blk_decode_int(W, p, end, 5) < 0) break;
                continue;  // table size update
            }
            if (name_lit && !mark_literal(W, p, end, true, lit_bits, name_bits)) break;
            if (!mark_literal(W, p, end, false, lit_bits, name_bits)) break;
        }
    }
}

// block-wide exclusive scan of one value per thread (kMarkThreads threads); *total = the block's sum
__device__ __forceinline__ uint32_t block_excl_scan(uint32_t v, uint32_t* sh, uint32_t* total) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint32_t incl = wave_incl_scan(v);
    if (lane == 63) sh[wave] = incl;
    __syncthreads();
    uint32_t base = 0, sum = 0;
    for (int k = 0; k < (int)(kMarkThreads / 64); ++k) {
        base += k < wave ? sh[k] : 0u;
        sum += sh[k];
    }
    __syncthreads();
    *total = sum;
    return base + incl - v;
}

// marks per chunk of kChunkWords bitmap words
__global__ __launch_bounds__(kMarkThreads) void blk_count_kernel(const uint32_t* __restrict__ lit_bits, uint64_t nwords,
                                                                uint32_t* __restrict__ chunk_sum) {
    __shared__ uint32_t sh[kMarkThreads / 64];
    const uint64_t w0 = (uint64_t)blockIdx.x * kChunkWords + threadIdx.x * (kChunkWords / kMarkThreads);
    uint32_t c = 0;
#pragma unroll
    for (uint32_t k = 0; k < kChunkWords / kMarkThreads; ++k)
        c += w0 + k < nwords ? (uint32_t)__builtin_popcount(lit_bits[w0 + k]) : 0u;
    uint32_t total;
    (void)block_excl_scan(c, sh, &total);
    if (threadIdx.x == 0) chunk_sum[blockIdx.x] = total;
}

// exclusive scan of the chunk sums in place (one block); *n_lit = the number of literals
__global__ __launch_bounds__(kMarkThreads) void blk_chunk_scan_kernel(uint32_t* __restrict__ chunk_sum, uint32_t nchunks,
                                                                     uint32_t* __restrict__ n_lit) {
    __shared__ uint32_t sh[kMarkThreads / 64];
    uint32_t carry = 0;
    for (uint32_t c0 = 0; c0 < nchunks; c0 += kMarkThreads) {
        const uint32_t i = c0 + threadIdx.x;
        const uint32_t v = i < nchunks ? chunk_sum[i] : 0u;
        uint32_t total;
        const uint32_t ex = block_excl_scan(v, sh, &total);
        if (i < nchunks) chunk_sum[i] = carry + ex;
        carry += total;
    }
    if (threadIdx.x == 0) *n_lit = carry;
}

// per bitmap word: the marks before it (word_pre), and the literal list in position order: lit_off[r],
// and bit r of lnames for the names
__global__ __launch_bounds__(kMarkThreads) void blk_list_kernel(const uint32_t* __restrict__ lit_bits,
                                                               const uint32_t* __restrict__ name_bits, uint64_t nwords,
                                                               const uint32_t* __restrict__ chunk_pre,
                                                               uint32_t* __restrict__ word_pre,
                                                               uint32_t* __restrict__ lit_off, uint32_t* __restrict__ lnames,
                                                               const uint32_t* __restrict__ pfx_bits, uint32_t pfx_alt,
                                                               uint32_t pfx_name, uint8_t* __restrict__ prefix_of) {
    __shared__ uint32_t sh[kMarkThreads / 64];
    constexpr uint32_t K = kChunkWords / kMarkThreads;
    const uint64_t w0 = (uint64_t)blockIdx.x * kChunkWords + threadIdx.x * K;
    uint32_t bits[K], c = 0;
#pragma unroll
    for (uint32_t k = 0; k < K; ++k) {
        bits[k] = w0 + k < nwords ? lit_bits[w0 + k] : 0u;
        c += (uint32_t)__builtin_popcount(bits[k]);
    }
    uint32_t total;
    uint32_t r = chunk_pre[blockIdx.x] + block_excl_scan(c, sh, &total);
#pragma unroll
    for (uint32_t k = 0; k < K; ++k) {
        if (w0 + k >= nwords) break;
        word_pre[w0 + k] = r;
        uint32_t m = bits[k];
        const uint32_t nm = m ? name_bits[w0 + k] : 0u;
        const uint32_t pm = m && prefix_of ? pfx_bits[w0 + k] : 0u;
        while (m) {
            const uint32_t bit = (uint32_t)__builtin_ctz(m);
            m &= m - 1u;
            lit_off[r] = (uint32_t)(32u * (w0 + k) + bit);
            if ((nm >> bit) & 1u) atomicOr(lnames + (r >> 5), 1u << (r & 31));
            if (prefix_of) prefix_of[r] = (uint8_t)(((pm >> bit) & 1u) ? pfx_alt : ((nm >> bit) & 1u) ? pfx_name : 7u);
            ++r;
        }
    }
}
uint64_t literal_list_chunks(uint64_t nwords) { return (nwords + kChunkWords - 1) / kChunkWords; }

hipError_t launch_literal_list(const uint32_t* lit_bits, const uint32_t* name_bits, const uint32_t* pfx_bits, uint32_t pfx_alt,
                               uint32_t pfx_name, uint64_t nwords, uint32_t* chunk, uint32_t* word_pre, uint32_t* list, uint32_t* lnames,
                               uint8_t* prefix_of, hipStream_t stream) {
    const uint64_t nchunks = literal_list_chunks(nwords);
    hipLaunchKernelGGL(blk_count_kernel, dim3((uint32_t)nchunks), dim3(kMarkThreads), 0, stream, lit_bits, nwords, chunk);
    hipLaunchKernelGGL(blk_chunk_scan_kernel, dim3(1), dim3(kMarkThreads), 0, stream, chunk, (uint32_t)nchunks,
                       chunk + nchunks);
    hipLaunchKernelGGL(blk_list_kernel, dim3((uint32_t)nchunks), dim3(kMarkThreads), 0, stream, lit_bits, name_bits, nwords,
                       chunk, word_pre, list, lnames, pfx_bits, pfx_alt, pfx_name, prefix_of);
    return hipGetLastError();
}

uint64_t hpack_conn_scratch(uint32_t table_size) {
    return sizeof(TableState) + (uint64_t)tbl_entries(table_size) * sizeof(Entry) + 2 * tbl_ring(table_size);
}

hipError_t launch_hpack_blocks(const uint8_t* in, uint64_t in_size, const uint32_t* blk_off, const uint32_t* conn_first,
                               uint32_t nconn, uint32_t table_size, uint8_t* arena, const uint64_t* arena_off,
                               uint32_t* name_off, uint32_t* name_len, uint32_t* value_off, uint32_t* value_len,
                               uint8_t* fflags, uint32_t* nfields, int32_t* bstatus, hhuff_request_t* req,
                               hhuff_response_t* res, const uint8_t* trailers, uint8_t* scratch, uint32_t flags,
                               hipStream_t stream) {
    if (nconn == 0) return hipSuccess;
    BlkArgs A{in, in_size, blk_off, conn_first, nconn, table_size, arena, arena_off, name_off, name_len, value_off,
              value_len, fflags, nfields, bstatus, scratch, hpack_conn_scratch(table_size), flags, req,
              nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, res, trailers};
    // workspace (the library's stream-ordered pool): field sources for every slot (block byte);
    // with the literal pre-pass (inputs below 4 GiB: u32 positions) its bitmaps, word prefixes, chunk sums,
    // the literal list and results, and the decoded bytes
    const uint64_t nslots = in_size;
    const bool prepass = in_size > 0 && in_size < (1ull << 32);
    const uint64_t nwords = (in_size + 31) / 32, nchunks = (nwords + kChunkWords - 1) / kChunkWords;
    const uint64_t n_max = (2 * in_size) / 3 + 2;  // a field with two literals takes >= 3 bytes
    auto up = [](uint64_t x) { return (x + 255) & ~255ull; };
    uint64_t o = 0;
    const uint64_t o_lit = o;
    if (prepass) o += up(4 * nwords);
    const uint64_t o_name = o;
    if (prepass) o += up(4 * nwords);
    const uint64_t o_lnames = o;
    if (prepass) o += up(4 * ((n_max + 31) / 32));
    const uint64_t zero_end = o;  // [0, zero_end) starts zeroed
    const uint64_t o_fsn = o;
    o += up(8 * nslots + 8);
    const uint64_t o_fsv = o;
    o += up(8 * nslots + 8);
    const uint64_t o_pre = o, o_chunk = o_pre + (prepass ? up(4 * nwords) : 0);
    const uint64_t o_list = o_chunk + (prepass ? up(4 * nchunks + 4) : 0);
    const uint64_t o_len = o_list + (prepass ? up(4 * n_max) : 0);
    const uint64_t o_pay = o_len + (prepass ? up(4 * n_max) : 0);
    const uint64_t o_cons = o_pay + (prepass ? up(4 * n_max) : 0);
    const uint64_t o_st = o_cons + (prepass ? up(4 * n_max) : 0);
    const uint64_t o_ws = o_st + (prepass ? up(n_max) : 0);
    const uint64_t o_out = o_ws + (prepass ? up(literals_dev_ws((uint32_t)n_max, in_size)) : 0);
    o = o_out + (prepass ? up((8 * in_size) / 5 + 64) : 0);
    uint8_t* work = nullptr;
    hipError_t e = work_alloc((void**)&work, o, stream);
    if (e != hipSuccess) return e;
    A.fsrc_n = reinterpret_cast<uint64_t*>(work + o_fsn);
    A.fsrc_v = reinterpret_cast<uint64_t*>(work + o_fsv);
    e = hipMemsetAsync(work, 0, zero_end, stream);
    if (e == hipSuccess && prepass) {
        uint32_t* lit_bits = reinterpret_cast<uint32_t*>(work + o_lit);
        uint32_t* name_bits = reinterpret_cast<uint32_t*>(work + o_name);
        uint32_t* lnames = reinterpret_cast<uint32_t*>(work + o_lnames);
        uint32_t* word_pre = reinterpret_cast<uint32_t*>(work + o_pre);
        uint32_t* chunk = reinterpret_cast<uint32_t*>(work + o_chunk);
        uint32_t* n_lit = chunk + nchunks;
        uint32_t* list = reinterpret_cast<uint32_t*>(work + o_list);
        hipLaunchKernelGGL(blk_mark_kernel, dim3(2048), dim3(kMarkThreads), 0, stream, in, in_size, blk_off, conn_first,
                           nconn, lit_bits, name_bits);
        e = hipGetLastError();
        if (e == hipSuccess)
            e = launch_literal_list(lit_bits, name_bits, nullptr, 7u, 7u, nwords, chunk, word_pre, list, lnames, nullptr, stream);
        if (e == hipSuccess)
            e = launch_literals_dev(in, in_size, list, (uint32_t)n_max, n_lit, 7u, kLitNoRawCopy, lnames, work + o_out,
                                    reinterpret_cast<uint32_t*>(work + o_len), reinterpret_cast<uint32_t*>(work + o_pay),
                                    reinterpret_cast<uint32_t*>(work + o_cons), work + o_st, work + o_ws, stream);
        A.lit_bits = lit_bits;
        A.word_pre = word_pre;
        A.lit_len = reinterpret_cast<const uint32_t*>(work + o_len);
        A.lit_pay = reinterpret_cast<const uint32_t*>(work + o_pay);
        A.lit_cons = reinterpret_cast<const uint32_t*>(work + o_cons);
        A.lit_st = work + o_st;
        A.lit_out = work + o_out;
    }
    if (e == hipSuccess) {
        const uint32_t blocks = min((nconn + kBlkThreads - 1u) / kBlkThreads, 65535u);
        if (req)
            hipLaunchKernelGGL(hpack_walk_kernel<kWalkReq>, dim3(blocks), dim3(kBlkThreads), 0, stream, A);
        else if (res)
            hipLaunchKernelGGL(hpack_walk_kernel<kWalkResp>, dim3(blocks), dim3(kBlkThreads), 0, stream, A);
        else
            hipLaunchKernelGGL(hpack_walk_kernel<kWalkPlain>, dim3(blocks), dim3(kBlkThreads), 0, stream, A);
        hipLaunchKernelGGL(blk_copy_kernel, dim3(4096), dim3(256), 0, stream, A);
        hipLaunchKernelGGL(blk_table_kernel, dim3((uint32_t)(((uint64_t)nconn + 3) / 4)), dim3(256), 0, stream, A);
        e = hipGetLastError();
    }
    const hipError_t f = hipFreeAsync(work, stream);
    return e != hipSuccess ? e : f;
}

}  // namespace hhuff
