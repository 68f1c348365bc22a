// QPACK decoding on the GPU (QPACK half): h2o's QPACK decoder, lib/http3/qpack.c.
//   encoder stream  h2o_qpack_decoder_handle_input (:420-485) -- insert with static / dynamic name
//                   reference (:289-348), insert with a literal name (:352-393), duplicate (:395-406),
//                   set dynamic table capacity (:408-418) -- into one dynamic table per connection
//                   (header_table_insert :166-190, header_table_evict :153-164)
//   field sections  h2o_qpack_parse_request's reading of a section (:830-858): parse_decode_context
//                   (:754-799), check_decode_context_blocked (:801-820), then decode_header (:652-752)
//                   field after field (resolve_static / resolve_dynamic / _postbase :506-557, literals
//                   :559-629)
//
// Decomposition.  Unlike HPACK, a QPACK field section never changes the dynamic table: only the encoder
// stream does.  A step runs as passes on the stream:
//   literal pre-pass       qpack_mark_kernel (one lane per encoder stream or section) marks every string
//                          literal -- instructions and field lines are readable without the table -- and
//                          the literal kernels decode them all, balanced across connections;
//   qpack_encoder_kernel   one lane per connection applies its encoder-stream instructions in order, on
//                          integers only: an entry is a pair of REFERENCES to where its name and value bytes
//                          are (a pre-decoded literal, the input, the static table, or an entry's ring);
//   qpack_table_kernel     one wave per connection whose table changed writes the live entries' bytes back
//                          to back into its other ring and points the entries there;
//   qpack_sections_kernel  one lane per field SECTION (many per connection) decodes it against that table,
//                          recording each field string's source; qpack_copy_kernel (one wave per section)
//                          moves the bytes into the arena.
// The table lives in per-connection scratch in HBM: an entry ring of header_table_size / 32 + 1 records
// {name source, value source, lengths, soft bits}, oldest first, absolute index = base_offset + position as
// in h2o (base_offset starts at 1, :143), and two byte rings of header_table_size bytes (live entries hold
// at most max_size <= header_table_size bytes).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

#include "hhuff_device.h"
#include "hhuff.h"
#include "hhuff_launch.h"
#include "hhuff_request.h"

namespace hhuff {
namespace {
__device__ const uint32_t q_dec_lut[1u << HHUFF_LUT_BITS] = HHUFF_DEC_LUT_INIT;
__device__ const uint32_t q_kinfo[31] = HHUFF_ONES_KINFO_INIT;
__device__ const uint32_t q_ones[HHUFF_ONES_NENT] = HHUFF_ONES_ENT_INIT;
__device__ const uint32_t q_name_invalid[8] = HHUFF_NAME_INVALID_INIT;
__device__ const uint32_t q_value_invalid[8] = HHUFF_VALUE_INVALID_INIT;
__device__ const uint8_t q_static_bytes[HHUFF_QSTATIC_NBYTES] = HHUFF_QSTATIC_BYTES_INIT;
__device__ const uint16_t q_static_ent[99 * 4] = HHUFF_QSTATIC_ENT_INIT;

constexpr uint32_t kQStaticCount = 99;  // h2o_qpack_static_table (include/h2o/token_table.h)
constexpr int32_t kDF = HHUFF_QPK_DECOMPRESSION_FAILED;
constexpr int32_t kQIncomplete = -1;       // H2O_HTTP3_ERROR_INCOMPLETE (http3_common.h:77)
constexpr int32_t kErrInvalidChar = -254;  // H2O_HTTP2_ERROR_INVALID_HEADER_CHAR
constexpr uint32_t kEntryOverhead = 32;    // HEADER_ENTRY_SIZE_OFFSET (qpack.c:32)
constexpr int64_t kQuicIntMax = 4611686018427387903LL;  // PTLS_QUICINT_MAX
constexpr int64_t kIntIncomplete = -255, kIntBad = -9;
}  // namespace

struct QpkArgs {
    const uint8_t* in;
    uint64_t in_size;
    const uint32_t *enc_off, *enc_len, *sec_off, *conn_first, *num_blocked;
    uint32_t nconn, nsec, T;  // T = header_table_size
    uint64_t max_blocked;
    uint8_t* arena;
    const uint64_t* arena_off;
    uint32_t *name_off, *name_len, *value_off, *value_len;
    uint8_t* fflags;
    uint32_t* nfields;
    int32_t* sstatus;
    uint64_t* req_insert_count;
    int32_t* enc_status;
    uint32_t* enc_consumed;
    uint64_t* insert_count;
    uint8_t* scratch;
    uint64_t conn_scratch;
    uint32_t flags;
    // pre-decoded encoder-stream literals (launch_qpack's pre-pass): bit p of lit_bits marks a literal whose
    // header starts at input byte p; word_pre[w] counts the marks before word w; literal r has the literal
    // kernels' results lit_len / lit_st, its bytes at lit_out + floor(8 payload / 5) (Huffman) or in the
    // input (raw).  NULL lit_bits: every literal is decoded in place.
    const uint32_t* lit_bits;
    const uint32_t* word_pre;
    const uint32_t* lit_len;
    const uint8_t* lit_st;
    const uint8_t* lit_pfx;  // the prefix literal r was decoded with
    const uint8_t* lit_out;
    // deferred section copies (with the pre-pass): per field slot, the address of its name's / value's
    // bytes (0: already in the arena); qpack_copy_kernel moves them.  NULL: the sections kernel copies.
    uint64_t* fsrc_n;
    uint64_t* fsrc_v;
    // h2o_qpack_parse_request mode (hhuff_qpack_parse_requests): per section its stream id and record
    const uint64_t* stream_id;
    hhuff_qpack_request_t* qreq;
    // h2o_qpack_parse_response mode (hhuff_qpack_parse_responses): per section its record (and stream_id)
    hhuff_qpack_response_head_t* qres;
};

// Byte sources of table entries and field strings: kind in the top 3 bits, offset below.  Every source stays
// valid until the call's last pass has run; between calls the entries' sources are all kQScr (their
// connection's ring in scratch), so a caller may keep scratch anywhere (offsets, not addresses).
constexpr uint64_t kQLit = 0;              // lit_out offset (a literal the pre-pass decoded, or decoded in place)
constexpr uint64_t kQStatic = 1ull << 61;  // static-table bytes
constexpr uint64_t kQScr = 2ull << 61;     // scratch offset (a ring: bytes an earlier call's table pass wrote)
constexpr uint64_t kQIn = 3ull << 61;      // input offset (a raw literal)
constexpr uint64_t kQOff = (1ull << 61) - 1;

__device__ __forceinline__ const uint8_t* q_src(const QpkArgs& A, uint64_t s) {
    const uint64_t o = s & kQOff;
    switch (s >> 61) {
        case 0: return A.lit_out + o;
        case 1: return q_static_bytes + o;
        case 2: return A.scratch + o;
        default: return A.in + o;
    }
}

// per-connection scratch: [QState 64 B][entry ring E x 32 B][ring 0][ring 1] (rings: T rounded up to 16 B).
// Live entries hold at most max_size <= T bytes, so the table pass (qpack_table_kernel) writes them back to
// back into the ring they do not use now, reading their sources from the other one.
struct QState {
    int64_t base_offset;
    uint64_t total_inserts, num_bytes, max_size;
    uint32_t start, num, ring, failed;  // ring: which ring holds the entries' bytes between calls
    uint32_t dirty, pad[3];             // dirty: entries inserted by this call (the table pass rewrites)
};
static_assert(sizeof(QState) == 64, "QState layout");
struct QEntry {  // one dynamic-table entry: references to its name and value bytes
    uint64_t nsrc, vsrc;
    uint32_t nl, vl, soft, pad;
};
static_assert(sizeof(QEntry) == 32, "QEntry layout");

__host__ __device__ __forceinline__ uint32_t qpk_ring_bytes(uint32_t T) { return ((T < 16u ? 16u : T) + 15u) & ~15u; }
__host__ __device__ __forceinline__ uint32_t qpk_entries(uint32_t T) { return T / kEntryOverhead + 1u; }

// h2o_hpack_decode_int (lib/http2/hpack.c:52-83) at in[p], bounded by end
__device__ int64_t q_hpack_int(const uint8_t* __restrict__ in, uint64_t& p, uint64_t end, uint32_t prefix_bits) {
    if (p >= end) return kIntIncomplete;
    const uint64_t pmax = (1u << prefix_bits) - 1u;
    uint64_t v = in[p++] & pmax;
    if (v != pmax) return (int64_t)v;
    uint32_t shift = 0;
    for (; shift < 56; shift += 7) {
        if (p == end) return kIntIncomplete;
        const uint32_t b = in[p++];
        v += (uint64_t)(b & 127u) << shift;
        if (!(b & 128u)) return (int64_t)v;
    }
    if (p == end) return kIntIncomplete;
    if (in[p] & 128u) return kIntBad;
    v += (uint64_t)(in[p++] & 127u) << shift;
    if (v > 0x7FFFFFFFFFFFFFFFull) return kIntBad;
    return (int64_t)v;
}

// decode_int (qpack.c:215-220): 0, kQIncomplete or kDF
__device__ __forceinline__ int32_t q_int(int64_t& v, const uint8_t* in, uint64_t& p, uint64_t end, uint32_t prefix) {
    v = q_hpack_int(in, p, end, prefix);
    if (v < 0) return v == kIntIncomplete ? kQIncomplete : kDF;
    return 0;
}

// h2o_hpack_validate_header_name (hpack.c:163-192): false on an upper-case letter, soft name bit otherwise
template <class Get>
__device__ bool q_valid_name(Get get, uint64_t n, uint32_t& soft) {
    bool bad = n == 0;
    for (uint64_t i = 0; i < n; ++i) {
        const uint32_t c = get(i);
        if ((q_name_invalid[c >> 5] >> (c & 31)) & 1u) {
            if (c - 'A' < 26u) return false;
            bad = true;
        }
    }
    if (bad) soft |= 0x1u;
    return true;
}

// h2o_hpack_validate_header_value (hpack.c:194-221) with the whole-value rule (:110-115)
template <class Get>
__device__ void q_valid_value(Get get, uint64_t n, uint32_t& soft) {
    bool bad = false;
    if (n != 0) {
        const uint32_t f = get(0), l = get(n - 1);
        bad = f == ' ' || f == '\t' || l == ' ' || l == '\t';
    }
    for (uint64_t i = 0; !bad && i < n; ++i) {
        const uint32_t c = get(i);
        bad = ((q_value_invalid[c >> 5] >> (c & 31)) & 1u) != 0;
    }
    if (bad) soft |= 0x2u;
}

// h2o_lookup_token on a raw name (qpack.c:585) can only change a verdict for the pseudo-header tokens
// (every other token is a valid lower-case name): :authority :method :path :protocol :scheme :status
template <class Get>
__device__ bool q_pseudo_token(Get get, uint64_t n) {
    if (n < 5 || n > 10 || get(0) != ':') return false;
    const char* const tok[6] = {":authority", ":method", ":path", ":protocol", ":scheme", ":status"};
    const uint8_t len[6] = {10, 7, 5, 9, 7, 7};
    for (int k = 0; k < 6; ++k) {
        if (len[k] != n) continue;
        bool eq = true;
        for (uint64_t i = 1; eq && i < n; ++i) eq = get(i) == (uint8_t)tok[k][i];
        if (eq) return true;
    }
    return false;
}

// sink with first / last byte tracking over a RegSink (soft bits need them, hpack.c:136-152)
struct ArenaSinkFL {
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
};

struct QTable {  // one connection's table, as the kernels see it
    QEntry* ent;
    uint32_t E;
    QState s;
    __device__ __forceinline__ uint32_t slot(uint32_t k) const {
        const uint32_t i = s.start + k;
        return i >= E ? i - E : i;
    }
    __device__ __forceinline__ QEntry get(uint32_t k) const { return ent[slot(k)]; }  // k-th oldest live entry
    __device__ __forceinline__ int64_t total() const { return s.base_offset + (int64_t)s.num; }  // :321-324
    __device__ __forceinline__ bool resolve_abs(int64_t index, QEntry& e) const {  // resolve_dynamic_abs :201-213
        if (index < s.base_offset || index - s.base_offset >= (int64_t)s.num) return false;
        e = get((uint32_t)(index - s.base_offset));
        return true;
    }
    __device__ void evict(uint64_t delta) {  // header_table_evict (:153-164)
        while (s.num != 0 && s.num_bytes + delta > s.max_size) {
            const uint2 l = *reinterpret_cast<const uint2*>(&ent[s.start].nl);
            s.num_bytes -= (uint64_t)l.x + l.y + kEntryOverhead;
            s.start = s.start + 1 == E ? 0u : s.start + 1;
            --s.num;
            ++s.base_offset;
        }
    }
    // header_table_insert (:166-190): the entry's bytes are references; the table pass writes them
    __device__ void commit(const QEntry& e) {
        const uint64_t add = (uint64_t)e.nl + e.vl + kEntryOverhead;
        evict(add);
        ent[slot(s.num)] = e;
        ++s.num;
        s.num_bytes += add;
        ++s.total_inserts;
        s.dirty = 1;
    }
};

// pre-pass literal marks (qpack_mark_kernel): names are the 5-bit-prefix literals (encoder stream) and the
// 3-bit-prefix ones (sections, also in p3_bits); everything else is a value (7-bit prefix)
// the pre-decoded literal whose header is at input byte p, or -1: not marked, decoded with another prefix
// (input regions that overlap), or a verdict other than success (the in-place path then reproduces the
// reference's exact failure)
__device__ __forceinline__ int64_t q_pre(const QpkArgs& A, uint64_t p, uint32_t prefix) {
    const uint32_t w = A.lit_bits[p >> 5], m = 1u << (p & 31);
    if (!(w & m)) return -1;
    const uint32_t r = A.word_pre[p >> 5] + (uint32_t)__builtin_popcount(w & (m - 1u));
    return ((A.lit_st[r] >> 2) & 7u) == 0 && A.lit_pfx[r] == prefix ? (int64_t)r : -1;
}

// An encoder-stream string literal (H flag at bit `prefix`, length, payload at p after the header): its
// source and length.  Pre-decoded (pre >= 0): the pre-pass results.  Otherwise decoded here -- a Huffman
// payload into lit_out at the place the pre-pass would have used (floor(8 p / 5)), a raw one validated
// and referenced in the input -- with the reference's verdicts (qpack.c:222-237, :362-378).
__device__ bool q_enc_string(const QpkArgs& A, bool huff, bool is_name, uint64_t p, uint64_t n, int64_t pre,
                             uint64_t& src, uint32_t& len, uint32_t& soft, const DecTables& T) {
    if (pre >= 0) {
        len = A.lit_len[pre];
        soft |= A.lit_st[pre] & 3u;
        src = huff ? kQLit | ((p * 8u) / 5u) : kQIn | p;
        return true;
    }
    if (huff) {
        if (n > kMaxStrLen) return false;
        ArenaSinkFL sk{RegSink{}, 0u, 0u};
        sk.s.init(const_cast<uint8_t*>(A.lit_out) + (p * 8u) / 5u);
        const DecResult d = decode_core(GlobalSource{A.in, A.in_size}, (uint32_t)p, (uint32_t)n, sk, T);
        if (!d.ok) return false;
        sk.s.finish();
        soft |= soft_bits(is_name, d.len, d.flags, sk.first, sk.last);
        len = d.len;
        src = kQLit | ((p * 8u) / 5u);
        return true;
    }
    const uint8_t* s = A.in + p;
    if (is_name) {
        if (!q_valid_name([&](uint64_t i) { return (uint32_t)s[i]; }, n, soft)) return false;
    } else {
        q_valid_value([&](uint64_t i) { return (uint32_t)s[i]; }, n, soft);
    }
    len = (uint32_t)n;
    src = kQIn | p;
    return true;
}

// the value half of an insert (decode_value_and_insert :273-287)
__device__ int32_t q_value_and_insert(QTable& t, const QpkArgs& A, QEntry e, bool vhuff, uint64_t vp, uint64_t vlen,
                                      int64_t pre, const DecTables& T) {
    if (!q_enc_string(A, vhuff, false, vp, vlen, pre, e.vsrc, e.vl, e.soft, T)) return kDF;
    if ((uint64_t)e.nl + e.vl + kEntryOverhead > t.s.max_size) return kDF;  // header exceeds table size (:278-281)
    t.commit(e);
    return 0;
}

// h2o_qpack_decoder_handle_input (qpack.c:420-485) over in[p, end)
__device__ int32_t q_handle_input(QTable& t, const QpkArgs& A, uint64_t p, uint64_t end, uint32_t& consumed,
                                  uint64_t& insert_count, const DecTables& T) {
    const uint8_t* in = A.in;
    const uint64_t p0 = p;
    uint64_t done = p;
    const uint64_t old_total = t.s.total_inserts;
    int32_t ret = 0;
    insert_count = 0;
    while (p != end && ret == 0) {
        const uint32_t b = in[p];
        switch (b >> 5) {
            default: {  // insert with name reference (:430-444)
                int64_t name_index, value_len;
                const bool name_is_static = (b & 0x40u) != 0;
                if ((ret = q_int(name_index, in, p, end, 6)) != 0) goto Exit;
                if (p == end) goto Exit;
                const int64_t vpre = q_pre(A, p, 7);
                const bool vhuff = (in[p] & 0x80u) != 0;
                if ((ret = q_int(value_len, in, p, end, 7)) != 0) goto Exit;
                if (!((uint64_t)value_len <= end - p)) goto Exit;
                QEntry e{};
                if (name_is_static) {  // insert_token_header (:289-300): soft starts at 0
                    if ((uint64_t)name_index >= kQStaticCount) {
                        ret = kDF;
                    } else {
                        const uint32_t k = 4u * (uint32_t)name_index;
                        e.nsrc = kQStatic | q_static_ent[k];
                        e.nl = q_static_ent[k + 1];
                        ret = q_value_and_insert(t, A, e, vhuff, p, (uint64_t)value_len, vpre, T);
                    }
                } else {  // dynamic (:335-348): token names carry no name bit, literal names keep theirs
                    const int64_t base_index = t.total() - 1;
                    QEntry r;
                    if (name_index > base_index || !t.resolve_abs(base_index - name_index, r)) {
                        ret = kDF;
                    } else {
                        e.nsrc = r.nsrc;
                        e.nl = r.nl;
                        e.soft = r.soft & 0x1u;
                        ret = q_value_and_insert(t, A, e, vhuff, p, (uint64_t)value_len, vpre, T);
                    }
                }
                p += (uint64_t)value_len;
            } break;
            case 2:
            case 3: {  // insert without name reference (:446-462, :352-393)
                int64_t name_len, value_len;
                const bool nhuff = (b & 0x20u) != 0;
                const int64_t npre = q_pre(A, p, 5);
                if ((ret = q_int(name_len, in, p, end, 5)) != 0) goto Exit;
                if (!((uint64_t)name_len < end - p)) goto Exit;
                const uint64_t qn = p;
                p += (uint64_t)name_len;
                const int64_t vpre = q_pre(A, p, 7);
                const bool vhuff = (in[p] & 0x80u) != 0;
                if ((ret = q_int(value_len, in, p, end, 7)) != 0) goto Exit;
                if (!((uint64_t)value_len <= end - p)) goto Exit;
                QEntry e{};
                if (!q_enc_string(A, nhuff, true, qn, (uint64_t)name_len, npre, e.nsrc, e.nl, e.soft, T)) {
                    ret = kDF;
                } else {
                    // a name h2o_lookup_token knows goes in as a token header with soft bits 0 (:383-384)
                    if (e.soft) {
                        const uint8_t* nb = q_src(A, e.nsrc);
                        if (q_pseudo_token([&](uint64_t i) { return (uint32_t)nb[i]; }, e.nl)) e.soft = 0;
                    }
                    ret = q_value_and_insert(t, A, e, vhuff, p, (uint64_t)value_len, vpre, T);
                }
                p += (uint64_t)value_len;
            } break;
            case 0: {  // duplicate (:463-468, :395-406)
                int64_t index;
                if ((ret = q_int(index, in, p, end, 5)) != 0) goto Exit;
                if (index >= (int64_t)t.s.num)
                    ret = kDF;
                else
                    t.commit(t.get(t.s.num - 1u - (uint32_t)index));
            } break;
            case 1: {  // set dynamic table capacity (:469-474, :408-418)
                int64_t max_size;
                if ((ret = q_int(max_size, in, p, end, 5)) != 0) goto Exit;
                if (max_size > (int64_t)A.T) {
                    ret = kDF;
                } else {
                    t.s.max_size = (uint64_t)max_size;
                    t.evict(0);
                }
            } break;
        }
        done = p;
    }
Exit:
    if (ret == kQIncomplete) ret = 0;
    if (ret == 0 && old_total != t.s.total_inserts) insert_count = t.s.total_inserts;
    consumed = (uint32_t)(done - p0);
    return ret;
}

__device__ __forceinline__ QTable q_table(const QpkArgs& A, uint64_t c) {
    uint8_t* scr = A.scratch + c * A.conn_scratch;
    QTable t{reinterpret_cast<QEntry*>(scr + sizeof(QState)), qpk_entries(A.T), {}};
    t.s = *reinterpret_cast<const QState*>(scr);
    return t;
}

__device__ __forceinline__ void load_dec_tables(uint32_t* s_lut, uint32_t* s_kinfo, uint32_t* s_ones) {
    for (uint32_t k = threadIdx.x; k < (1u << HHUFF_LUT_BITS) / 4; k += blockDim.x)
        reinterpret_cast<uint4*>(s_lut)[k] = reinterpret_cast<const uint4*>(q_dec_lut)[k];
    for (uint32_t k = threadIdx.x; k < HHUFF_ONES_NENT; k += blockDim.x) s_ones[k] = q_ones[k];
    if (threadIdx.x < 31) s_kinfo[threadIdx.x] = q_kinfo[threadIdx.x];
    __syncthreads();
}

__global__ __launch_bounds__(256) void qpack_encoder_kernel(QpkArgs A) {
    __shared__ __attribute__((aligned(16))) uint32_t s_lut[1u << HHUFF_LUT_BITS];
    __shared__ uint32_t s_kinfo[32];
    __shared__ uint32_t s_ones[HHUFF_ONES_NENT];
    load_dec_tables(s_lut, s_kinfo, s_ones);
    DecTables T;  // assigned, not brace-initialised (see hhuff_blocks.hip)
    T.lut = s_lut;
    T.kinfo = s_kinfo;
    T.ones = s_ones;
    for (uint64_t c = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; c < A.nconn; c += (uint64_t)gridDim.x * blockDim.x) {
        QState* ps = reinterpret_cast<QState*>(A.scratch + c * A.conn_scratch);
        if (!(A.flags & HHUFF_QPK_CONTINUE)) {  // h2o_qpack_create_decoder (:240-252)
            QState s0{};
            s0.base_offset = 1;
            s0.max_size = A.T;
            *ps = s0;
        }
        QTable t = q_table(A, c);
        t.s.dirty = 0;
        int32_t st = 0;
        uint32_t consumed = 0;
        uint64_t ic = 0;
        if (t.s.failed) {
            st = HHUFF_QPK_SKIPPED;
        } else if (A.enc_len[c]) {
            const uint64_t p = A.enc_off[c];
            st = q_handle_input(t, A, p, p + A.enc_len[c], consumed, ic, T);
            t.s.failed = st != 0;
        }
        A.enc_status[c] = st;
        A.enc_consumed[c] = consumed;
        A.insert_count[c] = ic;
        *ps = t.s;
    }
}

// Table pass: one wave per connection whose table took entries this call writes the live entries' bytes,
// oldest first, back to back into the ring they do not use now and points the entries there; the field
// sections (and the next call, HHUFF_QPK_CONTINUE) read only scratch.
__global__ __launch_bounds__(256) void qpack_table_kernel(QpkArgs A) {
    const int lane = threadIdx.x & 63;
    const uint64_t c = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    if (c >= A.nconn) return;
    const uint64_t base = c * A.conn_scratch;
    QState* ps = reinterpret_cast<QState*>(A.scratch + base);
    const QState s = *ps;
    if (!s.dirty) return;
    const uint32_t E = qpk_entries(A.T);
    QEntry* ent = reinterpret_cast<QEntry*>(A.scratch + base + sizeof(QState));
    const uint32_t nring = s.ring ^ 1u;
    const uint64_t rbase = base + sizeof(QState) + (uint64_t)E * sizeof(QEntry) + nring * (uint64_t)qpk_ring_bytes(A.T);
    uint32_t carry = 0;
    for (uint32_t k0 = 0; k0 < s.num; k0 += 64) {
        const uint32_t k = k0 + (uint32_t)lane;
        const bool live = k < s.num;
        uint32_t i = s.start + k;
        i = i >= E ? i - E : i;
        QEntry e{};
        if (live) e = ent[i];
        const uint32_t sz = live ? e.nl + e.vl : 0u;
        const uint32_t dst = carry + wave_excl_scan(sz, lane);
        carry += (uint32_t)__builtin_amdgcn_readlane((int)(dst - carry + sz), 63);
        uint8_t* d = A.scratch + rbase + dst;
        wave_copy64(q_src(A, e.nsrc), d, live ? e.nl : 0u, lane);
        wave_copy64(q_src(A, e.vsrc), d + e.nl, live ? e.vl : 0u, lane);
        if (live) {
            ent[i].nsrc = kQScr | (rbase + dst);
            ent[i].vsrc = kQScr | (rbase + dst + e.nl);
        }
    }
    if (lane == 0) ps->ring = nring;
}

// ---- field sections ----

struct QCtx {
    int64_t ric, base;
};

// parse_decode_context (qpack.c:754-799)
__device__ int32_t q_parse_context(const QTable& t, uint32_t max_entries, QCtx& ctx, const uint8_t* in, uint64_t& p,
                                   uint64_t end) {
    int64_t ric, delta;
    if (q_int(ric, in, p, end, 8) != 0) return kDF;
    if (ric > 0) {
        if (max_entries == 0) return kDF;
        const uint32_t full_range = 2 * max_entries;
        const uint64_t max_value = t.s.total_inserts + max_entries;
        const uint64_t rounded = max_value / full_range * full_range;
        ric = (int64_t)((uint64_t)ric + rounded - 1);
        if ((uint64_t)ric > max_value) {
            if (ric <= (int64_t)full_range) return kDF;
            ric -= full_range;
        }
        if (ric == 0) return kDF;
        if (ric > kQuicIntMax) return kDF;
    }
    ctx.ric = ric;
    if (p >= end) return kDF;
    const bool sign = (in[p] & 0x80u) != 0;
    if (q_int(delta, in, p, end, 7) != 0) return kDF;
    if (delta > kQuicIntMax) return kDF;
    ctx.base = sign ? ric - delta - 1 : ric + delta;
    if (ctx.base < 0) return kDF;
    return 0;
}

// resolve_dynamic / resolve_dynamic_postbase (qpack.c:523-557)
__device__ bool q_dyn(const QTable& t, const QCtx& ctx, const uint8_t* in, uint64_t& p, uint64_t end, uint32_t prefix,
                      bool postbase, QEntry& e) {
    int64_t off, index;
    if (q_int(off, in, p, end, prefix) != 0) return false;
    if (postbase) {
        if (off > INT64_MAX - ctx.base - 1) return false;
        index = ctx.base + off + 1;
    } else {
        if (off >= ctx.base) return false;
        index = ctx.base - off;
    }
    if (ctx.ric < index) return false;
    return t.resolve_abs(index, e);
}

struct QArena {
    uint8_t* a;
    uint64_t cur, end;
};

// a field string's n bytes at source `src` go to arena[off, off + n): qpack_copy_kernel moves them
// (fs = their address)
__device__ __forceinline__ int32_t q_copy(const QpkArgs& A, QArena& R, uint64_t src, uint32_t n, uint32_t& off,
                                          uint64_t& fs) {
    if (R.cur + n > R.end) return HHUFF_QPK_ARENA;
    off = (uint32_t)R.cur;
    fs = (uint64_t)(uintptr_t)q_src(A, src);
    R.cur += n;
    return 0;
}

// decode_header_value_literal (qpack.c:603-629) / decode_header_name_literal (:559-601, prefix 3)
__device__ int32_t q_literal(const QpkArgs& A, QArena& R, uint32_t& soft, uint64_t& p, uint64_t end, bool is_name,
                             uint32_t& off, uint32_t& len, uint64_t& fs, const DecTables& T) {
    const uint8_t* in = A.in;
    if (!is_name && !(p < end)) return kDF;
    const uint32_t prefix = is_name ? 3u : 7u;
    const bool huff = ((in[p] >> prefix) & 1u) != 0;
    const int64_t pre = q_pre(A, p, prefix);
    int64_t n;
    if (q_int(n, in, p, end, prefix) != 0) return kDF;
    if ((int64_t)(end - p) < n) return kDF;
    fs = 0;
    if (pre >= 0) {  // decoded and validated by the pre-pass; the reference's order of checks holds
        if (R.cur + (huff ? ((uint64_t)n * 8u) / 5u : (uint64_t)n) > R.end) return HHUFF_QPK_ARENA;
        len = A.lit_len[pre];
        soft |= A.lit_st[pre] & 3u;
        off = (uint32_t)R.cur;
        fs = (uint64_t)(uintptr_t)(huff ? A.lit_out + (p * 8u) / 5u : in + p);
        R.cur += len;
        p += (uint64_t)n;
        return 0;
    }
    if (huff) {
        if (R.cur + ((uint64_t)n * 8u) / 5u > R.end) return HHUFF_QPK_ARENA;
        if ((uint64_t)n > kMaxStrLen) return kDF;
        ArenaSinkFL sk{RegSink{}, 0u, 0u};
        sk.s.init(R.a + R.cur);
        const DecResult d = decode_core(GlobalSource{A.in, A.in_size}, (uint32_t)p, (uint32_t)n, sk, T);
        if (!d.ok) return kDF;
        sk.s.finish();
        soft |= soft_bits(is_name, d.len, d.flags, sk.first, sk.last);
        len = d.len;
    } else {
        const uint8_t* src = in + p;
        auto get = [&](uint64_t i) { return (uint32_t)src[i]; };
        if (is_name) {  // tokens are taken as they are; anything else is validated (:583-588)
            if (!q_pseudo_token(get, (uint64_t)n) && !q_valid_name(get, (uint64_t)n, soft)) return kDF;
        } else {
            q_valid_value(get, (uint64_t)n, soft);
        }
        if (R.cur + (uint64_t)n > R.end) return HHUFF_QPK_ARENA;
        uint8_t* d = R.a + R.cur;
        copy16([&](uint32_t i) { return src[i]; }, [&](uint32_t i, uint8_t v) { d[i] = v; }, (uint32_t)n);
        len = (uint32_t)n;
    }
    off = (uint32_t)R.cur;
    R.cur += len;
    p += (uint64_t)n;
    return 0;
}

// decode_header (qpack.c:652-752): 0 / kErrInvalidChar = a field was produced
__device__ int32_t q_field(const QpkArgs& A, const QTable& t, const QCtx& ctx, uint64_t& p, uint64_t end, QArena& R,
                           uint32_t& noff, uint32_t& nlen, uint32_t& voff, uint32_t& vlen, uint32_t& soft_out,
                           uint64_t& fn, uint64_t& fv, const DecTables& T) {
    const uint8_t* in = A.in;
    uint32_t soft = 0;
    int32_t r;
    QEntry e;
    const uint32_t kind = in[p] >> 4;
    switch (kind) {
        case 12:
        case 13:
        case 14:
        case 15: {  // indexed field line, static (:659-669)
            int64_t si;
            if (q_int(si, in, p, end, 6) != 0 || (uint64_t)si >= kQStaticCount) return kDF;
            const uint32_t k = 4u * (uint32_t)si;
            nlen = q_static_ent[k + 1];
            if ((r = q_copy(A, R, kQStatic | q_static_ent[k], nlen, noff, fn)) != 0) return r;
            vlen = q_static_ent[k + 3];
            if ((r = q_copy(A, R, kQStatic | q_static_ent[k + 2], vlen, voff, fv)) != 0) return r;
        } break;
        case 8:
        case 9:
        case 10:
        case 11:  // indexed field line, dynamic (:670-682)
        case 1:   // indexed field line, post-base (:713-722)
            if (!q_dyn(t, ctx, in, p, end, kind == 1 ? 4u : 6u, kind == 1, e)) return kDF;
            if ((r = q_copy(A, R, e.nsrc, e.nl, noff, fn)) != 0) return r;
            if ((r = q_copy(A, R, e.vsrc, e.vl, voff, fv)) != 0) return r;
            nlen = e.nl;
            vlen = e.vl;
            soft = e.soft;
            break;
        case 5:
        case 7: {  // literal field line, static name reference (:683-692)
            int64_t si;
            if (q_int(si, in, p, end, 4) != 0 || (uint64_t)si >= kQStaticCount) return kDF;
            const uint32_t k = 4u * (uint32_t)si;
            nlen = q_static_ent[k + 1];
            if ((r = q_copy(A, R, kQStatic | q_static_ent[k], nlen, noff, fn)) != 0) return r;
            if ((r = q_literal(A, R, soft, p, end, false, voff, vlen, fv, T)) != 0) return r;
        } break;
        case 4:
        case 6:  // literal field line, dynamic name reference (:693-704)
        case 0:  // literal field line, post-base name reference (:723-733)
            if (!q_dyn(t, ctx, in, p, end, kind == 0 ? 3u : 4u, kind == 0, e)) return kDF;
            if ((r = q_copy(A, R, e.nsrc, e.nl, noff, fn)) != 0) return r;
            nlen = e.nl;
            soft = e.soft & 0x1u;
            if ((r = q_literal(A, R, soft, p, end, false, voff, vlen, fv, T)) != 0) return r;
            break;
        default:  // 2, 3: literal field line with a literal name (:705-712)
            if ((r = q_literal(A, R, soft, p, end, true, noff, nlen, fn, T)) != 0) return r;
            if ((r = q_literal(A, R, soft, p, end, false, voff, vlen, fv, T)) != 0) return r;
            break;
    }
    soft_out = soft;
    return soft ? kErrInvalidChar : 0;
}

// h2o_hpack_encode_int (hpack.c:757-772) of v with a 7-bit prefix behind 0x80: send_header_ack (qpack.c:642-649)
__device__ __forceinline__ uint32_t q_header_ack(uint64_t v, uint8_t* out) {
    uint32_t n = 0;
    if (v < 127u) {
        out[n++] = (uint8_t)(0x80u | v);
        return n;
    }
    out[n++] = 0xFFu;
    v -= 127u;
    while (v >= 128u) {
        out[n++] = (uint8_t)(0x80u | (v & 0x7Fu));
        v >>= 7;
    }
    out[n++] = (uint8_t)v;
    return n;
}

__device__ __forceinline__ void q_req_store(hhuff_qpack_request_t* out, const ReqState& r, int32_t st, uint64_t ric,
                                            uint64_t stream_id) {
    req_store(&out->req, r);
    out->datagram_flow_id = r.dfid;
    uint8_t ack[16] = {};
    const uint32_t n = ((st == 0 || st == kErrInvalidChar) && ric != 0) ? q_header_ack(stream_id, ack) : 0u;
    out->ack_len = n;
    uint2* a2 = reinterpret_cast<uint2*>(out->ack);  // 8-byte aligned records: two 8-byte stores
    uint32_t w[4];
    __builtin_memcpy(w, ack, 16);
    a2[0] = make_uint2(w[0], w[1]);
    a2[1] = make_uint2(w[2], w[3]);
}

// The HTTP/3 rules as a call of their own: inlined into the sections kernel (11K instructions, SGPRs spilled
// to VGPR lanes), the compiler lost the err_desc code of a rejected connection-specific field on gfx950
// (the request record said 0 where h2o says h2o_hpack_err_unexpected_connection_specific_header), while the
// same source compiled for the host, and inlined into the HPACK walk, is right.  The rules' source is clean
// under ASan + UBSan on the host and equal to the oracle field for field (tests/rules_host.cpp); A/B builds
// with -DHHUFF_H3_INLINE inline them again (tests/test_rules_host.py documents the GPU result).
#ifdef HHUFF_H3_INLINE
#define HHUFF_H3_CALL __forceinline__
#else
#define HHUFF_H3_CALL __noinline__
#endif
__device__ HHUFF_H3_CALL int32_t req_field_h3(ReqState& r, uint32_t cls, const uint8_t* value, uint32_t vl, uint32_t soft,
                                             int32_t k, bool& header) {
    return req_field<true>(r, cls, value, vl, soft, k, header);
}

__device__ HHUFF_H3_CALL int32_t resp_field_h3(RespState& r, uint32_t cls, const uint8_t* value, uint32_t vl, uint32_t soft,
                                              int32_t k, bool& header) {
    return resp_field<true>(r, cls, value, vl, soft, k, header);
}

// h2o_qpack_parse_response's record: the Section Acknowledgment only after a clean parse (qpack.c:876-881)
__device__ __forceinline__ void q_res_store(hhuff_qpack_response_head_t* out, const RespState& r, int32_t st, uint64_t ric,
                                            uint64_t stream_id) {
    resp_store(&out->res, r);
    uint8_t ack[16] = {};
    const uint32_t n = (st == 0 && ric != 0) ? q_header_ack(stream_id, ack) : 0u;
    out->ack_len = n;
    out->reserved = 0u;
    uint2* a2 = reinterpret_cast<uint2*>(out->ack);
    uint32_t w[4];
    __builtin_memcpy(w, ack, 16);
    a2[0] = make_uint2(w[0], w[1]);
    a2[1] = make_uint2(w[2], w[3]);
}

constexpr int kSecPlain = 0, kSecReq = 1, kSecResp = 2;  // qpack_sections_kernel modes

// REQ: h2o_qpack_parse_request (qpack.c:830-858) -- each field also runs h2o_hpack_parse_request's rules
// (hhuff_request.h, the HTTP/3 arguments of lib/http3/server.c:1540-1545), a rule's hard error is
// normalised to DECOMPRESSION_FAILED (:852-853), and the record gets the Section Acknowledgment (:856).
// RESP: h2o_qpack_parse_response (:860-882) as lib/common/http3client.c:542 calls it -- a response head,
// h2o_hpack_parse_response's rules (a status and a datagram-flow-id out-parameter), the same normalisation
template <int MODE>
__global__ __launch_bounds__(256) void qpack_sections_kernel(QpkArgs A) {
    constexpr bool REQ = MODE == kSecReq, RESP = MODE == kSecResp;
    __shared__ __attribute__((aligned(16))) uint32_t s_lut[1u << HHUFF_LUT_BITS];
    __shared__ uint32_t s_kinfo[32];
    __shared__ uint32_t s_ones[HHUFF_ONES_NENT];
    load_dec_tables(s_lut, s_kinfo, s_ones);
    DecTables T;  // assigned, not brace-initialised (see hhuff_blocks.hip)
    T.lut = s_lut;
    T.kinfo = s_kinfo;
    T.ones = s_ones;
    const uint32_t max_entries = A.T / kEntryOverhead;
    for (uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; k < A.nsec; k += (uint64_t)gridDim.x * blockDim.x) {
        // the section's connection: the last c with conn_first[c] <= k
        uint32_t lo = 0, hi = A.nconn;  // invariant: conn_first[lo] <= k < conn_first[hi]
        while (hi - lo > 1) {
            const uint32_t mid = (lo + hi) >> 1;
            if (A.conn_first[mid] <= k)
                lo = mid;
            else
                hi = mid;
        }
        const QTable t = q_table(A, lo);
        A.nfields[k] = 0;
        A.req_insert_count[k] = 0;
        ReqState rq;
        RespState rs;
        if (REQ) rq.reset();
        if (RESP) rs.reset(false);
        if (t.s.failed) {
            A.sstatus[k] = HHUFF_QPK_SKIPPED;
            if (REQ) q_req_store(A.qreq + k, rq, HHUFF_QPK_SKIPPED, 0u, 0u);
            if (RESP) q_res_store(A.qres + k, rs, HHUFF_QPK_SKIPPED, 0u, 0u);
            continue;
        }
        uint64_t p = A.sec_off[k];
        const uint64_t end = A.sec_off[k + 1];
        QCtx ctx{0, 0};
        int32_t st = q_parse_context(t, max_entries, ctx, A.in, p, end);
        if (st == 0) {
            A.req_insert_count[k] = (uint64_t)ctx.ric;
            // check_decode_context_blocked (:801-820); the max_blocked limit is applied per connection in
            // section order by qpack_blocked_kernel (every parked stream raises num_blocked)
            if (!(ctx.ric < t.total())) st = HHUFF_QPK_BLOCKED;
        }
        QArena R{A.arena, A.arena_off[k], min(A.arena_off[k + 1], kArenaLimit)};  // field offsets are u32
        const uint32_t slot = A.sec_off[k];
        uint32_t nf = 0;
        if (RESP && st == 0 && p == end) {  // a head without fields: missing :status (hpack.c:652-655), normalised
            rs.err = HHUFF_HERR_MISSING_PSEUDO;
            st = kDF;
        }
        while (st == 0 && p != end) {
            uint32_t no = 0, nl = 0, vo = 0, vl = 0, soft = 0;
            uint64_t fn = 0, fv = 0;
            const int32_t rc = q_field(A, t, ctx, p, end, R, no, nl, vo, vl, soft, fn, fv, T);
            if (rc != 0 && rc != kErrInvalidChar) {
                st = rc;
                // h2o_hpack_parse_request: *err_desc = decode_err (hpack.c:523-525)
                if (REQ) rq.err = rc == HHUFF_QPK_ARENA ? HHUFF_HERR_NONE : HHUFF_HERR_DECODE;
                if (RESP) rs.err = rc == HHUFF_QPK_ARENA ? HHUFF_HERR_NONE : HHUFF_HERR_DECODE;
                break;
            }
            bool header = false;
            int32_t rr = 0;
            if (REQ || RESP) {  // the bytes where they lie: a source (fn / fv), or the arena (decoded in place)
                const uint8_t* np = fn ? reinterpret_cast<const uint8_t*>(fn) : A.arena + no;
                const uint8_t* vp = fv ? reinterpret_cast<const uint8_t*>(fv) : A.arena + vo;
                if (REQ) rr = req_field_h3(rq, req_name_class(np, nl), vp, vl, soft, (int32_t)nf, header);
                if (RESP) rr = resp_field_h3(rs, req_name_class(np, nl), vp, vl, soft, (int32_t)nf, header);
            }
            A.fsrc_n[slot + nf] = fn;
            A.fsrc_v[slot + nf] = fv;
            A.name_off[slot + nf] = no;
            A.name_len[slot + nf] = nl;
            A.value_off[slot + nf] = vo;
            A.value_len[slot + nf] = vl;
            A.fflags[slot + nf] = (uint8_t)(soft | (header ? HHUFF_FIELD_HEADER : 0u));
            ++nf;
            if (rr != 0) {  // normalize_error_code (qpack.c:822-828): a rule's H2 error fails the section
                st = kDF;
                break;
            }
        }
        if (REQ) {
            if (st == 0 && rq.err != HHUFF_HERR_NONE) st = kErrInvalidChar;  // hpack.c:636-637
            q_req_store(A.qreq + k, rq, st, (uint64_t)ctx.ric, A.stream_id[k]);
        }
        if (RESP) {
            if (st == 0 && rs.err != HHUFF_HERR_NONE) st = kErrInvalidChar;  // hpack.c:745-747
            q_res_store(A.qres + k, rs, st, (uint64_t)ctx.ric, A.stream_id[k]);
        }
        A.nfields[k] = nf;
        A.sstatus[k] = st;
    }
}

// Copy pass: 64 sections per wave (wave_copy_fields), their fields' name / value bytes into the arena.
__global__ __launch_bounds__(256) void qpack_copy_kernel(QpkArgs A) {
    const int lane = threadIdx.x & 63;
    const uint32_t nw = gridDim.x * 4u;
    for (uint32_t k0 = (blockIdx.x * 4u + (threadIdx.x >> 6)) * 64u; k0 < A.nsec; k0 += nw * 64u) {
        const uint32_t k = k0 + (uint32_t)lane;
        const uint32_t s0 = k < A.nsec ? A.sec_off[k] : 0u, nf = k < A.nsec ? A.nfields[k] : 0u;
        wave_copy_fields(s0, nf, lane, [&](uint32_t f, bool val, const uint8_t*& src, uint8_t*& dst, uint32_t& len) {
            const uint64_t fs = val ? A.fsrc_v[f] : A.fsrc_n[f];
            src = reinterpret_cast<const uint8_t*>(fs);
            dst = A.arena + (val ? A.value_off[f] : A.name_off[f]);
            len = fs ? (val ? A.value_len[f] : A.name_len[f]) : 0u;
        });
    }
}

// check_decode_context_blocked's slot limit (qpack.c:801-820) across one step's sections of a connection:
// h2o raises conn->num_qpack_blocked for every stream it parks (lib/http3/server.c:1553), so the blocked
// sections of a connection, in section order, take the free slots one by one; the first one that finds
// num_blocked >= max_blocked fails with QPACK_DECOMPRESSION_FAILED.  One lane per connection.
__global__ __launch_bounds__(256) void qpack_blocked_kernel(QpkArgs A) {
    for (uint64_t c = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; c < A.nconn; c += (uint64_t)gridDim.x * blockDim.x) {
        uint64_t nb = A.num_blocked ? A.num_blocked[c] : 0u;
        for (uint32_t k = A.conn_first[c]; k < A.conn_first[c + 1]; ++k) {
            if (A.sstatus[k] != HHUFF_QPK_BLOCKED) continue;
            if (nb >= A.max_blocked)
                A.sstatus[k] = kDF;
            else
                ++nb;
        }
    }
}

// ---- encoder-stream literal pre-pass ----
// An encoder stream's instructions are readable without the table (name indexes and literal lengths are
// explicit, qpack.c:420-474), so one lane per connection finds every literal the walk could reach and the
// literal kernels decode them all together, balanced across connections; the walk (qpack_encoder_kernel)
// then copies bytes instead of running a Huffman decoder per lane.  Marks past a table-dependent error (an
// index the table does not hold) are decoded and unused.

struct QMarks {
    uint32_t *lit, *name, *p3;
};

// the literal with `prefix`-bit length at p inside [p, end): mark it, step over it
__device__ __forceinline__ bool q_mark_literal(const uint8_t* in, uint64_t& p, uint64_t end, uint32_t prefix,
                                               const QMarks& M) {
    if (p >= end) return false;
    uint64_t q = p;
    const int64_t n = q_hpack_int(in, q, end, prefix);
    if (n < 0 || (uint64_t)n > end - q) return false;
    const uint32_t w = (uint32_t)(p >> 5), m = 1u << (p & 31);
    atomicOr(M.lit + w, m);
    if (prefix != 7) atomicOr(M.name + w, m);
    if (prefix == 3) atomicOr(M.p3 + w, m);
    p = q + (uint64_t)n;
    return true;
}

// one lane per encoder stream (items [0, nconn)) or field section (the rest)
__global__ __launch_bounds__(256) void qpack_mark_kernel(QpkArgs A, QMarks M) {
    const uint8_t* in = A.in;
    const uint64_t nitems = (uint64_t)A.nconn + A.nsec;
    for (uint64_t c = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; c < nitems; c += (uint64_t)gridDim.x * blockDim.x) {
        if (c >= A.nconn) {  // a section: the decode context, then the representation switch of q_field
            const uint64_t k = c - A.nconn;
            uint64_t p = A.sec_off[k];
            const uint64_t end = A.sec_off[k + 1];
            bool go = q_hpack_int(in, p, end, 8) >= 0 && p < end && q_hpack_int(in, p, end, 7) >= 0;
            while (go && p < end) {
                const uint32_t kind = in[p] >> 4;
                if (kind >= 8) {  // indexed, static or dynamic
                    go = q_hpack_int(in, p, end, 6) >= 0;
                } else if (kind == 1) {  // indexed, post-base
                    go = q_hpack_int(in, p, end, 4) >= 0;
                } else if (kind == 2 || kind == 3) {  // literal name, then the value
                    go = q_mark_literal(in, p, end, 3, M) && q_mark_literal(in, p, end, 7, M);
                } else {  // name reference (static / dynamic 4 bits, post-base 3), then the value
                    go = q_hpack_int(in, p, end, kind == 0 ? 3 : 4) >= 0 && q_mark_literal(in, p, end, 7, M);
                }
            }
            continue;
        }
        uint64_t p = A.enc_off[c];
        const uint64_t end = p + A.enc_len[c];
        bool go = true;
        while (go && p < end) {  // the instruction switch of q_handle_input
            const uint32_t b = in[p];
            switch (b >> 5) {
                default:  // insert with name reference: index, then the value
                    go = q_hpack_int(in, p, end, 6) >= 0 && q_mark_literal(in, p, end, 7, M);
                    break;
                case 2:
                case 3:  // insert with a literal name: the name (5-bit prefix), then the value
                    go = q_mark_literal(in, p, end, 5, M) && q_mark_literal(in, p, end, 7, M);
                    break;
                case 0:
                case 1: go = q_hpack_int(in, p, end, 5) >= 0; break;  // duplicate, set capacity
            }
        }
    }
}

uint64_t qpack_conn_scratch(uint32_t header_table_size) {
    return sizeof(QState) + (uint64_t)qpk_entries(header_table_size) * sizeof(QEntry) +
           2ull * qpk_ring_bytes(header_table_size);
}

hipError_t launch_qpack(const uint8_t* in, uint64_t in_size, const uint32_t* enc_off, const uint32_t* enc_len,
                        const uint32_t* sec_off, const uint32_t* conn_first, uint32_t nconn, uint32_t nsec,
                        uint32_t header_table_size, uint64_t max_blocked, const uint32_t* num_blocked, uint8_t* arena,
                        const uint64_t* arena_off, uint32_t* name_off, uint32_t* name_len, uint32_t* value_off,
                        uint32_t* value_len, uint8_t* fflags, uint32_t* nfields, int32_t* sstatus,
                        uint64_t* req_insert_count, int32_t* enc_status, uint32_t* enc_consumed, uint64_t* insert_count,
                        uint8_t* scratch, uint32_t flags, hipStream_t stream, const uint64_t* stream_id,
                        hhuff_qpack_request_t* qreq, hhuff_qpack_response_head_t* qres) {
    if (nconn == 0) return hipSuccess;
    QpkArgs A{in, in_size, enc_off, enc_len, sec_off, conn_first, num_blocked, nconn, nsec, header_table_size,
              max_blocked, arena, arena_off, name_off, name_len, value_off, value_len, fflags, nfields, sstatus,
              req_insert_count, enc_status, enc_consumed, insert_count, scratch, qpack_conn_scratch(header_table_size),
              flags, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, stream_id, qreq, qres};
    // workspace: the literal pre-pass's bitmaps, word prefixes, chunk sums, the literal list with each
    // literal's prefix, the literal kernels' results and decoded bytes (positions are u32: in_size < 2^32,
    // checked by the C ABI), and the field slots' byte sources
    const uint64_t nwords = in_size / 32 + 1, nchunks = literal_list_chunks(nwords);
    const uint64_t n_max = in_size + 2;  // every literal header takes a byte
    auto up = [](uint64_t x) { return (x + 255) & ~255ull; };
    const uint64_t o_lit = 0, o_name = o_lit + up(4 * nwords), o_p3 = o_name + up(4 * nwords);
    const uint64_t o_lnames = o_p3 + up(4 * nwords);
    const uint64_t zero_end = o_lnames + up(4 * ((n_max + 31) / 32));  // [0, zero_end) starts zeroed
    const uint64_t o_pre = zero_end, o_chunk = o_pre + up(4 * nwords), o_list = o_chunk + up(4 * nchunks + 4);
    const uint64_t o_pfx = o_list + up(4 * n_max), o_len = o_pfx + up(n_max), o_pay = o_len + up(4 * n_max);
    const uint64_t o_cons = o_pay + up(4 * n_max), o_st = o_cons + up(4 * n_max), o_ws = o_st + up(n_max);
    const uint64_t o_out = o_ws + up(literals_dev_ws((uint32_t)n_max, in_size));
    const uint64_t o_fsn = o_out + up((8 * in_size) / 5 + 64), o_fsv = o_fsn + up(8 * in_size + 8);
    const uint64_t wbytes = o_fsv + up(8 * in_size + 8);  // field slots: one per input byte
    uint8_t* work = nullptr;
    hipError_t e = hipSuccess;
    {
        e = work_alloc((void**)&work, wbytes, stream);
        if (e == hipSuccess) e = hipMemsetAsync(work, 0, zero_end, stream);
        uint32_t* lit_bits = reinterpret_cast<uint32_t*>(work + o_lit);
        uint32_t* name_bits = reinterpret_cast<uint32_t*>(work + o_name);
        uint32_t* chunk = reinterpret_cast<uint32_t*>(work + o_chunk);
        uint32_t* list = reinterpret_cast<uint32_t*>(work + o_list);
        uint32_t* word_pre = reinterpret_cast<uint32_t*>(work + o_pre);
        uint32_t* p3_bits = reinterpret_cast<uint32_t*>(work + o_p3);
        if (e == hipSuccess) {
            const uint64_t items = (uint64_t)nconn + nsec;
            hipLaunchKernelGGL(qpack_mark_kernel, dim3((uint32_t)std::min<uint64_t>((items + 255) / 256, 65535)), dim3(256),
                               0, stream, A, QMarks{lit_bits, name_bits, p3_bits});
            e = hipGetLastError();
        }
        if (e == hipSuccess)  // prefixes: section names 3, encoder-stream names 5, values 7
            e = launch_literal_list(lit_bits, name_bits, p3_bits, 3u, 5u, nwords, chunk, word_pre, list,
                                    reinterpret_cast<uint32_t*>(work + o_lnames), work + o_pfx, stream);
        if (e == hipSuccess)
            e = launch_literals_dev(in, in_size, list, (uint32_t)n_max, chunk + nchunks, 7u,
                                    HHUFF_LIT_QPACK | kLitNoRawCopy, reinterpret_cast<uint32_t*>(work + o_lnames),
                                    work + o_out, reinterpret_cast<uint32_t*>(work + o_len),
                                    reinterpret_cast<uint32_t*>(work + o_pay), reinterpret_cast<uint32_t*>(work + o_cons),
                                    work + o_st, work + o_ws, stream, work + o_pfx);
        A.lit_bits = lit_bits;
        A.word_pre = word_pre;
        A.lit_len = reinterpret_cast<const uint32_t*>(work + o_len);
        A.lit_st = work + o_st;
        A.lit_pfx = work + o_pfx;
        A.lit_out = work + o_out;
        A.fsrc_n = reinterpret_cast<uint64_t*>(work + o_fsn);
        A.fsrc_v = reinterpret_cast<uint64_t*>(work + o_fsv);
    }
    if (e == hipSuccess) {
        hipLaunchKernelGGL(qpack_encoder_kernel, dim3(std::min((nconn + 255u) / 256u, 65535u)), dim3(256), 0, stream, A);
        hipLaunchKernelGGL(qpack_table_kernel, dim3((uint32_t)(((uint64_t)nconn + 3) / 4)), dim3(256), 0, stream, A);
        e = hipGetLastError();
    }
    if (e == hipSuccess && nsec != 0) {
        if (qres)
            hipLaunchKernelGGL(qpack_sections_kernel<kSecResp>, dim3(std::min((nsec + 255u) / 256u, 65535u)), dim3(256), 0, stream, A);
        else if (qreq)
            hipLaunchKernelGGL(qpack_sections_kernel<kSecReq>, dim3(std::min((nsec + 255u) / 256u, 65535u)), dim3(256), 0, stream, A);
        else
            hipLaunchKernelGGL(qpack_sections_kernel<kSecPlain>, dim3(std::min((nsec + 255u) / 256u, 65535u)), dim3(256), 0,
                               stream, A);
        hipLaunchKernelGGL(qpack_copy_kernel, dim3(std::min((nsec + 255u) / 256u, 4096u)), dim3(256), 0, stream, A);
        hipLaunchKernelGGL(qpack_blocked_kernel, dim3(std::min((nconn + 255u) / 256u, 65535u)), dim3(256), 0, stream, A);
        e = hipGetLastError();
    }
    if (work) {
        const hipError_t f = hipFreeAsync(work, stream);
        if (e == hipSuccess) e = f;
    }
    return e;
}

}  // namespace hhuff
