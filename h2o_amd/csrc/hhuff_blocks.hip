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
};

// per-connection scratch: [TableState 32 B][byte ring, table_size rounded to 16][entry ring]
struct TableState {
    uint32_t start, num, whead, failed;
    uint64_t size, cap;
};

// h2o_hpack_decode_int (hpack.c:52-83) at in[*p], bounded by end
__device__ int64_t blk_decode_int(const uint8_t* __restrict__ in, uint64_t& p, uint64_t end, uint32_t prefix_bits) {
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
    __device__ __forceinline__ void put(const uint8_t* src, uint32_t n) {
        for (uint32_t i = 0; i < n; ++i) {
            ring[whead] = src[i];
            whead = whead + 1 == R ? 0u : whead + 1;
        }
    }
    __device__ __forceinline__ void copy_out(uint32_t off, uint32_t n, uint8_t* dst) const {
        for (uint32_t i = 0; i < n; ++i) {
            dst[i] = ring[off];
            off = off + 1 == R ? 0u : off + 1;
        }
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
__device__ int blk_string(const BlkArgs& A, uint64_t& p, uint64_t end, bool is_name, uint32_t& soft, uint64_t& cur,
                          uint64_t aend, uint32_t& off, uint32_t& len, const DecTables& T) {
    if (p >= end) return kStrFail;
    const bool huff = (A.in[p] & 0x80u) != 0;
    const int64_t n = blk_decode_int(A.in, p, end, 7);
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
        const DecResult r = decode_core(GlobalSource{A.in, A.in_size}, (uint32_t)p, (uint32_t)n, fl, T);
        if (!r.ok) return kStrFail;
        fl.s.finish();
        soft |= soft_bits(is_name, r.len, r.flags, fl.first, fl.last);
        len = r.len;
    } else {
        const uint8_t* src = A.in + p;
        if (is_name) {
            if (n == 0 || src[0] != ':') {  // h2o_hpack_validate_header_name (hpack.c:163-192)
                bool bad = n == 0, upper = false;
                for (int64_t i = 0; i < n; ++i) {
                    const uint32_t c = src[i];
                    if ((b_name_invalid[c >> 5] >> (c & 31)) & 1u) {
                        if (c - 'A' < 26u) {
                            upper = true;
                            break;
                        }
                        bad = true;
                    }
                }
                if (upper) return kStrUpper;
                if (bad) soft |= 0x1u;
            }
        } else {  // h2o_hpack_validate_header_value (hpack.c:194-221), whole-value rule :110-115
            bool bad = n != 0 && (src[0] == ' ' || src[0] == '\t' || src[n - 1] == ' ' || src[n - 1] == '\t');
            for (int64_t i = 0; !bad && i < n; ++i) {
                const uint32_t c = src[i];
                bad = ((b_value_invalid[c >> 5] >> (c & 31)) & 1u) != 0;
            }
            if (bad) soft |= 0x2u;
        }
        if (cur + (uint64_t)n > aend) return kStrArena;
        for (int64_t i = 0; i < n; ++i) A.arena[cur + i] = src[i];
        len = (uint32_t)n;
    }
    off = (uint32_t)cur;
    cur += len;
    p += (uint64_t)n;
    return kStrOk;
}

// one field (h2o_hpack_decode_header): 0 / kErrInvalidChar = a field was produced
__device__ int32_t blk_field(const BlkArgs& A, DynTable& t, uint64_t& p, uint64_t end, uint64_t& cur, uint64_t aend,
                             uint32_t& noff, uint32_t& nlen, uint32_t& voff, uint32_t& vlen, uint32_t& soft_out,
                             const DecTables& T) {
    int64_t index = 0;
    bool value_indexed = false, do_index = false;
    for (;;) {
        if (p >= end) return kErrCompression;
        const uint32_t b = A.in[p];
        if (b >= 128) {  // indexed header field
            if ((index = blk_decode_int(A.in, p, end, 7)) <= 0) return kErrCompression;
            value_indexed = true;
        } else if (b >= 64) {  // literal with incremental indexing
            if (b == 64)
                ++p;
            else if ((index = blk_decode_int(A.in, p, end, 6)) <= 0)
                return kErrCompression;
            do_index = true;
        } else if (b < 32) {  // literal without indexing / never indexed
            if ((b & 0xFu) == 0)
                ++p;
            else if ((index = blk_decode_int(A.in, p, end, 4)) <= 0)
                return kErrCompression;
        } else {  // dynamic table size update
            const int64_t c = blk_decode_int(A.in, p, end, 5);
            if (c < 0 || (uint64_t)c > t.maxcap) return kErrCompression;
            t.cap = (uint64_t)c;
            while (t.num != 0 && t.size > t.cap) t.evict_one();
            continue;
        }
        break;
    }
    uint32_t soft = 0;
    if (index > 0) {
        if (index <= 61) {
            const uint32_t k = 4u * (uint32_t)(index - 1);
            const uint32_t no = b_static_ent[k], nl = b_static_ent[k + 1];
            if (cur + nl > aend) return kBlkArena;
            for (uint32_t i = 0; i < nl; ++i) A.arena[cur + i] = b_static_bytes[no + i];
            noff = (uint32_t)cur;
            nlen = nl;
            cur += nl;
            if (value_indexed) {
                const uint32_t vo = b_static_ent[k + 2], vl = b_static_ent[k + 3];
                if (cur + vl > aend) return kBlkArena;
                for (uint32_t i = 0; i < vl; ++i) A.arena[cur + i] = b_static_bytes[vo + i];
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
    } else {
        const int r = blk_string(A, p, end, true, soft, cur, aend, noff, nlen, T);
        if (r == kStrArena) return kBlkArena;
        if (r != kStrOk) return r == kStrUpper ? kErrProtocol : kErrCompression;
    }
    if (!value_indexed) {
        soft &= ~0x2u;
        const int r = blk_string(A, p, end, false, soft, cur, aend, voff, vlen, T);
        if (r == kStrArena) return kBlkArena;
        if (r != kStrOk) return kErrCompression;
    }
    if (do_index) t.add(A.arena + noff, nlen, A.arena + voff, vlen, soft);
    soft_out = soft;
    return soft ? kErrInvalidChar : 0;
}

__global__ __launch_bounds__(256) void hpack_blocks_kernel(BlkArgs A) {
    __shared__ __attribute__((aligned(16))) uint32_t s_lut[1u << HHUFF_LUT_BITS];
    __shared__ uint32_t s_kinfo[32];
    __shared__ uint32_t s_ones[HHUFF_ONES_NENT];
    for (uint32_t k = threadIdx.x; k < (1u << HHUFF_LUT_BITS) / 4; k += blockDim.x)
        reinterpret_cast<uint4*>(s_lut)[k] = reinterpret_cast<const uint4*>(b_dec_lut)[k];
    for (uint32_t k = threadIdx.x; k < HHUFF_ONES_NENT; k += blockDim.x) s_ones[k] = b_ones[k];
    if (threadIdx.x < 31) s_kinfo[threadIdx.x] = b_kinfo[threadIdx.x];
    __syncthreads();
    const DecTables T{s_lut, s_kinfo, s_ones};
    const uint32_t R = A.table_size, E = A.table_size / kEntryOverhead + 1;
    for (uint64_t c = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; c < A.nconn; c += (uint64_t)gridDim.x * blockDim.x) {
        uint8_t* scr = A.scratch + c * A.conn_scratch;
        TableState* ts = reinterpret_cast<TableState*>(scr);
        uint8_t* ring = scr + sizeof(TableState);
        DynTable t{ring, reinterpret_cast<uint4*>(ring + ((R + 15u) & ~15u)), R, E, 0u, 0u, 0u, 0u, A.table_size,
                   A.table_size};
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
            if (failed) {
                A.bstatus[b] = kBlkSkipped;
                continue;
            }
            uint64_t p = A.blk_off[b];
            const uint64_t end = A.blk_off[b + 1];
            uint64_t cur = A.arena_off[b];
            const uint64_t aend = min(A.arena_off[b + 1], kArenaLimit);  // field offsets are u32
            const uint32_t slot = A.blk_off[b];
            uint32_t nf = 0;
            int32_t st = 0;
            while (p != end) {
                uint32_t no = 0, nl = 0, vo = 0, vl = 0, soft = 0;
                const int32_t rc = blk_field(A, t, p, end, cur, aend, no, nl, vo, vl, soft, T);
                if (rc != 0 && rc != kErrInvalidChar) {
                    st = rc;
                    break;
                }
                A.name_off[slot + nf] = no;
                A.name_len[slot + nf] = nl;
                A.value_off[slot + nf] = vo;
                A.value_len[slot + nf] = vl;
                A.fflags[slot + nf] = (uint8_t)soft;
                ++nf;
            }
            A.nfields[b] = nf;
            A.bstatus[b] = st;
            failed = st != 0;
        }
        *ts = TableState{t.start, t.num, t.whead, failed ? 1u : 0u, t.size, t.cap};
    }
}

uint64_t hpack_conn_scratch(uint32_t table_size) {
    const uint64_t R = ((uint64_t)table_size + 15u) & ~15ull;
    return sizeof(TableState) + R + 16ull * (table_size / kEntryOverhead + 1u);
}

hipError_t launch_hpack_blocks(const uint8_t* in, uint64_t in_size, const uint32_t* blk_off, const uint32_t* conn_first,
                               uint32_t nconn, uint32_t table_size, uint8_t* arena, const uint64_t* arena_off,
                               uint32_t* name_off, uint32_t* name_len, uint32_t* value_off, uint32_t* value_len,
                               uint8_t* fflags, uint32_t* nfields, int32_t* bstatus, uint8_t* scratch, uint32_t flags,
                               hipStream_t stream) {
    if (nconn == 0) return hipSuccess;
    BlkArgs A{in, in_size, blk_off, conn_first, nconn, table_size, arena, arena_off, name_off, name_len, value_off,
              value_len, fflags, nfields, bstatus, scratch, hpack_conn_scratch(table_size), flags};
    const uint32_t blocks = min((nconn + 255u) / 256u, 65535u);
    hipLaunchKernelGGL(hpack_blocks_kernel, dim3(blocks), dim3(256), 0, stream, A);
    return hipGetLastError();
}

}  // namespace hhuff
