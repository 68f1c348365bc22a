// Response header encoders on the GPU (encode side).
//
// HTTP/2: h2o_hpack_flatten_response (lib/http2/hpack.c:1137-1177), h2o_hpack_flatten_trailers
// (:1179-1196) and, on the client side, h2o_hpack_flatten_request (:1044-1096) for many connections, each with its encoder dynamic table (do_encode_header :858-937,
// header_table_add :277-317 with at most 32 entries, header_table_adjust_size :839-856).
// What a field becomes depends on the table, and the table on every earlier field of the connection, so
// the table work is sequential per connection -- but it needs no output bytes: only lengths and equality.
//   1. prep (hpe_prep_kernel, one lane per header): a hash of the name and of the value, the Huffman code
//      bits of each (h2o_hpack_encode_string's verdict and length, hpack.c:816-837), the token facts
//      do_encode_header reads (static name index, dont_compress); strings longer than kLongStr go to
//      long_bits_kernel, one wave per string;
//   2. the walk (hpe_table_kernel, one lane per connection): the table's lengths and hashes sit in LDS, a
//      field compares them with all 32 slots at once (no branch per entry) and checks the bytes of the
//      candidates only; it yields each field's representation, byte length and place in the response.
//      Table entries are references to the bytes (this call's input, or the connection's ring);
//   3. emit (hpe_emit_kernel, one lane per field and one per response head): every field writes its bytes
//      at its place -- prefix integers, raw copies, Huffman codes (encode_core) -- through a register sink;
//      payloads longer than kLongStr are left to long_payload_kernel (one wave per string, OR-placed code
//      bits in LDS), so no lane walks a long string alone;
//   4. frames (hpe_frames_kernel, one workgroup per response longer than max_frame_size): the payload moves
//      apart for the CONTINUATION frame headers, last chunk first (fixup_frame_headers :1012-1042);
//   5. the table pass (hpe_ring_kernel, one wave per connection) copies the live entries' bytes into the
//      connection's other ring, so the next call (HHUFF_ENC_CONTINUE) reads only scratch.
// HTTP/3: h2o_qpack_flatten_response without an encoder-stream buffer (below): stateless per response.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

#include "hhuff.h"
#include "hhuff_device.h"
#include "hhuff_launch.h"
#include "hhuff_tables.h"

namespace hhuff {
namespace {
__device__ const uint32_t e_enc_code[256] = HHUFF_ENC_CODE_INIT;
__device__ const uint8_t e_enc_nbits[256] = HHUFF_ENC_NBITS_INIT;
__device__ const uint8_t e_static_bytes[HHUFF_STATIC_NBYTES] = HHUFF_STATIC_BYTES_INIT;
__device__ const uint16_t e_static_ent[61 * 4] = HHUFF_STATIC_ENT_INIT;
__device__ const uint8_t __attribute__((aligned(16))) e_server[16] = {'s', 'e', 'r', 'v', 'e', 'r'};

constexpr uint32_t kOverhead = 32;     // HEADER_TABLE_ENTRY_SIZE_OFFSET (hpack.c:30)
constexpr uint32_t kTableOffset = 62;  // HEADER_TABLE_OFFSET (hpack.c:29)
constexpr uint32_t kMaxEntries = 32;   // header_table_add(..., 32) (hpack.c:921)
constexpr uint32_t kInitialCap = 4096; // conn->_output_header_table.hpack_capacity (connection.c:1847)
constexpr uint32_t kRing = 4096;       // live entry bytes never exceed the capacity (<= 4096)
constexpr uint32_t kServerIndex = 54;  // H2O_TOKEN_SERVER's http2_static_table_name_index
constexpr uint32_t kLongStr = 256;     // strings longer than this are hashed / coded by a whole wave

// info word of a prepped string pair
constexpr uint32_t kInfoStatic = 0x7Fu;  // static name index (tokens only)
constexpr uint32_t kInfoTokDc = 1u << 8;  // token flag dont_compress (cookie, set-cookie)
constexpr uint32_t kInfoTok = 1u << 9;
constexpr uint32_t kInfoHdrDc = 1u << 10;
constexpr uint32_t kInfoBad = 1u << 11;  // a string past in_size
constexpr uint32_t kInfoFastShift = 12;  // bits 12-19: h2o_hpack_flatten_request's one-byte reference, 0 = none
constexpr uint32_t kInfoFastOwn = 1u << 20;  // ... for one of its own fields (:method, :scheme, :path)

// op code of a field
constexpr uint32_t kOpIndexed = 0, kOpIdxName = 1, kOpNever = 2, kOpNewName = 3;
constexpr uint32_t kOpAsIs = 1u << 9;  // the value goes as it is (encode_as_is, hpack.c:806-814)
constexpr uint32_t kOpFast = 1u << 10; // one byte (bits 11-18): flatten_request's static references
constexpr uint32_t kOpSkip = 1u << 31;

// byte sources of a table entry's name / value
constexpr uint64_t kSrcIn = 0;               // input offset (added in this call)
constexpr uint64_t kSrcScr = 1ull << 62;     // scratch offset (a ring: added by an earlier call)
constexpr uint64_t kSrcConst = 2ull << 62;   // e_server
constexpr uint64_t kSrcOff = (1ull << 62) - 1;

struct EncState {
    uint32_t start, num, ring, failed;
    uint32_t size, cap, pad0, pad1;
};
struct EncEntry {
    uint64_t nsrc, vsrc;
    uint32_t nl, vl, nh, vh;
    uint32_t tok, pad;
};
static_assert(sizeof(EncState) == 32 && sizeof(EncEntry) == 40, "scratch records");
constexpr uint64_t kConnScratch = sizeof(EncState) + kMaxEntries * sizeof(EncEntry) + 2 * kRing;
static_assert(kConnScratch % 16 == 0, "scratch alignment");
}  // namespace

// Strings too long for one lane: their hash / code bits (long_bits_kernel) and their payloads
// (long_payload_kernel) are done by a wave each.
struct LongWork {
    uint32_t* bits;  // [1 + cap]: count, then item << 1 | which (0 name, 1 value)
    uint4* jobs;     // payloads {source offset, length, destination address lo, hi | Huffman << 31}
    uint32_t* njobs;
    uint32_t cap, jcap;
};

struct HpeArgs {
    const uint8_t* in;
    uint64_t in_size;
    const hhuff_hpack_header_t* hdr;
    uint32_t nhdr;
    const hhuff_hpack_response_t* res;
    const uint32_t* conn_first;
    uint32_t nconn, nres;
    uint32_t server_off, server_len;
    uint8_t* out;
    const uint64_t* out_off;
    uint32_t* out_len;
    uint32_t* headers_size;
    int32_t* rstatus;
    uint8_t* scratch;
    uint32_t flags;
    // workspace
    uint4* rec;      // [nhdr + 1] {name hash, value hash, name code bits, value code bits}; item nhdr: server
    uint32_t* info;  // [nhdr + 1]
    uint4* op;       // [nhdr] {dst lo, dst hi, code, 0}
    uint4* plan;     // [2 nres] {base lo, base hi, payload, total} {size update or ~0, server code, server pos, cl len}
    uint32_t* big;   // [nres + 1]: count, then the responses longer than their max_frame_size
    LongWork lw;
};

namespace {
__device__ __forceinline__ const uint8_t* hpe_src(const HpeArgs& A, uint64_t s) {
    const uint64_t o = s & kSrcOff;
    switch (s >> 62) {
        case 0: return A.in + o;
        case 1: return A.scratch + o;
        default: return e_server + o;
    }
}

__device__ __forceinline__ uint32_t int_len(uint32_t v, uint32_t p) {  // h2o_hpack_encode_int's length (hpack.c:757-772)
    const uint32_t pmax = (1u << p) - 1u;
    if (v < pmax) return 1;
    v -= pmax;
    uint32_t n = 2;
    while (v >= 128) {
        v >>= 7;
        ++n;
    }
    return n;
}

__device__ __forceinline__ bool huff_wins(uint32_t len, uint32_t bits) {  // hpack.c:789-791, :799-800
    return len != 0 && bits <= 8u * len - 8u;
}

__device__ __forceinline__ uint32_t str_len(uint32_t len, uint32_t bits) {  // h2o_hpack_encode_string's length
    if (huff_wins(len, bits)) {
        const uint32_t hb = (bits + 7u) >> 3;
        return int_len(hb, 7) + hb;
    }
    return int_len(len, 7) + len;
}

__device__ __forceinline__ uint32_t digits(uint64_t v) {
    uint32_t n = 1;
    while (v >= 10) {
        v /= 10;
        ++n;
    }
    return n;
}

// String hash: sum over the 4-byte words w_k (bytes 4k .. 4k+3, zero past the end) of mix(w_k, k), mixed with
// the length -- a function of the bytes alone that any split of the words computes alike, so one lane and a
// whole wave agree.  Used as a prefilter only: the bytes of a candidate are always compared.
__device__ __forceinline__ uint32_t mix32(uint32_t x) {
    x ^= x >> 16;
    x *= 0x7feb352du;
    x ^= x >> 15;
    x *= 0x846ca68bu;
    x ^= x >> 16;
    return x;
}
__device__ __forceinline__ uint32_t word_term(uint32_t w, uint32_t k) { return mix32(w ^ (k * 0x9E3779B9u)); }
__device__ __forceinline__ uint32_t hash_final(uint32_t sum, uint32_t len) { return mix32(sum ^ (len * 0x85EBCA6Bu)); }

// the 4 bytes of word k of string p (length len), zero past the end; code bits of its bytes
__device__ __forceinline__ uint32_t string_word(const uint8_t* p, uint32_t len, uint32_t k, const uint8_t* nbits, uint32_t& bits) {
    uint32_t w = 0;
    const uint32_t a = 4u * k;
    if (a + 4u <= len) {
        __builtin_memcpy(&w, p + a, 4);
        bits = nbits[w & 0xFFu] + nbits[(w >> 8) & 0xFFu] + nbits[(w >> 16) & 0xFFu] + nbits[w >> 24];
    } else {
        bits = 0;
        for (uint32_t j = 0; j < 4; ++j)
            if (a + j < len) {
                const uint32_t b = p[a + j];
                w |= b << (8 * j);
                bits += nbits[b];
            }
    }
    return w;
}

__device__ __forceinline__ void hash_bits_lane(const uint8_t* p, uint32_t len, const uint8_t* nbits, uint32_t& h, uint32_t& bits) {
    uint32_t sum = 0;
    bits = 0;
    for (uint32_t k = 0; 4u * k < len; ++k) {
        uint32_t b;
        sum += word_term(string_word(p, len, k, nbits, b), k);
        bits += b;
    }
    h = hash_final(sum, len);
}

__device__ __forceinline__ bool lit_eq(const uint8_t* a, const char* lit, uint32_t n) {
    for (uint32_t k = 0; k < n; ++k)
        if (a[k] != (uint8_t)lit[k]) return false;
    return true;
}

// byte equality without an early exit: 16-byte loads issue back to back, one wait covers them
__device__ __forceinline__ bool bytes_eq(const uint8_t* a, const uint8_t* b, uint32_t n) {
#ifdef HHUFF_HPE_NOVERIFY  // ablation only (wrong on a hash collision): what the walk's byte checks cost
    return true;
#endif
    uint32_t diff = 0, k = 0;
    for (; k + 16u <= n; k += 16u) {
        uint4 x, y;
        __builtin_memcpy(&x, a + k, 16);
        __builtin_memcpy(&y, b + k, 16);
        diff |= (x.x ^ y.x) | (x.y ^ y.y) | (x.z ^ y.z) | (x.w ^ y.w);
    }
    for (; k < n; ++k) diff |= (uint32_t)(a[k] ^ b[k]);
    return diff == 0;
}

// h2o_hpack_flatten_request's one-byte static references (hpack.c:950-985 for its own fields, :1083-1086 for
// accept-encoding among the headers) as an info word; the walk applies them by the field's place
__device__ __forceinline__ uint32_t request_fast(const uint8_t* n, uint32_t nl, const uint8_t* v, uint32_t vl) {
    uint32_t b = 0, own = kInfoFastOwn;
    if (nl == 7 && lit_eq(n, ":method", 7)) {
        b = vl == 3 && lit_eq(v, "GET", 3) ? 0x82u : vl == 4 && lit_eq(v, "POST", 4) ? 0x83u : 0u;
    } else if (nl == 7 && lit_eq(n, ":scheme", 7)) {
        b = vl == 5 && lit_eq(v, "https", 5) ? 0x87u : vl == 4 && lit_eq(v, "http", 4) ? 0x86u : 0u;
    } else if (nl == 5 && lit_eq(n, ":path", 5)) {
        b = vl == 1 && v[0] == '/' ? 0x84u : vl == 11 && lit_eq(v, "/index.html", 11) ? 0x85u : 0u;
    } else if (nl == 15 && vl == 13 && lit_eq(n, "accept-encoding", 15) && lit_eq(v, "gzip, deflate", 13)) {
        b = 0x90u, own = 0u;
    }
    return b ? (b << kInfoFastShift | own) : 0u;
}

__device__ __forceinline__ void push_long_bits(const LongWork& L, uint32_t item, uint32_t which) {
    const uint32_t j = atomicAdd(L.bits, 1u);
    if (j < L.cap) L.bits[1 + j] = item << 1 | which;
}
}  // namespace

// 1. prep: one lane per header (item nhdr: the server name under the server token)
__global__ __launch_bounds__(256) void hpe_prep_kernel(HpeArgs A) {
    __shared__ uint8_t s_nbits[256];
    s_nbits[threadIdx.x] = e_enc_nbits[threadIdx.x];
    __syncthreads();
    for (uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x; i <= A.nhdr; i += (uint64_t)gridDim.x * 256u) {
        uint32_t nh, vh, nb = 0, vb = 0, info;
        const uint8_t *n, *v;
        uint32_t nl, vl;
        bool bad;
        if (i == A.nhdr) {
            bad = (uint64_t)A.server_off + A.server_len > A.in_size;
            n = e_server, nl = 6, v = A.in + A.server_off, vl = bad ? 0u : A.server_len;
            info = kServerIndex | kInfoTok | (bad ? kInfoBad : 0u);
        } else {
            const hhuff_hpack_header_t H = A.hdr[i];
            bad = (uint64_t)H.name_off + H.name_len > A.in_size || (uint64_t)H.value_off + H.value_len > A.in_size;
            nl = bad ? 0u : H.name_len, vl = bad ? 0u : H.value_len;
            n = A.in + H.name_off, v = A.in + H.value_off;
            info = (bad ? kInfoBad : 0u) | ((H.flags & HHUFF_HDR_DONT_COMPRESS) ? kInfoHdrDc : 0u);
            if (H.flags & HHUFF_HDR_TOKEN) {
                // lib/common/token_table.h: a token's http2_static_table_name_index is the first static
                // entry with its name; dont_compress is set for cookie and set-cookie
                uint32_t sidx = 0;
                for (uint32_t k = 0; k < 61 && sidx == 0; ++k)
                    if (e_static_ent[4 * k + 1] == nl && bytes_eq(e_static_bytes + e_static_ent[4 * k], n, nl)) sidx = k + 1;
                const bool dc = (nl == 6 && lit_eq(n, "cookie", 6)) || (nl == 10 && lit_eq(n, "set-cookie", 10));
                info |= kInfoTok | sidx | (dc ? kInfoTokDc : 0u) | request_fast(n, nl, v, vl);
            }
        }
        if (nl > kLongStr) {
            push_long_bits(A.lw, (uint32_t)i, 0);
            nh = 0;
        } else {
            hash_bits_lane(n, nl, s_nbits, nh, nb);
        }
        if (vl > kLongStr) {
            push_long_bits(A.lw, (uint32_t)i, 1);
            vh = 0;
        } else {
            hash_bits_lane(v, vl, s_nbits, vh, vb);
        }
        A.rec[i] = make_uint4(nh, vh, nb, vb);
        A.info[i] = info;
        if (i < A.nhdr) A.op[i] = make_uint4(0u, 0u, kOpSkip, 0u);  // a header no response lists writes nothing
    }
}

// Long strings' hash and code bits, one wave per string (the sums of hash_bits_lane split over the lanes):
// rec[item].x / .z for a name, .y / .w for a value.  HASH = false: the bits only (QPACK).
template <bool HASH>
__global__ __launch_bounds__(256) void long_bits_kernel(const uint8_t* in, const hhuff_hpack_header_t* hdr, uint32_t nhdr,
                                                        uint32_t server_off, uint32_t server_len, uint4* rec, LongWork L) {
    __shared__ uint8_t s_nbits[256];
    s_nbits[threadIdx.x] = e_enc_nbits[threadIdx.x];
    __syncthreads();
    const int lane = threadIdx.x & 63;
    const uint32_t n = min(L.bits[0], L.cap);
    for (uint32_t j = blockIdx.x * 4u + (threadIdx.x >> 6); j < n; j += gridDim.x * 4u) {
        const uint32_t e = L.bits[1 + j], item = e >> 1, which = e & 1u;
        const uint8_t* p;
        uint32_t len;
        if (item == nhdr) {
            p = in + server_off, len = server_len;
        } else {
            const hhuff_hpack_header_t H = hdr[item];
            p = in + (which ? H.value_off : H.name_off), len = which ? H.value_len : H.name_len;
        }
        uint32_t sum = 0, bits = 0;
        for (uint32_t k = (uint32_t)lane; 4u * k < len; k += 64u) {
            uint32_t b;
            const uint32_t w = string_word(p, len, k, s_nbits, b);
            if (HASH) sum += word_term(w, k);
            bits += b;
        }
#pragma unroll
        for (int d = 32; d > 0; d >>= 1) {
            sum += (uint32_t)__shfl_xor((int)sum, d);
            bits += (uint32_t)__shfl_xor((int)bits, d);
        }
        if (lane == 0) {
            uint32_t* r = reinterpret_cast<uint32_t*>(rec + item);
            if (HASH) r[which] = hash_final(sum, len);
            r[2 + which] = bits;
        }
    }
}

namespace {
// One wave codes src[0 .. len) into dst: ceil(bits / 8) bytes, the last padded with the EOS prefix
// (hpack.c:795-798).  Rounds of 256 input bytes, 4 per lane: a lane's four codes are OR-placed at their
// stream bit in the wave's LDS stage (place_bits), the stage's whole words go out, the partial last word
// moves to the front.  stage: kStageWords + 4 words of LDS, zero on entry, left zero.
constexpr uint32_t kStageWords = 256;  // >= 256 bytes x 30 bits / 32 + 1
__device__ void wave_huff_long(const uint8_t* src, uint32_t len, uint8_t* dst, const uint2* enc, uint32_t* stage, int lane) {
    const uint32_t obase = lds_addr(stage);
    uint32_t cb = 0;       // bits in stage word 0 carried from the last round
    uint64_t flushed = 0;  // bytes of dst written
    for (uint32_t r0 = 0; r0 < len; r0 += 256u) {
        const uint32_t a = r0 + 4u * (uint32_t)lane;
        uint2 e[4];
        uint32_t n = 0;
#pragma unroll
        for (uint32_t j = 0; j < 4; ++j) {
            e[j] = a + j < len ? enc[src[a + j]] : make_uint2(0u, 0u);
            n += e[j].y;
        }
        const uint32_t off = wave_excl_scan(n, lane);
        const uint32_t tb = cb + off;
        const uint32_t n01 = e[0].y + e[1].y, n23 = e[2].y + e[3].y;
        if (max(max(e[0].y, e[1].y), max(e[2].y, e[3].y)) > 16u) {
            place_bits(obase, tb, (uint64_t)e[0].x << e[1].y | e[1].x, n01);
            place_bits(obase, tb + n01, (uint64_t)e[2].x << e[3].y | e[3].x, n23);
        } else {
            place_bits(obase, tb, ((uint64_t)(e[0].x << e[1].y | e[1].x) << n23) | (e[2].x << e[3].y | e[3].x), n);
        }
        wave_lds_sync();
        const uint32_t total = cb + (uint32_t)__builtin_amdgcn_readlane((int)(off + n), 63);
        const bool last = r0 + 256u >= len;
        const uint32_t whole = total >> 5;
        for (uint32_t w = (uint32_t)lane; w < whole; w += 64u) {  // MSB-first words -> stream bytes
            const uint32_t v = __builtin_bswap32(stage[w]);
            __builtin_memcpy(dst + flushed + 4u * w, &v, 4);
        }
        const uint32_t tail = stage[whole];
        wave_lds_sync();
        for (uint32_t w = (uint32_t)lane; w <= whole; w += 64u) stage[w] = 0u;
        wave_lds_sync();
        flushed += 4ull * whole;
        cb = total & 31u;
        if (last) {
            if (lane == 0 && cb) {
                const uint32_t v = tail | (~0u >> cb);  // EOS-prefix padding of the last byte
                for (uint32_t b = 0; b < (cb + 7u) >> 3; ++b) dst[flushed + b] = (uint8_t)(v >> (24 - 8 * b));
            }
        } else if (lane == 0) {
            stage[0] = tail;
        }
        wave_lds_sync();
    }
}
}  // namespace

// Payloads of long strings (HPACK literals and QPACK flatten_string payloads), one wave per string
__global__ __launch_bounds__(256) void long_payload_kernel(const uint8_t* in, LongWork L) {
    __shared__ uint2 s_enc[256];
    __shared__ uint32_t s_stage[4][kStageWords + 4];
    s_enc[threadIdx.x] = make_uint2(e_enc_code[threadIdx.x], e_enc_nbits[threadIdx.x]);
    for (uint32_t k = threadIdx.x; k < 4 * (kStageWords + 4); k += 256) (&s_stage[0][0])[k] = 0u;
    __syncthreads();
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const uint32_t n = min(*L.njobs, L.jcap);
    for (uint32_t j = blockIdx.x * 4u + (uint32_t)wv; j < n; j += gridDim.x * 4u) {
        const uint4 job = L.jobs[j];
        uint8_t* dst = reinterpret_cast<uint8_t*>((uint64_t)(job.w & 0x7FFFFFFFu) << 32 | job.z);  // an address in `out`
        if (job.w >> 31)
            wave_huff_long(in + job.x, job.y, dst, s_enc, s_stage[wv], lane);
        else
            wave_copy64(in + job.x, dst, lane == 0 ? job.y : 0u, lane);
    }
}

namespace {
// 2. the walk's table: lengths and hashes in LDS ({nl | token << 31, vl, nh, vh} of slot s at
// s_meta[s * 64 + lane]), byte sources in the connection's scratch entries
struct EncTable {
    EncEntry* ent;
    uint4* meta;  // this lane's column: meta[s * 64]
    uint32_t start, num, size, cap;
    __device__ __forceinline__ uint32_t slot(uint32_t k) const { return (start + k) & (kMaxEntries - 1); }
    __device__ __forceinline__ void evict_one() {  // header_table_evict_one (hpack.c:263-275)
        --num;
        const uint4 q = meta[slot(num) * 64];
        size -= (q.x & 0x7FFFFFFFu) + q.y + kOverhead;
    }
    __device__ void add(const EncEntry& e) {  // header_table_add (hpack.c:277-317), at most 32 entries
        const uint32_t add = e.nl + e.vl + kOverhead;
        while (num != 0 && size + add > cap) evict_one();
        while (num >= kMaxEntries) evict_one();
        if (num == 0 && add > cap) return;
        start = (start + kMaxEntries - 1) & (kMaxEntries - 1);
#ifndef HHUFF_HPE_NOENTST  // ablation only: what the entries' global stores cost the walk
        ent[start] = e;
#endif
        meta[start * 64] = make_uint4(e.nl | (e.tok << 31), e.vl, e.nh, e.vh);
        size += add;
        ++num;
    }
};

struct FieldIn {  // what the walk reads of a field
    uint32_t noff, nl, voff, vl;
    uint4 rc;
    uint32_t info;
};

__device__ __forceinline__ FieldIn load_field(const HpeArgs& A, uint32_t h) {
    const hhuff_hpack_header_t H = A.hdr[h];
    return FieldIn{H.name_off, H.name_len, H.value_off, H.value_len, A.rec[h], A.info[h]};
}

// do_encode_header (hpack.c:858-937): returns the op code and its byte length, and updates the table as
// h2o does.  The scan over the entries (:864-890) is done for all 32 slots at once on lengths and hashes;
// the candidates' bytes are then compared in h2o's order (newest first).
__device__ uint32_t hpe_field(const HpeArgs& A, EncTable& t, const FieldIn& F, uint64_t nsrc, uint64_t vsrc, uint32_t& len) {
    const bool tok = (F.info & kInfoTok) != 0;
    const uint32_t key = F.nl | (tok ? 0x80000000u : 0u);
    const uint32_t kmask = tok ? 0xFFFFFFFFu : 0x7FFFFFFFu;  // a token name is compared by pointer (:870-872)
    uint32_t nm = 0, fm = 0;
#pragma unroll
    for (uint32_t k = 0; k < kMaxEntries; ++k) {
        const uint4 q = t.meta[t.slot(k) * 64];
        const bool n_ok = k < t.num && (q.x & kmask) == key && q.z == F.rc.x;
        nm |= (uint32_t)n_ok << k;
        fm |= (uint32_t)(n_ok && q.y == F.vl && q.w == F.rc.y) << k;
    }
    const uint8_t* np = hpe_src(A, nsrc);
    const uint8_t* vp = hpe_src(A, vsrc);
    while (fm) {
        const uint32_t k = __builtin_ctz(fm);
        const EncEntry& e = t.ent[t.slot(k)];
        if (bytes_eq(np, hpe_src(A, e.nsrc), F.nl) && bytes_eq(vp, hpe_src(A, e.vsrc), F.vl)) {
            len = int_len(k + kTableOffset, 7);  // indexed (:881-884)
            return kOpIndexed | ((k + kTableOffset) << 2);
        }
        fm &= fm - 1u;
    }
    uint32_t name_index = F.info & kInfoStatic;  // tokens: the static index; others: the newest name match (:875-876)
    if (!tok) {
        while (nm) {
            const uint32_t k = __builtin_ctz(nm);
            if (bytes_eq(np, hpe_src(A, t.ent[t.slot(k)].nsrc), F.nl)) {
                name_index = k + kTableOffset;
                break;
            }
            nm &= nm - 1u;
        }
    }
    bool dc = (F.info & kInfoHdrDc) != 0;
    if (!dc && tok) dc = (F.info & kInfoTokDc) != 0;  // :892-893
    if (dc) dc = F.vl < 20;                           // :894-895
    uint32_t code;
    if (name_index != 0) {
        code = (dc ? kOpNever : kOpIdxName) | (name_index << 2);
        len = int_len(name_index, dc ? 4u : 6u);
    } else {
        code = kOpNewName;
        len = 1u + str_len(F.nl, F.rc.z);
    }
    if (dc) {
        len += int_len(F.vl, 7) + F.vl;
        code |= kOpAsIs;
    } else {
        len += str_len(F.vl, F.rc.w);
        t.add(EncEntry{nsrc, vsrc, F.nl, F.vl, F.rc.x, F.rc.y, tok ? 1u : 0u, 0u});
    }
    return code;
}
}  // namespace

// 2. the walk: one lane per connection, its responses in order
__global__ __launch_bounds__(64) void hpe_table_kernel(HpeArgs A) {
    __shared__ uint4 s_meta[kMaxEntries * 64];
    const uint32_t lane = threadIdx.x;
    const uint64_t c = (uint64_t)blockIdx.x * 64u + lane;
    if (c >= A.nconn) return;
    uint8_t* scr = A.scratch + c * kConnScratch;
    EncState* ts = reinterpret_cast<EncState*>(scr);
    EncState s0{0u, 0u, 0u, 0u, 0u, kInitialCap, 0u, 0u};
    if (A.flags & HHUFF_ENC_CONTINUE) s0 = *ts;
    EncTable t{reinterpret_cast<EncEntry*>(scr + sizeof(EncState)), s_meta + lane, s0.start, s0.num, s0.size, s0.cap};
    for (uint32_t k = 0; k < t.num; ++k) {
        const EncEntry& e = t.ent[t.slot(k)];
        t.meta[t.slot(k) * 64] = make_uint4(e.nl | (e.tok << 31), e.vl, e.nh, e.vh);
    }
    bool failed = s0.failed != 0;
    const uint4 srv_rc = A.rec[A.nhdr];
    const uint32_t srv_info = A.info[A.nhdr];
    // a malformed conn_first cannot send the walk past the response array
    const uint32_t r1 = min(A.conn_first[c + 1], A.nres), r0 = min(A.conn_first[c], r1);
    hhuff_hpack_response_t R{};
    uint64_t base = 0, limit = 0;
    if (r0 < r1) {  // (res and out_off may be NULL when the call has no responses)
        R = A.res[r0];
        base = A.out_off[r0];
        limit = A.out_off[r0 + 1];
    }
    for (uint32_t r = r0; r < r1; ++r) {
        // the next response's record and region are in flight while this one is walked
        const uint32_t rn = r + 1 < r1 ? r + 1 : r;
        const hhuff_hpack_response_t Rn = A.res[rn];
        const uint64_t base_n = limit, limit_n = A.out_off[rn + 1];
        const bool trailers = (R.flags & HHUFF_RES_TRAILERS) != 0;
        const bool request = !trailers && (R.flags & HHUFF_RES_REQUEST);  // h2o_hpack_flatten_request
        const bool head = !trailers && !request;                          // :status, server, content-length
        const bool server = head && (R.flags & HHUFF_RES_SERVER) && A.server_len != 0;
        const uint32_t h0 = R.hdr_first, h1 = R.hdr_first + R.nhdr;
        const uint32_t own_end = request ? h0 + R.status : h0;  // a request's own fields: method .. expect
        int32_t st = 0;
        if (failed) {
            st = HHUFF_RES_SKIPPED;
        } else if ((uint64_t)R.hdr_first + R.nhdr > A.nhdr || limit < base ||  // header range / region malformed
                   (head && (R.status < 100 || R.status > 999)) || (request && R.status > R.nhdr) ||
                   R.max_frame_size < 16384u ||
                   R.max_frame_size > 0xFFFFFFu || (server && (srv_info & kInfoBad))) {
            st = HHUFF_RES_EINVAL;
        }
        uint32_t pos = 0, su = ~0u, scode = 0, spos = 0, cll = 0;
        if (st == 0) {
            if (R.header_table_size < t.cap) {  // header_table_adjust_size (:839-856)
                t.cap = R.header_table_size;
                while (t.num != 0 && t.size > t.cap) t.evict_one();
                su = t.cap;
                pos += int_len(su, 5);
            }
            if (head) {
                const uint32_t s = R.status;  // encode_status (:437-466)
                pos += (s == 200 || s == 204 || s == 206 || s == 304 || s == 400 || s == 404 || s == 500) ? 1u : 5u;
            }
            if (server) {  // :1159-1163, encode_header_token(H2O_TOKEN_SERVER)
                uint32_t l;
                spos = pos;
                const FieldIn S{0u, 6u, A.server_off, A.server_len, srv_rc, srv_info};
                scode = hpe_field(A, t, S, kSrcConst, kSrcIn | A.server_off, l);
                pos += l;
            }
            FieldIn cur = h0 < h1 ? load_field(A, h0) : FieldIn{};
            for (uint32_t h = h0; h < h1; ++h) {
                const FieldIn nxt = h + 1 < h1 ? load_field(A, h + 1) : cur;  // in flight while this one is walked
                if (cur.info & kInfoBad) {  // a string past in_size: the response is refused (the table no longer
                    st = HHUFF_RES_EINVAL;  // matters: the connection fails with it)
                    break;
                }
                uint32_t l, code;
                const uint32_t fast = (cur.info >> kInfoFastShift) & 0xFFu;
                if (request && fast && (cur.info & kInfoTok) && ((cur.info & kInfoFastOwn) != 0) == (h < own_end)) {
                    code = kOpFast | fast << 11;  // encode_method / _scheme / _path, accept-encoding: no table
                    l = 1;
                } else {
                    code = hpe_field(A, t, cur, kSrcIn | cur.noff, kSrcIn | cur.voff, l);
                }
                const uint64_t dst = base + 9u + pos;
#ifndef HHUFF_HPE_NOOPST  // ablation only: what the per-field op stores cost the walk
                A.op[h] = make_uint4((uint32_t)dst, (uint32_t)(dst >> 32), code, 0u);
#endif
                pos += l;
                cur = nxt;
            }
            if (head && R.content_length != ~0ull) {  // encode_content_length (:468-485)
                cll = 3u + digits(R.content_length);
                pos += cll;
            }
            const uint32_t M = R.max_frame_size;
            const uint64_t total = 9ull + pos + (pos > M ? 9ull * ((pos - 1u) / M) : 0ull);
            if (st == 0 && total > limit - base) st = HHUFF_RES_SPACE;
            if (st == 0) {
                A.out_len[r] = (uint32_t)total;
                A.headers_size[r] = pos;
                A.plan[2 * r] = make_uint4((uint32_t)base, (uint32_t)(base >> 32), pos, (uint32_t)total);
                A.plan[2 * r + 1] = make_uint4(su, server ? scode : kOpSkip, spos, cll);
                if (pos > M) A.big[1 + atomicAdd(A.big, 1u)] = r;
            }
        }
        if (st != 0) {
            A.out_len[r] = 0;
            A.headers_size[r] = 0;
            A.plan[2 * r + 1] = make_uint4(~0u, kOpSkip, 0u, 0u);
            A.plan[2 * r] = make_uint4(0u, 0u, 0u, 0u);
            if ((uint64_t)R.hdr_first + R.nhdr <= A.nhdr)  // a malformed range is not touched
                for (uint32_t h = h0; h < h1; ++h) A.op[h] = make_uint4(0u, 0u, kOpSkip, 0u);
            failed = true;
        }
        A.rstatus[r] = st;
        R = Rn;
        base = base_n;
        limit = limit_n;
    }
    *ts = EncState{t.start, t.num, s0.ring, failed ? 1u : 0u, t.size, t.cap, 0u, 0u};
}

namespace {
__device__ __forceinline__ void sink_int(RegSink& sink, uint32_t first, uint32_t v, uint32_t p) {  // hpack.c:757-772
    const uint32_t pmax = (1u << p) - 1u;
    if (v < pmax) {
        sink.put1(first | v);
        return;
    }
    sink.put1(first | pmax);
    v -= pmax;
    while (v >= 128) {
        sink.put1(0x80u | (v & 127u));
        v >>= 7;
    }
    sink.put1(v);
}

__device__ __forceinline__ void sink_raw(RegSink& sink, const GlobalSource& src, uint32_t s, uint32_t len) {
    uint32_t a = s & ~3u, rem = len, skip = s & 3u;
    while (rem) {
        const uint32_t w = src.word(a) >> (8 * skip);
        const uint32_t k = min(4u - skip, rem);
        sink.push(w, k);
        rem -= k;
        a += 4;
        skip = 0;
    }
}

// The payload of a string literal: written here, or -- longer than kLongStr -- handed to
// long_payload_kernel while the sink steps over its bytes.
__device__ __forceinline__ void sink_payload(RegSink& sink, const GlobalSource& src, uint32_t s, uint32_t len, bool huff,
                                             uint32_t hb, const uint2* enc, const LongWork& L) {
    if (len > kLongStr) {
        sink.finish();
        const uint64_t d = (uint64_t)sink.p;
        const uint32_t j = atomicAdd(L.njobs, 1u);
        if (j < L.jcap) L.jobs[j] = make_uint4(s, len, (uint32_t)d, (uint32_t)(d >> 32) | (huff ? 0x80000000u : 0u));
        sink.init(sink.p + (huff ? hb : len));
    } else if (huff) {
        encode_core(src, s, len, sink, enc);  // flushes the sink
    } else {
        sink_raw(sink, src, s, len);
    }
}

// h2o_hpack_encode_string (hpack.c:816-837) of in[s .. s + len) whose code is `bits` long
__device__ __forceinline__ void sink_string(RegSink& sink, const GlobalSource& src, uint32_t s, uint32_t len, uint32_t bits,
                                            const uint2* enc, const LongWork& L) {
    const bool huff = huff_wins(len, bits);
    const uint32_t hb = (bits + 7u) >> 3;
    sink_int(sink, huff ? 0x80u : 0u, huff ? hb : len, 7);
    sink_payload(sink, src, s, len, huff, hb, enc, L);
}

__device__ void emit_field(const GlobalSource& src, uint8_t* dst, uint32_t code, uint32_t noff, uint32_t nl, uint32_t voff,
                           uint32_t vl, uint4 rc, const uint2* enc, const LongWork& L) {
    if (code & kOpFast) {
        *dst = (uint8_t)(code >> 11);
        return;
    }
    RegSink sink;
    sink.init(dst);
    const uint32_t kind = code & 3u, idx = (code >> 2) & 0x7Fu;
    switch (kind) {
        case kOpIndexed:
            sink_int(sink, 0x80u, idx, 7);
            sink.finish();
            return;
        case kOpIdxName: sink_int(sink, 0x40u, idx, 6); break;
        case kOpNever: sink_int(sink, 0x10u, idx, 4); break;
        default:
            sink.put1(0x40u);
            sink_string(sink, src, noff, nl, rc.z, enc, L);
            break;
    }
    if (code & kOpAsIs) {  // encode_as_is (:806-814)
        sink_int(sink, 0u, vl, 7);
        sink_payload(sink, src, voff, vl, false, 0u, enc, L);
    } else {
        sink_string(sink, src, voff, vl, rc.w, enc, L);
    }
    sink.finish();
}

__device__ __forceinline__ void put_frame_header(uint8_t* d, uint32_t len, uint32_t type, uint32_t flags, uint32_t sid) {
    d[0] = (uint8_t)(len >> 16);  // h2o_http2_encode_frame_header (lib/http2/frame.c:68-79)
    d[1] = (uint8_t)(len >> 8);
    d[2] = (uint8_t)len;
    d[3] = (uint8_t)type;
    d[4] = (uint8_t)flags;
    d[5] = (uint8_t)(sid >> 24);
    d[6] = (uint8_t)(sid >> 16);
    d[7] = (uint8_t)(sid >> 8);
    d[8] = (uint8_t)sid;
}
}  // namespace

// 3. emit: items 0 .. nhdr-1 are fields, nhdr .. nhdr+nres-1 response heads (frame header, table size
//    update, :status, server, and the content-length at the end)
__global__ __launch_bounds__(256) void hpe_emit_kernel(HpeArgs A) {
    __shared__ uint2 s_enc[256];
    s_enc[threadIdx.x] = make_uint2(e_enc_code[threadIdx.x], e_enc_nbits[threadIdx.x]);
    __syncthreads();
    const GlobalSource src{A.in, A.in_size};
    const uint64_t items = (uint64_t)A.nhdr + A.nres;
    for (uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x; i < items; i += (uint64_t)gridDim.x * 256u) {
        if (i < A.nhdr) {
            const uint4 o = A.op[i];
            if (o.z & kOpSkip) continue;
            const hhuff_hpack_header_t H = A.hdr[i];
            emit_field(src, A.out + ((uint64_t)o.y << 32 | o.x), o.z, H.name_off, H.name_len, H.value_off, H.value_len,
                       A.rec[i], s_enc, A.lw);
            continue;
        }
        const uint32_t r = (uint32_t)(i - A.nhdr);
        const uint4 p0 = A.plan[2 * r], p1 = A.plan[2 * r + 1];
        if (p0.w == 0) continue;  // failed
        const hhuff_hpack_response_t R = A.res[r];
        uint8_t* base = A.out + ((uint64_t)p0.y << 32 | p0.x);
        const bool trailers = (R.flags & HHUFF_RES_TRAILERS) != 0;
        const uint32_t es = (trailers || (R.flags & HHUFF_RES_END_STREAM)) ? 1u : 0u;
        if (p0.z <= R.max_frame_size) put_frame_header(base, p0.z, 1u, 4u | es, R.stream_id);  // else hpe_frames_kernel
        RegSink sink;
        sink.init(base + 9);
        if (p1.x != ~0u) sink_int(sink, 0x20u, p1.x, 5);  // Dynamic Table Size Update (:852-853)
        if (!trailers && !(R.flags & HHUFF_RES_REQUEST)) {
            const uint32_t s = R.status;  // encode_status (:437-466)
            const uint32_t c = s == 200 ? 8 : s == 204 ? 9 : s == 206 ? 10 : s == 304 ? 11 : s == 400 ? 12 : s == 404 ? 13 : s == 500 ? 14 : 0;
            if (c) {
                sink.put1(0x80u | c);
            } else {
                sink.put1(8u);
                sink.put1(3u);
                sink.put1('0' + s / 100);
                sink.put1('0' + s / 10 % 10);
                sink.put1('0' + s % 10);
            }
        }
        sink.finish();
        if (!(p1.y & kOpSkip))
            emit_field(src, base + 9 + p1.z, p1.y, 0u, 6u, A.server_off, A.server_len, A.rec[A.nhdr], s_enc, A.lw);
        if (p1.w) {  // encode_content_length (:468-485): literal without indexing, name index 28, raw digits
            uint8_t* d = base + 9 + p0.z - p1.w;
            d[0] = 0x0f;
            d[1] = 0x0d;
            d[2] = (uint8_t)(p1.w - 3u);
            uint64_t v = R.content_length;
            for (uint32_t k = p1.w - 1; k >= 3; --k) {
                d[k] = (uint8_t)('0' + v % 10);
                v /= 10;
            }
        }
    }
}

// 4. frames: one workgroup per listed response; chunk j (>= 1) of the payload moves up by 9 j bytes,
//    last chunk first and each chunk top-down through LDS, so no byte is overwritten before it is read
__global__ __launch_bounds__(256) void hpe_frames_kernel(HpeArgs A) {
    __shared__ uint8_t s_buf[8192];
    const uint32_t nbig = A.big[0];
    for (uint32_t b = blockIdx.x; b < nbig; b += gridDim.x) {
        const uint32_t r = A.big[1 + b];
        const uint4 p0 = A.plan[2 * r];
        const hhuff_hpack_response_t R = A.res[r];
        uint8_t* base = A.out + ((uint64_t)p0.y << 32 | p0.x);
        const uint32_t P = p0.z, M = R.max_frame_size;
        const uint32_t k = (P + M - 1u) / M;
        for (uint32_t j = k - 1; j >= 1; --j) {
            const uint64_t lo = 9ull + (uint64_t)j * M, hi = 9ull + min((uint64_t)(j + 1) * M, (uint64_t)P);
            const uint64_t shift = 9ull * j;
            for (uint64_t top = hi; top > lo;) {
                const uint64_t bot = top - lo > sizeof(s_buf) ? top - sizeof(s_buf) : lo;
                for (uint64_t q = bot + threadIdx.x; q < top; q += 256) s_buf[q - bot] = base[q];
                __syncthreads();
                for (uint64_t q = bot + threadIdx.x; q < top; q += 256) base[q + shift] = s_buf[q - bot];
                __syncthreads();
                top = bot;
            }
            if (threadIdx.x == 0) {
                const bool last = j == k - 1;
                put_frame_header(base + (uint64_t)j * (M + 9u), last ? (uint32_t)(hi - lo) : M, 9u, last ? 4u : 0u,
                                 R.stream_id);
            }
            __syncthreads();
        }
        if (threadIdx.x == 0) {
            const uint32_t es = ((R.flags & HHUFF_RES_TRAILERS) || (R.flags & HHUFF_RES_END_STREAM)) ? 1u : 0u;
            put_frame_header(base, M, 1u, es, R.stream_id);
        }
        __syncthreads();
    }
}

// 5. the table pass: one wave per connection writes its live entries' bytes, newest first, into the ring
//    they do not use now and points the entries there (as blk_table_kernel does for the decoder)
__global__ __launch_bounds__(256) void hpe_ring_kernel(HpeArgs A) {
    const int lane = threadIdx.x & 63;
    const uint64_t c = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    if (c >= A.nconn) return;
    const uint64_t base = c * kConnScratch;
    EncState* ts = reinterpret_cast<EncState*>(A.scratch + base);
    EncEntry* ent = reinterpret_cast<EncEntry*>(A.scratch + base + sizeof(EncState));
    const EncState s = *ts;
    const uint32_t nring = s.ring ^ 1u;
    const uint64_t rbase = base + sizeof(EncState) + kMaxEntries * sizeof(EncEntry) + (uint64_t)nring * kRing;
    uint32_t carry = 0;
    for (uint32_t k0 = 0; k0 < s.num; k0 += 64) {
        const uint32_t k = k0 + (uint32_t)lane;
        const bool live = k < s.num;
        const uint32_t i = (s.start + k) & (kMaxEntries - 1);
        EncEntry e{};
        if (live) e = ent[i];
        const uint32_t sz = live ? e.nl + e.vl : 0u;
        const uint32_t dst = carry + wave_excl_scan(sz, lane);
        carry += (uint32_t)__builtin_amdgcn_readlane((int)(dst - carry + sz), 63);
        uint8_t* d = A.scratch + rbase + dst;
        wave_copy64(hpe_src(A, e.nsrc), d, live ? e.nl : 0u, lane);
        wave_copy64(hpe_src(A, e.vsrc), d + e.nl, live ? e.vl : 0u, lane);
        if (live) {
            ent[i].nsrc = kSrcScr | (rbase + dst);
            ent[i].vsrc = kSrcScr | (rbase + dst + e.nl);
        }
    }
    if (lane == 0) ts->ring = nring;
}

// ---------------------------------------------------------------------------------------------------
// HTTP/3 response HEADERS frames: h2o_qpack_flatten_response (lib/http3/qpack.c:1352-1399) as h2o's HTTP/3
// server calls it (lib/http3/server.c:1680-1683), without an encoder-stream buffer: the encoder's dynamic
// table stays empty (do_flatten_header inserts only with one, :1175-1176), so a field is a static reference
// or a literal and a response depends on nothing but itself -- no sequential walk:
//   qpe_size_kernel (one lane per header): h2o_qpack_lookup_static for token names (lib/common/token_table.h:
//     the static entry with the name and value, else the first with the name), the representation and the
//     code bits of its literals (long ones: long_bits_kernel);
//   qpe_layout_kernel (one lane per response): the fields' byte lengths (flatten_string's Huffman verdict
//     from the code bits), status, server, content-length and datagram-flow-id fields, the field positions,
//     the section length and the frame header's varint;
//   qpe_emit_kernel (one lane per field and per response head): the bytes, in place (long payloads:
//     long_payload_kernel).
// ---------------------------------------------------------------------------------------------------
namespace {
__device__ const uint8_t q_static_bytes[HHUFF_QSTATIC_NBYTES] = HHUFF_QSTATIC_BYTES_INIT;
__device__ const uint16_t q_static_ent[99 * 4] = HHUFF_QSTATIC_ENT_INIT;
__device__ const uint8_t __attribute__((aligned(16))) q_dfid_name[16] = {'d', 'a', 't', 'a', 'g', 'r', 'a', 'm',
                                                                         '-', 'f', 'l', 'o', 'w', '-', 'i', 'd'};

constexpr uint32_t kQStaticIdx = 0, kQStaticRef = 1, kQLiteral = 2;  // representations (code bits 0-1)
constexpr uint32_t kQDc = 1u << 9;                                     // dont_compress
constexpr uint32_t kQBad = 1u << 30;                                   // a string past in_size
}  // namespace

struct QpeArgs {
    const uint8_t* in;
    uint64_t in_size;
    const hhuff_hpack_header_t* hdr;
    uint32_t nhdr;
    const hhuff_qpack_response_t* res;
    uint32_t nres;
    uint32_t server_off, server_len;
    uint8_t* out;
    const uint64_t* out_off;
    uint32_t* out_len;
    uint32_t* header_len;
    int32_t* rstatus;
    // workspace
    uint4* rec;   // [nhdr + 1] {0, code, name code bits, value code bits}; item nhdr: the server name
    uint2* dst;   // [nhdr] the field's output offset (lo, hi); hi = ~0 when its response failed
    uint4* plan;  // [2 nres] {base lo, base hi, section length, frame total} {status size, server size, cl size, dfid size}
    LongWork lw;
};

namespace {
// flatten_string (qpack.c:1042-1066): its length with prefix p, Huffman when not dont_compress and shorter
__device__ __forceinline__ uint32_t q_str_len(uint32_t len, uint32_t bits, uint32_t p, bool dc) {
    if (!dc && huff_wins(len, bits)) {
        const uint32_t hb = (bits + 7u) >> 3;
        return int_len(hb, p) + hb;
    }
    return int_len(len, p) + len;
}

__device__ __forceinline__ uint32_t code_bits(const uint8_t* p, uint32_t len) {
    uint32_t bits = 0;
    for (uint32_t k = 0; k < len; ++k) bits += e_enc_nbits[p[k]];
    return bits;
}

// do_flatten_header (:1148-1213) with an empty dynamic table: the length of the field
__device__ __forceinline__ uint32_t q_field_len(uint32_t code, uint32_t nl, uint32_t vl, uint32_t nbits, uint32_t vbits) {
    const uint32_t kind = code & 3u, idx = (code >> 2) & 0x7Fu;
    const bool dc = (code & kQDc) != 0;
    if (kind == kQStaticIdx) return int_len(idx, 6);                                  // flatten_static_indexed
    if (kind == kQStaticRef) return int_len(idx, 4) + q_str_len(vl, vbits, 7, dc);    // flatten_static_nameref
    return q_str_len(nl, nbits, 3, false) + q_str_len(vl, vbits, 7, dc);             // flatten_without_nameref
}

// flatten_string on a RegSink: `first` holds the bits above the H bit
__device__ __forceinline__ void q_sink_string(RegSink& sink, const GlobalSource& src, uint32_t first, uint32_t s, uint32_t len,
                                              uint32_t bits, uint32_t p, bool dc, const uint2* enc, const LongWork& L) {
    const bool huff = !dc && huff_wins(len, bits);
    const uint32_t hb = (bits + 7u) >> 3;
    if (huff)
        sink_int(sink, (first & ~((1u << p) - 1u)) | (1u << p), hb, p);
    else
        sink_int(sink, first & ~((2u << p) - 1u), len, p);
    sink_payload(sink, src, s, len, huff, hb, enc, L);
}

__device__ __forceinline__ void q_emit_field(RegSink& sink, const GlobalSource& src, uint32_t code, uint32_t noff, uint32_t nl, uint32_t voff,
                             uint32_t vl, uint32_t nbits, uint32_t vbits, const uint2* enc, const LongWork& L) {
    const uint32_t kind = code & 3u, idx = (code >> 2) & 0x7Fu;
    const bool dc = (code & kQDc) != 0;
    if (kind == kQStaticIdx) {
        sink_int(sink, 0xc0u, idx, 6);
        return;
    }
    if (kind == kQStaticRef)
        sink_int(sink, 0x50u | (dc ? 0x20u : 0u), idx, 4);
    else
        q_sink_string(sink, src, 0x20u | (dc ? 0x10u : 0u), noff, nl, nbits, 3, false, enc, L);
    q_sink_string(sink, src, 0u, voff, vl, vbits, 7, dc, enc, L);
}

__device__ __forceinline__ uint32_t q_status_index(uint32_t s) {  // INDEXED_STATUS (:1362-1377)
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

__device__ const uint64_t q_pow10[20] = {1ull, 10ull, 100ull, 1000ull, 10000ull, 100000ull, 1000000ull, 10000000ull,
                                         100000000ull, 1000000000ull, 10000000000ull, 100000000000ull, 1000000000000ull,
                                         10000000000000ull, 100000000000000ull, 1000000000000000ull,
                                         10000000000000000ull, 100000000000000000ull, 1000000000000000000ull,
                                         10000000000000000000ull};
// digit k (most significant first) of the n-digit decimal v
__device__ __forceinline__ uint32_t q_digit(uint64_t v, uint32_t n, uint32_t k) {
    return '0' + (uint32_t)((v / q_pow10[n - 1 - k]) % 10u);
}
// the decimal digits of v ("%u" / "%zu"): their count, and their code bits in `bits`
__device__ __forceinline__ uint32_t q_digits(uint64_t v, uint32_t& bits) {
    uint32_t n = 1;
    while (n < 20 && v >= q_pow10[n]) ++n;
    bits = 0;
    for (uint32_t k = 0; k < n; ++k) bits += e_enc_nbits[q_digit(v, n, k)];
    return n;
}

// a field whose value is the decimal of v (status / content-length): static name reference `idx`
__device__ __forceinline__ uint32_t q_local_len(uint32_t idx, uint32_t n, uint32_t bits) {
    return int_len(idx, 4) + q_str_len(n, bits, 7, false);
}
__device__ __forceinline__ void q_emit_local(RegSink& sink, uint32_t idx, uint64_t v, const uint2* enc) {
    uint32_t bits;
    const uint32_t n = q_digits(v, bits);
    sink_int(sink, 0x50u, idx, 4);
    if (huff_wins(n, bits)) {
        sink_int(sink, 0x80u, (bits + 7u) >> 3, 7);
        uint64_t acc = 0;  // <= 20 digits x 6 bits: flushed a byte at a time
        uint32_t an = 0;
        for (uint32_t k = 0; k < n; ++k) {
            const uint2 e = enc[q_digit(v, n, k)];
            acc = acc << e.y | e.x;
            an += e.y;
            while (an >= 8) {
                an -= 8;
                sink.put1((uint32_t)(acc >> an) & 0xFFu);
            }
        }
        if (an) sink.put1((uint32_t)((acc << (8 - an)) | (0xFFu >> an)) & 0xFFu);  // EOS prefix padding (hpack.c:795-798)
    } else {
        sink_int(sink, 0u, n, 7);
        for (uint32_t k = 0; k < n; ++k) sink.put1(q_digit(v, n, k));
    }
}

__device__ __forceinline__ uint32_t q_varint_len(uint64_t v) { return v <= 63 ? 1u : v <= 16383 ? 2u : v <= 1073741823 ? 4u : 8u; }
}  // namespace

__global__ __launch_bounds__(256) void qpe_size_kernel(QpeArgs A) {
    for (uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x; i <= A.nhdr; i += (uint64_t)gridDim.x * 256u) {
        if (i < A.nhdr) A.dst[i] = make_uint2(0u, ~0u);  // a header no response lists writes nothing
        if (i == A.nhdr) {  // the server name: static name reference 92 (:1387-1389)
            const bool bad = (uint64_t)A.server_off + A.server_len > A.in_size;
            uint32_t vb = 0;
            if (!bad && A.server_len > kLongStr)
                push_long_bits(A.lw, (uint32_t)i, 1);
            else if (!bad)
                vb = code_bits(A.in + A.server_off, A.server_len);
            A.rec[i] = make_uint4(0u, kQStaticRef | (92u << 2) | (bad ? kQBad : 0u), 0u, vb);
            continue;
        }
        const hhuff_hpack_header_t H = A.hdr[i];
        if ((uint64_t)H.name_off + H.name_len > A.in_size || (uint64_t)H.value_off + H.value_len > A.in_size) {
            A.rec[i] = make_uint4(0u, kQBad, 0u, 0u);
            continue;
        }
        const uint8_t* n = A.in + H.name_off;
        const uint8_t* v = A.in + H.value_off;
        int32_t sidx = -1;
        bool exact = false;
        if (H.flags & HHUFF_HDR_TOKEN) {  // h2o_qpack_lookup_static[token] (flatten_header :1219-1224)
            for (uint32_t k = 0; k < 99 && !exact; ++k) {
                if (q_static_ent[4 * k + 1] != H.name_len || !bytes_eq(q_static_bytes + q_static_ent[4 * k], n, H.name_len))
                    continue;
                if (sidx < 0) sidx = (int32_t)k;
                if (q_static_ent[4 * k + 3] == H.value_len && bytes_eq(q_static_bytes + q_static_ent[4 * k + 2], v, H.value_len)) {
                    sidx = (int32_t)k;
                    exact = true;
                }
            }
        }
        const bool dc = (H.flags & HHUFF_HDR_DONT_COMPRESS) != 0;
        const uint32_t code = (sidx >= 0 ? (exact ? kQStaticIdx : kQStaticRef) | ((uint32_t)sidx << 2) : kQLiteral) | (dc ? kQDc : 0u);
        uint32_t nb = 0, vb = 0;
        if (sidx < 0) {  // the name is a literal
            if (H.name_len > kLongStr)
                push_long_bits(A.lw, (uint32_t)i, 0);
            else
                nb = code_bits(n, H.name_len);
        }
        if (!(sidx >= 0 && exact) && !dc) {  // the value may be Huffman-coded
            if (H.value_len > kLongStr)
                push_long_bits(A.lw, (uint32_t)i, 1);
            else
                vb = code_bits(v, H.value_len);
        }
        A.rec[i] = make_uint4(0u, code, nb, vb);
    }
}

__global__ __launch_bounds__(256) void qpe_layout_kernel(QpeArgs A) {
    for (uint64_t r = (uint64_t)blockIdx.x * 256u + threadIdx.x; r < A.nres; r += (uint64_t)gridDim.x * 256u) {
        const hhuff_qpack_response_t R = A.res[r];
        const bool request = (R.flags & HHUFF_QRES_REQUEST) != 0;  // h2o_qpack_flatten_request: its own fields are
        const bool server = !request && (R.flags & HHUFF_RES_SERVER) && A.server_len != 0;  // headers of the list
        const bool dfid = (R.flags & HHUFF_QRES_DATAGRAM) != 0;
        const uint4 sr = A.rec[A.nhdr];
        // a header range past the call's headers or a region that ends before it starts: EINVAL
        const bool malformed = (uint64_t)R.hdr_first + R.nhdr > A.nhdr || A.out_off[r + 1] < A.out_off[r];
        bool bad = malformed || (server && (sr.y & kQBad)) || (dfid && (uint64_t)R.dfid_off + R.dfid_len > A.in_size);
        uint32_t bits;
        const uint32_t si = request ? 0u : q_status_index(R.status);
        uint32_t st_len = si ? int_len(si, 6) : 0u;
        if (!si && !request) {
            const uint32_t n = q_digits((uint16_t)R.status, bits);
            st_len = q_local_len(24, n, bits);
        }
        const uint32_t sv_len = server ? q_field_len(sr.y & ~kQBad, 0, A.server_len, 0, sr.w) : 0u;
        uint32_t cl_len = 0;
        if (!request && R.content_length != ~0ull) {
            if (R.content_length == 0) {
                cl_len = 1;
            } else {
                const uint32_t n = q_digits(R.content_length, bits);
                cl_len = q_local_len(4, n, bits);
            }
        }
        uint32_t df_len = 0;
        if (dfid && !bad)
            df_len = q_field_len(kQLiteral, 16, R.dfid_len, code_bits(q_dfid_name, 16), code_bits(A.in + R.dfid_off, R.dfid_len));
        const uint32_t h0 = R.hdr_first, h1 = R.hdr_first + R.nhdr;
        uint64_t body = 2u + st_len + sv_len + cl_len;  // after the section prefix 00 00
        for (uint32_t h = h0; h < h1 && !bad; ++h) {
            const uint4 rc = A.rec[h];
            if (rc.y & kQBad) {
                bad = true;
                break;
            }
            const hhuff_hpack_header_t H = A.hdr[h];
            body += q_field_len(rc.y, H.name_len, H.value_len, rc.z, rc.w);
        }
        body += df_len;
        const uint64_t base = A.out_off[r];
        int32_t st = bad ? HHUFF_RES_EINVAL : 0;
        const uint64_t total = 1u + q_varint_len(body) + body;
        if (st == 0 && (total > A.out_off[r + 1] - base || body > 0xFFFFFFFFull)) st = HHUFF_RES_SPACE;
        if (st == 0) {
            uint64_t o = base + 1u + q_varint_len(body) + 2u + st_len + sv_len + cl_len;
            for (uint32_t h = h0; h < h1; ++h) {
                A.dst[h] = make_uint2((uint32_t)o, (uint32_t)(o >> 32));
                const uint4 rc = A.rec[h];
                const hhuff_hpack_header_t H = A.hdr[h];
                o += q_field_len(rc.y, H.name_len, H.value_len, rc.z, rc.w);
            }
            A.plan[2 * r] = make_uint4((uint32_t)base, (uint32_t)(base >> 32), (uint32_t)body, (uint32_t)total);
            A.plan[2 * r + 1] = make_uint4(st_len, sv_len, cl_len, df_len);
            A.out_len[r] = (uint32_t)total;
            A.header_len[r] = (uint32_t)body;
        } else {
            for (uint32_t h = h0; h < h1 && !malformed; ++h) A.dst[h] = make_uint2(0u, ~0u);
            A.plan[2 * r] = make_uint4(0u, 0u, 0u, 0u);
            A.out_len[r] = 0;
            A.header_len[r] = 0;
        }
        A.rstatus[r] = st;
    }
}

__global__ __launch_bounds__(256) void qpe_emit_kernel(QpeArgs A) {
    __shared__ uint2 s_enc[256];
    s_enc[threadIdx.x] = make_uint2(e_enc_code[threadIdx.x], e_enc_nbits[threadIdx.x]);
    __syncthreads();
    const GlobalSource src{A.in, A.in_size};
    const uint64_t items = (uint64_t)A.nhdr + A.nres;
    for (uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x; i < items; i += (uint64_t)gridDim.x * 256u) {
        if (i < A.nhdr) {
            const uint2 o = A.dst[i];
            if (o.y == ~0u) continue;
            const hhuff_hpack_header_t H = A.hdr[i];
            const uint4 rc = A.rec[i];
            RegSink sink;
            sink.init(A.out + ((uint64_t)o.y << 32 | o.x));
            q_emit_field(sink, src, rc.y, H.name_off, H.name_len, H.value_off, H.value_len, rc.z, rc.w, s_enc, A.lw);
            sink.finish();
            continue;
        }
        const uint32_t r = (uint32_t)(i - A.nhdr);
        const uint4 p0 = A.plan[2 * r], p1 = A.plan[2 * r + 1];
        if (p0.w == 0) continue;
        const hhuff_qpack_response_t R = A.res[r];
        uint8_t* base = A.out + ((uint64_t)p0.y << 32 | p0.x);
        RegSink sink;
        sink.init(base);
        sink.put1(0x01u);  // H2O_HTTP3_FRAME_TYPE_HEADERS, then the length as a QUIC varint (finalize_flatten :1303-1307)
        const uint32_t vl = q_varint_len(p0.z);
        const uint32_t tag = vl == 1 ? 0x00u : vl == 2 ? 0x40u : vl == 4 ? 0x80u : 0xC0u;
        for (uint32_t k = 0; k < vl; ++k) {
            const uint32_t b = k + 4 < vl ? 0u : (p0.z >> (8 * (vl - 1 - k))) & 0xFFu;
            sink.put1(k == 0 ? (b | tag) : b);
        }
        sink.put1(0u);  // Required Insert Count 0
        sink.put1(0u);  // Delta Base 0
        const uint32_t si = q_status_index(R.status);
        if (R.flags & HHUFF_QRES_REQUEST) {
        } else if (si) {
            sink_int(sink, 0xc0u, si, 6);
        } else {
            q_emit_local(sink, 24, (uint16_t)R.status, s_enc);
        }
        if (p1.y) {
            const uint4 sr = A.rec[A.nhdr];
            q_emit_field(sink, src, sr.y & ~kQBad, 0u, 0u, A.server_off, A.server_len, 0u, sr.w, s_enc, A.lw);
        }
        if (p1.z) {
            if (R.content_length == 0)
                sink_int(sink, 0xc0u, 4, 6);
            else
                q_emit_local(sink, 4, R.content_length, s_enc);
        }
        sink.finish();
        if (p1.w) {  // datagram-flow-id last (:1396-1398): a literal with its name (no static entry)
            RegSink s2;
            s2.init(base + p0.w - p1.w);
            const GlobalSource nsrc{q_dfid_name, 16};
            q_sink_string(s2, nsrc, 0x20u, 0u, 16u, code_bits(q_dfid_name, 16), 3, false, s_enc, A.lw);
            q_sink_string(s2, src, 0u, R.dfid_off, R.dfid_len, code_bits(A.in + R.dfid_off, R.dfid_len), 7, false, s_enc, A.lw);
            s2.finish();
        }
    }
}

uint64_t hpenc_conn_scratch() { return kConnScratch; }

namespace {
// the long-string lists: bits [1 + 2 nhdr + 2] (a header's name and value, the server name) and payload jobs
// [2 nhdr + 2 nres + 2] (a field's name and value, a response head's server and datagram-flow-id values)
struct LongCaps {
    uint32_t bits, jobs;
};
LongCaps long_caps(uint32_t nhdr, uint32_t nres) { return LongCaps{2u * nhdr + 2u, 2u * nhdr + 2u * nres + 2u}; }
uint64_t long_ws_bytes(uint32_t nhdr, uint32_t nres) {
    const LongCaps c = long_caps(nhdr, nres);
    return 16ull * c.jobs + 4ull * (c.bits + 1) + 16;
}
LongWork long_ws(uint8_t* p, uint32_t nhdr, uint32_t nres) {
    const LongCaps c = long_caps(nhdr, nres);
    LongWork L;
    L.jobs = reinterpret_cast<uint4*>(p);
    L.bits = reinterpret_cast<uint32_t*>(p + 16ull * c.jobs);
    L.njobs = L.bits + 1 + c.bits;
    L.cap = c.bits;
    L.jcap = c.jobs;
    return L;
}
}  // namespace

hipError_t launch_hpack_flatten(const uint8_t* in, uint64_t in_size, const hhuff_hpack_header_t* hdr, uint32_t nhdr,
                                const hhuff_hpack_response_t* res, const uint32_t* conn_first, uint32_t nconn, uint32_t nres,
                                uint32_t server_off, uint32_t server_len, uint8_t* out, const uint64_t* out_off,
                                uint32_t* out_len, uint32_t* headers_size, int32_t* rstatus, uint8_t* scratch,
                                uint32_t flags, hipStream_t stream) {
    if (nconn == 0) return hipSuccess;
    const uint64_t lw_bytes = long_ws_bytes(nhdr, nres);
    const uint64_t ws_bytes = 16ull * (nhdr + 1) + 16ull * nhdr + 32ull * nres + lw_bytes + 4ull * (nhdr + 1) + 4ull * (nres + 1) + 64;
    uint8_t* ws = nullptr;
    hipError_t e = work_alloc((void**)&ws, ws_bytes, stream);
    if (e != hipSuccess) return e;
    HpeArgs A{in, in_size, hdr, nhdr, res, conn_first, nconn, nres, server_off, server_len, out, out_off, out_len,
              headers_size, rstatus, scratch, flags, nullptr, nullptr, nullptr, nullptr, nullptr, LongWork{}};
    uint8_t* p = ws;
    A.rec = reinterpret_cast<uint4*>(p);
    p += 16ull * (nhdr + 1);
    A.op = reinterpret_cast<uint4*>(p);
    p += 16ull * nhdr;
    A.plan = reinterpret_cast<uint4*>(p);
    p += 32ull * nres;
    A.lw = long_ws(p, nhdr, nres);
    p += lw_bytes;
    A.info = reinterpret_cast<uint32_t*>(p);
    p += 4ull * (nhdr + 1);
    A.big = reinterpret_cast<uint32_t*>(p);
    e = hipMemsetAsync(A.big, 0, 4, stream);
    if (e == hipSuccess) e = hipMemsetAsync(A.lw.bits, 0, 4, stream);
    if (e == hipSuccess) e = hipMemsetAsync(A.lw.njobs, 0, 4, stream);
    const uint32_t gp = (uint32_t)std::min<uint64_t>((nhdr + 256ull) / 256u, 8192ull);
    if (e == hipSuccess) {
        hipLaunchKernelGGL(hpe_prep_kernel, dim3(gp), dim3(256), 0, stream, A);
        e = hipGetLastError();
    }
    if (e == hipSuccess) {
        hipLaunchKernelGGL(long_bits_kernel<true>, dim3(256), dim3(256), 0, stream, in, hdr, nhdr, server_off, server_len,
                           A.rec, A.lw);
        e = hipGetLastError();
    }
    if (e == hipSuccess) {
        hipLaunchKernelGGL(hpe_table_kernel, dim3((nconn + 63u) / 64u), dim3(64), 0, stream, A);
        e = hipGetLastError();
    }
    if (e == hipSuccess && (uint64_t)nhdr + nres != 0) {
        const uint32_t ge = (uint32_t)std::min<uint64_t>(((uint64_t)nhdr + nres + 255u) / 256u, 16384ull);
        hipLaunchKernelGGL(hpe_emit_kernel, dim3(ge), dim3(256), 0, stream, A);
        e = hipGetLastError();
    }
    if (e == hipSuccess) {
        hipLaunchKernelGGL(long_payload_kernel, dim3(512), dim3(256), 0, stream, in, A.lw);
        e = hipGetLastError();
    }
    if (e == hipSuccess && nres != 0) {
        hipLaunchKernelGGL(hpe_frames_kernel, dim3(std::min(nres, 512u)), dim3(256), 0, stream, A);
        e = hipGetLastError();
    }
    if (e == hipSuccess) {
        hipLaunchKernelGGL(hpe_ring_kernel, dim3((nconn + 3u) / 4u), dim3(256), 0, stream, A);
        e = hipGetLastError();
    }
    const hipError_t f = hipFreeAsync(ws, stream);
    return e != hipSuccess ? e : f;
}

hipError_t launch_qpack_flatten(const uint8_t* in, uint64_t in_size, const hhuff_hpack_header_t* hdr, uint32_t nhdr,
                                const hhuff_qpack_response_t* res, uint32_t nres, uint32_t server_off, uint32_t server_len,
                                uint8_t* out, const uint64_t* out_off, uint32_t* out_len, uint32_t* header_len,
                                int32_t* rstatus, hipStream_t stream) {
    if (nres == 0) return hipSuccess;
    const uint64_t lw_bytes = long_ws_bytes(nhdr, nres);
    const uint64_t ws_bytes = 16ull * (nhdr + 1) + 32ull * nres + lw_bytes + 8ull * nhdr + 64;
    uint8_t* ws = nullptr;
    hipError_t e = work_alloc((void**)&ws, ws_bytes, stream);
    if (e != hipSuccess) return e;
    QpeArgs A{in, in_size, hdr, nhdr, res, nres, server_off, server_len, out, out_off, out_len, header_len, rstatus,
              nullptr, nullptr, nullptr, LongWork{}};
    uint8_t* p = ws;
    A.rec = reinterpret_cast<uint4*>(p);
    p += 16ull * (nhdr + 1);
    A.plan = reinterpret_cast<uint4*>(p);
    p += 32ull * nres;
    A.lw = long_ws(p, nhdr, nres);
    p += lw_bytes;
    A.dst = reinterpret_cast<uint2*>(p);
    e = hipMemsetAsync(A.lw.bits, 0, 4, stream);
    if (e == hipSuccess) e = hipMemsetAsync(A.lw.njobs, 0, 4, stream);
    const uint32_t gs = (uint32_t)std::min<uint64_t>((nhdr + 256ull) / 256u, 16384ull);
    if (e == hipSuccess) {
        hipLaunchKernelGGL(qpe_size_kernel, dim3(gs), dim3(256), 0, stream, A);
        e = hipGetLastError();
    }
    if (e == hipSuccess) {
        hipLaunchKernelGGL(long_bits_kernel<false>, dim3(256), dim3(256), 0, stream, in, hdr, nhdr, server_off, server_len,
                           A.rec, A.lw);
        e = hipGetLastError();
    }
    if (e == hipSuccess) {
        hipLaunchKernelGGL(qpe_layout_kernel, dim3((uint32_t)std::min<uint64_t>((nres + 255ull) / 256u, 16384ull)), dim3(256), 0,
                           stream, A);
        e = hipGetLastError();
    }
    if (e == hipSuccess) {
        const uint32_t ge = (uint32_t)std::min<uint64_t>(((uint64_t)nhdr + nres + 255u) / 256u, 16384ull);
        hipLaunchKernelGGL(qpe_emit_kernel, dim3(ge), dim3(256), 0, stream, A);
        e = hipGetLastError();
    }
    if (e == hipSuccess) {
        hipLaunchKernelGGL(long_payload_kernel, dim3(512), dim3(256), 0, stream, in, A.lw);
        e = hipGetLastError();
    }
    const hipError_t f = hipFreeAsync(ws, stream);
    return e != hipSuccess ? e : f;
}
}  // namespace hhuff
