// hhuff HIP kernels for gfx950 (MI355X) and their launchers.
//
// Work decomposition (both directions): one lane per string, 64 consecutive strings per wave
// ("tile"), waves grid-stride over the batch.  Staged variant: a wave copies its tile's input span
// into LDS with 16-byte coalesced loads (1 KiB per wave instruction), every lane decodes / encodes its
// string from LDS into an LDS output stage, then the wave writes the tile's output back:
//   * implicit contiguous layout (out_off == NULL, in_len == NULL): the tile's output regions tile one
//     contiguous range of `out`, written with coalesced 16-byte stores (byte-exact at the two edges);
//   * explicit destinations / (offset, length) pairs: each lane copies its own string (dword stores,
//     LDS position congruent to the destination mod 4).
// Tiles whose span exceeds the stage, and batches of long strings, use the direct variant: lanes read
// their input from global memory and write through a register accumulator with dword stores.
// The decode LUT (32 KiB) + leading-ones tables / encode table (4 KiB) live in LDS per workgroup.
//
// Reference semantics: lib/http2/hpack.c:117-156 (decode), :774-804 (encode); see hhuff_device.h.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "hhuff_device.h"
#include "hhuff_launch.h"

namespace hhuff {

__device__ const uint32_t g_dec_lut[1u << HHUFF_LUT_BITS] = HHUFF_DEC_LUT_INIT;
__device__ const uint32_t g_kinfo[31] = HHUFF_ONES_KINFO_INIT;
__device__ const uint32_t g_ones[HHUFF_ONES_NENT] = HHUFF_ONES_ENT_INIT;
__device__ const uint32_t g_enc_code[256] = HHUFF_ENC_CODE_INIT;
__device__ const uint8_t g_enc_nbits[256] = HHUFF_ENC_NBITS_INIT;

// ------------------------------------------------------------------------------------------------
// tile helpers
// ------------------------------------------------------------------------------------------------
struct Tile {
    uint32_t i;       // this lane's string
    bool valid;       // i < n
    uint32_t s, len;  // input offset and length
    uint32_t lo, hi;  // input span of the tile's non-empty strings
};

__device__ __forceinline__ Tile load_tile(uint64_t base, int lane, uint32_t n, const uint32_t* __restrict__ in_off,
                                          const uint32_t* __restrict__ in_len) {
    Tile t;
    t.i = (uint32_t)base + lane;
    t.valid = t.i < n;
    t.s = 0;
    t.len = 0;
    if (t.valid) {
        t.s = in_off[t.i];
        t.len = in_len ? in_len[t.i] : in_off[t.i + 1] - t.s;
    }
    const bool has = t.valid && t.len != 0;
    t.lo = wave_min_u32(has ? t.s : 0xFFFFFFFFu);
    t.hi = wave_max_u32(has ? t.s + t.len : 0u);
    return t;
}

// Stage [a0, a0 + span) of `in` into LDS (16-byte loads; bytes past in_size read as 0).
__device__ __forceinline__ void stage_span(uint32_t* stage, const uint8_t* __restrict__ in, uint64_t in_size, uint32_t a0,
                                           uint32_t span, int lane) {
    for (uint32_t k = (uint32_t)lane * 16u; k < span; k += 64u * 16u) {
        const uint64_t g = (uint64_t)a0 + k;
        uint4 v;
        if (g + 16 <= in_size) {
            v = *reinterpret_cast<const uint4*>(in + g);
        } else {
            uint32_t w[4] = {0, 0, 0, 0};
            for (uint32_t b = 0; b < 16; ++b)
                if (g + b < in_size) w[b >> 2] |= (uint32_t)in[g + b] << (8 * (b & 3));
            v = make_uint4(w[0], w[1], w[2], w[3]);
        }
        *reinterpret_cast<uint4*>(reinterpret_cast<uint8_t*>(stage) + k) = v;
    }
}

// Write LDS bytes [0, ospan) to global [gbase, gbase + ospan) (gbase 16-aligned), keeping only the
// global bytes in [keep_lo, keep_hi); 16-byte stores for whole chunks, byte stores at the edges.
__device__ __forceinline__ void region_copy(uint8_t* __restrict__ out, uint64_t gbase, const uint8_t* lds, uint32_t ospan,
                                            uint64_t keep_lo, uint64_t keep_hi, int lane) {
    for (uint32_t k = (uint32_t)lane * 16u; k < ospan; k += 64u * 16u) {
        const uint64_t g = gbase + k;
        if (g >= keep_lo && g + 16 <= keep_hi) {
            *reinterpret_cast<uint4*>(out + g) = *reinterpret_cast<const uint4*>(lds + k);
        } else {
            for (uint32_t b = 0; b < 16; ++b)
                if (g + b >= keep_lo && g + b < keep_hi) out[g + b] = lds[k + b];
        }
    }
}

// Copy `n` bytes from LDS `src` to global `dst`, where src == dst (mod 4).
__device__ __forceinline__ void lane_copy(uint8_t* __restrict__ dst, const uint8_t* src, uint32_t n) {
    uint32_t head = (4u - ((uint32_t)(uintptr_t)dst & 3u)) & 3u;
    head = min(head, n);
    for (uint32_t j = 0; j < head; ++j) dst[j] = src[j];
    dst += head;
    src += head;
    n -= head;
    const uint32_t nw = n >> 2;
    for (uint32_t j = 0; j < nw; ++j)
        reinterpret_cast<uint32_t*>(dst)[j] = reinterpret_cast<const uint32_t*>(src)[j];
    dst += 4 * nw;
    src += 4 * nw;
    for (uint32_t j = 0; j < (n & 3u); ++j) dst[j] = src[j];
}

// RegSink that also remembers the first and last byte (direct decode path).
struct RegSinkFL : RegSink {
    uint32_t first, last;
    __device__ __forceinline__ void put1(uint32_t b) {
        first = cnt == 0 ? (b & 0xFFu) : first;
        last = b & 0xFFu;
        RegSink::put1(b);
    }
    __device__ __forceinline__ void put12(uint32_t syms, bool two) {
        first = cnt == 0 ? (syms & 0xFFu) : first;
        last = (two ? (syms >> 8) : syms) & 0xFFu;
        RegSink::put12(syms, two);
    }
};

// ------------------------------------------------------------------------------------------------
// decode
// ------------------------------------------------------------------------------------------------
struct DecArgs {
    const uint8_t* in;
    uint64_t in_size;
    const uint32_t* in_off;
    const uint32_t* in_len;
    uint32_t n;
    const uint32_t* is_name_bits;
    uint8_t* out;
    const uint32_t* out_off;
    uint32_t* out_len;
    uint8_t* status;
};

__device__ __forceinline__ void load_dec_tables(uint32_t* s_lut, uint32_t* s_kinfo, uint32_t* s_ones, int nthreads) {
    for (uint32_t k = threadIdx.x; k < (1u << HHUFF_LUT_BITS) / 4; k += nthreads)
        reinterpret_cast<uint4*>(s_lut)[k] = reinterpret_cast<const uint4*>(g_dec_lut)[k];
    for (uint32_t k = threadIdx.x; k < HHUFF_ONES_NENT; k += nthreads) s_ones[k] = g_ones[k];
    if (threadIdx.x < 31) s_kinfo[threadIdx.x] = g_kinfo[threadIdx.x];
}

// direct variant for one lane: global input, register sink straight to `dst`
__device__ __forceinline__ void decode_direct(const DecArgs& A, uint32_t s, uint32_t len, bool is_name, uint8_t* dst,
                                              const DecTables& T, uint32_t& ol, uint8_t& st) {
    if (len > kMaxStrLen) {
        ol = kFailLen;
        st = kStatusTooLong;
        return;
    }
    RegSinkFL sink;
    sink.init(dst);
    sink.first = sink.last = 0;
    DecResult r = decode_core(GlobalSource{A.in, A.in_size}, s, len, sink, T);
    if (r.ok) {
        sink.finish();
        ol = r.len;
        st = soft_bits(is_name, r.len, r.flags, sink.first, sink.last);
    } else {
        ol = kFailLen;
        st = kStatusFail;
    }
}

template <int WAVES, int IN_STAGE, int OUT_STAGE>
__global__ __launch_bounds__(WAVES * 64) void decode_staged_kernel(DecArgs A) {
    __shared__ __attribute__((aligned(16))) uint32_t s_lut[1u << HHUFF_LUT_BITS];
    __shared__ uint32_t s_kinfo[32];
    __shared__ uint32_t s_ones[HHUFF_ONES_NENT];
    __shared__ __attribute__((aligned(16))) uint32_t s_in[WAVES][IN_STAGE / 4];
    __shared__ __attribute__((aligned(16))) uint8_t s_out[WAVES][OUT_STAGE + 256];  // + a trash dword per lane
    load_dec_tables(s_lut, s_kinfo, s_ones, WAVES * 64);
    __syncthreads();
    const DecTables T{s_lut, s_kinfo, s_ones};
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint32_t* stage = s_in[wave];
    uint8_t* obuf = s_out[wave];
    const bool region = A.in_len == nullptr && A.out_off == nullptr;
    const uint64_t stride = (uint64_t)gridDim.x * WAVES * 64;
    for (uint64_t base = ((uint64_t)blockIdx.x * WAVES + wave) * 64; base < A.n; base += stride) {
        const Tile t = load_tile(base, lane, A.n, A.in_off, A.in_len);
        const bool is_name = t.valid && A.is_name_bits ? ((A.is_name_bits[t.i >> 5] >> (t.i & 31)) & 1u) : false;
        const uint32_t a0 = t.lo & ~15u;
        const uint32_t span = t.hi > t.lo ? ((t.hi + 15u) & ~15u) - a0 : 0u;
        // output stage layout
        uint64_t dst_g = 0, obase = 0, olo = 0, ohi = 0;
        uint32_t op0, ospan;
        if (region) {
            olo = dec_slot(t.lo);
            ohi = dec_slot(t.hi);
            obase = olo & ~15ull;
            ospan = t.hi > t.lo ? (uint32_t)(ohi - obase) : 0u;
            op0 = t.len ? (uint32_t)(dec_slot(t.s) - obase) : 0u;
        } else {
            dst_g = A.out_off ? (uint64_t)(t.valid ? A.out_off[t.i] : 0u) : dec_slot(t.s);
            const uint32_t cap = t.valid ? (uint32_t)(((uint64_t)min(t.len, kMaxStrLen) * 8u) / 5u) + 3u : 0u;
            const uint32_t pre = wave_excl_scan(cap, lane);
            ospan = __shfl(pre + cap, 63, 64);
            op0 = pre + ((uint32_t)(((uintptr_t)A.out + dst_g) - pre) & 3u);
        }
        uint32_t ol = 0;
        uint8_t st = 0;
        if (span <= IN_STAGE && ospan <= OUT_STAGE) {
            stage_span(stage, A.in, A.in_size, a0, span, lane);
            wave_lds_sync();
            {
                const bool act = t.valid && t.len <= kMaxStrLen;
                const uint32_t rel = t.len ? t.s - a0 : 0u;
                const uint32_t last = span ? span - 4u : 0u;
                const DecResult r =
                    decode_staged_lane(stage, last, rel, t.len, act, obuf, op0, OUT_STAGE + 4u * (uint32_t)lane, T);
                if (t.valid && t.len > kMaxStrLen) {
                    ol = kFailLen;
                    st = kStatusTooLong;
                } else if (r.ok) {
                    ol = r.len;
                    const uint32_t first = r.len ? obuf[op0] : 0u, lastc = r.len ? obuf[op0 + r.len - 1] : 0u;
                    st = soft_bits(is_name, r.len, r.flags, first, lastc);
                } else {
                    ol = kFailLen;
                    st = kStatusFail;
                }
            }
            wave_lds_sync();
            if (region) {
                region_copy(A.out, obase, obuf, ospan, olo, ohi, lane);
            } else if (t.valid && ol != kFailLen) {
                lane_copy(A.out + dst_g, obuf + op0, ol);
            }
            wave_lds_sync();
        } else if (t.valid) {
            const uint64_t d = A.out_off ? (uint64_t)A.out_off[t.i] : dec_slot(t.s);
            decode_direct(A, t.s, t.len, is_name, A.out + d, T, ol, st);
        }
        if (t.valid) {
            A.out_len[t.i] = ol;
            A.status[t.i] = st;
        }
    }
}

template <int WAVES>
__global__ __launch_bounds__(WAVES * 64) void decode_direct_kernel(DecArgs A) {
    __shared__ __attribute__((aligned(16))) uint32_t s_lut[1u << HHUFF_LUT_BITS];
    __shared__ uint32_t s_kinfo[32];
    __shared__ uint32_t s_ones[HHUFF_ONES_NENT];
    load_dec_tables(s_lut, s_kinfo, s_ones, WAVES * 64);
    __syncthreads();
    const DecTables T{s_lut, s_kinfo, s_ones};
    const uint64_t stride = (uint64_t)gridDim.x * WAVES * 64;
    for (uint64_t i = (uint64_t)blockIdx.x * WAVES * 64 + threadIdx.x; i < A.n; i += stride) {
        const uint32_t s = A.in_off[i];
        const uint32_t len = A.in_len ? A.in_len[i] : A.in_off[i + 1] - s;
        const bool is_name = A.is_name_bits ? ((A.is_name_bits[i >> 5] >> (i & 31)) & 1u) : false;
        const uint64_t d = A.out_off ? (uint64_t)A.out_off[i] : dec_slot(s);
        uint32_t ol;
        uint8_t st;
        decode_direct(A, s, len, is_name, A.out + d, T, ol, st);
        A.out_len[i] = ol;
        A.status[i] = st;
    }
}

// ------------------------------------------------------------------------------------------------
// encode
// ------------------------------------------------------------------------------------------------
struct EncArgs {
    const uint8_t* in;
    uint64_t in_size;
    const uint32_t* in_off;
    const uint32_t* in_len;
    uint32_t n;
    uint8_t* out;
    const uint32_t* out_off;
    uint32_t* out_len;
    uint8_t* status;
};

__device__ __forceinline__ void load_enc_table(uint2* s_enc, int nthreads) {
    for (uint32_t k = threadIdx.x; k < 256; k += nthreads) s_enc[k] = make_uint2(g_enc_code[k], g_enc_nbits[k]);
}

__device__ __forceinline__ void finish_encode(const EncArgs& A, uint32_t i, uint32_t len, uint32_t ol) {
    A.out_len[i] = ol;
    if (A.status) A.status[i] = ol == kFailLen ? (len > kMaxStrLen ? kStatusTooLong : kStatusFail) : 0;
}

template <int WAVES, int STAGE>
__global__ __launch_bounds__(WAVES * 64) void encode_staged_kernel(EncArgs A) {
    __shared__ __attribute__((aligned(16))) uint2 s_enc[512];  // 256..511: bytes outside a string
    __shared__ __attribute__((aligned(16))) uint32_t s_in[WAVES][STAGE / 4];
    __shared__ __attribute__((aligned(16))) uint32_t s_out[WAVES][STAGE / 4 + 4];
    for (uint32_t k = threadIdx.x; k < 512; k += WAVES * 64)
        s_enc[k] = k < 256 ? make_uint2(g_enc_code[k], g_enc_nbits[k]) : make_uint2(0u, 0u);
    __syncthreads();
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint32_t* stage = s_in[wave];
    uint32_t* obuf32 = s_out[wave];
    const uint8_t* obuf = reinterpret_cast<const uint8_t*>(obuf32);
    const bool region = A.in_len == nullptr && A.out_off == nullptr;
    const uint64_t stride = (uint64_t)gridDim.x * WAVES * 64;
    for (uint64_t base = ((uint64_t)blockIdx.x * WAVES + wave) * 64; base < A.n; base += stride) {
        const Tile t = load_tile(base, lane, A.n, A.in_off, A.in_len);
        const uint32_t a0 = t.lo & ~15u;
        const uint32_t span = t.hi > t.lo ? ((t.hi + 15u) & ~15u) - a0 : 0u;
        uint64_t dst_g = 0;
        uint32_t op0, ospan;
        if (region) {  // output slot = input offset: the output stage mirrors the input stage
            ospan = span;
            op0 = t.len ? t.s - a0 : 0u;
        } else {
            dst_g = A.out_off ? (uint64_t)(t.valid ? A.out_off[t.i] : 0u) : (uint64_t)t.s;
            const uint32_t cap = t.valid ? min(t.len, kMaxStrLen) + 3u : 0u;
            const uint32_t pre = wave_excl_scan(cap, lane);
            ospan = __shfl(pre + cap, 63, 64);
            op0 = pre + ((uint32_t)(((uintptr_t)A.out + dst_g) - pre) & 3u);
        }
        uint32_t ol = kFailLen;
        if (span <= STAGE && ospan <= STAGE) {
            stage_span(stage, A.in, A.in_size, a0, span, lane);
            for (uint32_t k = (uint32_t)lane * 16u; k < ospan + 16u; k += 64u * 16u)
                *reinterpret_cast<uint4*>(reinterpret_cast<uint8_t*>(obuf32) + k) = make_uint4(0u, 0u, 0u, 0u);
            wave_lds_sync();
            const bool act = t.valid && t.len != 0 && t.len <= kMaxStrLen;
            const uint32_t r = encode_staged_lane(stage, span ? span - 4u : 0u, t.len ? t.s - a0 : 0u, t.len, act, obuf32,
                                                  op0, s_enc);
            if (act) ol = r;
            wave_lds_sync();
            if (region) {
                region_copy(A.out, a0, obuf, ospan, t.lo, t.hi, lane);
            } else if (t.valid && ol != kFailLen) {
                lane_copy(A.out + dst_g, obuf + op0, ol);
            }
            wave_lds_sync();
        } else if (t.valid && t.len <= kMaxStrLen) {
            RegSink sink;
            sink.init(A.out + (A.out_off ? (uint64_t)A.out_off[t.i] : (uint64_t)t.s));
            ol = encode_core(GlobalSource{A.in, A.in_size}, t.s, t.len, sink, s_enc);
        }
        if (t.valid) finish_encode(A, t.i, t.len, ol);
    }
}

template <int WAVES>
__global__ __launch_bounds__(WAVES * 64) void encode_direct_kernel(EncArgs A) {
    __shared__ __attribute__((aligned(16))) uint2 s_enc[256];
    load_enc_table(s_enc, WAVES * 64);
    __syncthreads();
    const uint64_t stride = (uint64_t)gridDim.x * WAVES * 64;
    for (uint64_t i = (uint64_t)blockIdx.x * WAVES * 64 + threadIdx.x; i < A.n; i += stride) {
        const uint32_t s = A.in_off[i];
        const uint32_t len = A.in_len ? A.in_len[i] : A.in_off[i + 1] - s;
        uint32_t ol = kFailLen;
        if (len <= kMaxStrLen) {
            RegSink sink;
            sink.init(A.out + (A.out_off ? (uint64_t)A.out_off[i] : (uint64_t)s));
            ol = encode_core(GlobalSource{A.in, A.in_size}, s, len, sink, s_enc);
        }
        finish_encode(A, (uint32_t)i, len, ol);
    }
}

// ------------------------------------------------------------------------------------------------
// string-literal framing: HPACK h2o_hpack_encode_string (hpack.c:816-837) and QPACK flatten_string
// (qpack.c:1042-1066), batched.  Per string: Huffman iff not flagged raw and strictly shorter
// (hpack.c:818-821, qpack.c:1046), then [first byte with the H bit | prefix integer][payload].
// One lane per string, direct global path: a bit-count pass fixes the header length, then the payload
// is written behind it through the register sink (any destination alignment).
// ------------------------------------------------------------------------------------------------
struct FlatArgs {
    const uint8_t* in;
    uint64_t in_size;
    const uint32_t* in_off;
    const uint32_t* in_len;
    uint32_t n;
    const uint8_t* first_bytes;
    uint32_t prefix_bits;
    const uint32_t* raw_bits;
    uint8_t* out;
    const uint32_t* out_off;
    uint32_t* out_len;
};

// RFC 7541 5.1 prefix integer (hpack.c:757-772) OR-ed into first byte h0: up to 6 bytes for v < 2^32
__device__ __forceinline__ void push_prefix_int(RegSink& sink, uint32_t h0, uint32_t v, uint32_t p) {
    const uint32_t pmax = (1u << p) - 1u;
    uint64_t hb;
    uint32_t hn = 1;
    if (v < pmax) {
        hb = h0 | v;
    } else {
        hb = h0 | pmax;
        v -= pmax;
        while (v >= 128) {
            hb |= (uint64_t)(0x80u | (v & 127u)) << (8 * hn);
            ++hn;
            v >>= 7;
        }
        hb |= (uint64_t)v << (8 * hn);
        ++hn;
    }
    sink.push((uint32_t)hb, min(hn, 4u));
    if (hn > 4) sink.push((uint32_t)(hb >> 32), hn - 4);
}

__device__ __forceinline__ uint32_t count_code_bits(const GlobalSource& src, uint32_t start, uint32_t len,
                                                    const uint2* __restrict__ enc) {
    uint32_t bits = 0;
    const uint32_t end = start + len;
    for (uint32_t a = start & ~3u; a < end; a += 4) {
        const uint32_t w = src.word(a);
#pragma unroll
        for (uint32_t k = 0; k < 4; ++k) {
            const uint32_t pos = a + k;
            bits += (pos >= start && pos < end) ? enc[(w >> (8 * k)) & 0xFFu].y : 0u;
        }
    }
    return bits;
}

template <int WAVES>
__global__ __launch_bounds__(WAVES * 64) void flatten_direct_kernel(FlatArgs A) {
    __shared__ __attribute__((aligned(16))) uint2 s_enc[256];
    load_enc_table(s_enc, WAVES * 64);
    __syncthreads();
    const uint32_t p = A.prefix_bits;
    const GlobalSource src{A.in, A.in_size};
    const uint64_t stride = (uint64_t)gridDim.x * WAVES * 64;
    for (uint64_t i = (uint64_t)blockIdx.x * WAVES * 64 + threadIdx.x; i < A.n; i += stride) {
        const uint32_t s = A.in_off[i];
        const uint32_t len = A.in_len ? A.in_len[i] : A.in_off[i + 1] - s;
        const uint32_t first = A.first_bytes ? A.first_bytes[i] : 0u;
        const bool raw = A.raw_bits ? ((A.raw_bits[i >> 5] >> (i & 31)) & 1u) : false;
        RegSink sink;
        sink.init(A.out + (A.out_off ? (uint64_t)A.out_off[i] : (uint64_t)s + 11u * i));
        if (len > kMaxStrLen) {
            A.out_len[i] = kFailLen;
            continue;
        }
        const uint32_t bits = (raw || len == 0) ? 0u : count_code_bits(src, s, len, s_enc);
        const bool huff = !raw && len != 0 && bits <= 8 * len - 8;  // ceil(bits / 8) < len (hpack.c:799-800)
        if (huff) {
            push_prefix_int(sink, (first & ~((1u << p) - 1u)) | (1u << p), (bits + 7) >> 3, p);  // qpack.c:1054-1056
            encode_core(src, s, len, sink, s_enc);
        } else {
            push_prefix_int(sink, first & ~((2u << p) - 1u), len, p);  // qpack.c:1048-1049 (hpack.c:806-814)
            uint32_t a = s & ~3u, rem = len;
            uint32_t skip = s & 3u;
            while (rem) {
                const uint32_t w = src.word(a) >> (8 * skip);
                const uint32_t k = min(4u - skip, rem);
                sink.push(w, k);
                rem -= k;
                a += 4;
                skip = 0;
            }
            sink.finish();
        }
        A.out_len[i] = sink.count();
    }
}

// ------------------------------------------------------------------------------------------------
// launch configuration (LDS per workgroup in brackets)
//   decode staged:        16 waves/WG, 3 KiB in + 4.5 KiB out per wave   [~158 KiB, 1 WG/CU]
//   decode staged (long):  6 waves/WG, 8 KiB in + 12.9 KiB out per wave [~144 KiB, 1 WG/CU]
//   decode direct:         4 waves/WG, tables only                        [~17.5 KiB]
//   encode staged:        16 waves/WG, 3.5 KiB in + out per wave          [~114 KiB, 1 WG/CU]
//   encode staged (long):  8 waves/WG, 8 KiB in + out per wave            [~130 KiB, 1 WG/CU]
//   encode direct:         4 waves/WG                                      [2 KiB]
// The variant is picked from the mean bytes per string (in_size / n).
// ------------------------------------------------------------------------------------------------
#define DEC_S decode_staged_kernel<16, 3072, 4608>
#define DEC_L decode_staged_kernel<6, 8192, 12928>
#define DEC_D decode_direct_kernel<4>
#define ENC_S encode_staged_kernel<16, 3584>
#define ENC_L encode_staged_kernel<8, 8192>
#define ENC_D encode_direct_kernel<4>
#define FLAT_D flatten_direct_kernel<4>

enum Variant { kDecS, kDecL, kDecD, kEncS, kEncL, kEncD, kFlatD, kNumVariants };

static const void* variant_fn(int v) {
    switch (v) {
        case kDecS: return (const void*)DEC_S;
        case kDecL: return (const void*)DEC_L;
        case kDecD: return (const void*)DEC_D;
        case kEncS: return (const void*)ENC_S;
        case kEncL: return (const void*)ENC_L;
        case kFlatD: return (const void*)FLAT_D;
        default: return (const void*)ENC_D;
    }
}
static int variant_threads(int v) {
    switch (v) {
        case kDecS:
        case kEncS: return 1024;
        case kDecL: return 384;
        case kEncL: return 512;
        default: return 256;
    }
}

static int grid_for(int v, int device, uint32_t n) {
    static int cache[64][kNumVariants] = {};
    if (device < 0 || device >= 64) device = 0;
    if (cache[device][v] == 0) {
        int per_cu = 0, cus = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, variant_fn(v), variant_threads(v), 0) != hipSuccess ||
            per_cu < 1)
            per_cu = 1;
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess || cus < 1) cus = 256;
        cache[device][v] = per_cu * cus;
    }
    const uint64_t per_block = (uint64_t)variant_threads(v);
    const uint64_t blocks = ((uint64_t)n + per_block - 1) / per_block;
    const int g = cache[device][v];
    return (int)(blocks < (uint64_t)g ? (blocks ? blocks : 1) : g);
}

static int current_device() {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) dev = 0;
    return dev;
}

static int pick_decode(uint64_t in_size, uint32_t n) {
    const uint64_t mean = n ? in_size / n : 0;  // in_size bounds the bytes the batch can address
    if (mean <= 40) return kDecS;
    if (mean <= 128) return kDecL;
    return kDecD;
}
static int pick_encode(uint64_t in_size, uint32_t n) {
    const uint64_t mean = n ? in_size / n : 0;
    if (mean <= 52) return kEncS;
    if (mean <= 120) return kEncL;
    return kEncD;
}

hipError_t launch_decode(const uint8_t* in, uint64_t in_size, const uint32_t* in_off, const uint32_t* in_len, uint32_t n,
                         const uint32_t* is_name_bits, uint8_t* out, const uint32_t* out_off, uint32_t* out_len,
                         uint8_t* status, hipStream_t stream) {
    if (n == 0) return hipSuccess;
    DecArgs A{in, in_size, in_off, in_len, n, is_name_bits, out, out_off, out_len, status};
    const int v = pick_decode(in_size, n);
    const int grid = grid_for(v, current_device(), n);
    switch (v) {
        case kDecS: hipLaunchKernelGGL(DEC_S, dim3(grid), dim3(1024), 0, stream, A); break;
        case kDecL: hipLaunchKernelGGL(DEC_L, dim3(grid), dim3(384), 0, stream, A); break;
        default: hipLaunchKernelGGL(DEC_D, dim3(grid), dim3(256), 0, stream, A); break;
    }
    return hipGetLastError();
}

hipError_t launch_encode(const uint8_t* in, uint64_t in_size, const uint32_t* in_off, const uint32_t* in_len, uint32_t n,
                         uint8_t* out, const uint32_t* out_off, uint32_t* out_len, uint8_t* status, hipStream_t stream) {
    if (n == 0) return hipSuccess;
    EncArgs A{in, in_size, in_off, in_len, n, out, out_off, out_len, status};
    const int v = pick_encode(in_size, n);
    const int grid = grid_for(v, current_device(), n);
    switch (v) {
        case kEncS: hipLaunchKernelGGL(ENC_S, dim3(grid), dim3(1024), 0, stream, A); break;
        case kEncL: hipLaunchKernelGGL(ENC_L, dim3(grid), dim3(512), 0, stream, A); break;
        default: hipLaunchKernelGGL(ENC_D, dim3(grid), dim3(256), 0, stream, A); break;
    }
    return hipGetLastError();
}

hipError_t launch_flatten(const uint8_t* in, uint64_t in_size, const uint32_t* in_off, const uint32_t* in_len, uint32_t n,
                          const uint8_t* first_bytes, uint32_t prefix_bits, const uint32_t* raw_bits, uint8_t* out,
                          const uint32_t* out_off, uint32_t* out_len, hipStream_t stream) {
    if (n == 0) return hipSuccess;
    FlatArgs A{in, in_size, in_off, in_len, n, first_bytes, prefix_bits, raw_bits, out, out_off, out_len};
    const int grid = grid_for(kFlatD, current_device(), n);
    hipLaunchKernelGGL(FLAT_D, dim3(grid), dim3(256), 0, stream, A);
    return hipGetLastError();
}

int grid_size(int device, int which) { return grid_for(which == 0 ? kDecS : kEncS, device, 0xFFFFFFFFu); }

}  // namespace hhuff
