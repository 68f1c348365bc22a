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
#include <stdlib.h>
#include <algorithm>
#include <atomic>
#include <mutex>
#include <type_traits>
#include <vector>

#include "hhuff_device.h"
#include "hhuff_launch.h"

namespace hhuff {

// A/B builds only (tools/ab.py build NAME -DHHUFF_AB_VARIANTS=1 ..., include path tools/ab): the variant kernels
// measured and not adopted live in tools/ab/, out of libhhuff.so.  A flag that selects one implies the switch.
#if !defined(HHUFF_AB_VARIANTS)
#if defined(HHUFF_STREAM_RK) || defined(HHUFF_STREAM2) || (defined(HHUFF_ENC_INPLACE) && HHUFF_ENC_INPLACE) || \
    (defined(HHUFF_DEC_SW) && HHUFF_DEC_SW) || (defined(HHUFF_DEC_RUN) && HHUFF_DEC_RUN)
#define HHUFF_AB_VARIANTS 1
#else
#define HHUFF_AB_VARIANTS 0
#endif
#endif
__device__ const uint32_t g_dec_lut[1u << HHUFF_LUT_BITS] = HHUFF_DEC_LUT_INIT;
__device__ const uint32_t g_name_invalid[8] = HHUFF_NAME_INVALID_INIT;    // raw-literal validity bitmaps
__device__ const uint32_t g_value_invalid[8] = HHUFF_VALUE_INVALID_INIT;  // (hpack.c:171-180, 200-209)
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

// The 16 bytes at g when they cross in_size (bytes past it read as 0).  A rolled loop over the < 16 bytes
// that exist: unrolled, the 16 bounds checks were hoisted as 64-bit lane + b constants that held ~30
// VGPRs for the whole kernel (and spilled), for a path taken once per launch.
__device__ __forceinline__ uint4 load16_tail(const uint8_t* __restrict__ in, uint64_t in_size, uint64_t g) {
    const uint32_t rem = g < in_size ? (uint32_t)min(in_size - g, (uint64_t)16) : 0u;
    const uint8_t* p = in + g;
    uint64_t lo = 0, hi = 0;
#pragma unroll 1
    for (uint32_t b = 0; b < rem; ++b) {
        const uint64_t x = p[b];
        if (b < 8) lo |= x << (8u * b);
        else hi |= x << (8u * (b - 8u));
    }
    return make_uint4((uint32_t)lo, (uint32_t)(lo >> 32), (uint32_t)hi, (uint32_t)(hi >> 32));
}

constexpr int kVmWait0 = 0x0F70;  // s_waitcnt vmcnt(0) (expcnt, lgkmcnt untouched)

// Stage [a0, a0 + span) of `in` into a wave's LDS stage with LDS-DMA (global_load_lds_dwordx4: 16 B a lane to
// the wave-uniform base + 16 lane, no VGPRs), every 1-KiB chunk in flight at once, then one wait; the chunk
// holding the input's end goes through registers (bytes past in_size read as 0).  (A loop of load / wait /
// ds_write paid one memory latency per KiB; register staging of all chunks spilled in flatten_pl_kernel.)
template <int NCH>
__device__ __forceinline__ void stage_span_dma_issue(uint32_t* stage, const uint8_t* __restrict__ in, uint64_t in_size,
                                                     uint32_t a0, uint32_t span, int lane) {
    const uint64_t av = in_size > (uint64_t)a0 ? in_size - a0 : 0u;
    const uint32_t avail = av > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)av;
    const uint32_t sb = lds_addr(stage);
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
        const uint32_t k = (uint32_t)c * 1024u + (uint32_t)lane * 16u;
        if (k < span && k + 16u <= avail)
            __builtin_amdgcn_global_load_lds((const void*)(in + a0 + k), (lds_u8*)(size_t)(sb + (uint32_t)c * 1024u), 16, 0, 0);
    }
}
// waits for every memory operation in flight (the DMA with them), then the chunk at the input's end
template <int NCH>
__device__ __forceinline__ void stage_span_dma_finish(uint32_t* stage, const uint8_t* __restrict__ in, uint64_t in_size,
                                                      uint32_t a0, uint32_t span, int lane) {
    const uint64_t av = in_size > (uint64_t)a0 ? in_size - a0 : 0u;
    const uint32_t avail = av > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)av;
    __builtin_amdgcn_s_waitcnt(kVmWait0);
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
        const uint32_t k = (uint32_t)c * 1024u + (uint32_t)lane * 16u;
        if (k < span && k + 16u > avail)
            *reinterpret_cast<uint4*>(reinterpret_cast<uint8_t*>(stage) + k) = load16_tail(in, in_size, (uint64_t)a0 + k);
    }
}
template <int NCH>
__device__ __forceinline__ void stage_span_dma(uint32_t* stage, const uint8_t* __restrict__ in, uint64_t in_size,
                                               uint32_t a0, uint32_t span, int lane) {
    stage_span_dma_issue<NCH>(stage, in, in_size, a0, span, lane);
    stage_span_dma_finish<NCH>(stage, in, in_size, a0, span, lane);
}

// Software pipelining across tiles: the next tile's offsets (and is-name word / destination) and its
// input span are loaded into registers while the current tile is decoded or encoded from LDS, so the
// wave never sits on a global-memory round trip between tiles.  Nothing on the LDS path of a tile
// issues a global load, so no vmcnt wait there can be held up by the prefetch.

// Phase timing (profile builds only, -DHHUFF_PROFILE): shader cycles per phase summed over waves,
// read back with hhuff_debug_prof() (tools/ab.py prof).  s_memtime costs a little itself.
#ifdef HHUFF_PROFILE
__device__ unsigned long long g_prof[2][8];
#define PROF_DECL                                      \
    uint64_t prof_t = __builtin_readcyclecounter();    \
    uint64_t prof_a[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#define PROF_MARK(k)                                          \
    do {                                                      \
        const uint64_t prof_n = __builtin_readcyclecounter(); \
        prof_a[k] += prof_n - prof_t;                         \
        prof_t = prof_n;                                      \
    } while (0)
#define PROF_FLUSH(kern) \
    if (lane == 0)       \
        for (int prof_k = 0; prof_k < 8; ++prof_k) atomicAdd(&g_prof[kern][prof_k], (unsigned long long)prof_a[prof_k]);
#else
#define PROF_DECL
#define PROF_MARK(k) \
    do {             \
    } while (0)
#define PROF_FLUSH(kern)
#endif

struct TileIn {  // per-lane prefetched fields of one tile
    uint32_t s, len, name_word, dst;
};

// No VALU writes on purpose: the index is clamped (a lane past n loads string n - 1's fields, which
// finish_tile then ignores) and absent arrays read in_off instead, so every load issues unconditionally
// and its register is written by the load alone; consume_tile() then uses all four words where the
// tile is planned.  With the loads under `if (i < n)` and zero defaults, or with a loaded word left
// unused, the compiler copied (PHI), re-zeroed or reused those registers and put a vmcnt wait in front
// of each write -- a memory round trip per tile, behind the span loads just issued or the stores.
__device__ __forceinline__ TileIn issue_tile(uint64_t base, int lane, uint32_t n, const uint32_t* __restrict__ in_off,
                                             const uint32_t* __restrict__ in_len, const uint32_t* __restrict__ name_bits,
                                             const uint32_t* __restrict__ out_off) {
    const uint64_t i = min(base + (uint64_t)lane, (uint64_t)n - 1u);  // n >= 1 in every kernel
    TileIn r;
    r.s = in_off[i];
    r.len = in_len ? in_len[i] : in_off[i + 1];  // end offset for the contiguous layout (minus s later)
    r.name_word = name_bits ? name_bits[i >> 5] : in_off[i];
    r.dst = out_off ? out_off[i] : in_off[i];
    return r;
}
// the words of a prefetched tile are all waited for here, where its offsets are needed anyway
__device__ __forceinline__ void consume_tile(const TileIn& t) {
    __asm__ volatile("" : : "v"(t.s), "v"(t.len), "v"(t.name_word), "v"(t.dst));
}

__device__ __forceinline__ Tile finish_tile(uint64_t base, int lane, uint32_t n, const TileIn& in, bool pairs) {
    consume_tile(in);
    Tile t;
    t.i = (uint32_t)base + lane;
    t.valid = (uint64_t)base + lane < n;
    t.s = in.s;
    t.len = t.valid ? (pairs ? in.len : in.len - in.s) : 0u;
    if (!pairs) {
        // contiguous layout: the span runs from the first string's start to the last one's end (empty
        // strings add no bytes), two lane reads instead of two wave reductions
        const uint64_t last = min((uint64_t)n - 1u - base, (uint64_t)63);
        t.lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)in.s);
        t.hi = (uint32_t)__builtin_amdgcn_readlane((int)in.len, (int)last);
        if (t.hi == t.lo) t.lo = 0xFFFFFFFFu, t.hi = 0u;  // no bytes: as the reductions would report
        return t;
    }
    const bool has = t.valid && t.len != 0;
    t.lo = wave_min_u32(has ? t.s : 0xFFFFFFFFu);
    t.hi = wave_max_u32(has ? t.s + t.len : 0u);
    return t;
}

#ifndef HHUFF_NT_LOAD  // A/B: tile spans fetched with streaming (non-temporal) loads
#define HHUFF_NT_LOAD 0
#endif
template <int NCH>
struct SpanPrefetch {  // up to NCH x 1 KiB of a tile's input span, 16 B per lane per KiB
    uint4 v[NCH];
    __device__ __forceinline__ void issue(const uint8_t* __restrict__ in, uint64_t in_size, uint32_t a0, uint32_t span,
                                          int lane) {
        // bytes readable from a0 on, clamped to 32 bits (a0 <= in_size): every test below is 32-bit
        const uint64_t av = in_size > (uint64_t)a0 ? in_size - a0 : 0u;
        const uint32_t avail = av > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)av;
        const uint8_t* src = in + a0;
#pragma unroll
        for (int c = 0; c < NCH; ++c) {
            const uint32_t k = (uint32_t)c * 1024u + (uint32_t)lane * 16u;
#if HHUFF_NT_LOAD  // A/B: the span as streaming loads (read once)
            if (k < span && k + 16u <= avail) {
                typedef unsigned int u32x4l __attribute__((ext_vector_type(4)));
                const u32x4l x = __builtin_nontemporal_load(reinterpret_cast<const u32x4l*>(src + k));
                v[c] = make_uint4(x.x, x.y, x.z, x.w);
            }
#else
            if (k < span && k + 16u <= avail) v[c] = *reinterpret_cast<const uint4*>(src + k);
#endif
        }
    }
    template <bool kSwap = false>  // kSwap: store big-endian dwords (the v5 decode window reads them)
    __device__ __forceinline__ void commit(uint32_t* stage, const uint8_t* __restrict__ in, uint64_t in_size, uint32_t a0,
                                           uint32_t span, int lane) {
#pragma unroll
        for (int c = 0; c < NCH; ++c) {
            const uint32_t k = (uint32_t)c * 1024u + (uint32_t)lane * 16u;
            if (k < span) {
                const uint64_t g = (uint64_t)a0 + k;
                uint4 x = v[c];
                if (g + 16 > in_size) x = load16_tail(in, in_size, g);  // the chunk holding the input's end
                if (kSwap) x = make_uint4(bswap32(x.x), bswap32(x.y), bswap32(x.z), bswap32(x.w));
                *reinterpret_cast<uint4*>(reinterpret_cast<uint8_t*>(stage) + k) = x;
            }
        }
    }
};

// Deferred region edges.  Writing the (at most two) 16-byte chunks a tile's output region shares with
// its neighbours byte by byte costs a serial LDS round trip per byte; measured, it was 11 % of both c4
// kernels.  Instead the tile writes every whole chunk with 16-B stores, and the lanes holding its first
// and last chunk record them {bytes, address, byte range} in `rec` (2 per tile) straight from their
// registers; edge_fix_kernel writes the recorded byte ranges after the kernel (neighbouring tiles'
// ranges in one chunk are disjoint, so dword / byte stores suffice).
// decode_select_kernel's verdict: which of the two kernels launched behind it does the work
constexpr uint32_t kGateStaged = 0u, kGateStream = 1u;

// The staged/stream verdict from decode_select_kernel's partial sums; called by one whole wave.
// Prices: ps per string and per byte of each kernel (DecArgs::price) -- staged per tile-padded byte (64 x
// the tile's longest string), stream per byte.  Measured per device at its first mixed-length decode
// (decode_prices: both kernels timed on two fixed-length probe batches); one MI355X gave ~40 / 1.07 and
// ~184 / 1.15.
__device__ __forceinline__ uint32_t select_verdict(const uint64_t* __restrict__ part, const float (&price)[4]) {
    constexpr uint32_t kB = 64;  // kSelBlocks
    const uint32_t lane = threadIdx.x & 63;
    uint64_t pad = part[lane], sum = part[kB + lane], cnt = part[2 * kB + lane];
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        pad += (uint64_t)__shfl_xor((long long)pad, d);
        sum += (uint64_t)__shfl_xor((long long)sum, d);
        cnt += (uint64_t)__shfl_xor((long long)cnt, d);
    }
    const double staged = (double)price[0] * (double)cnt + (double)price[1] * (double)pad,
                 streamed = (double)price[2] * (double)cnt + (double)price[3] * (double)sum;
    return streamed < staged ? kGateStream : kGateStaged;
}

struct EdgeRec {
    uint4 v;
    uint4 m;  // {address lo, address hi, lo, hi}: bytes [lo, hi) of the chunk are ours (lo >= hi: none)
};

#ifndef HHUFF_NT_STORE  // output pieces as streaming (non-temporal) 16-B stores: c4 decode -2.1 %, encode -0.9 %,
                        // c2 -3 %, c3 / c5 level (profiles/r05t_nt_store_ab.jsonl; with the per-string lengths and
                        // statuses streamed too, HHUFF_NT_RES, c4 decode gains less)
#define HHUFF_NT_STORE 1
#endif
#ifndef HHUFF_STREAM_NT
#define HHUFF_STREAM_NT 0
#endif
#ifndef HHUFF_STATUS_DW  // staged decode: a tile's status bytes stored as dwords
#define HHUFF_STATUS_DW 0
#endif
// result stores the kernel never reads back: streaming (non-temporal) with HHUFF_NT_STORE (HHUFF_NT_RES=1 also for
// the per-string lengths and statuses)
#ifndef HHUFF_NT_RES
#define HHUFF_NT_RES 0
#endif
typedef unsigned int hh_u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void st16_out(uint8_t* p, uint4 v) {
#if HHUFF_NT_STORE
    __builtin_nontemporal_store(hh_u32x4{v.x, v.y, v.z, v.w}, reinterpret_cast<hh_u32x4*>(p));
#else
    *reinterpret_cast<uint4*>(p) = v;
#endif
}
// bytes [lo, hi) of the 16-B chunk v (in registers) to global g (16-B aligned): whole dwords as dword stores, the
// partial dword at each end as byte stores -- at most 10 predicated stores
__device__ __forceinline__ void store_range16r(uint8_t* __restrict__ g, uint4 v, uint32_t lo, uint32_t hi) {
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (uint32_t k = 0; k < 4; ++k)
        if (lo <= 4u * k && 4u * k + 4u <= hi) *reinterpret_cast<uint32_t*>(g + 4u * k) = w[k];
    const uint64_t q0 = (uint64_t)v.y << 32 | v.x, q1 = (uint64_t)v.w << 32 | v.z;
    auto byte_at = [&](uint32_t a) { return (uint32_t)((a < 8u ? q0 : q1) >> (8u * (a & 7u))); };
    const uint32_t e0 = min(hi, (lo + 3u) & ~3u);
    const uint32_t s1 = max(max(lo, hi & ~3u), e0);
#pragma unroll
    for (uint32_t j = 0; j < 3; ++j) {
        if (lo + j < e0) g[lo + j] = (uint8_t)byte_at(lo + j);
        if (s1 + j < hi) g[s1 + j] = (uint8_t)byte_at(s1 + j);
    }
}
template <class T>
__device__ __forceinline__ void st_res(T* p, T v) {
#if HHUFF_NT_RES
    __builtin_nontemporal_store(v, p);
#else
    *p = v;
#endif
}

// Write LDS bytes [0, ospan) to global [gbase, gbase + ospan) (gbase 16-aligned), keeping only the
// global bytes in [keep_lo, keep_hi); 16-byte stores for whole chunks, byte stores at the edges.
// (Measured: batching the LDS reads of all chunks, or taking the edge bytes from the loaded registers,
// made the c4 decode 3.5 % slower -- register pressure / code size in the 16-wave staged kernels.)
#ifndef HHUFF_EDGE_BYTES
// 1: a tile's two shared 16-B chunks are stored one byte a lane (lanes 0-15 the first chunk, 16-31 the last: one
// LDS byte read and one byte-store instruction a tile); 0: by byte range from the chunk's registers (<= 10
// predicated stores each)
#define HHUFF_EDGE_BYTES 1
#endif
// The region's two edge chunks (first and last; the whole region is [gbase, gbase + ospan), gbase 16-aligned),
// one byte a lane: lanes 0-15 the first chunk, lanes 16-31 the last, each storing its byte when it lies in
// [keep_lo, keep_hi) and its chunk is partial (a full chunk went out whole).
template <bool SWAP>
__device__ __forceinline__ void edge_bytes(uint8_t* __restrict__ out, uint64_t gbase, const uint8_t* lds, uint32_t ospan,
                                           uint64_t keep_lo, uint64_t keep_hi, int lane) {
    if (ospan == 0 || lane >= 32) return;
    const uint32_t kl = (ospan - 1u) & ~15u, b = (uint32_t)lane & 15u;
    const uint32_t k = lane < 16 ? 0u : kl;
    const uint64_t g = gbase + k, G = g + b;
    const bool part = !(g >= keep_lo && g + 16 <= keep_hi);
    if ((lane < 16 || kl != 0) && part && G >= keep_lo && G < keep_hi) out[G] = lds[k + (SWAP ? b ^ 3u : b)];
}
// SWAP: the LDS bytes are MSB-first words (the encode stage), byte-swapped in registers on the way out.
// G: the LDS reads of G chunks ahead of their stores (one LDS round trip per G chunks; 4 (G - 1) more VGPRs)
template <int NCH, bool SWAP = false, int G = 1>
__device__ __forceinline__ void region_copy(uint8_t* __restrict__ out, uint64_t gbase, const uint8_t* lds, uint32_t ospan,
                                            uint64_t keep_lo, uint64_t keep_hi, int lane) {
    auto put = [&](uint32_t k, uint4 v) {
        const uint64_t g = gbase + k;
        if (SWAP) v = make_uint4(bswap32(v.x), bswap32(v.y), bswap32(v.z), bswap32(v.w));
        if (g >= keep_lo && g + 16 <= keep_hi) {
            st16_out(out + g, v);
        } else if (!HHUFF_EDGE_BYTES) {  // a chunk shared with a neighbouring tile: only this tile's bytes
            const uint32_t lo = keep_lo > g ? (uint32_t)min(keep_lo - g, (uint64_t)16) : 0u;
            const uint32_t hi = keep_hi > g ? (uint32_t)min(keep_hi - g, (uint64_t)16) : 0u;
            if (hi > lo) store_range16r(out + g, v, lo, hi);
        }
    };
    for (uint32_t k = (uint32_t)lane * 16u; k < ospan; k += (uint32_t)G * 64u * 16u) {
        uint4 v[G];
#pragma unroll
        for (int j = 0; j < G; ++j) {
            const uint32_t kj = k + (uint32_t)j * 64u * 16u;
            v[j] = kj < ospan ? *reinterpret_cast<const uint4*>(lds + kj) : make_uint4(0u, 0u, 0u, 0u);
        }
#pragma unroll
        for (int j = 0; j < G; ++j) {
            const uint32_t kj = k + (uint32_t)j * 64u * 16u;
            if (kj < ospan) put(kj, v[j]);
        }
    }
    if (HHUFF_EDGE_BYTES) edge_bytes<SWAP>(out, gbase, lds, ospan, keep_lo, keep_hi, lane);
}

// (SWAP as region_copy)
template <bool SWAP = false>
__device__ __forceinline__ void region_copy_deferred(uint8_t* __restrict__ out, uint64_t gbase, const uint8_t* lds,
                                                     uint32_t ospan, uint64_t keep_lo, uint64_t keep_hi, int lane,
                                                     EdgeRec* __restrict__ rec) {
    const uint32_t kl = ospan ? (ospan - 1u) & ~15u : 0u;  // the last chunk
    for (uint32_t k = (uint32_t)lane * 16u; k < ospan; k += 64u * 16u) {
        const uint64_t g = gbase + k;
        uint4 v = *reinterpret_cast<const uint4*>(lds + k);
        if (SWAP) v = make_uint4(bswap32(v.x), bswap32(v.y), bswap32(v.z), bswap32(v.w));
        const bool full = g >= keep_lo && g + 16 <= keep_hi;
        if (full) st16_out(out + g, v);  // (streaming: the output is not read again by the kernel)
        if (k == 0 || k == kl) {
            const uint32_t lo = keep_lo > g ? (uint32_t)(keep_lo - g) : 0u;
            const uint32_t hi = keep_hi - g < 16 ? (uint32_t)(keep_hi - g) : 16u;
            EdgeRec* r = rec + (k == 0 ? 0 : 1);
            r->v = v;
            r->m = make_uint4((uint32_t)g, (uint32_t)(g >> 32), full ? 0u : lo, full ? 0u : hi);
            if (kl == 0) rec[1].m = make_uint4(0u, 0u, 0u, 0u);
        }
    }
    if (ospan == 0 && lane == 0) {
        rec[0].m = make_uint4(0u, 0u, 0u, 0u);
        rec[1].m = make_uint4(0u, 0u, 0u, 0u);
    }
}

// one thread per (record, dword)
__global__ void edge_fix_kernel(uint8_t* __restrict__ out, const EdgeRec* __restrict__ rec, uint64_t nrec,
                                const uint32_t* __restrict__ gate) {
    if (gate && *gate != kGateStaged) return;  // the staged kernel did not run: no records were written
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < 4 * nrec; i += (uint64_t)gridDim.x * blockDim.x) {
        const EdgeRec& r = rec[i >> 2];
        const uint4 m = r.m;
        const uint32_t w = (uint32_t)(i & 3), lo = max(m.z, 4u * w), hi = min(m.w, 4u * w + 4u);
        if (lo >= hi) continue;
        const uint32_t word = reinterpret_cast<const uint32_t*>(&r.v)[w];
        uint8_t* g = out + (((uint64_t)m.y << 32) | m.x);
        if (hi - lo == 4) {
            *reinterpret_cast<uint32_t*>(g + lo) = word;
        } else {
            for (uint32_t x = lo; x < hi; ++x) g[x] = (uint8_t)(word >> (8u * (x & 3u)));
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
    EdgeRec* edges;  // region layout: 2 records per 64-string tile (deferred edges), or NULL
    uint32_t* gate;        // NULL, or the device-side kernel choice (kGate*), written by the staged kernel
    const uint64_t* sel;   // decode_select_kernel's partial sums [3][kSelBlocks] (with gate)
    uint32_t* pk_off;      // packed mode (decode_staged_kernel<.., true>): u32[n + 1] output places
    const uint32_t* n_dev;  // NULL, or the string count in device memory (n an upper bound)
    // strings of kSplitMin bytes or more are listed here for split_decode_kernel instead of decoded by one lane
    // (NULL: every string decoded where it is met)
    uint32_t* split_list = nullptr;
    uint32_t* split_n = nullptr;
    uint32_t split_cap = 0;
    uint32_t split_min = 0xFFFFFFFFu;  // Huffman bytes from which a string is listed
    // strings of big_min bytes or more go to a second list, decoded by a whole block each (NULL: none)
    uint32_t* big_list = nullptr;
    uint32_t* big_n = nullptr;
    uint32_t big_cap = 0;
    uint32_t big_min = 0xFFFFFFFFu;
    // with gate: the staged / stream prices select_verdict uses, ps per string and per (tile-padded) byte --
    // the fitted defaults, or the device's calibration (calibrate_prices)
    float price[4] = {40.0f, 1.07f, 184.0f, 1.15f};
    // stream kernel: strings a wave takes from the batch counter at a time (stream_claim)
    uint32_t claim = 64;
};

__device__ __forceinline__ void load_dec_tables(uint32_t* s_lut, uint32_t* s_kinfo, uint32_t* s_ones, int nthreads) {
    for (uint32_t k = threadIdx.x; k < (1u << HHUFF_LUT_BITS) / 4; k += nthreads)
        reinterpret_cast<uint4*>(s_lut)[k] = reinterpret_cast<const uint4*>(g_dec_lut)[k];
    for (uint32_t k = threadIdx.x; k < HHUFF_ONES_NENT; k += nthreads) s_ones[k] = g_ones[k];
    if (threadIdx.x < 31) s_kinfo[threadIdx.x] = g_kinfo[threadIdx.x];
}

// a string long enough for split_decode_kernel goes to its list (when the launch has one) instead of being
// decoded by this lane; a full list leaves it here
__device__ __forceinline__ bool split_push(const DecArgs& A, uint32_t i, uint32_t len) {
    if (A.split_list == nullptr || len < A.split_min || len > kMaxStrLen) return false;
    if (A.big_list != nullptr && len >= A.big_min) {
        const uint32_t b = atomicAdd(A.big_n, 1u);
        if (b < A.big_cap) {
            A.big_list[b] = i;
            return true;
        }
    }
    const uint32_t k = atomicAdd(A.split_n, 1u);
    if (k >= A.split_cap) return false;
    A.split_list[k] = i;
    return true;
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

// Packed output (PACKED, contiguous layout): the 64 strings of a tile are written back to back in string
// order -- the wave's exclusive prefix sum of the decoded lengths places them -- from the tile's bound
// position G = floor(8 * in_off[first string] / 5) on, so the kernel writes exactly the decoded bytes (the
// slot layout writes whole floor(8 len / 5) slots).  pk_off[i] = G + place.  Tile runs never overlap: a
// tile's decoded bytes fit the slot region of its input span.
//
// LDS per wave is one buffer of IN + OUT + 256 (+16 slack) bytes whose halves swap roles from tile to tile
// in packed mode:
//   even tile: input [0, IN), slot output [IN, IN + OUT), trash [IN + OUT, Z); packed run at [c0, c0 + T),
//              c0 = G mod 16 (left end);
//   odd tile:  slot output [0, OUT), trash [OUT, OUT + 256), input [OUT + 256, Z); packed run right-aligned
//              (the largest c0 <= Z - T with c0 = G mod 16).
// The compaction moves each lane's string from its slot to its place in two passes: first every byte
// whose destination lies in the free half (the input / trash area of this tile), then the rest.  Each
// destination of the second pass holds, as a source, only bytes the first pass has already read (the
// run starts at least IN bytes away from the slots it is built from), so lanes copying in lock step
// never overwrite a source another lane still needs.  The next tile's input then goes into the other
// half, beside the packed run, before the run's 16-B stores are issued (the pipeline order of the slot
// layout, whose commit also precedes the stores).
#ifndef HHUFF_DEC_COPY_G  // decode_staged_kernel's slot-layout copy-out: chunks whose LDS reads go ahead of their stores
#define HHUFF_DEC_COPY_G 1
#endif
#ifndef HHUFF_DEC_TI_TOP  // decode_staged_kernel: the tile-after-next's offsets issued at the loop top, consumed in
#define HHUFF_DEC_TI_TOP 1   // the same trip (c4 decode -2.2 %, c2 -1.5 %; profiles/r06v_decode_ti_top_ab.jsonl)
#endif
template <int WAVES, int IN_STAGE, int OUT_STAGE, bool PACKED>
__global__ __launch_bounds__(WAVES * 64) void decode_staged_kernel(DecArgs A) {
    constexpr uint32_t Z = IN_STAGE + OUT_STAGE + 256u;  // + 16 slack: the run's last 16-B chunk may read past Z
    static_assert(OUT_STAGE <= 2 * IN_STAGE + 480 && Z % 16 == 0, "packed compaction needs OUT <= 2 IN");
    if (A.n_dev) A.n = *A.n_dev;  // the count lives in device memory (literal pre-passes)
    // one LDS object, window LUT first: its byte offsets then fit the ds_read address with no base add
    struct __attribute__((aligned(16))) Smem {
        uint32_t lut[1u << HHUFF_LUT_BITS];
        uint32_t kinfo[32];
        uint32_t ones[(HHUFF_ONES_NENT + 3) & ~3];
        uint8_t buf[WAVES][Z + 16];
    };
    if (A.gate) {  // mixed-length batch: price both kernels from the sampled tiles (decode_select_kernel)
        __shared__ uint32_t verdict;
        if (threadIdx.x < 64) {
            const uint32_t g = select_verdict(A.sel, A.price);
            if (threadIdx.x == 0) {
                verdict = g;
                if (blockIdx.x == 0) *A.gate = g;  // read by edge_fix_kernel and the stream kernel, launched after
            }
        }
        __syncthreads();
        if (verdict != kGateStaged) return;  // block-uniform
    }
    __shared__ Smem sm;
    uint32_t* s_lut = sm.lut;
    uint32_t* s_kinfo = sm.kinfo;
    uint32_t* s_ones = sm.ones;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint64_t stride = (uint64_t)gridDim.x * WAVES * 64;
    uint64_t base = ((uint64_t)blockIdx.x * WAVES + wave) * 64;
    load_dec_tables(s_lut, s_kinfo, s_ones, WAVES * 64);
    __syncthreads();
    const DecTables T{s_lut, s_kinfo, s_ones};
    uint8_t* const buf = sm.buf[wave];
    const uint32_t bufa = lds_addr(buf);
    const bool region = A.in_len == nullptr && A.out_off == nullptr;
    const bool pairs = A.in_len != nullptr;
    if (base >= A.n) return;

    // per-tile layout: input span and output stage extent.  Per lane: the string and its stage offset;
    // wave-uniform (SGPRs): the tile's input span [lo, hi) and everything derived from it.
    struct Plan {
        uint32_t s, len, op0;    // per lane
        uint32_t lo, hi, ospan;  // wave-uniform
        uint32_t ib, ob;         // byte offsets of the input and slot-output stages in the wave's buffer
        uint64_t dst_g;          // explicit destinations
        bool valid, fits;
        __device__ __forceinline__ uint32_t a0() const { return lo & ~15u; }
        __device__ __forceinline__ uint32_t span() const { return hi > lo ? ((hi + 15u) & ~15u) - a0() : 0u; }
        __device__ __forceinline__ uint64_t olo() const { return dec_slot(lo); }
        __device__ __forceinline__ uint64_t ohi() const { return dec_slot(hi); }
        __device__ __forceinline__ uint64_t obase() const { return olo() & ~15ull; }
    };
    auto plan = [&](uint64_t b, const TileIn& ti, uint32_t par) {
        Plan P;
        const Tile t = finish_tile(b, lane, A.n, ti, pairs);
        P.s = t.s;
        P.len = t.len;
        P.valid = t.valid;
        P.lo = __builtin_amdgcn_readfirstlane(t.lo);
        P.hi = __builtin_amdgcn_readfirstlane(t.hi);
        P.ib = par ? OUT_STAGE + 256u : 0u;
        P.ob = par ? 0u : IN_STAGE;
        P.dst_g = 0;
        if (region) {
            P.ospan = P.hi > P.lo ? (uint32_t)(P.ohi() - P.obase()) : 0u;
            P.op0 = t.len ? (uint32_t)(dec_slot(t.s) - P.obase()) : 0u;
        } else {
            P.dst_g = A.out_off ? (uint64_t)ti.dst : dec_slot(t.s);
            const uint32_t cap = t.valid ? (uint32_t)(((uint64_t)min(t.len, kMaxStrLen) * 8u) / 5u) + 3u : 0u;
            const uint32_t pre = wave_excl_scan(cap, lane);
            P.ospan = (uint32_t)__builtin_amdgcn_readlane((int)(pre + cap), 63);
            P.op0 = pre + ((uint32_t)(((uintptr_t)A.out + P.dst_g) - pre) & 3u);
        }
        P.fits = P.span() <= IN_STAGE && P.ospan <= OUT_STAGE;
        return P;
    };

    // Software pipeline over the wave's tiles (cur = being decoded, nxt = span prefetched into registers,
    // ti = offsets of the tile after).  Every wait on a global load sits between the current tile's steps
    // and its stores: the vmcnt counter also counts stores, so a load consumed right after the previous
    // tile's stores would wait for their writes to land.
    SpanPrefetch<(IN_STAGE + 1023) / 1024> pf;
    uint32_t par = 0;  // layout parity of the current tile (packed mode alternates)
    TileIn ti = issue_tile(base, lane, A.n, A.in_off, A.in_len, A.is_name_bits, A.out_off);
    Plan cur = plan(base, ti, 0);
    uint32_t cur_name = ti.name_word;
    if (cur.fits) pf.issue(A.in, A.in_size, cur.a0(), cur.span(), lane);
    bool have_next = base + stride < A.n;
    ti = issue_tile(base + stride, lane, A.n, A.in_off, A.in_len, A.is_name_bits, A.out_off);
    if (cur.fits) pf.template commit<true>(reinterpret_cast<uint32_t*>(buf + cur.ib), A.in, A.in_size, cur.a0(), cur.span(), lane);
    Plan nxt;
    uint32_t nxt_name = 0;
    if (have_next) {
        nxt = plan(base + stride, ti, PACKED ? 1u : 0u);
        nxt_name = ti.name_word;
        if (nxt.fits) pf.issue(A.in, A.in_size, nxt.a0(), nxt.span(), lane);
#if !HHUFF_DEC_TI_TOP
        ti = issue_tile(base + 2 * stride, lane, A.n, A.in_off, A.in_len, A.is_name_bits, A.out_off);
#endif
    }
    PROF_DECL
    for (;;) {
        const uint64_t nbase = base + stride;
#if HHUFF_DEC_TI_TOP
        // the offsets of the tile after next, issued at the top and consumed at this tile's plan step below: no
        // loaded register lives across the loop's back edge, where a PHI copy would wait for it behind this
        // tile's stores (the ISA had s_waitcnt vmcnt(3) / (2) there, in front of two such copies)
        ti = issue_tile(nbase + stride, lane, A.n, A.in_off, A.in_len, A.is_name_bits, A.out_off);
#endif
        // ---- the current tile: steps and verdicts ----
        const Plan& t = cur;
        const uint32_t ti_i = (uint32_t)base + (uint32_t)lane;
        const bool is_name = t.valid && A.is_name_bits ? ((cur_name >> (ti_i & 31)) & 1u) : false;
        uint32_t* stage = reinterpret_cast<uint32_t*>(buf + cur.ib);
        uint8_t* obuf = buf + cur.ob;
        uint32_t ol = 0;
        uint8_t st = 0;
        uint64_t G = 0;        // packed: the tile's run start in `out`
        uint32_t place = 0, T_run = 0, c0 = 0;
        bool listed = false;
        PROF_MARK(0);
        if (cur.fits) {
            wave_lds_sync();
            const bool act = t.valid && t.len <= kMaxStrLen;
            const uint32_t rel = t.len ? t.s - cur.a0() : 0u;
            const DecResult r = decode_staged_lane_v7(stage, rel, t.len, act, obuf, cur.op0, OUT_STAGE + 4u * (uint32_t)lane, T);
            PROF_MARK(1);  // steps
            if (t.valid && t.len > kMaxStrLen) {
                ol = kFailLen;
                st = kStatusTooLong;
            } else if (r.ok) {
                ol = r.len;
                const uint32_t first = r.len ? obuf[cur.op0] : 0u, lastc = r.len ? obuf[cur.op0 + r.len - 1] : 0u;
                st = soft_bits(is_name, r.len, r.flags, first, lastc);
            } else {
                ol = kFailLen;
                st = kStatusFail;
            }
            if constexpr (PACKED) {
                // places: wave prefix sum of the kept lengths; then the two-pass compaction (see above)
                const uint32_t keep = (t.valid && ol != kFailLen) ? ol : 0u;
                place = wave_excl_scan(keep, lane);
                T_run = (uint32_t)__builtin_amdgcn_readlane((int)(place + keep), 63);
                G = dec_slot((uint32_t)__builtin_amdgcn_readfirstlane((int)t.s));
                const uint32_t g15 = (uint32_t)G & 15u;
                if (par == 0) {
                    c0 = g15;
                } else {
                    c0 = ((Z - T_run) & ~15u) | g15;
                    if (c0 > Z - T_run) c0 -= 16u;
                }
                const uint32_t D = c0 + place, S = cur.ob + cur.op0;
                const uint32_t rend = (c0 + T_run + 15u) & ~15u;
                // bytes [0, cut) of the string go to destinations below `edge`, the rest above it
                const uint32_t edge = par == 0 ? IN_STAGE : OUT_STAGE;
                const uint32_t cut = D >= edge ? 0u : min(keep, edge - D);
                const uint32_t a0 = par == 0 ? 0u : cut, a1 = par == 0 ? cut : keep;  // pass 1: the free half
                if (par == 0)
                    lds_zero(buf, 0u, min(rend, IN_STAGE), lane);
                else
                    lds_zero(buf, max(c0 & ~15u, OUT_STAGE), rend, lane);
                wave_lds_sync();
                lds_move_or(bufa + S + a0, bufa + D + a0, a1 - a0);
                const uint32_t b0 = par == 0 ? cut : 0u, b1 = par == 0 ? keep : cut;
                if (__builtin_amdgcn_ballot_w64(b1 > b0) != 0) {  // pass 2: its sources were all read in pass 1
                    wave_lds_sync();
                    if (par == 0)
                        lds_zero(buf, IN_STAGE, rend, lane);
                    else
                        lds_zero(buf, c0 & ~15u, OUT_STAGE, lane);
                    wave_lds_sync();
                    lds_move_or(bufa + S + b0, bufa + D + b0, b1 - b0);
                }
            }
            wave_lds_sync();
            PROF_MARK(2);  // verdicts
        } else if (!PACKED && t.valid) {
            if (split_push(A, ti_i, t.len)) {
                listed = true;  // split_decode_kernel writes its results
            } else {
                const uint64_t d = A.out_off ? cur.dst_g : dec_slot(t.s);
                decode_direct(A, t.s, t.len, is_name, A.out + d, T, ol, st);
            }
            PROF_MARK(6);  // direct path
        } else if (PACKED) {
            // a tile larger than the stages: count first (lengths fix the places), then decode into place
            CountSink cs;
            cs.init();
            bool ok = false;
            if (t.valid && t.len <= kMaxStrLen) {
                const DecResult r = decode_core(GlobalSource{A.in, A.in_size}, t.s, t.len, cs, T);
                ok = r.ok;
                ol = ok ? r.len : kFailLen;
                st = ok ? soft_bits(is_name, r.len, r.flags, cs.first, cs.last) : kStatusFail;
            } else if (t.valid) {
                ol = kFailLen;
                st = kStatusTooLong;
            }
            const uint32_t keep = ok ? ol : 0u;
            place = wave_excl_scan(keep, lane);
            G = dec_slot((uint32_t)__builtin_amdgcn_readfirstlane((int)t.s));
            if (ok && keep) {
                RegSink sink;
                sink.init(A.out + G + place);
                (void)decode_core(GlobalSource{A.in, A.in_size}, t.s, t.len, sink, T);
                sink.finish();
            }
            PROF_MARK(6);
        }
        // ---- the next tile: commit its span (its input half is free), plan + prefetch the one after ----
        Plan nn;
        uint32_t nn_name = 0;
        bool have_nn = false;
        if (have_next && nxt.fits)
            pf.template commit<true>(reinterpret_cast<uint32_t*>(buf + nxt.ib), A.in, A.in_size, nxt.a0(), nxt.span(), lane);
        have_nn = have_next && nbase + stride < A.n;
        // planned and reloaded on every path (issue_tile clamps its index): ti is consumed and redefined
        // at one place, so no wait for it lands behind the span loads issued here
        nn = plan(nbase + stride, ti, PACKED ? par : 0u);
        nn_name = ti.name_word;
        if (have_nn && nn.fits) pf.issue(A.in, A.in_size, nn.a0(), nn.span(), lane);
#if !HHUFF_DEC_TI_TOP
        ti = issue_tile(nbase + 2 * stride, lane, A.n, A.in_off, A.in_len, A.is_name_bits, A.out_off);
#endif
        PROF_MARK(3);  // commit + plan
        // ---- the current tile: stores ----
#if defined(HHUFF_X_NOSTORE) || defined(HHUFF_X_NOSTORE_OUT)  // ablations (output wrong by design): no output stores
        if (false) {
#else
        if (cur.fits) {
#endif
            if (PACKED) {
                const uint64_t gb = G & ~15ull;
                const uint32_t ps = (uint32_t)(((G + T_run + 15u) & ~15ull) - gb);
                if (A.edges)
                    region_copy_deferred(A.out, gb, buf + c0 - ((uint32_t)G & 15u), ps, G, G + T_run, lane,
                                         A.edges + 2 * (base >> 6));
                else
                    region_copy<(OUT_STAGE + 1023) / 1024>(A.out, gb, buf + c0 - ((uint32_t)G & 15u), ps, G, G + T_run, lane);
            } else if (region) {
                if (A.edges)
                    region_copy_deferred(A.out, cur.obase(), obuf, cur.ospan, cur.olo(), cur.ohi(), lane,
                                         A.edges + 2 * (base >> 6));
                else
                    region_copy<(OUT_STAGE + 1023) / 1024, false, HHUFF_DEC_COPY_G>(A.out, cur.obase(), obuf, cur.ospan,
                                                                                           cur.olo(), cur.ohi(), lane);
            } else if (t.valid && ol != kFailLen) {
                lane_copy(A.out + cur.dst_g, obuf + cur.op0, ol);
            }
            wave_lds_sync();
        } else if (A.edges && lane == 0) {  // direct path: no edges to defer
            A.edges[2 * (base >> 6)].m = make_uint4(0u, 0u, 0u, 0u);
            A.edges[2 * (base >> 6) + 1].m = make_uint4(0u, 0u, 0u, 0u);
        }
#if HHUFF_STATUS_DW
        // a whole tile's status bytes as 16 dword stores (4 lanes' bytes each) instead of 64 byte stores; a listed
        // string's byte is 0 here and written by split_decode_kernel, which runs after this kernel
        const bool st_dw = !PACKED && base + 64u <= A.n && (((uintptr_t)(A.status + base)) & 3u) == 0;  // (uniform)
        if (st_dw) {
            uint32_t sv = (t.valid && !listed ? (uint32_t)st : 0u) << (8u * ((uint32_t)lane & 3u));
            sv |= (uint32_t)__shfl_xor((int)sv, 1);
            sv |= (uint32_t)__shfl_xor((int)sv, 2);
            if ((lane & 3) == 0) *reinterpret_cast<uint32_t*>(A.status + base + (uint32_t)lane) = sv;
            if (t.valid && !listed) A.out_len[ti_i] = ol;
        } else
#endif
#if defined(HHUFF_X_NOSTORE) || defined(HHUFF_X_NOSTORE_LEN)  // (no length / status stores)
        if (false) {
#else
        if (t.valid && !listed) {
#endif
            st_res(A.out_len + ti_i, ol);
            st_res(A.status + ti_i, st);
            if (PACKED) {
                A.pk_off[ti_i] = (uint32_t)(G + place);
                if (ti_i == A.n - 1) A.pk_off[A.n] = (uint32_t)(G + place + (ol != kFailLen ? ol : 0u));
            }
        }
        PROF_MARK(4);  // stores
        if (!have_next) {
            PROF_FLUSH(0);
            break;
        }
        cur = nxt;
        cur_name = nxt_name;
        nxt = nn;
        nxt_name = nn_name;
        have_next = have_nn;
        base = nbase;
        if (PACKED) par ^= 1u;
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
        if (split_push(A, (uint32_t)i, len)) continue;
        uint32_t ol;
        uint8_t st;
        decode_direct(A, s, len, is_name, A.out + d, T, ol, st);
        A.out_len[i] = ol;
        A.status[i] = st;
    }
}

// ------------------------------------------------------------------------------------------------
// Split decode of long strings (SURVEY §7 hard part 2: h2o takes header values up to H2O_MAX_REQLEN).  A
// string of kSplitMin bytes or more would keep one lane busy for its whole length; here one wave decodes it.
// The string's bits are cut into 64 segments of `seg` bits (a dword multiple).  Huffman codes self-
// synchronise: a lane that starts decoding a lead of 64..kSplitLead bits before its segment at an arbitrary bit
// is, with high probability, on the true symbol boundaries by the time it reaches its segment.
//   pass A: lane k decodes from max(k seg - lead, 0) to the first symbol boundary at or after
//           (k + 1) seg (the last active lane: to the string's end, with the padding rule, hpack.c:132-133),
//           and counts the symbols that start at or after k seg: f_k = the first of them, e_k = where it stops;
//   check:  lane k agrees with lane k - 1 iff f_k == e_{k-1}; a lane that does not decodes again from
//           e_{k-1}, a true boundary (lane 0 starts at bit 0), until no lane changes;
//   pass B: a wave prefix sum of the counts places each lane's symbols; lane k decodes [f_k, e_k) again and
//           writes them (register sink, any alignment).
// Same results as decode_core (hpack.c:117-156): EOS on the true path fails the string (hpack.c:88-89), the
// soft bits come from all symbols' flags and the first and last byte.
// ------------------------------------------------------------------------------------------------
constexpr uint32_t kSplitMin = 4096;     // Huffman bytes: strings this long go to split_decode_kernel
constexpr uint32_t kSplitMinFew = 512;   // the same in batches of <= 16 strings (latency: one lane would take them)
constexpr uint32_t kSplitLead = 256;  // bits decoded before a long segment (synchronisation lag: mean 37, p99 193)

struct SegWalk {
    uint32_t f, e;        // first counted symbol's start, stop position (bits from the string's start)
    uint32_t cnt, flags;  // counted symbols, their invalid-char flags (decode_core's encoding)
    uint32_t first, last; // first / last counted symbol
    bool eos, end_ok;     // an EOS among the counted symbols; (last segment) the padding rule held
};

constexpr int kSplitNW = 16;  // window dwords per lane (split_decode_kernel, one_string_kernel)
// a dword-aligned 16-B load; at the end of the input, the bytes that exist
__device__ __forceinline__ uint4 load16_bounded(const uint8_t* __restrict__ in, uint64_t in_size, uint64_t a) {
    if (a + 16 <= in_size) {
        typedef uint32_t u32x4a __attribute__((ext_vector_type(4), aligned(4)));  // dword-aligned 16-B load
        const u32x4a v = *reinterpret_cast<const u32x4a*>(in + a);
        return make_uint4(v.x, v.y, v.z, v.w);
    }
    return load16_tail(in, in_size, a);
}
// A dword-aligned 16-B window piece of a split string: from global memory (bounded at the input's end) or from
// a string staged in LDS (one_string_kernel; reads clamped to its last dword).
__device__ __forceinline__ uint4 split_piece(const GlobalSource& src, uint64_t a) {
    return load16_bounded(src.in, src.in_size, a);
}
__device__ __forceinline__ uint4 split_piece(const LdsSource& src, uint64_t a) {
    const uint32_t b = (uint32_t)a;
    return make_uint4(src.word(b), src.word(b + 4u), src.word(b + 8u), src.word(b + 12u));
}

// Decode the string's bits (string at byte s, TB bits) from p0; count (and with EMIT write) the symbols that
// start in [kstart, pstop); stop at the first boundary >= pstop, or at the string's end when pstop >= TB.
// A lane's next kSplitNW input dwords go into its LDS window `win` (kSplitNW + 1 dwords, odd stride) in
// rounds -- one 16-B load round trip for the wave per window, the next window prefetched into registers
// during the round -- and the lane steps until its window runs out.  Away from kstart and pstop a step is
// decode_staged_lane_v7's bulk step (two LUT lookups, 1-4 symbols, no per-symbol checks); within 26 bits of
// either, and for codes longer than the window LUT, it is the checked single-lookup step.
template <bool EMIT, class Src>
__device__ __forceinline__ SegWalk seg_walk(const Src& src, uint32_t s, uint32_t TB, uint32_t p0, uint32_t kstart,
                                            uint32_t pstop, bool act, uint32_t* win, RegSink& sink,
                                            const DecTables& T) {
    constexpr uint32_t NW = kSplitNW;
    SegWalk r{0xFFFFFFFFu, 0u, 0u, 0u, 0u, 0u, false, false};
    auto take = [&](uint32_t p, uint32_t sym, uint32_t fl) {  // one symbol starting at p
        if (p < kstart) return;
        r.f = min(r.f, p);
        r.first = r.cnt == 0 ? sym : r.first;
        r.last = sym;
        r.cnt += 1;
        r.flags |= fl;
        if (EMIT) sink.put1(sym);
    };
    const lds_u32* wl = (const lds_u32*)win;
    uint4 pf[NW / 4];
    uint64_t pfa = ~0ull;
    uint32_t p = p0;
    bool live = act;
    for (;;) {
        if (!__any(live)) break;
        const uint64_t abit = 8ull * s + p;
        const uint64_t wa = (abit >> 5) << 2;
        if (live) {
            if (wa != pfa) {
#pragma unroll
                for (int j = 0; j < (int)NW / 4; ++j) pf[j] = split_piece(src, wa + 16u * j);
            }
#pragma unroll
            for (int j = 0; j < (int)NW / 4; ++j) {
                win[4 * j + 0] = bswap32(pf[j].x);
                win[4 * j + 1] = bswap32(pf[j].y);
                win[4 * j + 2] = bswap32(pf[j].z);
                win[4 * j + 3] = bswap32(pf[j].w);
            }
            // a lane leaves the round with its next bit in dword NW - 1: that window comes next
            pfa = wa + 4u * (NW - 1);
#pragma unroll
            for (int j = 0; j < (int)NW / 4; ++j) pf[j] = split_piece(src, pfa + 16u * j);
        }
        uint32_t q = (uint32_t)(abit & 31u);  // bit of the window; x0..x2 hold dwords qd..qd + 2
        uint32_t qd = 0, x0 = wl[0], x1 = wl[1], x2 = wl[2];
        auto advance = [&](uint32_t cons) {  // cons <= 30: at most one dword boundary crossed
            q += cons;
            p += cons;
            const bool adv = (q >> 5) != qd;
            x0 = adv ? x1 : x0;
            x1 = adv ? x2 : x1;
            qd = q >> 5;
            x2 = wl[qd + 2];  // (qd <= NW - 2 while the lane steps: inside the NW + 1 dwords)
        };
        while (live) {
            if (p >= pstop) {  // (pstop >= TB: p == TB, no bits left, the padding rule holds)
                live = false;
                r.end_ok = !r.eos;
                break;
            }
            // bulk run: every symbol of a step's two lookups starts before pstop (hence inside the string),
            // and either all of them are counted (p >= kstart) or none is (p + 26 < kstart)
            for (;;) {
                const uint32_t cm = p >= kstart ? 0xFFFFFFFFu : 0u;
                const uint32_t lim = cm ? pstop : kstart;
                if (p + 26u >= lim || q >= 32u * (NW - 1)) break;
                const uint32_t wz = (q & 31u) ? __builtin_amdgcn_alignbit(x0, x1, 32u - (q & 31u)) : x0;
                const uint32_t e = T.lut[wz >> (32 - HHUFF_LUT_BITS)];
                if (e & kLong) break;
                uint32_t cons = lut_l12(e);
                const uint32_t eb = T.lut[(wz << cons) >> (32 - HHUFF_LUT_BITS)];
                const uint32_t bm = (eb & kLong) ? 0u : 0xFFFFFFFFu;
                cons += lut_l12(eb) & bm;
                const uint32_t ne = (e >> 28) & 3u, nb = (eb >> 28) & 3u & bm;
                const uint32_t lb = nb == 2u ? lut_sym2(eb) : eb;
                const uint32_t le = ne == 2u ? lut_sym2(e) : e;
                r.f = min(r.f, p | ~cm);
                r.first = (cm && r.cnt == 0) ? (e & 0xFFu) : r.first;
                r.last = cm ? (nb ? lb : le) & 0xFFu : r.last;
                r.cnt += (ne + nb) & cm;
                r.flags |= ((e >> 24) | (e >> 26) | (((eb >> 24) | (eb >> 26)) & bm)) & 3u & cm;
                if (EMIT) {  // pass B starts at kstart: every bulk step is counted
                    sink.put12(lut_pair(e), ne == 2u);
                    if (nb) sink.put12(lut_pair(eb), nb == 2u);
                }
                advance(cons);
            }
            if (p >= pstop) continue;
            if (q >= 32u * (NW - 1)) break;  // the window runs out: next round
            // one checked step
            const uint32_t w = (q & 31u) ? __builtin_amdgcn_alignbit(x0, x1, 32u - (q & 31u)) : x0;
            const uint32_t e = T.lut[w >> (32 - HHUFF_LUT_BITS)];
            const uint32_t R = TB - p;
            uint32_t cons;
            bool stop = false;
            if (e & kLong) {
                const uint32_t k = min((uint32_t)__builtin_clz(~w | 1u), 30u);
                const uint32_t ki = T.kinfo[k];
                const uint32_t le = T.ones[(ki & 0xFFFFu) + (((w << (k + 1)) >> 1) >> (31 - (ki >> 16)))];
                const uint32_t L = (le >> 9) & 31u;
                const uint32_t sym = le & 0x1FFu;
                stop = L > R;  // the string's end: padding
                if (!stop && sym == kEos && p >= kstart) {  // EOS inside the string (hpack.c:88-89)
                    r.eos = true;
                    stop = true;
                }
                if (!stop && sym != kEos) take(p, sym, (le >> 14) & 3u);
                cons = L;
            } else {
                const uint32_t L1 = lut_l1(e);
                stop = L1 > R;  // fewer bits left than the next code: padding
                const uint32_t L12 = lut_l12(e);
                if (!stop) take(p, e & 0xFFu, (e >> 24) & 3u);
                // the second symbol only when it starts before the stop and fits the string
                const bool two = (e & kHas2) && L12 <= R && p + L1 < pstop;
                if (!stop && two) take(p + L1, lut_sym2(e) & 0xFFu, (e >> 26) & 3u);
                cons = two ? L12 : L1;
            }
            if (stop) {  // at most 7 bits of padding, all ones (mkhufftbl.py:374-381)
                live = false;
                r.end_ok = !r.eos && R <= 7u && ((w >> 24) | (0xFFu >> R)) == 0xFFu;
                break;
            }
            advance(cons);
        }
    }
    r.e = p;
    if (r.f == 0xFFFFFFFFu) r.f = p;  // no symbol starts in the segment
    if (pstop < TB) r.end_ok = false;
    return r;
}

// One wave decodes the string at src bytes [s, s + len) into dst (any alignment, global or LDS); every lane
// returns the output length (kFailLen on failure) and the status byte.
template <class Src>
__device__ __forceinline__ void split_decode_wave(const Src& src, uint32_t s, uint32_t len, bool is_name, uint8_t* dst,
                                                  const DecTables& T, uint32_t lane, uint32_t& ol, uint8_t& st,
                                                  uint32_t* win) {
    // every lane walks its string bits through its LDS window (win: kSplitNW + 1 dwords)
    auto walk = [&](auto emit, uint32_t p0, uint32_t kstart, uint32_t pstop, bool act, RegSink& sink) {
        return seg_walk<decltype(emit)::value>(src, s, 8u * len, p0, kstart, pstop, act, win, sink, T);
    };
    using NoEmit = std::integral_constant<bool, false>;
    using Emit = std::integral_constant<bool, true>;
    const uint32_t TB = 8u * len;
    if (TB == 0) {  // an empty string decodes to nothing (hpack.c:117-156 with no bits)
        ol = 0;
        st = soft_bits(is_name, 0u, 0u, 0u, 0u);
        return;
    }
    const uint32_t seg = (uint32_t)(((uint64_t)TB + 64u * 32u - 1u) / (64u * 32u)) * 32u;  // bits, a dword multiple
    // lead: the bits a lane decodes before its segment.  Longer leads fail to synchronise less often (header
    // text: 17 % of starts at 64 bits, 3.6 % at 128, ~0.2 % at 256), and every failure costs a sequential
    // re-walk of a segment; short segments (per-string calls) take short leads
    const uint32_t lead = seg <= 64u ? 64u : (seg <= 256u ? 128u : kSplitLead);
    const uint32_t ks = lane * seg;
    const bool act = ks < TB;
    const bool lastl = act && ks + seg >= TB;
    const uint32_t pstop = lastl ? TB : ks + seg;
    RegSink none;
    none.init(nullptr);
    SegWalk w = walk(NoEmit{}, ks > lead ? ks - lead : 0u, ks, pstop, act, none);
    // agree with the lane before: lane k starts where lane k - 1 stopped
    for (int it = 0; it < 64; ++it) {
        const uint32_t pe = (uint32_t)__shfl_up((int)w.e, 1, 64);
        const bool bad = act && lane > 0 && w.f != pe;
        if (__builtin_amdgcn_ballot_w64(bad) == 0) break;
        const SegWalk w2 = walk(NoEmit{}, pe, pe, pstop, bad, none);
        if (bad) w = w2;
    }
    const uint32_t cnt = act ? w.cnt : 0u;
    const uint32_t place = wave_excl_scan(cnt, (int)lane);
    const uint32_t total = (uint32_t)__builtin_amdgcn_readlane((int)(place + cnt), 63);
    const bool eos = __builtin_amdgcn_ballot_w64(act && w.eos) != 0;
    const bool end_ok = __builtin_amdgcn_ballot_w64(lastl && w.end_ok) != 0;
    const bool ok = !eos && end_ok;
    uint32_t fl = act ? w.flags : 0u;
    fl |= (uint32_t)__shfl_xor((int)fl, 1, 64);
    fl |= (uint32_t)__shfl_xor((int)fl, 2, 64);
    fl |= (uint32_t)__shfl_xor((int)fl, 4, 64);
    fl |= (uint32_t)__shfl_xor((int)fl, 8, 64);
    fl |= (uint32_t)__shfl_xor((int)fl, 16, 64);
    fl |= (uint32_t)__shfl_xor((int)fl, 32, 64);
    // first byte: the first lane with symbols; last byte: the last one
    const uint64_t has = __builtin_amdgcn_ballot_w64(cnt != 0);
    uint32_t first = 0, last = 0;
    if (has) {
        first = (uint32_t)__shfl((int)w.first, (int)__builtin_ctzll(has), 64);
        last = (uint32_t)__shfl((int)w.last, 63 - (int)__builtin_clzll(has), 64);
    }
    {
        const bool em = ok && act && cnt != 0;
        RegSink sink;
        sink.init(dst + place);
        (void)walk(Emit{}, w.f, w.f, pstop, em, sink);
        if (em) sink.finish();
    }
    ol = ok ? total : kFailLen;
    st = ok ? soft_bits(is_name, total, fl & 3u, first, last) : kStatusFail;
}

// The same with the whole block (W waves, 64 W segments of at least 128 bits) on one string: lone very long
// strings (a 1-MB value on one wave walks 16 KB per lane).  The agree-with-the-lane-before check crosses waves
// through LDS (sx[0]: each wave's last e) with a block barrier per round; the wave totals, flags and first /
// last bytes meet in sx[1..4].  Every thread of the block calls it with the same string.
template <int W, class Src>
__device__ __forceinline__ void split_decode_block(const Src& src, uint32_t s, uint32_t len, bool is_name,
                                                   uint8_t* dst, const DecTables& T, uint32_t* win,
                                                   uint32_t (&sx)[5][W], uint32_t& ol, uint8_t& st) {
    const uint32_t t = threadIdx.x, lane = t & 63u, wave = t >> 6;
    auto walk = [&](auto emit, uint32_t p0, uint32_t kstart, uint32_t pstop, bool act, RegSink& sink) {
        return seg_walk<decltype(emit)::value>(src, s, 8u * len, p0, kstart, pstop, act, win, sink, T);
    };
    using NoEmit = std::integral_constant<bool, false>;
    using Emit = std::integral_constant<bool, true>;
    const uint32_t TB = 8u * len;
    if (TB == 0) {
        ol = 0;
        st = soft_bits(is_name, 0u, 0u, 0u, 0u);
        return;
    }
    constexpr uint32_t N = 64u * W;
    const uint32_t seg = max((uint32_t)(((uint64_t)TB + N * 32u - 1u) / (N * 32u)) * 32u, 128u);
    const uint32_t lead = seg <= 64u ? 64u : (seg <= 256u ? 128u : kSplitLead);
    const uint32_t ks = t * seg;
    const bool act = ks < TB;
    const bool lastl = act && ks + seg >= TB;
    const uint32_t pstop = lastl ? TB : ks + seg;
    RegSink none;
    none.init(nullptr);
    SegWalk w = walk(NoEmit{}, ks > lead ? ks - lead : 0u, ks, pstop, act, none);
    for (uint32_t it = 0; it < N; ++it) {
        if (lane == 63u) sx[0][wave] = w.e;
        __syncthreads();
        uint32_t pe = (uint32_t)__shfl_up((int)w.e, 1, 64);
        if (lane == 0u) pe = wave ? sx[0][wave - 1u] : 0u;
        const bool bad = act && t > 0u && w.f != pe;
        if (!__syncthreads_or(bad)) break;
        const SegWalk w2 = walk(NoEmit{}, pe, pe, pstop, bad, none);
        if (bad) w = w2;
    }
    const uint32_t cnt = act ? w.cnt : 0u;
    const uint32_t place = wave_excl_scan(cnt, (int)lane);
    uint32_t fl = act ? w.flags : 0u;
    fl |= (act && w.eos ? 4u : 0u) | (lastl && w.end_ok ? 8u : 0u);
    fl |= (uint32_t)__shfl_xor((int)fl, 1, 64);
    fl |= (uint32_t)__shfl_xor((int)fl, 2, 64);
    fl |= (uint32_t)__shfl_xor((int)fl, 4, 64);
    fl |= (uint32_t)__shfl_xor((int)fl, 8, 64);
    fl |= (uint32_t)__shfl_xor((int)fl, 16, 64);
    fl |= (uint32_t)__shfl_xor((int)fl, 32, 64);
    const uint64_t has = __builtin_amdgcn_ballot_w64(cnt != 0);
    uint32_t wf = 0x100u, wl = 0x100u;  // 0x100: no symbol in the wave
    if (has) {
        wf = (uint32_t)__shfl((int)w.first, (int)__builtin_ctzll(has), 64) & 0xFFu;
        wl = (uint32_t)__shfl((int)w.last, 63 - (int)__builtin_clzll(has), 64) & 0xFFu;
    }
    const uint32_t wtot = (uint32_t)__builtin_amdgcn_readlane((int)(place + cnt), 63);
    if (lane == 0u) {
        sx[1][wave] = wtot;
        sx[2][wave] = wf;
        sx[3][wave] = wl;
        sx[4][wave] = fl;
    }
    __syncthreads();
    uint32_t pre = 0, total = 0, F = 0, first = 0x100u, last = 0x100u;
#pragma unroll
    for (uint32_t k = 0; k < (uint32_t)W; ++k) {
        const uint32_t v = sx[1][k];
        pre += k < wave ? v : 0u;
        total += v;
        F |= sx[4][k];
        first = first == 0x100u ? sx[2][k] : first;
        last = sx[3][k] != 0x100u ? sx[3][k] : last;
    }
    first &= 0xFFu;
    last &= 0xFFu;
    const bool ok = !(F & 4u) && (F & 8u);
    {
        const bool em = ok && act && cnt != 0;
        RegSink sink;
        sink.init(dst + pre + place);
        (void)walk(Emit{}, w.f, w.f, pstop, em, sink);
        if (em) sink.finish();
    }
    ol = ok ? total : kFailLen;
    st = ok ? soft_bits(is_name, total, F & 3u, first, last) : kStatusFail;
}

// BIG: the block list (a block per string), else the one-wave list
template <int WAVES, bool BIG>
__global__ __launch_bounds__(WAVES * 64) void split_decode_kernel(DecArgs A) {
    __shared__ __attribute__((aligned(16))) uint32_t s_lut[1u << HHUFF_LUT_BITS];
    __shared__ uint32_t s_kinfo[32];
    __shared__ uint32_t s_ones[HHUFF_ONES_NENT];
    __shared__ uint32_t s_win[WAVES * 64][kSplitNW + 1];
    __shared__ uint32_t s_x[5][WAVES];
    const uint32_t nl = BIG ? 0u : min(*A.split_n, A.split_cap);
    const uint32_t nb = BIG ? min(*A.big_n, A.big_cap) : 0u;
    if (blockIdx.x * WAVES >= nl && blockIdx.x >= nb) return;  // (block-uniform) nothing listed for it
    load_dec_tables(s_lut, s_kinfo, s_ones, WAVES * 64);
    __syncthreads();
    const DecTables T{s_lut, s_kinfo, s_ones};
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
    const GlobalSource src{A.in, A.in_size};
    for (uint32_t j = blockIdx.x; j < nb; j += gridDim.x) {  // block-uniform: the big strings, a block each
        const uint32_t i = A.big_list[j];
        const uint32_t s = A.in_off[i];
        const uint32_t len = A.in_len ? A.in_len[i] : A.in_off[i + 1] - s;
        const bool is_name = A.is_name_bits ? ((A.is_name_bits[i >> 5] >> (i & 31)) & 1u) : false;
        const uint64_t d = A.out_off ? (uint64_t)A.out_off[i] : dec_slot(s);
        uint32_t ol;
        uint8_t st;
        split_decode_block<WAVES>(src, s, len, is_name, A.out + d, T, s_win[threadIdx.x], s_x, ol, st);
        if (threadIdx.x == 0) {
            A.out_len[i] = ol;
            A.status[i] = st;
        }
    }
    for (uint32_t j = blockIdx.x * WAVES + wave; j < nl; j += gridDim.x * WAVES) {  // the one-wave strings
        const uint32_t i = A.split_list[j];
        const uint32_t s = A.in_off[i];
        const uint32_t len = A.in_len ? A.in_len[i] : A.in_off[i + 1] - s;  // split_min <= len <= kMaxStrLen
        const bool is_name = A.is_name_bits ? ((A.is_name_bits[i >> 5] >> (i & 31)) & 1u) : false;
        const uint64_t d = A.out_off ? (uint64_t)A.out_off[i] : dec_slot(s);
        uint32_t ol;
        uint8_t st;
        split_decode_wave(src, s, len, is_name, A.out + d, T, lane, ol, st, s_win[threadIdx.x]);
        if (lane == 0) {
            A.out_len[i] = ol;
            A.status[i] = st;
        }
    }
}

// ------------------------------------------------------------------------------------------------
// Streaming decode (long and mixed lengths).  The staged kernels give a tile of 64 strings one lane
// each and run it as long as its longest string; with Zipf-like lengths (c3) a tile idles most of its
// lanes, and strings longer than a stage share fall back to decode_direct_kernel.  Here every lane owns
// one string at a time and a private window: NW input dwords and an OUT-byte output buffer in LDS.
// A round
//   1. gives idle lanes the next strings of the wave's batch (waves take batches of 64 from a global
//      counter, so waves finish together too);
//   2. loads each lane's next window: NW dwords from its current byte (dword-aligned), byte-swapped;
//   3. runs v7 bulk steps as far as the window allows (or to 27 bits before the string end) and, where
//      the string ends inside the window, v5's checked tail with the padding rule (hpack.c:132-133);
//   4. flushes the lane's whole output chunks with 16-B stores at 16-B aligned destinations -- the LDS
//      buffer holds byte g of the output at offset g % 16 -- and carries the partial last chunk over;
//      a string's first (head) and last (tail) chunks are written byte / dword-wise, only the bytes it
//      produced, so neighbouring slots are never touched.
// Lanes share nothing but the tables: no barriers, and a lane never waits for another lane's string.
// Same results as decode_core (hpack.c:117-156) for every layout (implicit slots, pairs, explicit dst).
// ------------------------------------------------------------------------------------------------

// bytes [lo, hi) of the 16-B LDS chunk `c` to global `g` (16-B aligned): whole dwords as dword stores, the
// partial dword at each end (at most 3 bytes each) as byte stores -- a fixed set of at most 10 predicated
// stores, where per-dword byte loops issued up to 16 (the wave runs the union of its lanes' paths)
__device__ __forceinline__ void store_range16(uint8_t* __restrict__ g, const uint8_t* c, uint32_t lo, uint32_t hi) {
    const uint4 v = *reinterpret_cast<const uint4*>(c);
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (uint32_t k = 0; k < 4; ++k)
        if (lo <= 4u * k && 4u * k + 4u <= hi) *reinterpret_cast<uint32_t*>(g + 4u * k) = w[k];
    const uint64_t q0 = (uint64_t)v.y << 32 | v.x, q1 = (uint64_t)v.w << 32 | v.z;
    auto byte_at = [&](uint32_t a) { return (uint32_t)((a < 8u ? q0 : q1) >> (8u * (a & 7u))); };
    const uint32_t e0 = min(hi, (lo + 3u) & ~3u);            // head partial dword: [lo, e0)
    const uint32_t s1 = max(max(lo, hi & ~3u), e0);           // tail partial dword: [s1, hi)
#pragma unroll
    for (uint32_t j = 0; j < 3; ++j) {
        if (lo + j < e0) g[lo + j] = (uint8_t)byte_at(lo + j);
        if (s1 + j < hi) g[s1 + j] = (uint8_t)byte_at(s1 + j);
    }
}

// 1: the prefetched window lands before the flush stores, removing the loop-top wait that also waits for them.
// Measured slower (c3 decode 0.293 -> 0.296 ms, c5 0.426 -> 0.449, profiles/r04ak_stream_early_ab.log): the
// window's loads, not the stores, are what that wait is for, and landing them earlier only shortens their time
#ifndef HHUFF_STREAM_EARLY
#define HHUFF_STREAM_EARLY 0
#endif
#ifndef HHUFF_STREAM_TAILWHOLE  // 1 (default): a string's last output chunk as one 16-B store when it lies in the
#define HHUFF_STREAM_TAILWHOLE 1  // string's own slot: c3 decode -1.1 %, c5 -1.5 %, write traffic unchanged
#endif                            // (profiles/r06i_stream_tail_whole_ab.jsonl, r06i_c3_decode_pmc.txt)

// SEG: flush granularity -- whole SEG-byte aligned output segments leave before a string's end
template <int WAVES, int NW, int OUT, int SEG = 16>
__global__ __launch_bounds__(WAVES * 64) void decode_stream_kernel(DecArgs A, unsigned long long* __restrict__ counter) {
    static_assert(NW >= 8 && NW % 4 == 0 && OUT % 16 == 0, "window shape");
    // per round a lane consumes <= 32 (NW - 2) bits: <= 32 (NW - 2) / 5 symbols after <= 15 carried bytes,
    // plus the byte the second-symbol store may touch; the last byte of the buffer is the trash byte
    static_assert(SEG >= 16 && (SEG & (SEG - 1)) == 0 && SEG - 1 + (32 * (NW - 2)) / 5 + 2 < OUT,
                  "output buffer too small for a window");
    constexpr uint32_t kWS = NW + 1;  // odd dword stride: lanes at the same q hit distinct banks
    struct __attribute__((aligned(16))) Smem {
        uint32_t lut[1u << HHUFF_LUT_BITS];
        uint32_t kinfo[32];
        uint32_t ones[(HHUFF_ONES_NENT + 3) & ~3];
        uint8_t out[WAVES * 64][OUT];
        uint32_t win[WAVES * 64][kWS];  // [0]: the dword before the window (read, never used)
    };
    if (A.gate && *A.gate != kGateStream) return;  // block-uniform: decode_select_kernel chose the staged kernel
    __shared__ Smem sm;
    load_dec_tables(sm.lut, sm.kinfo, sm.ones, WAVES * 64);
    __syncthreads();
    const DecTables T{sm.lut, sm.kinfo, sm.ones};
    const int lane = threadIdx.x & 63;
#if HHUFF_STREAM_TAILWHOLE
    const bool slots = A.out_off == nullptr && A.in_len == nullptr;  // implicit output slots floor(8 in_off / 5)
#endif
    uint32_t* win = &sm.win[threadIdx.x][1];
    const lds_u32* st = (const lds_u32*)win;
    uint8_t* obuf = sm.out[threadIdx.x];
    const uint32_t ob = lds_addr(obuf), trash = ob + OUT - 1u;
    constexpr int32_t kLimW = 32 * (NW - 2) - 30;  // bulk steps start below this window bit
    constexpr int32_t kFinal = 32 * (NW - 2);      // a string ending at or before this bit ends in the window

    // per-lane string state
    uint4 pfv[NW / 4];       // the prefetched next window (its input address: pfa)
    uint64_t pfa = ~0ull;
    bool busy = false, head = false, is_name = false;
    uint32_t i = 0, s = 0, len = 0, P = 0, ocnt = 0, flags = 0, first = 0, lastb = 0, fail = 0;
    uint64_t dst = 0;
    // wave batch
    uint64_t bnext = 0, bend = 0;
    bool qdone = false;
    const uint64_t nwork = A.n_dev ? (uint64_t)*A.n_dev : (uint64_t)A.n;
    PROF_DECL  // profile builds: phases take / window / bulk / tail / flush in slot 0 (the staged kernel's)

    for (;;) {
        // ---- 1. idle lanes take strings ----
        for (int it = 0; it < 2; ++it) {
            const uint64_t need = __builtin_amdgcn_ballot_w64(!busy);
            if (need == 0) break;
            if (bnext >= bend) {
                if (qdone) break;
                uint64_t b = 0;
                if (lane == 0) b = atomicAdd(counter, (unsigned long long)A.claim);
                b = ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(b >> 32)) << 32) |
                    (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)b);
                if (b >= nwork) {
                    qdone = true;
                    break;
                }
                bnext = b;
                bend = min(b + A.claim, nwork);
            }
            const uint32_t rank = (uint32_t)__builtin_amdgcn_mbcnt_hi((uint32_t)(need >> 32),
                                                                      __builtin_amdgcn_mbcnt_lo((uint32_t)need, 0u));
            if (!busy && bnext + rank < bend) {
                i = (uint32_t)(bnext + rank);
                s = A.in_off[i];
                len = A.in_len ? A.in_len[i] : A.in_off[i + 1] - s;
                is_name = A.is_name_bits ? ((A.is_name_bits[i >> 5] >> (i & 31)) & 1u) : false;
                dst = A.out_off ? (uint64_t)A.out_off[i] : dec_slot(s);
                if (len > kMaxStrLen) {
                    A.out_len[i] = kFailLen;
                    A.status[i] = kStatusTooLong;
                } else if (!split_push(A, i, len)) {
                    busy = true;
                    head = (dst & (SEG - 1u)) != 0;
                    P = ocnt = flags = first = lastb = fail = 0;
                }
            }
            bnext = min(bend, bnext + (uint64_t)__builtin_popcountll(need));
        }
        if (!__any(busy)) {
            if (qdone) {
                PROF_FLUSH(0);
                break;
            }
            continue;
        }
        PROF_MARK(0);

        // ---- 2. the lane's window: NW dwords from its current byte (dword-aligned) ----
        // A round that does not finish its string stops with its next byte at wb + 4 (NW - 3) (bulk steps
        // run to bit 32 (NW - 2) - 30 and overshoot by < 32), so that window was prefetched into registers
        // at the start of the round before: its loads had the whole round to land.
        const uint64_t cur = (uint64_t)s + (P >> 3);
        const uint64_t wb = cur & ~3ull;
        const uint64_t rem = (uint64_t)len * 8u - P;  // string bits left
        if (busy) {
            if (wb != pfa) {
#pragma unroll
                for (int j = 0; j < NW / 4; ++j) pfv[j] = load16_bounded(A.in, A.in_size, wb + 16u * j);
            }
#pragma unroll
            for (int j = 0; j < NW / 4; ++j) {
                win[4 * j + 0] = bswap32(pfv[j].x);
                win[4 * j + 1] = bswap32(pfv[j].y);
                win[4 * j + 2] = bswap32(pfv[j].z);
                win[4 * j + 3] = bswap32(pfv[j].w);
            }
            // the string goes on past this window: fetch the next one now
            pfa = rem + 8u * (uint32_t)(cur - wb) + (P & 7u) > 32u * (NW - 2) ? wb + 4u * (NW - 3) : ~0ull;
            if (pfa != ~0ull) {
#pragma unroll
                for (int j = 0; j < NW / 4; ++j) pfv[j] = load16_bounded(A.in, A.in_size, pfa + 16u * j);
            }
        }
        int32_t pm = busy ? (int32_t)(8u * (uint32_t)(cur - wb) + (P & 7u)) - 1 : -1;
        const int32_t pm0 = pm;
        PROF_MARK(1);
        const int32_t end = busy ? (int32_t)min((uint64_t)(pm + 1) + rem, (uint64_t)0x40000000u) : 0;
        const bool fin = busy && end <= kFinal;
        const uint32_t h0 = (uint32_t)((dst + ocnt) & (SEG - 1u));  // buffer offset of this round's first byte
        uint32_t o = ob + h0;
        int32_t q = pm >> 5;
        uint32_t x0 = st[q], x1 = st[q + 1], x2 = st[q + 2];
        uint32_t accb = 0, acc1 = 0, acc2 = 0, accl = 0, parked = busy ? 0u : 1u;
        int32_t lim = busy ? min(end - 26, kLimW) : (int32_t)0x80000000;
        auto advance = [&](int32_t cons) {
            pm += cons;
            const int32_t qn = pm >> 5;
            const bool adv = qn != q;
            x0 = adv ? x1 : x0;
            x1 = adv ? x2 : x1;
            q = qn;
            x2 = st[q + 2];
        };

        // ---- 3a. bulk (decode_staged_lane_v7's step) ----
        auto bstep = [&](bool longchk) {
            if (pm < lim) {
                const uint32_t w = __builtin_amdgcn_alignbit(x0, x1, ~(uint32_t)pm);
                const uint32_t e = T.lut[w >> (32 - HHUFF_LUT_BITS)];
                const uint32_t sl = (uint32_t)((int32_t)e >> 31);
                uint32_t cons = lut_l12(e);  // LONG entries carry L12 = 0
#if HHUFF_DEC_READ_FIRST
                {  // the second lookup ahead of the first entry's byte stores (decode_staged_lane_v7)
                    const uint32_t wb2 = w << cons;
                    const uint32_t eb = T.lut[wb2 >> (32 - HHUFF_LUT_BITS)];
                    bulk_put2(o, e, trash);
                    o += (e >> 28) & 3u;
                    accb |= e;
                    bulk_put2(o, eb, trash);
                    o += (eb >> 28) & 3u;
                    accb |= eb;
                    cons += lut_l12(eb);
                }
#else
                bulk_put2(o, e, trash);
                o += (e >> 28) & 3u;
                accb |= e;
                {
                    const uint32_t wb2 = w << cons;
                    const uint32_t eb = T.lut[wb2 >> (32 - HHUFF_LUT_BITS)];
                    bulk_put2(o, eb, trash);
                    o += (eb >> 28) & 3u;
                    accb |= eb;
                    cons += lut_l12(eb);
                }
#endif
                if (longchk && __builtin_amdgcn_ballot_w64(sl != 0u) != 0) {
                    if (sl) {
                        const uint32_t k = min((uint32_t)__builtin_clz(~w | 1u), 30u);
                        const uint32_t ki = T.kinfo[k];
                        const uint32_t le = T.ones[(ki & 0xFFFFu) + (((w << (k + 1)) >> 1) >> (31 - (ki >> 16)))];
                        const int32_t L = (le >> 9) & 31u;
                        const uint32_t fits = (uint32_t)((L + pm - end) >> 31);
                        const uint32_t eos = (le & 0x1FFu) == kEos ? 0xFFFFFFFFu : 0u;
                        const uint32_t okm = fits & ~eos;
                        fail |= fits & eos & 1u;  // EOS inside the string (hpack.c:88-89)
                        lds_st8(sel_bits(okm, o, trash), le);
                        o -= okm;
                        accl |= le & okm;
                        cons = okm & (uint32_t)L;
                        parked |= ~okm & 1u;
                        lim = (int32_t)sel_bits(okm, (uint32_t)lim, 0x80000000u);
                    }
                }
                advance((int32_t)cons);
            }
        };
        for (;;) {
            bstep(false);
            bstep(true);
            if (!__any(pm < lim)) break;
        }
        PROF_MARK(2);

        // ---- 3b. tail: lanes whose string ends in this window ----
        int32_t c = (fin && !parked) ? pm - end : 0x40000000;
        if (__any(fin)) {
            int32_t prog = 0;
            auto step = [&](bool longchk) {
                const uint32_t w = __builtin_amdgcn_alignbit(x0, x1, ~(uint32_t)pm);
                const uint32_t e = T.lut[w >> (32 - HHUFF_LUT_BITS)];
                const int32_t L1 = lut_l1(e), L12 = lut_l12(e);
                const int32_t s1 = L1 + c, s2 = L12 + c;
                const uint32_t m1 = (uint32_t)((s1 & ~(int32_t)e) >> 31);
                const uint32_t m2 = (uint32_t)((s2 & (int32_t)(e << 1)) >> 31);
                int32_t cons = (int32_t)sel_bits(m2, (uint32_t)L12, m1 & (uint32_t)L1);
                lds_st8(sel_bits(m1, o - m2, trash), lut_sym2(e));
                lds_st8(sel_bits(m1, o, trash), e);
                o = o - m1 - m2;
                acc1 |= e & m1;
                acc2 |= e & m2;
                {
                    const uint32_t wb2 = w << cons;
                    const uint32_t eb = T.lut[wb2 >> (32 - HHUFF_LUT_BITS)];
                    const int32_t cb = c + cons;
                    const int32_t L1b = lut_l1(eb), L12b = lut_l12(eb);
                    const uint32_t m1b = (uint32_t)(((L1b + cb) & ~(int32_t)eb) >> 31);
                    const uint32_t m2b = (uint32_t)(((L12b + cb) & (int32_t)(eb << 1)) >> 31);
                    lds_st8(sel_bits(m1b, o - m2b, trash), lut_sym2(eb));
                    lds_st8(sel_bits(m1b, o, trash), eb);
                    o = o - m1b - m2b;
                    acc1 |= eb & m1b;
                    acc2 |= eb & m2b;
                    cons += (int32_t)sel_bits(m2b, (uint32_t)L12b, m1b & (uint32_t)L1b);
                }
                const bool lact = (s1 & (int32_t)e) < 0;
                uint32_t consl = 0;
                if (longchk && __builtin_amdgcn_ballot_w64(lact) != 0) {
                    if (lact) {
                        const uint32_t k = min((uint32_t)__builtin_clz(~w | 1u), 30u);
                        const uint32_t ki = T.kinfo[k];
                        const uint32_t le = T.ones[(ki & 0xFFFFu) + (((w << (k + 1)) >> 1) >> (31 - (ki >> 16)))];
                        const int32_t L = (le >> 9) & 31u;
                        const uint32_t fits = (uint32_t)((L + c) >> 31);
                        const uint32_t eos = (le & 0x1FFu) == kEos ? 0xFFFFFFFFu : 0u;
                        const uint32_t okm = fits & ~eos;
                        fail |= fits & eos & 1u;
                        lds_st8(sel_bits(okm, o, trash), le);
                        o -= okm;
                        accl |= le & okm;
                        consl = okm & (uint32_t)L;
                        c = (int32_t)sel_bits(okm, (uint32_t)c, 0x40000000u);
                    }
                }
                cons |= (int32_t)consl;
                c += cons;
                advance(cons);
                prog = cons;
            };
            step(true);
            for (;;) {
                step(false);
                step(true);
                if (!__any(prog != 0)) break;
            }
        }

        PROF_MARK(3);
#if HHUFF_STREAM_EARLY
        // land the prefetched window before this round's flush stores: loads and stores share one in-order
        // counter on gfx950, so a wait for it next round, behind the stores, would wait for them too
#pragma unroll
        for (int j = 0; j < NW / 4; ++j) {
            uint32_t a0 = pfv[j].x, a1 = pfv[j].y, a2 = pfv[j].z, a3 = pfv[j].w;
            asm volatile("" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3) :: "memory");
            pfv[j] = make_uint4(a0, a1, a2, a3);
        }
#endif
        // ---- 4. flush whole chunks, carry the partial one; finish strings ----
        if (busy) {
            flags |= ((accb >> 24) | (accb >> 26) | (acc1 >> 24) | (acc2 >> 26) | (accl >> 14)) & 3u;
            const uint32_t nb = o - ob;  // buffer bytes: h0 carried (or, at a string's start, foreign) + produced
            const uint32_t made = nb - h0;
            if (made) {
                if (ocnt == 0) first = obuf[h0];
                lastb = obuf[nb - 1u];
            }
            const bool done = parked || fin;
            const bool ok = fin && !parked && !fail && [&] {
                const uint32_t R = ~(uint32_t)c;
                const uint32_t w = __builtin_amdgcn_alignbit(x0, x1, ~(uint32_t)pm);
                return R <= 7 && (w | (0xFFFFFFFFu >> (R & 31u))) == 0xFFFFFFFFu;
            }();
            uint8_t* gchunk = A.out + ((dst + ocnt) & ~(uint64_t)(SEG - 1));
            const uint32_t hs = head ? (uint32_t)(dst & (SEG - 1u)) : 0u;  // head segment: the string starts here
#ifdef HHUFF_X_NOSTORE
            if (false) {
#else
            if (!done || ok) {  // a failed string's output is unspecified: skip its last stores
#endif
                // whole 16-B chunks now: all of them at the string's end, else those of whole segments
                const uint32_t nfull = done ? nb >> 4 : (nb / SEG) * (SEG / 16u);
                for (uint32_t k = 0; k < nfull; ++k) {
                    const uint32_t c0 = 16u * k;
                    if (c0 + 16u <= hs) continue;  // foreign bytes before the string
                    if (c0 < hs)
                        store_range16(gchunk + c0, obuf + c0, hs - c0, 16u);
                    else
#if HHUFF_STREAM_NT  // A/B: the flush's whole chunks as streaming stores
                        st16_out(gchunk + c0, *reinterpret_cast<const uint4*>(obuf + c0));
#else
                        *reinterpret_cast<uint4*>(gchunk + c0) = *reinterpret_cast<const uint4*>(obuf + c0);
#endif
                }
                const uint32_t c0 = 16u * nfull;
                if (done) {
                    const uint32_t lo = hs > c0 ? hs - c0 : 0u;
#if HHUFF_STREAM_TAILWHOLE
                    // implicit slots: the last chunk goes out whole when all of it lies in this string's slot (the
                    // bytes past the output are the slot's unused tail, unspecified) -- one 16-B store, not <= 10
                    const bool whole = slots && lo == 0u && nb > c0 &&
                                       (uint64_t)(gchunk - A.out) + c0 + 16u <= dec_slot((uint64_t)s + len);
                    if (whole)
                        *reinterpret_cast<uint4*>(gchunk + c0) = *reinterpret_cast<const uint4*>(obuf + c0);
                    else
#endif
                    if (nb - c0 > lo) store_range16(gchunk + c0, obuf + c0, lo, nb - c0);
                } else if (nfull) {  // carry the partial segment to the buffer's start
                    head = false;
                    for (uint32_t r = 0; c0 + 16u * r < nb; ++r)
                        *reinterpret_cast<uint4*>(obuf + 16u * r) = *reinterpret_cast<const uint4*>(obuf + c0 + 16u * r);
                }
            }
            ocnt += made;
            P += (uint32_t)(pm - pm0);
            if (done) {
#ifndef HHUFF_X_NOSTORE
                A.out_len[i] = ok ? ocnt : kFailLen;
                A.status[i] = ok ? soft_bits(is_name, ocnt, flags, first, lastb) : kStatusFail;
#endif
                busy = false;
            }
        }
        PROF_MARK(4);
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
    EdgeRec* edges;  // region layout, encode_staged_kernel: 2 records per 64-string tile, or NULL
    uint32_t* pk_off;  // packed mode (encode_staged_kernel<.., true>): u32[n + 1] output places
};

__device__ __forceinline__ void load_enc_table(uint2* s_enc, int nthreads) {
    for (uint32_t k = threadIdx.x; k < 256; k += nthreads) s_enc[k] = make_uint2(g_enc_code[k], g_enc_nbits[k]);
}

__device__ __forceinline__ void finish_encode(const EncArgs& A, uint32_t i, uint32_t len, uint32_t ol) {
    st_res(A.out_len + i, ol);
    if (A.status) st_res(A.status + i, (uint8_t)(ol == kFailLen ? (len > kMaxStrLen ? kStatusTooLong : kStatusFail) : 0));
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

// Packed output (PACKED, contiguous layout): as decode_staged_kernel's -- the tile's encoded strings back to
// back in string order from G = in_off[first string of the tile], failed strings taking no bytes.  The
// strings are encoded into their slots (the output stage mirrors the input) and then moved to their places
// in the input stage, which is free once the tile is encoded (the next span is committed after the
// stores); no two regions overlap, so one pass suffices.
template <int WAVES, int STAGE, bool PACKED>
__global__ __launch_bounds__(WAVES * 64) void encode_staged_kernel(EncArgs A) {
    __shared__ __attribute__((aligned(16))) uint2 s_enc[512];  // 256..511: bytes outside a string
    // + 32 B: a packed run starts up to 15 B into the stage and its last 16-B chunk may end 15 B past it
    __shared__ __attribute__((aligned(16))) uint32_t s_in[WAVES][STAGE / 4 + 8];
    __shared__ __attribute__((aligned(16))) uint32_t s_out[WAVES][STAGE / 4 + 4];
    for (uint32_t k = threadIdx.x; k < 512; k += WAVES * 64)
        s_enc[k] = k < 256 ? make_uint2(g_enc_code[k], g_enc_nbits[k]) : make_uint2(0u, 0u);
    __syncthreads();
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint32_t* stage = s_in[wave];
    uint32_t* obuf32 = s_out[wave];
    const uint8_t* obuf = reinterpret_cast<const uint8_t*>(obuf32);
    const bool region = A.in_len == nullptr && A.out_off == nullptr;
    const bool pairs = A.in_len != nullptr;
    const uint64_t stride = (uint64_t)gridDim.x * WAVES * 64;
    uint64_t base = ((uint64_t)blockIdx.x * WAVES + wave) * 64;
    if (base >= A.n) return;

    struct Plan {
        Tile t;
        uint32_t a0, span, op0, ospan;
        uint64_t dst_g;
        bool fits;
    };
    auto plan = [&](uint64_t b, const TileIn& ti) {
        Plan P;
        P.t = finish_tile(b, lane, A.n, ti, pairs);
        const Tile& t = P.t;
        P.a0 = t.lo & ~15u;
        P.span = t.hi > t.lo ? ((t.hi + 15u) & ~15u) - P.a0 : 0u;
        P.dst_g = 0;
        if (region) {  // output slot = input offset: the output stage mirrors the input stage
            P.ospan = P.span;
            P.op0 = t.len ? t.s - P.a0 : 0u;
        } else {
            P.dst_g = A.out_off ? (uint64_t)ti.dst : (uint64_t)t.s;
            const uint32_t cap = t.valid ? min(t.len, kMaxStrLen) + 3u : 0u;
            const uint32_t pre = wave_excl_scan(cap, lane);
            P.ospan = (uint32_t)__builtin_amdgcn_readlane((int)(pre + cap), 63);
            P.op0 = pre + ((uint32_t)(((uintptr_t)A.out + P.dst_g) - pre) & 3u);
        }
        P.fits = P.span <= STAGE && P.ospan <= STAGE;
        return P;
    };

    // Software pipeline: cur = being encoded (span in the stage), nxt = planned, span in flight in pf,
    // ti = offsets of the tile after nxt.  Every wait on a global load sits between a tile's encode and its
    // stores, never right after stores: vmcnt counts stores too, so a load consumed after the stores
    // would wait for their writes to land.
    SpanPrefetch<(STAGE + 1023) / 1024> pf;
    TileIn ti = issue_tile(base, lane, A.n, A.in_off, A.in_len, nullptr, A.out_off);
    Plan cur = plan(base, ti);
    if (cur.fits) pf.issue(A.in, A.in_size, cur.a0, cur.span, lane);
    ti = issue_tile(base + stride, lane, A.n, A.in_off, A.in_len, nullptr, A.out_off);
    if (cur.fits) pf.commit(stage, A.in, A.in_size, cur.a0, cur.span, lane);
    Plan nxt;
    bool nxt_pf = false;  // nxt's span is in pf (issued, not committed)
    if (base + stride < A.n) {
        nxt = plan(base + stride, ti);
        if (nxt.fits) {
            pf.issue(A.in, A.in_size, nxt.a0, nxt.span, lane);
            nxt_pf = true;
        }
    }
    PROF_DECL
    for (;;) {
        const uint64_t nbase = base + stride;
        const bool have_next = nbase < A.n, have_nn = nbase + stride < A.n;
        ti = issue_tile(nbase + stride, lane, A.n, A.in_off, A.in_len, nullptr, A.out_off);  // clamped: always safe
        Plan nn;
        bool nn_pf = false, advanced = false;
        // commit nxt's span into the (free) stage, then plan the tile after it and put its span in flight
        auto advance = [&]() {
            PROF_MARK(2);
            if (nxt_pf) pf.commit(stage, A.in, A.in_size, nxt.a0, nxt.span, lane);
            PROF_MARK(3);  // commit
            nn = plan(nbase + stride, ti);  // on every path: ti is consumed at one place (see issue_tile)
            if (have_nn && nn.fits) {
                pf.issue(A.in, A.in_size, nn.a0, nn.span, lane);
                nn_pf = true;
            }
            PROF_MARK(7);  // plan + issue of the tile after next
            advanced = true;
        };
        // ---- the current tile ----
        const Tile& t = cur.t;
        uint32_t ol = kFailLen;
        PROF_MARK(0);
        if (cur.fits) {
            {
                for (uint32_t k = (uint32_t)lane * 16u; k < cur.ospan + 16u; k += 64u * 16u)
                    *reinterpret_cast<uint4*>(reinterpret_cast<uint8_t*>(obuf32) + k) = make_uint4(0u, 0u, 0u, 0u);
                wave_lds_sync();
                const bool act = t.valid && t.len != 0 && t.len <= kMaxStrLen;
                const uint32_t rel = t.len ? t.s - cur.a0 : 0u;
                const uint32_t last = cur.span ? cur.span - 4u : 0u;
                const uint32_t tb = encode_chunk_v2<HHUFF_ENC_OTHER_U>(stage, last, rel, t.len, act, lds_addr(obuf32), 8u * cur.op0, s_enc,
                                                    act ? 8 * t.len - 7 : 0xFFFFFFFFu, true);
                const uint32_t r = tb == kFailLen ? kFailLen : (tb + 7) >> 3;
                if (act) ol = r;
            }
            PROF_MARK(1);
            if constexpr (PACKED) {
                // the run goes to the input stage (free now), byte-swapped on the way (no stage_bswap pass)
                const uint32_t keep = ol != kFailLen ? ol : 0u;
                const uint32_t place = wave_excl_scan(keep, lane);
                const uint32_t T_run = (uint32_t)__builtin_amdgcn_readlane((int)(place + keep), 63);
                const uint64_t G = (uint32_t)__builtin_amdgcn_readfirstlane((int)t.s);
                const uint32_t g15 = (uint32_t)G & 15u;
                lds_zero(reinterpret_cast<uint8_t*>(stage), 0u, (g15 + T_run + 15u) & ~15u, lane);
                wave_lds_sync();
                lds_move_or<true>(lds_addr(obuf) + cur.op0, lds_addr(stage) + g15 + place, keep);
                wave_lds_sync();
                PROF_MARK(2);
                PROF_MARK(3);
                const uint64_t gb = G & ~15ull;
                const uint32_t ps = (uint32_t)(((G + T_run + 15u) & ~15ull) - gb);
                if (A.edges)
                    region_copy_deferred(A.out, gb, reinterpret_cast<const uint8_t*>(stage), ps, G, G + T_run, lane,
                                         A.edges + 2 * (base >> 6));
                else
                    region_copy<(STAGE + 1023) / 1024>(A.out, gb, reinterpret_cast<const uint8_t*>(stage), ps, G, G + T_run,
                                                       lane);
                if (t.valid) {
                    A.pk_off[t.i] = (uint32_t)(G + place);
                    if (t.i == A.n - 1) A.pk_off[A.n] = (uint32_t)(G + place + keep);
                }
            } else {
                // the input stage is free: commit the next span and plan the one after BEFORE this tile's
                // stores, so their vmcnt waits cover loads issued a tile ago, not the stores
                advance();
                wave_lds_sync();
                if (!(region && A.edges)) stage_bswap(obuf32, (cur.ospan + 15u) & ~15u, lane);
                wave_lds_sync();
                PROF_MARK(2);
            }
            if (PACKED) {
            } else if (region) {
                if (A.edges)  // the stage's MSB-first words are byte-swapped on the way out
                    region_copy_deferred<true>(A.out, cur.a0, obuf, cur.ospan, t.lo, t.hi, lane, A.edges + 2 * (base >> 6));
                else
                    region_copy<(STAGE + 1023) / 1024>(A.out, cur.a0, obuf, cur.ospan, t.lo, t.hi, lane);
            } else if (t.valid && ol != kFailLen) {
                lane_copy(A.out + cur.dst_g, obuf + cur.op0, ol);
            }
            wave_lds_sync();
            PROF_MARK(4);
        } else if (PACKED) {
            // a tile larger than the stage: code lengths first (they fix the places), then encode into place
            const GlobalSource src{A.in, A.in_size};
            const bool cand = t.valid && t.len != 0 && t.len <= kMaxStrLen;
            const uint32_t bits = cand ? count_code_bits(src, t.s, t.len, s_enc) : 0u;
            const bool ok = cand && bits <= 8u * t.len - 8u;  // ceil(bits / 8) < len (hpack.c:799-800)
            const uint32_t keep = ok ? (bits + 7u) >> 3 : 0u;
            if (ok) ol = keep;
            RegSink sink;
            const uint32_t place = wave_excl_scan(keep, lane);
            const uint64_t G = (uint32_t)__builtin_amdgcn_readfirstlane((int)t.s);
            if (ok) {
                sink.init(A.out + G + place);
                (void)encode_core(src, t.s, t.len, sink, s_enc);
            }
            if (t.valid) {
                A.pk_off[t.i] = (uint32_t)(G + place);
                if (t.i == A.n - 1) A.pk_off[A.n] = (uint32_t)(G + place + keep);
            }
            PROF_MARK(6);
        } else if (t.valid && t.len <= kMaxStrLen) {
            RegSink sink;
            sink.init(A.out + (A.out_off ? cur.dst_g : (uint64_t)t.s));
            ol = encode_core(GlobalSource{A.in, A.in_size}, t.s, t.len, sink, s_enc);
            PROF_MARK(6);
        }
        if (!cur.fits && A.edges && lane == 0) {  // direct path: no edges to defer
            A.edges[2 * (base >> 6)].m = make_uint4(0u, 0u, 0u, 0u);
            A.edges[2 * (base >> 6) + 1].m = make_uint4(0u, 0u, 0u, 0u);
        }
        if (t.valid) finish_encode(A, t.i, t.len, ol);
        PROF_MARK(5);
        if (!have_next) {
            PROF_FLUSH(1);
            break;
        }
        if (!advanced) advance();  // packed mode (the stage held the compaction) and direct tiles
        cur = nxt;
        nxt = nn;
        nxt_pf = nn_pf;
        base = nbase;
    }
}

// Length-sorted chunks (contiguous layout, deferred edges).  A staged tile of 64 consecutive strings runs
// as long as its longest string (U[24,72]: 71 of the mean 48 bytes' steps).  Here a workgroup stages the
// span of NS consecutive strings once (coalesced), counting-sorts their lengths in LDS and gives each of
// its waves 64 strings of about one length, so a wave's lock-step lasts about as long as its strings (wave
// w takes the w-th length group).  Two workgroups share a CU: while one waits at a barrier for its longest
// group, the other's waves keep the SIMDs busy.  Every string is encoded in place in the chunk's output
// stage (slot = input offset), which is then copied out whole.
constexpr uint32_t kSortBins = 128;  // whole dwords 0..126, and 127+
struct SortChunk {  // per thread: its string of a chunk and the chunk's input span
    uint32_t s, e, lo, hi;
};
__device__ __forceinline__ SortChunk sort_chunk_issue(const EncArgs& A, uint64_t cb, uint32_t t, uint32_t ns) {
    const uint64_t ic = min(cb + t, (uint64_t)A.n - 1u);  // clamped: every load issues
    return SortChunk{A.in_off[ic], A.in_off[ic + 1], A.in_off[min(cb, (uint64_t)A.n - 1u)],
                     A.in_off[min(cb + ns, (uint64_t)A.n)]};
}
#ifndef HHUFF_ENC_COPY_EARLY  // sorted encoder: the batched copy-out's reads issued right after barrier 3
#define HHUFF_ENC_COPY_EARLY 0
#endif
#ifndef HHUFF_ENC_SORTREC  // sorted encoder: one record read (place -> offset | length) before a lane's encode
#define HHUFF_ENC_SORTREC 0
#endif
#ifndef HHUFF_ENC_COPY_BATCH  // sorted encoder's copy-out: all LDS reads of a thread's chunks ahead of the stores
#define HHUFF_ENC_COPY_BATCH 1   // (c4 encode -2.0 %, c2 -3.8 %; 122 VGPRs, still 4 waves a SIMD: r06aa_encode_copy_batch_ab.jsonl)
#endif
#ifndef HHUFF_ENC_EARLY
// 1: the next chunk's offsets are loaded a chunk ahead and both they and the next span are waited for after
// barrier 3, before the chunk's stores (c4 encode 0.680 -> 0.655 ms, profiles/r04aa_encode_early_ab.log);
// 0: the round-3 order, where the compiler's vmcnt waits for those loads also waited for the stores
#define HHUFF_ENC_EARLY 1
#endif
// NS strings per chunk on NS / SPT threads (SPT strings a thread); CH bytes of stage.  SPT = 2 pairs the
// sorted ranks t and NS - 1 - t on thread t, so every lane encodes a short and a long string one after the
// other and the lanes' work (about twice the mean length) is even across the workgroup: no wave waits at the
// chunk's barriers for a longest length group.
#ifndef HHUFF_ENCO_SPT
#define HHUFF_ENCO_SPT 1
#endif
#ifndef HHUFF_ENCO_PAD  // A/B builds: extra LDS bytes per workgroup (fewer resident workgroups)
#define HHUFF_ENCO_PAD 0
#endif
template <int NS, int CH, int SPT = 1>
__global__ __launch_bounds__(NS / SPT) void encode_sorted_kernel(EncArgs A) {
    static_assert(SPT == 1 || SPT == 2, "one string a thread, or a sorted pair");
    constexpr uint32_t kSortStr = NS, NT = NS / SPT;
    constexpr int NV = (CH + 16 * NT - 1) / (16 * NT);  // 16-B span chunks per thread
    __shared__ __attribute__((aligned(16))) uint2 s_enc[512];  // 256..511: bytes outside a string
    __shared__ __attribute__((aligned(16))) uint32_t s_in[CH / 4 + 8];
    __shared__ __attribute__((aligned(16))) uint32_t s_out[CH / 4 + 8];
#if HHUFF_ENC_SORTREC
    // sorted place -> {offset in the span (14 bits) | length << 14}, written by the string's own thread once its
    // place is known, then overwritten with the encoded length (read back by that thread after barrier 3)
    static_assert(CH <= 16384, "14-bit span offsets");
    __shared__ uint32_t s_rec[kSortStr];
#else
    __shared__ uint2 s_str[kSortStr];  // {offset in the span, length} of chunk string t
    __shared__ uint16_t s_perm[kSortStr];
#endif
    __shared__ uint32_t s_bin[kSortBins];  // strings per bin, then the bins' first places
#if HHUFF_ENCO_PAD
    __shared__ uint32_t s_pad[HHUFF_ENCO_PAD / 4];
    if (A.n == 0xFFFFFFFFu) s_pad[threadIdx.x % (HHUFF_ENCO_PAD / 4)] = 0u;  // (never: keeps the bytes allocated)
#endif
    const uint32_t t = threadIdx.x, lane = t & 63u;
    for (uint32_t k = t; k < 512; k += NT) s_enc[k] = k < 256 ? make_uint2(g_enc_code[k], g_enc_nbits[k]) : make_uint2(0u, 0u);
    const uint64_t nch = ((uint64_t)A.n + kSortStr - 1) / kSortStr;
    uint64_t c = blockIdx.x;
    if (c >= nch) return;
    auto span_of = [](const SortChunk& q) { return q.hi > q.lo ? ((q.hi + 15u) & ~15u) - (q.lo & ~15u) : 0u; };
    auto issue_span = [&](uint4 (&v)[NV], const SortChunk& q) {
        const uint32_t a0 = q.lo & ~15u, span = span_of(q);
#pragma unroll
        for (int j = 0; j < NV; ++j) {
            const uint32_t k = (uint32_t)j * (16u * NT) + t * 16u;
            const uint64_t g = (uint64_t)a0 + k;
#if HHUFF_NT_LOAD
            if (k < span && span <= (uint32_t)CH && g + 16 <= A.in_size) {
                typedef unsigned int u32x4l __attribute__((ext_vector_type(4)));
                const u32x4l x = __builtin_nontemporal_load(reinterpret_cast<const u32x4l*>(A.in + g));
                v[j] = make_uint4(x.x, x.y, x.z, x.w);
            }
#else
            if (k < span && span <= (uint32_t)CH && g + 16 <= A.in_size) v[j] = *reinterpret_cast<const uint4*>(A.in + g);
#endif
        }
    };
    auto commit_span = [&](const uint4 (&v)[NV], const SortChunk& q) {
        const uint32_t a0 = q.lo & ~15u, span = span_of(q);
#pragma unroll
        for (int j = 0; j < NV; ++j) {
            const uint32_t k = (uint32_t)j * (16u * NT) + t * 16u;
            const uint64_t g = (uint64_t)a0 + k;
            if (k < span) *reinterpret_cast<uint4*>(reinterpret_cast<uint8_t*>(s_in) + k) =
                g + 16 <= A.in_size ? v[j] : load16_tail(A.in, A.in_size, g);
        }
    };
    auto issue_chunk = [&](SortChunk (&q)[SPT], uint64_t qb) {
#pragma unroll
        for (int u = 0; u < SPT; ++u) q[u] = sort_chunk_issue(A, qb, t + (uint32_t)u * NT, NS);
    };
    auto land = [](SortChunk (&q)[SPT]) {  // wait for a chunk's offsets here (see HHUFF_ENC_EARLY)
#pragma unroll
        for (int u = 0; u < SPT; ++u) __asm__ volatile("" : "+v"(q[u].s), "+v"(q[u].e), "+v"(q[u].lo), "+v"(q[u].hi) : : "memory");
    };
    for (uint32_t k = t; k < kSortBins; k += NT) s_bin[k] = 0u;  // then cleared by each chunk once every wave has read it
    __syncthreads();
    // prepare(q): chunk q's span into the input stage, the output stage zeroed from z0 on ([0, z0) is zero
    // already), its strings' {offset, length} and their ranks within their length bins.  Called once
    // nothing reads those areas any more (three barriers a chunk in all).
    uint4 pv[NV];
    uint32_t bin[SPT], rank[SPT];
#if HHUFF_ENC_SORTREC
    uint32_t mypos[SPT];
#endif
    auto prepare = [&](const SortChunk (&q)[SPT], uint64_t qb, uint32_t z0) {
        const uint32_t sp = span_of(q[0]);
        if (sp > (uint32_t)CH) return;  // workgroup-uniform: the per-thread path needs none of it
        commit_span(pv, q[0]);
        for (uint32_t k = z0 + t * 16u; k < sp + 16u; k += 16u * NT)
            *reinterpret_cast<uint4*>(reinterpret_cast<uint8_t*>(s_out) + k) = make_uint4(0u, 0u, 0u, 0u);
#pragma unroll
        for (int u = 0; u < SPT; ++u) {
            const uint32_t tt = t + (uint32_t)u * NT;
            const uint32_t ln = qb + tt < A.n ? q[u].e - q[u].s : 0u;
#if !HHUFF_ENC_SORTREC
            s_str[tt] = make_uint2(q[u].s - (q[0].lo & ~15u), ln);
#endif
            // counting sort by the bulk loop's trip count (encode_chunk_v2: dwords from the string's first
            // aligned dword to its end), which the wave's longest string sets
            bin[u] = ln ? min((q[u].s + ln - (q[u].s & ~3u)) >> 2, kSortBins - 1u) : 0u;
            rank[u] = atomicAdd(&s_bin[bin[u]], 1u);
        }
    };
    SortChunk cur[SPT];
    issue_chunk(cur, c * kSortStr);
    issue_span(pv, cur[0]);
    prepare(cur, c * kSortStr, 0u);
#if HHUFF_ENC_EARLY
    // the next chunk's offsets are loaded a chunk ahead (after barrier 2) and waited for after barrier 3,
    // before the chunk's stores: no load is then waited for behind a data-dependent number of stores
    SortChunk nxt[SPT];
    issue_chunk(nxt, (c + gridDim.x < nch ? c + gridDim.x : c) * kSortStr);
    land(nxt);  // (once)
#endif
    PROF_DECL  // profile builds: barrier 1 / ranks + barrier 2 / encode / barrier 3 + lengths / copy out / prepare
    for (;;) {
        const uint64_t cb = c * kSortStr;
        const uint32_t lo = cur[0].lo, hi = cur[0].hi, a0 = lo & ~15u, span = span_of(cur[0]);
        EdgeRec* rec = A.edges + 2 * c;  // two records a chunk (sorted_edge_recs)
        const uint64_t cn = c + gridDim.x;
        const bool more = cn < nch;
#if !HHUFF_ENC_EARLY
        SortChunk nxt[SPT];
        issue_chunk(nxt, (more ? cn : c) * kSortStr);  // in flight during this chunk
#endif
        const uint64_t cn2 = cn + gridDim.x;  // (HHUFF_ENC_EARLY) the chunk after next
        (void)cn2;
        __syncthreads();  // the chunk's stage, strings and ranks are in
        PROF_MARK(0);
        if (span > (uint32_t)CH) {  // (workgroup-uniform) a chunk larger than the stage: one thread per string
#pragma unroll
            for (int u = 0; u < SPT; ++u) {
                const uint64_t i = cb + t + (uint32_t)u * NT;
                const uint32_t len = i < A.n ? cur[u].e - cur[u].s : 0u;
                uint32_t ol = kFailLen;
                if (i < A.n && len <= kMaxStrLen) {
                    RegSink sink;
                    sink.init(A.out + cur[u].s);
                    ol = encode_core(GlobalSource{A.in, A.in_size}, cur[u].s, len, sink, s_enc);
                }
                if (i < A.n) finish_encode(A, (uint32_t)i, len, ol);
            }
            if (A.edges && t < 2) rec[t].m = make_uint4(0u, 0u, 0u, 0u);  // direct stores: no edges to defer
            if (!more) break;
            issue_span(pv, nxt[0]);
            prepare(nxt, cn * kSortStr, 0u);
#if HHUFF_ENC_EARLY
            {
                SortChunk nn[SPT];
                issue_chunk(nn, (cn2 < nch ? cn2 : cn) * kSortStr);
                land(nn);
#pragma unroll
                for (int u = 0; u < SPT; ++u) {
                    cur[u] = nxt[u];
                    nxt[u] = nn[u];
                }
            }
#else
#pragma unroll
            for (int u = 0; u < SPT; ++u) cur[u] = nxt[u];
#endif
            c = cn;
            continue;
        }
        {  // every wave scans the bin counts (two per lane)
            const uint32_t x0 = s_bin[2 * lane], x1 = s_bin[2 * lane + 1];
            const uint32_t ex = wave_excl_scan(x0 + x1, (int)lane);
#pragma unroll
            for (int u = 0; u < SPT; ++u) {
                const uint32_t eb = (uint32_t)__shfl((int)ex, (int)(bin[u] >> 1)), xb = (uint32_t)__shfl((int)x0, (int)(bin[u] >> 1));
#if HHUFF_ENC_SORTREC
                const uint32_t tt = t + (uint32_t)u * NT;
                const uint32_t ln = cb + tt < A.n ? cur[u].e - cur[u].s : 0u;
                mypos[u] = eb + ((bin[u] & 1u) ? xb : 0u) + rank[u];
                s_rec[mypos[u]] = (cur[u].s - (cur[0].lo & ~15u)) | (ln << 14);
#else
                s_perm[eb + ((bin[u] & 1u) ? xb : 0u) + rank[u]] = (uint16_t)(t + (uint32_t)u * NT);
#endif
            }
        }
        __syncthreads();
        PROF_MARK(1);
        for (uint32_t k = t; k < kSortBins; k += NT) s_bin[k] = 0u;  // read by every wave above: cleared for the next chunk
        if (more) issue_span(pv, nxt[0]);     // the next chunk's span: in flight during the encode
#if HHUFF_ENC_EARLY
        SortChunk nn[SPT];
        issue_chunk(nn, (cn2 < nch ? cn2 : (more ? cn : c)) * kSortStr);
#endif
        // sorted position t = 64 wave + lane: wave w encodes the w-th length group (SPT = 2: then also the
        // sorted position NS - 1 - t, so the pair's lengths add up to about twice the mean)
#pragma unroll
        for (int u = 0; u < SPT; ++u) {
#if HHUFF_ENC_SORTREC
            const uint32_t pj = u == 0 ? t : NS - 1u - t;
            const uint32_t rj = s_rec[pj];
            const uint2 sj = make_uint2(rj & 0x3FFFu, rj >> 14);
            const bool vj = true;  // a string past n has length 0
#else
            const uint32_t j = s_perm[u == 0 ? t : NS - 1u - t];
            const uint2 sj = s_str[j];
            const bool vj = cb + j < A.n;
#endif
            const bool act = vj && sj.y != 0 && sj.y <= kMaxStrLen;
            const uint32_t tb = encode_chunk_v2<HHUFF_ENC_SORTED_U>(s_in, span - 4u, sj.x, sj.y, act, lds_addr(s_out), 8u * sj.x, s_enc,
                                                act ? 8 * sj.y - 7 : 0xFFFFFFFFu, true);
            // the encoded length goes back to the string's own record (read by its own thread only), so the
            // lengths and statuses are stored in string order, coalesced
#if HHUFF_ENC_SORTREC
            s_rec[pj] = act && tb != kFailLen ? (tb + 7) >> 3 : kFailLen;
#else
            s_str[j].x = act && tb != kFailLen ? (tb + 7) >> 3 : kFailLen;
#endif
        }
        PROF_MARK(2);
        __syncthreads();
#if HHUFF_ENC_COPY_BATCH && HHUFF_ENC_COPY_EARLY
        // the copy-out's LDS reads right after barrier 3 (the stage is final; prepare() writes only past span),
        // so their latency runs under the next chunk's prepare and this chunk's length stores
        uint4 cv[NV];
#pragma unroll
        for (int jv = 0; jv < NV; ++jv) {
            const uint32_t k = (uint32_t)jv * (16u * NT) + t * 16u;
            if (k < span) cv[jv] = *reinterpret_cast<const uint4*>(reinterpret_cast<const uint8_t*>(s_out) + k);
        }
#endif
        uint32_t olen[SPT];
#pragma unroll
#if HHUFF_ENC_SORTREC
        for (int u = 0; u < SPT; ++u) olen[u] = s_rec[mypos[u]];
#else
        for (int u = 0; u < SPT; ++u) olen[u] = s_str[t + (uint32_t)u * NT].x;
#endif
#if HHUFF_ENC_EARLY
        // the next chunk goes in now, before this chunk's stores: its span loads (in flight since the encode
        // began) are then waited for with no store ahead of them in the memory counter
        if (more) prepare(nxt, cn * kSortStr, span);  // (overwrites this thread's records: olen read above)
        // the chunk after next's offsets are waited for here too, on every path: `nxt = nn` below then copies
        // registers with no load pending, not behind this chunk's stores
        land(nn);
        PROF_MARK(5);
#endif
#pragma unroll
        for (int u = 0; u < SPT; ++u) {
            const uint64_t i = cb + t + (uint32_t)u * NT;
            if (i < A.n) finish_encode(A, (uint32_t)i, cur[u].e - cur[u].s, olen[u]);
        }
        PROF_MARK(3);
        // the stage's MSB-first words, byte-swapped on the way out (each read chunk is zeroed for the next
        // chunk); the chunk's first and last 16-B chunks are deferred (edge_fix_kernel)
        const uint32_t kl = (span - 1u) & ~15u;
#if HHUFF_ENC_COPY_BATCH
        // every chunk's LDS read first (NV of them), then the stores: one LDS round trip a chunk, not one each
#if !HHUFF_ENC_COPY_EARLY
        uint4 cv[NV];
#pragma unroll
        for (int jv = 0; jv < NV; ++jv) {
            const uint32_t k = (uint32_t)jv * (16u * NT) + t * 16u;
            if (k < span) cv[jv] = *reinterpret_cast<const uint4*>(reinterpret_cast<const uint8_t*>(s_out) + k);
        }
#endif
#pragma unroll
        for (int jv = 0; jv < NV; ++jv) {
            const uint32_t k = (uint32_t)jv * (16u * NT) + t * 16u;
            if (k >= span) break;
            const uint64_t g = (uint64_t)a0 + k;
            uint4* sp = reinterpret_cast<uint4*>(reinterpret_cast<uint8_t*>(s_out) + k);
            uint4 v = cv[jv];
#else
        for (uint32_t k = t * 16u; k < span; k += 16u * NT) {
            const uint64_t g = (uint64_t)a0 + k;
            uint4* sp = reinterpret_cast<uint4*>(reinterpret_cast<uint8_t*>(s_out) + k);
            uint4 v = *sp;
#endif
            const bool full = g >= lo && g + 16 <= hi;
            // (a partial edge chunk stored one byte a lane below is zeroed there, after its bytes are read)
            if (full || A.edges || !HHUFF_EDGE_BYTES) *sp = make_uint4(0u, 0u, 0u, 0u);
            v = make_uint4(bswap32(v.x), bswap32(v.y), bswap32(v.z), bswap32(v.w));
            if (full) st16_out(A.out + g, v);
            if (k == 0 || k == kl) {
                const uint32_t elo = lo > g ? (uint32_t)(lo - g) : 0u;
                const uint32_t ehi = hi - g < 16 ? (uint32_t)(hi - g) : 16u;
                if (A.edges) {
                    EdgeRec* e = rec + (k == 0 ? 0 : 1);
                    e->v = v;
                    e->m = make_uint4((uint32_t)g, (uint32_t)(g >> 32), full ? 0u : elo, full ? 0u : ehi);
                } else if (!HHUFF_EDGE_BYTES && !full && ehi > elo) {  // small batches: the shared chunk's own bytes
                    store_range16r(A.out + g, v, elo, ehi);
                }
            }
        }
        if (HHUFF_EDGE_BYTES && !A.edges && t < 64u) {  // small batches: the two partial chunks, a byte a lane (wave 0)
            const uint8_t* so = reinterpret_cast<const uint8_t*>(s_out);
            edge_bytes<true>(A.out, a0, so, span, lo, hi, (int)t);
            // lane b read byte b ^ 3 of its chunk and zeroes byte b: every read lands before any lane's zeroing
            wave_lds_sync();
            if (t < 32u && span != 0) {  // zero the bytes read (the chunk was left in place above when partial)
                const uint32_t ke = t < 16u ? 0u : kl;
                if (!((uint64_t)a0 + ke >= lo && (uint64_t)a0 + ke + 16 <= hi))
                    reinterpret_cast<uint8_t*>(s_out)[ke + (t & 15u)] = 0;
            }
        }
        if (A.edges && t == 0 && (kl == 0 || span == 0)) rec[1].m = make_uint4(0u, 0u, 0u, 0u);  // one chunk, or none
        if (A.edges && t == 0 && span == 0) rec[0].m = make_uint4(0u, 0u, 0u, 0u);
        PROF_MARK(4);
        if (!more) {
            PROF_FLUSH(1);
            break;
        }
#if !HHUFF_ENC_EARLY
        // the stages are free (the input since the encode, the output but for this thread's chunks above):
        // the next chunk goes in before this chunk's stores have landed
        prepare(nxt, cn * kSortStr, span);
        PROF_MARK(5);
#endif
#pragma unroll
        for (int u = 0; u < SPT; ++u) {
            cur[u] = nxt[u];
#if HHUFF_ENC_EARLY
            nxt[u] = nn[u];
#endif
        }
        c = cn;
    }
}

// ------------------------------------------------------------------------------------------------
// Proportional-lane staged encode (contiguous layout, output slot = in_off: the wire / bench layout).
// A tile is K consecutive strings staged in LDS.  String j gets g_j = 1 + floor((64 - K) len_j / span)
// lanes, each encoding an equal share of the string, so every lane has about span / 64 bytes whatever
// the length mix (Zipf mixes, 512-B QPACK values).  Strings spread over several lanes take two passes:
// pass 1 counts each share's code bits, a wave scan turns the counts into each share's starting bit
// and the string's total (hence its verdict, hpack.c:799-800), pass 2 emits the shares into the
// OR-combined output stage.  Single-lane strings skip pass 1 and fail early as in encode_staged_kernel.
// Tiles whose span exceeds the stage (strings longer than ~STAGE / 1) fall back to the direct loop.
// ------------------------------------------------------------------------------------------------
// Proportional-lane tile size.  A tile of K strings whose span exceeds the stage falls back to the
// per-lane direct loop, and even a few such tiles set the kernel's tail (c3, Zipf 8..512 B: K = 16
// overflows 0.2 % of tiles and runs 45 % longer than K = 12, which never does), while uniform lengths
// want the largest K (fewer tiles; u64: 32 strings per tile 0.079 ms vs 21: 0.099).  So the host plans
// K0 (bytes per tile / mean, rounded down to 64 / m so that every string gets m lanes) and 64 one-wave
// blocks sample 4096 positions: for each candidate K <= K0 they count the K-string spans that would
// not fit.  Every encode_pl block then takes the largest candidate with no overflow in the sample.
constexpr uint32_t kPlCand[6] = {32u, 21u, 16u, 12u, 10u, 8u};
// input stage bytes per wave of encode_pl_kernel / flatten_pl_kernel: the planner's fit limit derives from it
// (a tile fits when its 16-B aligned span does: raw span + 30 <= kPlStage).  flatten_pl_kernel's output
// stage is kPlStage + 11 * 64 + 32 bytes, so a tile whose input fits always fits its framed output too.
constexpr uint32_t kPlStage = 3584u;
constexpr uint32_t kPlBlocks = 64;
__global__ __launch_bounds__(64) void encode_plan_kernel(const uint32_t* __restrict__ in_off, uint32_t n, uint32_t K0,
                                                         uint32_t limit, uint32_t* __restrict__ part) {
    const uint32_t lane = threadIdx.x;
    const uint64_t i = ((uint64_t)blockIdx.x * 64 + lane) * n / (kPlBlocks * 64);  // < n
    const uint32_t a = in_off[i];
    uint32_t e[6];
#pragma unroll
    for (int q = 0; q < 6; ++q)  // independent loads, issued back to back
        e[q] = kPlCand[q] <= K0 ? in_off[min(i + kPlCand[q], (uint64_t)n)] : a;
#pragma unroll
    for (int q = 0; q < 6; ++q) {
        const uint32_t over = (uint32_t)__popcll(__builtin_amdgcn_ballot_w64(e[q] - a > limit));
        if (lane == 0) part[q * kPlBlocks + blockIdx.x] = over;
    }
}
// one whole wave: the largest candidate <= K0 whose sampled spans all fit (else the smallest)
__device__ __forceinline__ uint32_t plan_tile_strings(const uint32_t* __restrict__ part, uint32_t K0) {
    const uint32_t lane = threadIdx.x & 63;
    uint32_t pick = kPlCand[5];
#pragma unroll
    for (int q = 5; q >= 0; --q) {
        uint32_t c = part[q * kPlBlocks + lane];
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) c += (uint32_t)__shfl_xor((int)c, d);
        if (kPlCand[q] <= K0 && c == 0) pick = kPlCand[q];
    }
    return pick < K0 ? pick : K0;
}

// Edge records of the proportional-lane kernels: 2 per tile of the planned K, allocated for the smallest K the
// plan can pick (rec_cap records); the records of tiles that K does not make are cleared here, so
// edge_fix_kernel reads all rec_cap of them
__device__ __forceinline__ void pl_clear_spare_edges(EdgeRec* edges, uint64_t ntiles, uint64_t rec_cap) {
    if (!edges) return;  // edges stored in the kernel
    const uint64_t nth = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t r = 2 * ntiles + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; r < rec_cap; r += nth)
        edges[r].m = make_uint4(0u, 0u, 0u, 0u);
}

#ifndef HHUFF_NB8  // pass 1 of the proportional-lane kernels counts with a byte table of code lengths
#define HHUFF_NB8 1
#endif
#ifndef HHUFF_PL_EARLY
// 1: the next span committed and the next offsets waited for before the tile's stores (with the clamped,
// unconditional offset loads: c5 encode 0.331 -> 0.320 ms, c3 0.226 -> 0.222, profiles/r04ac_pl_ab.log)
#define HHUFF_PL_EARLY 1
#endif
template <int WAVES, int STAGE>
__global__ __launch_bounds__(WAVES * 64) void encode_pl_kernel(EncArgs A, uint32_t K, const uint32_t* __restrict__ kplan,
                                                               uint64_t rec_cap) {
    struct __attribute__((aligned(16))) Smem {
        uint2 enc[512];  // 256..511: bytes outside a share
        uint32_t in[WAVES][STAGE / 4];
        uint32_t out[WAVES][STAGE / 4 + 4];
        uint32_t lmap[WAVES][64];
        uint8_t nb[272];  // code lengths for pass 1 (chunk_code_bits_nb); 256: outside the share
    };
    __shared__ Smem sm;
    __shared__ uint32_t s_k;
    for (uint32_t k = threadIdx.x; k < 512; k += WAVES * 64)
        sm.enc[k] = k < 256 ? make_uint2(g_enc_code[k], g_enc_nbits[k]) : make_uint2(0u, 0u);
    for (uint32_t k = threadIdx.x; k < 272; k += WAVES * 64) sm.nb[k] = k < 256 ? (uint8_t)g_enc_nbits[k] : (uint8_t)0;
    if (kplan && threadIdx.x < 64) {  // tile size from encode_plan_kernel's samples (K is then its ceiling)
        const uint32_t k = plan_tile_strings(kplan, K);
        if (threadIdx.x == 0) s_k = k;
    }
    __syncthreads();
    if (kplan) K = s_k;
    const uint2* s_enc = sm.enc;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint32_t* stage = sm.in[wave];
    uint32_t* obuf32 = sm.out[wave];
    const uint8_t* obuf = reinterpret_cast<const uint8_t*>(obuf32);
    uint32_t* lmap = sm.lmap[wave];
    const uint64_t ntiles = ((uint64_t)A.n + K - 1) / K;
    pl_clear_spare_edges(A.edges, ntiles, rec_cap);
    const uint64_t tstride = (uint64_t)gridDim.x * WAVES;
    uint64_t t = (uint64_t)blockIdx.x * WAVES + wave;
    if (t >= ntiles) return;

    struct Plan {
        uint64_t i0;
        uint32_t kt, s, e, lo, hi, a0, span;
        bool fits;
    };
    // every lane loads (index clamped; lanes past the tile's strings are never read): a load under a condition
    // with a zero default compiled to a register copy of the pending load, i.e. a wait right behind it
    auto issue = [&](uint64_t tt, uint32_t& s0, uint32_t& e0) {
        const uint64_t i = min(tt * K + min((uint32_t)lane, K - 1u), (uint64_t)A.n - 1u);
        s0 = A.in_off[i];
        e0 = A.in_off[i + 1];
    };
    auto plan = [&](uint64_t tt, uint32_t s0, uint32_t e0) {
        Plan P;
        P.i0 = tt * K;
        P.kt = (uint32_t)min<uint64_t>(K, A.n - P.i0);
        P.s = s0;
        P.e = e0;
        P.lo = (uint32_t)__shfl((int)s0, 0, 64);
        P.hi = (uint32_t)__shfl((int)e0, (int)P.kt - 1, 64);
        P.a0 = P.lo & ~15u;
        P.span = P.hi > P.lo ? ((P.hi + 15u) & ~15u) - P.a0 : 0u;
        P.fits = P.span <= STAGE;
        return P;
    };

    SpanPrefetch<(STAGE + 1023) / 1024> pf;
    uint32_t ns, ne;
    issue(t, ns, ne);
    Plan cur = plan(t, ns, ne);
    if (cur.fits) pf.issue(A.in, A.in_size, cur.a0, cur.span, lane);
    issue(min(t + tstride, ntiles - 1u), ns, ne);  // (unconditional: see issue)
    if (cur.fits) pf.commit(stage, A.in, A.in_size, cur.a0, cur.span, lane);
#if HHUFF_PL_EARLY
    __asm__ volatile("" : "+v"(ns), "+v"(ne) : : "memory");  // (once: no load pending at the loop head)
#endif
    for (;;) {
        const uint64_t tn = t + tstride;
        const bool have_next = tn < ntiles;
        Plan nxt;
        if (have_next) {
            nxt = plan(tn, ns, ne);
            if (nxt.fits) pf.issue(A.in, A.in_size, nxt.a0, nxt.span, lane);
        }
        issue(min(tn + tstride, ntiles - 1u), ns, ne);  // (unconditional: see issue)
        // ---- the current tile ----
        const bool own = (uint32_t)lane < cur.kt;
        const uint32_t len = own ? cur.e - cur.s : 0u;
        uint32_t ol = kFailLen;
        if (cur.fits) {
            for (uint32_t k = (uint32_t)lane * 16u; k < cur.span + 16u; k += 64u * 16u)
                *reinterpret_cast<uint4*>(reinterpret_cast<uint8_t*>(obuf32) + k) = make_uint4(0u, 0u, 0u, 0u);
            // lanes per string, first lane of each string, lane -> string map
            const uint32_t total = cur.hi - cur.lo;
            const uint32_t g = own ? 1u + (uint32_t)(((uint64_t)(64u - cur.kt) * len) / (total ? total : 1u)) : 0u;
            const uint32_t L = wave_excl_scan(g, lane);
            const uint32_t used = (uint32_t)__shfl((int)(L + g), (int)cur.kt - 1, 64);
            lmap[lane] = 0;
            wave_lds_sync();
            if (own) lmap[L] = (uint32_t)lane;
            wave_lds_sync();
            uint32_t j = lmap[lane];
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {  // inclusive max scan: the string whose first lane is at or below
                const uint32_t y = (uint32_t)__shfl_up((int)j, o, 64);
                if (lane >= o) j = max(j, y);
            }
            const bool act = (uint32_t)lane < used;
            const uint32_t sj = (uint32_t)__shfl((int)cur.s, (int)j, 64);
            const uint32_t lj = (uint32_t)__shfl((int)len, (int)j, 64);
            const uint32_t Lj = (uint32_t)__shfl((int)L, (int)j, 64);
            const uint32_t gj = (uint32_t)__shfl((int)g, (int)j, 64);
            const uint32_t sub = (uint32_t)lane - Lj;
            const uint32_t C = gj > 1 ? (((lj + gj - 1) / gj) + 3u) & ~3u : lj;
            const uint32_t c0 = min(sub * C, lj), c1 = min(sub * C + C, lj);
            const uint32_t cs = sj - cur.a0 + c0, clen = c1 - c0;
            const bool multi = gj > 1;
            const bool big = act && lj <= kMaxStrLen;
            const uint32_t last = cur.span ? cur.span - 4u : 0u;
            uint32_t off = 0, tot = 0;
            bool sfail = false;
            wave_lds_sync();
            if (__any(multi && big)) {  // pass 1: code bits of every share, then starting bits and totals
#if HHUFF_NB8
                const uint32_t b = chunk_code_bits_nb(stage, last, cs, clen, big && multi && clen != 0, sm.nb);
#else
                const uint32_t b = chunk_code_bits_v2(stage, last, cs, clen, big && multi && clen != 0, s_enc);
#endif
                const uint32_t x = wave_excl_scan(b, lane);
                const uint32_t xs = (uint32_t)__shfl((int)x, (int)Lj, 64);
                const uint32_t xe = (uint32_t)__shfl((int)(x + b), (int)(Lj + gj - 1), 64);
                off = x - xs;
                tot = xe - xs;
                sfail = multi && ((tot + 7u) >> 3) >= lj;
            }
            // pass 2: the shares' codes OR-ed into the MSB-first output stage (encode_chunk_v2); the share
            // holding the string's end pads it
            const uint32_t r = encode_chunk_v2<HHUFF_ENC_OTHER_U>(stage, last, cs, clen, big && !sfail && clen != 0, lds_addr(obuf32),
                                               8u * (sj - cur.a0) + off, s_enc, multi ? 0xFFFFFFFFu : 8u * lj - 7u,
                                               c1 == lj);
            uint32_t res = kFailLen;  // verdict of this lane's string, as seen by the string's first lane
            if (act && lj != 0 && lj <= kMaxStrLen) {
                if (multi) res = sfail ? kFailLen : (tot + 7u) >> 3;
                else res = r == kFailLen ? kFailLen : (r + 7u) >> 3;
            }
            ol = (uint32_t)__shfl((int)res, (int)L, 64);
            wave_lds_sync();
#if HHUFF_PL_EARLY
            // the stage is free (pass 2 is done): the next span goes in now, and the offsets of the tile after
            // next are waited for here, before this tile's stores -- a load waited for behind a data-dependent
            // number of stores waits for the stores too (vmcnt counts both, in order)
            if (have_next && nxt.fits) pf.commit(stage, A.in, A.in_size, nxt.a0, nxt.span, lane);
            __asm__ volatile("" : "+v"(ns), "+v"(ne) : : "memory");
#endif
            // byte-swapped on the way out; the (at most two) 16-B chunks shared with the neighbouring tiles
            // are deferred to edge_fix_kernel, or stored by byte range here (no records: small batches)
            if (A.edges)
                region_copy_deferred<true>(A.out, cur.a0, obuf, cur.span, cur.lo, cur.hi, lane, A.edges + 2 * t);
            else
                region_copy<(STAGE + 1023) / 1024, true>(A.out, cur.a0, obuf, cur.span, cur.lo, cur.hi, lane);
#if HHUFF_PL_EARLY
            // (the prefetch registers stay allocated across the copy: were they reused as its store data, the
            // next tile's loads into them would wait for those stores -- gfx950 orders no store-data reads)
#pragma unroll
            for (int k = 0; k < (STAGE + 1023) / 1024; ++k) {
                const uint4 q = pf.v[k];
                __asm__ volatile("" : : "v"(q.x), "v"(q.y), "v"(q.z), "v"(q.w));
            }
#endif
            wave_lds_sync();
        } else {
#if HHUFF_PL_EARLY
            __asm__ volatile("" : "+v"(ns), "+v"(ne) : : "memory");  // (as above, on this rare path too)
#endif
            if (own && len <= kMaxStrLen) {
                RegSink sink;
                sink.init(A.out + cur.s);
                ol = encode_core(GlobalSource{A.in, A.in_size}, cur.s, len, sink, s_enc);
            }
            if (A.edges && lane < 2) A.edges[2 * t + lane].m = make_uint4(0u, 0u, 0u, 0u);  // direct stores: no edges
        }
        if (own) finish_encode(A, (uint32_t)(cur.i0 + lane), len, ol);
        if (!have_next) break;
#if HHUFF_PL_EARLY
        if (!cur.fits && nxt.fits) pf.commit(stage, A.in, A.in_size, nxt.a0, nxt.span, lane);
#else
        if (nxt.fits) {
            pf.commit(stage, A.in, A.in_size, nxt.a0, nxt.span, lane);
        }
#endif
        cur = nxt;
        t = tn;
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
    EdgeRec* edges = nullptr;  // flatten_pl_kernel: 2 deferred-edge records per tile
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

// Prefix integer (hpack.c:757-772) as bytes, OR-ed into first byte h0; returns the byte count (<= 6).
__device__ __forceinline__ uint32_t prefix_int_bytes(uint32_t h0, uint32_t v, uint32_t p, uint64_t& hb) {
    const uint32_t pmax = (1u << p) - 1u;
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
    return hn;
}

// ------------------------------------------------------------------------------------------------
// Proportional-lane framing (QPACK flatten_string / HPACK h2o_hpack_encode_string) for the contiguous
// layout with the implicit output slots in_off[i] + 11 i.  Same share split as encode_pl_kernel; the
// bit-count pass runs for every string because the header's length depends on the Huffman length
// (qpack.c:1052-1060); raw fallbacks copy their shares after the raw header (qpack.c:1046-1051).
// ------------------------------------------------------------------------------------------------
// (Measured and rejected, profiles/r04ad_flatten_ab.log: the next tile's span DMA issued before this tile's
// stores -- the compiler then waits for that DMA before every LDS access of the copy-out: 0.342 -> 0.429 ms.)
template <int WAVES, int STAGE>
__global__ __launch_bounds__(WAVES * 64) void flatten_pl_kernel(FlatArgs A, uint32_t K, const uint32_t* __restrict__ kplan,
                                                                uint64_t rec_cap) {
    constexpr uint32_t OSTAGE = STAGE + 11u * 64u + 32u;
    struct __attribute__((aligned(16))) Smem {
        uint2 enc[512];
        uint32_t in[WAVES][STAGE / 4];
        uint32_t out[WAVES][OSTAGE / 4 + 4];
        uint32_t lmap[WAVES][64];
        uint8_t nb[272];  // code lengths for pass 1 (chunk_code_bits_nb)
    };
    __shared__ Smem sm;
    __shared__ uint32_t s_k;
    for (uint32_t k = threadIdx.x; k < 512; k += WAVES * 64)
        sm.enc[k] = k < 256 ? make_uint2(g_enc_code[k], g_enc_nbits[k]) : make_uint2(0u, 0u);
    for (uint32_t k = threadIdx.x; k < 272; k += WAVES * 64) sm.nb[k] = k < 256 ? (uint8_t)g_enc_nbits[k] : (uint8_t)0;
    if (kplan && threadIdx.x < 64) {  // tile size from encode_plan_kernel's samples (as encode_pl_kernel)
        const uint32_t k = plan_tile_strings(kplan, K);
        if (threadIdx.x == 0) s_k = k;
    }
    __syncthreads();
    if (kplan) K = s_k;
    const uint2* s_enc = sm.enc;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint32_t* stage = sm.in[wave];
    uint32_t* obuf32 = sm.out[wave];
    uint8_t* obuf = reinterpret_cast<uint8_t*>(obuf32);
    uint32_t* lmap = sm.lmap[wave];
    const uint32_t p = A.prefix_bits;
    const uint64_t ntiles = ((uint64_t)A.n + K - 1) / K;
    pl_clear_spare_edges(A.edges, ntiles, rec_cap);
    const uint64_t tstride = (uint64_t)gridDim.x * WAVES;
    uint64_t t = (uint64_t)blockIdx.x * WAVES + wave;
    if (t >= ntiles) return;

    // Software pipeline as encode_pl_kernel: the next tile's offsets, first bytes and raw bits, then its span,
    // are in flight while the current tile is framed.  The output stage holds MSB-first words (encode_chunk_v2
    // places code bits in them); prefix-integer headers and raw payload bytes go to their byte-swapped
    // positions (x ^ 3), and the region is byte-swapped on the way out.
    struct TIn {
        uint32_t s, e, first, raww;
    };
    auto issue = [&](uint64_t tt) {  // (clamped, unconditional loads: see encode_pl_kernel)
        TIn r;
        const uint64_t i = min(tt * K + min((uint32_t)lane, K - 1u), (uint64_t)A.n - 1u);
        r.s = A.in_off[i];
        r.e = A.in_off[i + 1];
        r.first = A.first_bytes ? A.first_bytes[i] : 0u;
        r.raww = A.raw_bits ? A.raw_bits[i >> 5] : 0u;
        return r;
    };
    struct Plan {
        uint64_t i0, olo, ohi, ob;
        uint32_t kt, lo, hi, a0, span, ospan;
        bool fits;
    };
    auto plan = [&](uint64_t tt, const TIn& x) {
        Plan P;
        P.i0 = tt * K;
        P.kt = (uint32_t)min<uint64_t>(K, A.n - P.i0);
        // wave-uniform: in SGPRs, so a plan kept across a tile costs no VGPRs
        P.lo = (uint32_t)__builtin_amdgcn_readfirstlane(__shfl((int)x.s, 0, 64));
        P.hi = (uint32_t)__builtin_amdgcn_readfirstlane(__shfl((int)x.e, (int)P.kt - 1, 64));
        P.a0 = P.lo & ~15u;
        P.span = P.hi > P.lo ? ((P.hi + 15u) & ~15u) - P.a0 : 0u;
        P.olo = (uint64_t)P.lo + 11u * P.i0;
        P.ohi = (uint64_t)P.hi + 11u * (P.i0 + P.kt);
        P.ob = P.olo & ~15ull;
        P.ospan = (uint32_t)(((P.ohi + 15u) & ~15ull) - P.ob);
        P.fits = P.span <= STAGE && P.ospan <= OSTAGE;
        return P;
    };
    // (the span is staged when its tile comes up: a register prefetch of it across the tile, as encode_pl_kernel
    // does, took this kernel past 128 VGPRs into scratch -- twice the HBM traffic)
    constexpr int NCH = (STAGE + 1023) / 1024;
    TIn cx = issue(t);
    // profile builds: stage issue / shares (+ the stage's wait) / pass 1 / header + pass 2 / raw copies /
    // copy-out / direct tiles / lengths, in the encode slot
    PROF_DECL
    for (;;) {
        const uint64_t tn = t + tstride;
        const bool have_next = tn < ntiles;
        const Plan cur = plan(t, cx);
        TIn nxi = issue(have_next ? tn : t);  // the next tile's offsets: in flight during this tile
        if (cur.fits) stage_span_dma<NCH>(stage, A.in, A.in_size, cur.a0, cur.span, lane);
        PROF_MARK(0);
        // ---- the current tile ----
        const uint32_t kt = cur.kt;
        const bool own = (uint32_t)lane < kt;
        const uint64_t i = cur.i0 + lane;
        const uint32_t s = cx.s, len = cx.e - cx.s, first = cx.first;
        const bool rawf = A.raw_bits ? ((cx.raww >> (i & 31)) & 1u) != 0 : false;
        uint32_t ol = kFailLen;
        if (cur.fits) {
            for (uint32_t k = (uint32_t)lane * 16u; k < cur.ospan + 16u; k += 64u * 16u)
                *reinterpret_cast<uint4*>(obuf + k) = make_uint4(0u, 0u, 0u, 0u);
            const uint32_t total = cur.hi - cur.lo;
            const uint32_t g = own ? 1u + (uint32_t)(((uint64_t)(64u - kt) * len) / (total ? total : 1u)) : 0u;
            const uint32_t L = wave_excl_scan(g, lane);
            const uint32_t used = (uint32_t)__shfl((int)(L + g), (int)kt - 1, 64);
            lmap[lane] = 0;
            wave_lds_sync();
            if (own) lmap[L] = (uint32_t)lane;
            wave_lds_sync();
            uint32_t j = lmap[lane];
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                const uint32_t y = (uint32_t)__shfl_up((int)j, o, 64);
                if (lane >= o) j = max(j, y);
            }
            const bool act = (uint32_t)lane < used;
            const uint32_t sj = (uint32_t)__shfl((int)s, (int)j, 64);
            const uint32_t lj = (uint32_t)__shfl((int)len, (int)j, 64);
            const uint32_t Lj = (uint32_t)__shfl((int)L, (int)j, 64);
            const uint32_t gj = (uint32_t)__shfl((int)g, (int)j, 64);
            const bool rj = __shfl((int)rawf, (int)j, 64) != 0;
            const uint32_t sub = (uint32_t)lane - Lj;
            const uint32_t C = gj > 1 ? (((lj + gj - 1) / gj) + 3u) & ~3u : lj;
            const uint32_t c0 = min(sub * C, lj), c1 = min(sub * C + C, lj);
            const uint32_t cs = sj - cur.a0 + c0, clen = c1 - c0;
            const bool ok = act && lj <= kMaxStrLen;
            const uint32_t last = cur.span ? cur.span - 4u : 0u;
            wave_lds_sync();
            PROF_MARK(1);
            // pass 1: code bits per share -> starting bit of each share, string totals, verdicts
#ifdef HHUFF_X_FLAT_NOCOUNT  // ablation (output wrong by design): no counting pass, every share 6 bits a byte
            const uint32_t b = ok && !rj ? 6u * clen : 0u;
#else
#if HHUFF_NB8
            const uint32_t b = chunk_code_bits_nb(stage, last, cs, clen, ok && !rj && clen != 0, sm.nb);
#else
            const uint32_t b = chunk_code_bits_v2(stage, last, cs, clen, ok && !rj && clen != 0, s_enc);
#endif
#endif
            PROF_MARK(2);
            const uint32_t x = wave_excl_scan(b, lane);
            const uint32_t xs = (uint32_t)__shfl((int)x, (int)Lj, 64);
            const uint32_t xe = (uint32_t)__shfl((int)(x + b), (int)(Lj + gj - 1), 64);
            const uint32_t tot = xe - xs;
            const bool huff = ok && !rj && lj != 0 && tot <= 8u * lj - 8u;  // ceil(bits / 8) < len (hpack.c:799-800)
            // header (the string's first lane) and payload offset in the slot
            const uint32_t fj = (uint32_t)__shfl((int)first, (int)j, 64);
            const uint32_t hlen = (tot + 7u) >> 3;
            uint64_t hb = 0;
            const uint32_t hn = huff ? prefix_int_bytes((fj & ~((1u << p) - 1u)) | (1u << p), hlen, p, hb)
                                     : prefix_int_bytes(fj & ~((2u << p) - 1u), lj, p, hb);
            const uint32_t orel = (uint32_t)((uint64_t)sj + 11u * (cur.i0 + j) - cur.ob);  // slot start in the out stage
            if (ok && sub == 0)
                for (uint32_t k = 0; k < hn; ++k) obuf[(orel + k) ^ 3u] = (uint8_t)(hb >> (8 * k));
            // pass 2: Huffman shares place their code bits; raw shares copy their bytes
            encode_chunk_v2<HHUFF_ENC_OTHER_U>(stage, last, cs, clen, huff && clen != 0, lds_addr(obuf32), 8u * (orel + hn) + (x - xs), s_enc,
                            0xFFFFFFFFu, c1 == lj);
            PROF_MARK(3);
            if (ok && !huff && clen) {
                const uint8_t* in8 = reinterpret_cast<const uint8_t*>(stage);
                for (uint32_t k = 0; k < clen; ++k) obuf[(orel + hn + c0 + k) ^ 3u] = in8[cs + k];
            }
            const uint32_t res = ok ? hn + (huff ? hlen : lj) : kFailLen;
            ol = (uint32_t)__shfl((int)res, (int)L, 64);
            wave_lds_sync();
            PROF_MARK(4);
            // the next tile's offsets are waited for here, before this tile's stores (not at the next tile's
            // plan, where the wait would cover the stores too)
            __asm__ volatile("" : "+v"(nxi.s), "+v"(nxi.e), "+v"(nxi.first), "+v"(nxi.raww) : : "memory");
#ifndef HHUFF_X_FLAT_NOSTORE  // ablation (output wrong by design): no output stores
            if (A.edges)
                region_copy_deferred<true>(A.out, cur.ob, obuf, cur.ospan, cur.olo, cur.ohi, lane, A.edges + 2 * t);
            else
                region_copy<1, true>(A.out, cur.ob, obuf, cur.ospan, cur.olo, cur.ohi, lane);
#endif
            wave_lds_sync();
            PROF_MARK(5);
        } else {
            __asm__ volatile("" : "+v"(nxi.s), "+v"(nxi.e), "+v"(nxi.first), "+v"(nxi.raww) : : "memory");
            if (own && len <= kMaxStrLen) {  // tile larger than the stage: one string per lane from global
                const uint64_t O = (uint64_t)s + 11u * i;  // output slot
                const GlobalSource src{A.in, A.in_size};
                RegSink sink;
                sink.init(A.out + O);
                const uint32_t bits = (rawf || len == 0) ? 0u : count_code_bits(src, s, len, s_enc);
                const bool huff = !rawf && len != 0 && bits <= 8 * len - 8;
                if (huff) {
                    push_prefix_int(sink, (first & ~((1u << p) - 1u)) | (1u << p), (bits + 7) >> 3, p);
                    encode_core(src, s, len, sink, s_enc);
                } else {
                    push_prefix_int(sink, first & ~((2u << p) - 1u), len, p);
                    uint32_t a = s & ~3u, rem = len, skip = s & 3u;
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
                ol = sink.count();
            }
            if (A.edges && lane < 2) A.edges[2 * t + lane].m = make_uint4(0u, 0u, 0u, 0u);  // direct stores: no edges
            PROF_MARK(6);
        }
        if (own) A.out_len[i] = ol;
        PROF_MARK(7);
        if (!have_next) {
            PROF_FLUSH(1);
            break;
        }
        cx = nxi;
        t = tn;
    }
}

// ------------------------------------------------------------------------------------------------
// String literals in header blocks: HPACK decode_string (hpack.c:223-261) and QPACK
// decode_header_{name,value}_literal (qpack.c:559-629).  Literal i starts at in[lit_off[i]]: the H flag
// at bit prefix_bits of that byte, the length as a prefix integer (h2o_hpack_decode_int, hpack.c:52-83),
// then the payload, all before in[lit_end[i]].  Three launches: parse the headers (payload offset and
// Huffman length per literal), the Huffman decode kernel over (payload, length) pairs, then a fix-up
// that validates and copies the raw literals (h2o_hpack_validate_header_name / _value, hpack.c:163-221)
// and folds the header verdicts into out_len / status.
// ------------------------------------------------------------------------------------------------
struct LitArgs {
    const uint8_t* in;
    uint64_t in_size;
    const uint32_t* lit_off;
    const uint32_t* lit_end;
    uint32_t n;
    uint32_t prefix_bits;
    uint32_t flags;
    const uint32_t* is_name_bits;
    uint8_t* out;
    uint32_t* out_len;
    uint32_t* pay_off;
    uint32_t* consumed;
    uint8_t* status;
    uint32_t* huff_len;  // workspace: Huffman payload length (0 for raw literals and errors)
    uint8_t* code;       // workspace: verdict | H flag << 3 | soft bits << 4
    const uint32_t* n_dev;  // NULL, or the literal count in device memory (n is then an upper bound)
    uint32_t* long_list;    // NULL, or: raw payloads longer than kLongRaw are validated by literal_long_kernel
    uint32_t* long_count;
    const uint8_t* prefix_of;  // NULL, or each literal's own prefix_bits
};

constexpr uint32_t kLongRaw = 512;  // raw payload bytes above which one wave validates the literal

enum : uint32_t { kLitIncomplete = 1, kLitBadInt = 2, kLitTruncated = 3, kLitHuffman = 4, kLitUpper = 5, kLitTooLong = 6 };

// header of literal i -> verdict (0 = ok); hdr = header bytes, len = payload bytes, huff = H flag
__device__ __forceinline__ uint32_t lit_header(const LitArgs& A, uint32_t i, bool& huff, uint32_t& hdr, uint32_t& len) {
    const uint64_t off = A.lit_off[i];
    const uint64_t end = A.lit_end ? min((uint64_t)A.lit_end[i], A.in_size) : A.in_size;
    huff = false;
    hdr = 0;
    len = 0;
    if (off >= end) return kLitIncomplete;
    const uint32_t p = A.prefix_of ? A.prefix_of[i] : A.prefix_bits;
    const uint32_t b0 = A.in[off];
    huff = ((b0 >> p) & 1u) != 0;
    const uint64_t pmax = (1u << p) - 1u;
    uint64_t v = b0 & pmax, q = off + 1;
    if (v == pmax) {
        bool done = false;
        uint32_t shift = 0;
        for (; shift < 56; shift += 7) {
            if (q == end) return kLitIncomplete;
            const uint32_t b = A.in[q++];
            v += (uint64_t)(b & 127u) << shift;
            if (!(b & 128u)) {
                done = true;
                break;
            }
        }
        if (!done) {  // the 9th octet (hpack.c:75-81)
            if (q == end) return kLitIncomplete;
            const uint32_t b = A.in[q];
            if (b & 128u) return kLitBadInt;
            v += (uint64_t)(b & 127u) << shift;
            ++q;
            if (v > 0x7FFFFFFFFFFFFFFFull) return kLitBadInt;
        }
    }
    if (v > end - q) return kLitTruncated;
    if (v > kMaxStrLen) return kLitTooLong;
    hdr = (uint32_t)(q - off);
    len = (uint32_t)v;
    return 0;
}

__device__ __forceinline__ bool pseudo_token(const uint8_t* s, uint32_t len) {  // lib/common/token_table.h
    const char* tok[6] = {":authority", ":method", ":path", ":protocol", ":scheme", ":status"};
    const uint32_t tl[6] = {10, 7, 5, 9, 7, 7};
    for (int k = 0; k < 6; ++k) {
        if (tl[k] != len) continue;
        bool eq = true;
        for (uint32_t j = 0; j < len && eq; ++j) eq = s[j] == (uint8_t)tok[k][j];
        if (eq) return true;
    }
    return false;
}

// Pass 1: headers; raw payloads are validated and copied here (they skip the Huffman kernel, which
// sees length 0 for them).  code[i] = verdict | H flag << 3 | soft bits << 4 for the fix-up.
__global__ void literal_parse_kernel(LitArgs A) {
    const uint64_t n = A.n_dev ? (uint64_t)*A.n_dev : (uint64_t)A.n;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        bool huff;
        uint32_t hdr, len;
        uint32_t v = lit_header(A, (uint32_t)i, huff, hdr, len);
        uint32_t soft = 0;
        if (v == 0 && !huff && A.long_list && len > kLongRaw) {  // one lane would walk it alone: defer
            A.long_list[atomicAdd(A.long_count, 1u)] = (uint32_t)i;
        } else if (v == 0 && !huff) {
            const bool is_name = A.is_name_bits ? ((A.is_name_bits[i >> 5] >> (i & 31)) & 1u) != 0 : false;
            const uint64_t s0 = (uint64_t)A.lit_off[i] + hdr;
            const uint8_t* src = A.in + s0;
            const bool skip = is_name && ((A.flags & 1u) ? pseudo_token(src, len) : (len != 0 && src[0] == ':'));
            const uint32_t* inval = is_name ? g_name_invalid : g_value_invalid;
            uint8_t* dst = A.out + (s0 * 8u) / 5u;
            // 16-byte aligned loads, four per round and no early exit: the loads of a long raw literal stay
            // in flight together (and the blocks pipeline, kLitNoRawCopy, stores nothing in between)
            const bool copy = !(A.flags & kLitNoRawCopy);
            bool anybad = false, softbad = false, upper = false;
            const uint64_t a0 = s0 & ~15ull, e0 = s0 + len;
            for (uint64_t ar = a0; ar < e0; ar += 64) {
                uint4 w4[4];
#pragma unroll
                for (uint32_t q = 0; q < 4; ++q) {
                    const uint64_t a = ar + 16u * q;
                    if (a + 16 <= A.in_size) {
                        w4[q] = *reinterpret_cast<const uint4*>(A.in + a);
                    } else {
                        uint32_t w[4] = {0, 0, 0, 0};
                        for (uint32_t k = 0; k < 16; ++k)
                            if (a + k < A.in_size) w[k >> 2] |= (uint32_t)A.in[a + k] << (8 * (k & 3));
                        w4[q] = make_uint4(w[0], w[1], w[2], w[3]);
                    }
                }
#pragma unroll
                for (uint32_t q = 0; q < 4; ++q) {
                    const uint32_t wv[4] = {w4[q].x, w4[q].y, w4[q].z, w4[q].w};
#pragma unroll
                    for (uint32_t k = 0; k < 16; ++k) {
                        const uint64_t pos = ar + 16u * q + k;
                        if (pos < s0 || pos >= e0) continue;
                        const uint32_t c = (wv[k >> 2] >> (8 * (k & 3))) & 0xFFu;
                        const bool bad = ((inval[c >> 5] >> (c & 31)) & 1u) != 0;
                        const bool up = bad && (c - 'A' < 26u);
                        anybad |= bad;
                        softbad |= bad && !up && !upper;  // names: only what precedes the first upper-case letter
                        upper |= up;
                        if (copy) dst[pos - s0] = (uint8_t)c;
                    }
                }
            }
            if (is_name) {
                if (!skip) {  // h2o_hpack_validate_header_name: empty -> soft; upper case -> hard error
                    soft = (len == 0 || softbad) ? 0x1 : 0u;
                    if (upper) v = kLitUpper;
                }
            } else {  // h2o_hpack_validate_header_value, with the whitespace rule (hpack.c:110-115)
                const bool ws = len != 0 && (src[0] == ' ' || src[0] == '\t' || src[len - 1] == ' ' || src[len - 1] == '\t');
                soft = (anybad || ws) ? 0x2 : 0u;
            }
        }
        A.pay_off[i] = A.lit_off[i] + hdr;
        A.huff_len[i] = (v == 0 && huff) ? len : 0u;
        A.consumed[i] = v == 0 ? hdr + len : 0u;
        A.code[i] = (uint8_t)(v | (huff ? 8u : 0u) | (soft << 4));
    }
}

// Long raw payloads (deferred by literal_parse_kernel): one wave per literal, 16 bytes per lane per round.  The
// name rule needs the first upper-case letter's position (h2o_hpack_validate_header_name stops there, soft
// errors count only before it), so lanes keep the first position of each kind and the wave takes minima.
__global__ __launch_bounds__(256) void literal_long_kernel(LitArgs A) {
    const int lane = threadIdx.x & 63;
    const uint32_t nl = *A.long_count;
    const bool copy = !(A.flags & kLitNoRawCopy);
    for (uint32_t w = blockIdx.x * 4u + (threadIdx.x >> 6); w < nl; w += gridDim.x * 4u) {
        const uint32_t i = A.long_list[w];
        bool huff;
        uint32_t hdr, len;
        (void)lit_header(A, i, huff, hdr, len);  // verdict 0, raw: checked by the parse kernel
        const bool is_name = A.is_name_bits ? ((A.is_name_bits[i >> 5] >> (i & 31)) & 1u) != 0 : false;
        const uint64_t s0 = (uint64_t)A.lit_off[i] + hdr, e0 = s0 + len;
        const uint8_t* src = A.in + s0;
        const bool skip = is_name && ((A.flags & 1u) ? pseudo_token(src, len) : (len != 0 && src[0] == ':'));
        const uint32_t* inval = is_name ? g_name_invalid : g_value_invalid;
        uint8_t* dst = A.out + (s0 * 8u) / 5u;
        uint32_t first_up = 0xFFFFFFFFu, first_soft = 0xFFFFFFFFu, anybad = 0;
        for (uint64_t a = s0 + 16u * (uint32_t)lane; a < e0; a += 1024) {
            uint8_t v[16];
#pragma unroll
            for (uint32_t k = 0; k < 16; ++k) v[k] = a + k < e0 ? A.in[a + k] : 0u;
#pragma unroll
            for (uint32_t k = 0; k < 16; ++k) {
                if (a + k >= e0) break;
                const uint32_t c = v[k];
                const bool bad = ((inval[c >> 5] >> (c & 31)) & 1u) != 0;
                const bool up = bad && (c - 'A' < 26u);
                const uint32_t pos = (uint32_t)(a + k - s0);
                anybad |= bad ? 1u : 0u;
                if (up) first_up = min(first_up, pos);
                if (bad && !up) first_soft = min(first_soft, pos);
                if (copy) dst[pos] = (uint8_t)c;
            }
        }
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            first_up = min(first_up, (uint32_t)__shfl_xor((int)first_up, d));
            first_soft = min(first_soft, (uint32_t)__shfl_xor((int)first_soft, d));
            anybad |= (uint32_t)__shfl_xor((int)anybad, d);
        }
        if (lane == 0) {
            uint32_t v = 0, soft = 0;
            if (is_name) {
                if (!skip) {  // h2o_hpack_validate_header_name: empty -> soft; upper case -> hard error
                    soft = first_soft < first_up ? 0x1u : 0u;
                    if (first_up != 0xFFFFFFFFu) v = kLitUpper;
                }
            } else {  // h2o_hpack_validate_header_value, with the whitespace rule (hpack.c:110-115)
                const bool ws = src[0] == ' ' || src[0] == '\t' || src[len - 1] == ' ' || src[len - 1] == '\t';
                soft = (anybad || ws) ? 0x2u : 0u;
            }
            A.consumed[i] = v == 0 ? hdr + len : 0u;
            A.code[i] = (uint8_t)(v | (soft << 4));
        }
    }
}

// Pass 3: fold the header / raw verdicts into out_len and status (the Huffman kernel ran in between).
__global__ void literal_fix_kernel(LitArgs A) {
    const uint64_t n = A.n_dev ? (uint64_t)*A.n_dev : (uint64_t)A.n;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t c = A.code[i];
        const uint32_t v = c & 7u, soft = c >> 4;
        if (v) {
            A.out_len[i] = kFailLen;
            A.status[i] = (uint8_t)(soft | kStatusFail | (v << 2));
        } else if (!(c & 8u)) {
            A.out_len[i] = A.consumed[i] - (A.pay_off[i] - A.lit_off[i]);
            A.status[i] = (uint8_t)soft;
        } else if (A.status[i] & kStatusFail) {  // h2o_hpack_decode_huffman returned SIZE_MAX
            A.status[i] = (uint8_t)(kStatusFail | (kLitHuffman << 2));
            A.consumed[i] = 0;
        }
    }
}

#if HHUFF_AB_VARIANTS
#include "hhuff_ab_decoders.h"
#endif
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
// A/B variants measured and not adopted: the store-wave staged decode, stream2, the
// register-output stream decode and the in-place sorted encoder -- tools/ab/hhuff_variants.h, in A/B builds only.
#if HHUFF_AB_VARIANTS
#include "hhuff_variants.h"
#endif

// (measured shapes, kept for the record: stream kernel waves / window dwords / output bytes per lane, c3 /
//  u400 decode ms: 12,12,96: 0.335 / 0.621; 16,8,64: 0.390 / 0.783; 8,16,112: 0.316 / 0.527.  Short-string
//  encode waves per block, c4 ms: 16: 0.83; 12: 0.93; 20 does not launch at 118 VGPRs.)
#ifndef HHUFF_ENCO_NS  // length-sorted encode chunks: strings per chunk, stage bytes (64 B a string: 4 per CU)
#define HHUFF_ENCO_NS 256
#define HHUFF_ENCO_CH 16384
#endif
#ifndef HHUFF_RK_W  // stream decode with register output: waves per block (16 x 6.4 KiB of windows + the LUT)
#define HHUFF_RK_W 16
#endif
#ifndef HHUFF_DECT  // stream decode: waves per block, window dwords, output bytes per lane
// 8 waves of 20-dword windows (the most the LDS holds beside the window table at these windows): against the
// round-4 shape of 6 x 24, c3 0.274 -> 0.244 ms, c5 0.436 -> 0.400 once the claims take ~11.5 KB each (9 or 10
// waves of 16-dword windows: c3 level, c5 +9 %; profiles/r05be_stream_shape_ab.jsonl).  Round 4, with
// 64-string claims, had 6 x 24 ahead of 8 x 16 (profiles/r04k_stream_shapes.log).
#define HHUFF_DECT_W 8
#define HHUFF_DECT_NW 20
#define HHUFF_DECT_OUT 144
#endif
#ifdef HHUFF_STREAM_RK
constexpr int kDecTWaves = HHUFF_RK_W;
#else
constexpr int kDecTWaves = HHUFF_DECT_W;
#endif
#ifndef HHUFF_ENC_INPLACE  // 1: the contiguous short-string encoder is encode_inplace_kernel (512 strings, pairs)
#define HHUFF_ENC_INPLACE 0
#endif
#ifndef HHUFF_ENCI_NS  // strings per chunk, stage bytes, strings per thread
#define HHUFF_ENCI_NS 512
#define HHUFF_ENCI_CH 28672
#define HHUFF_ENCI_SPT 2
#endif
#if HHUFF_ENC_INPLACE
constexpr int kEncOStr = HHUFF_ENCI_NS, kEncOThreads = HHUFF_ENCI_NS / HHUFF_ENCI_SPT;
#else
constexpr int kEncOStr = HHUFF_ENCO_NS, kEncOThreads = HHUFF_ENCO_NS / HHUFF_ENCO_SPT;
#endif
constexpr int kDecSWaves = 16, kEncSWaves = 16;
#define DEC_S decode_staged_kernel<kDecSWaves, 3072, 4608, false>
#ifndef HHUFF_DEC_SW  // 1: contiguous short-string decode through decode_staged_sw_kernel (a store wave)
#define HHUFF_DEC_SW 0
#endif

#define DEC_SW decode_staged_sw_kernel<3072, 4608, HHUFF_DEC_SW_NSW>
#ifndef HHUFF_DEC_RUN  // 1: the contiguous layout's stream decode runs decode_run_kernel (runs of HHUFF_RUN_RL strings)
#define HHUFF_DEC_RUN 0
#endif
#ifndef HHUFF_RUN_RL
#define HHUFF_RUN_RL 4
#endif
#define DEC_R decode_run_kernel<kDecTWaves, HHUFF_DECT_NW, HHUFF_DECT_OUT, HHUFF_RUN_RL>
#define DEC_L decode_staged_kernel<6, 8192, 12928, false>
#define DEC_SP decode_staged_kernel<kDecSWaves, 3072, 4608, true>
#define DEC_LP decode_staged_kernel<6, 8192, 12928, true>
#define DEC_D decode_direct_kernel<4>
#ifdef HHUFF_STREAM2  // A/B: the stream kernel with prefetched next strings, window in place (HHUFF_DECT_OUT: dwords)
#define DEC_T decode_stream2_kernel<kDecTWaves, HHUFF_DECT_NW, HHUFF_DECT_OUT>
#else
#ifndef HHUFF_DECT_SEG
#define HHUFF_DECT_SEG 16
#endif
#ifdef HHUFF_STREAM_RK  // A/B builds: register output, 16 waves (c3 0.437 / c5 0.687 ms against 0.294 / 0.430:
                        // the per-symbol register packing costs more than the occupancy gains, r05j_stream_rk_ab)
#define DEC_T decode_stream_rk_kernel<HHUFF_RK_W, HHUFF_DECT_NW>
#else
#define DEC_T decode_stream_kernel<kDecTWaves, HHUFF_DECT_NW, HHUFF_DECT_OUT, HHUFF_DECT_SEG>
#endif
#endif
#define ENC_S encode_staged_kernel<kEncSWaves, 3584, false>
#if HHUFF_ENC_INPLACE
#define ENC_O encode_inplace_kernel<HHUFF_ENCI_NS, HHUFF_ENCI_CH, HHUFF_ENCI_SPT>
#else
#define ENC_O encode_sorted_kernel<kEncOStr, HHUFF_ENCO_CH, HHUFF_ENCO_SPT>
#endif
#define ENC_L encode_staged_kernel<8, 8192, false>
#define ENC_SP encode_staged_kernel<kEncSWaves, 3584, true>
#define ENC_LP encode_staged_kernel<8, 8192, true>
#define ENC_D encode_direct_kernel<4>
#define FLAT_D flatten_direct_kernel<4>
#define ENC_P encode_pl_kernel<16, kPlStage>
#define FLAT_P flatten_pl_kernel<16, kPlStage>
#define FLAT_P_THREADS 1024

enum Variant { kDecS, kDecL, kDecD, kEncS, kEncL, kEncD, kFlatD, kEncP, kFlatP, kDecT, kDecSP, kDecLP, kEncSP, kEncLP,
               kEncO, kNumVariants };

static const void* variant_fn(int v) {
    switch (v) {
        case kDecS: return (const void*)DEC_S;
        case kDecL: return (const void*)DEC_L;
        case kDecSP: return (const void*)DEC_SP;
        case kDecLP: return (const void*)DEC_LP;
        case kEncSP: return (const void*)ENC_SP;
        case kEncLP: return (const void*)ENC_LP;
        case kDecD: return (const void*)DEC_D;
        case kDecT: return (const void*)DEC_T;
        case kEncS: return (const void*)ENC_S;
        case kEncO: return (const void*)ENC_O;
        case kEncL: return (const void*)ENC_L;
        case kFlatD: return (const void*)FLAT_D;
        case kEncP: return (const void*)ENC_P;
        case kFlatP: return (const void*)FLAT_P;
        default: return (const void*)ENC_D;
    }
}
static int variant_threads(int v) {
    switch (v) {
        case kDecS:
        case kDecSP: return kDecSWaves * 64;
        case kDecT: return kDecTWaves * 64;
        case kEncS:
        case kEncSP: return kEncSWaves * 64;
        case kDecL:
        case kDecLP: return 384;
        case kEncL:
        case kEncLP: return 512;
        case kEncO: return kEncOThreads;
        case kEncP: return 1024;
        case kFlatP: return FLAT_P_THREADS;
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

// Mixed lengths (Zipf 8..512 B): a staged tile of 64 strings runs as long as its longest
// string, while the stream kernel pays a per-string setup but never waits for another lane.  Which is
// faster depends on the length spread, and the lengths live in device memory: 64 one-wave blocks (on
// different CUs, so the scattered first touches do not queue behind one CU's address translation)
// sample 4 tiles each and write partial sums; the staged kernel, launched next, prices both kernels
// from them in every block (select_verdict), runs or exits, and its block 0 publishes the verdict for
// edge_fix_kernel and the stream kernel launched after it.  Block 0 here zeroes the work counter.
constexpr uint32_t kSelBlocks = 64, kSelTiles = 4;  // 256 sampled tiles, spread over 64 CUs
__global__ __launch_bounds__(64) void decode_select_kernel(DecArgs A, uint64_t* __restrict__ part,
                                                           unsigned long long* __restrict__ counter) {
    const uint64_t ntiles = ((uint64_t)A.n + 63) / 64;
    const uint64_t S = ntiles < kSelBlocks * kSelTiles ? ntiles : kSelBlocks * kSelTiles;
    const uint32_t lane = threadIdx.x;
    uint32_t len[kSelTiles];
    bool live[kSelTiles];
#pragma unroll
    for (uint32_t k = 0; k < kSelTiles; ++k) {  // independent coalesced loads, issued back to back
        const uint64_t t = (uint64_t)blockIdx.x * kSelTiles + k;
        const uint64_t i = (t < S ? t * ntiles / S : 0) * 64 + lane;
        live[k] = t < S && i < A.n;
        len[k] = live[k] ? (A.in_len ? A.in_len[i] : A.in_off[i + 1] - A.in_off[i]) : 0u;
    }
    uint64_t pad = 0, sum = 0, cnt = 0;
#pragma unroll
    for (uint32_t k = 0; k < kSelTiles; ++k) {
        const uint32_t l = min(len[k], kMaxStrLen + 1u);  // a failing length costs no more than that
        uint32_t mx = l;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) mx = max(mx, (uint32_t)__shfl_xor((int)mx, d));
        pad += 64ull * mx;
        sum += l;
        cnt += live[k] ? 1u : 0u;
    }
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        sum += (uint64_t)__shfl_xor((long long)sum, d);
        cnt += (uint64_t)__shfl_xor((long long)cnt, d);
    }
    if (lane == 0) {
        part[blockIdx.x] = pad;
        part[kSelBlocks + blockIdx.x] = sum;
        part[2 * kSelBlocks + blockIdx.x] = cnt;
        if (blockIdx.x == 0) *counter = 0ull;  // the stream kernel's work counter
    }
}

// The stream kernel's claim: about HHUFF_STREAM_CLAIM_BYTES of input a wave, 64 to 256 strings.  Every claim is
// one atomic on the batch counter, and waves wait for it: c3 (89-B mean) decodes 6.7 % faster taking 128
// strings a claim instead of 64 (6 waves a CU), 2 % faster again at 256 with 8 waves, while c5 (~400 B) loses
// 1 % at 128 and 24 % at 256 to the grid's tail (profiles/r05az_stream_claim_ab.jsonl, r05bg_stream_claim8_ab.jsonl).
#ifndef HHUFF_STREAM_CLAIM_BYTES
#define HHUFF_STREAM_CLAIM_BYTES 23040u
#endif
static uint32_t stream_claim(uint64_t in_size, uint32_t n) {
    const uint64_t mean = n ? std::max<uint64_t>(in_size / n, 1) : 1;
    const uint64_t c = HHUFF_STREAM_CLAIM_BYTES / mean;
    return c >= 256 ? 256u : c >= 192 ? 192u : c >= 128 ? 128u : 64u;
}
static int pick_decode(uint64_t in_size, uint32_t n) {
    const uint64_t mean = n ? in_size / n : 0;  // in_size bounds the bytes the batch can address
    if (mean <= 40) return kDecS;
    if (mean <= 128) return kDecL;
    return kDecT;  // u400: 2.35 ms (kDecL, tiles past the stage go direct) -> 0.53 ms
}
constexpr uint64_t kEncPlMean = 53;   // proportional-lane encode from this mean string length up
constexpr uint64_t kPlFill = 2560;    // mean bytes a proportional-lane tile is planned for (of kPlStage)
static uint64_t edge_recs(uint32_t n) { return 2 * (((uint64_t)n + 63) / 64); }

// Edge records come from a library-owned stream-ordered pool that keeps its memory between calls (the
// default pool's release threshold of 0 would hand it back to the driver at every synchronisation).
// hhuff_pool_trim() hands the kept memory back.
static std::mutex g_pool_mu;
static hipMemPool_t g_pools[64] = {};
static hipError_t pool_alloc(void** p, uint64_t bytes, hipStream_t stream) {
    std::mutex& mu = g_pool_mu;
    hipMemPool_t* pools = g_pools;
    const int dev = current_device();
    if (dev < 0 || dev >= 64) return hipErrorInvalidDevice;
    hipMemPool_t pool;
    {
        std::lock_guard<std::mutex> g(mu);
        if (!pools[dev]) {
            hipMemPoolProps props = {};
            props.allocType = hipMemAllocationTypePinned;
            props.location.type = hipMemLocationTypeDevice;
            props.location.id = dev;
            hipError_t e = hipMemPoolCreate(&pools[dev], &props);
            if (e != hipSuccess) return e;
            uint64_t keep = ~0ull;
            (void)hipMemPoolSetAttribute(pools[dev], hipMemPoolAttrReleaseThreshold, &keep);
        }
        pool = pools[dev];
    }
    return hipMallocFromPoolAsync(p, bytes, pool, stream);
}
// Edge records and edge_fix_kernel for batches of at least this many strings; below it the codec kernels store
// their regions' shared 16-B chunks themselves, one byte a lane (edge_bytes).  Default: never deferred -- the
// byte-lane edges measured c4 decode -5.5 %, c3 encode -5.3 %, c5 encode -5.6 %, flatten -6.6 %, c2 decode -9 %
// against the records and the fix-up kernel (profiles/r05ao_edge_bytes_ab.jsonl).  hhuff_set_edge_defer_min
// moves it (tests run both ways).
#ifndef HHUFF_DEFER_MIN
#define HHUFF_DEFER_MIN 0xFFFFFFFFu
#endif
static std::atomic<uint32_t> g_defer_min{HHUFF_DEFER_MIN};
uint32_t set_edge_defer_min(uint32_t n) { return g_defer_min.exchange(n); }
static bool defer_edges(uint32_t n) { return n >= g_defer_min.load(std::memory_order_relaxed); }
static hipError_t alloc_edges(EdgeRec** p, uint32_t n, hipStream_t stream) {
    return pool_alloc((void**)p, edge_recs(n) * sizeof(EdgeRec), stream);
}

// after a staged kernel launched with deferred edges: write them, release the records (stream order)
static hipError_t finish_deferred(uint8_t* out, EdgeRec* edges, uint32_t n, hipStream_t stream,
                                  const uint32_t* gate = nullptr, uint64_t recs = 0) {
    hipError_t e = hipGetLastError();
    if (e == hipSuccess) {
        const uint64_t nrec = recs ? recs : edge_recs(n);
        const uint32_t blocks = (uint32_t)min((4 * nrec + 255) / 256, (uint64_t)8192);
        hipLaunchKernelGGL(edge_fix_kernel, dim3(blocks), dim3(256), 0, stream, out, edges, nrec, gate);
        e = hipGetLastError();
    }
    const hipError_t f = hipFreeAsync(edges, stream);
    return e != hipSuccess ? e : f;
}

static bool use_pl_encode(uint64_t in_size, uint32_t n) {
    const uint64_t mean = n ? in_size / n : 0;
    return mean >= kEncPlMean;
}
static int pick_encode(uint64_t in_size, uint32_t n) {
    const uint64_t mean = n ? in_size / n : 0;
    if (mean <= 52) return kEncS;
    if (mean <= 120) return kEncL;
    return kEncD;
}

// Staged / stream prices of each device (select_verdict).  The launch path only reads them: the fitted
// defaults until hhuff_calibrate_decode_prices measures this device or hhuff_set_decode_prices pins values,
// so a decode never runs the probe (its allocations, frees and syncs) inside an asynchronous launch.
// The calibration decodes two probe batches of fixed-length strings with both kernels (zero bytes: '0'
// symbols to the end, so every string is decoded whole and then fails its padding), 131,072 x 48 B and
// 65,536 x 120 B (a 64-string tile of those still fits the staged kernel's stage), timed with events on a
// private stream (best of 3 after a warm-up); per kernel, per-string and per-byte costs solve
// t / n = a + b L on the two lengths.  A failed or implausible fit keeps the prices in effect.
constexpr float kDefPrices[4] = {40.0f, 1.07f, 184.0f, 1.15f};
static std::mutex g_price_mu;
static float g_prices[64][4];
static bool g_price_set[64];

static void prices_in_effect(int dev, float out[4]) {
    std::lock_guard<std::mutex> g(g_price_mu);
    const bool set = dev >= 0 && dev < 64 && g_price_set[dev];
    for (int k = 0; k < 4; ++k) out[k] = set ? g_prices[dev][k] : kDefPrices[k];
}

static void calibrate_prices(int dev) {
    float fit[4];
    constexpr uint32_t kN[2] = {131072u, 65536u}, kL[2] = {48u, 120u};
    const uint64_t bytes = (uint64_t)kN[1] * kL[1];
    hipStream_t s = nullptr;
    uint8_t *in = nullptr, *out = nullptr, *st = nullptr;
    uint32_t *off = nullptr, *olen = nullptr;
    unsigned long long* ctr = nullptr;
    hipEvent_t e0 = nullptr, e1 = nullptr;
    bool ok = hipStreamCreateWithFlags(&s, hipStreamNonBlocking) == hipSuccess &&
              hipMalloc((void**)&in, bytes + 64) == hipSuccess && hipMalloc((void**)&out, (bytes * 8) / 5 + 64) == hipSuccess &&
              hipMalloc((void**)&st, kN[0]) == hipSuccess && hipMalloc((void**)&off, 4ull * (kN[0] + 1)) == hipSuccess &&
              hipMalloc((void**)&olen, 4ull * kN[0]) == hipSuccess && hipMalloc((void**)&ctr, 8) == hipSuccess &&
              hipEventCreate(&e0) == hipSuccess && hipEventCreate(&e1) == hipSuccess &&
              hipMemsetAsync(in, 0, bytes + 64, s) == hipSuccess;
    double u[2][2] = {};  // [kernel][probe]: ms per string
    for (int p = 0; ok && p < 2; ++p) {
        std::vector<uint32_t> h(kN[p] + 1);
        for (uint32_t i = 0; i <= kN[p]; ++i) h[i] = i * kL[p];
        ok = hipMemcpyAsync(off, h.data(), 4ull * (kN[p] + 1), hipMemcpyHostToDevice, s) == hipSuccess &&
             hipStreamSynchronize(s) == hipSuccess;
        DecArgs A{in, (uint64_t)kN[p] * kL[p], off, nullptr, kN[p], nullptr, out, nullptr, olen, st,
                  nullptr, nullptr, nullptr, nullptr, nullptr};
        A.claim = stream_claim((uint64_t)kN[p] * kL[p], kN[p]);
        for (int k = 0; ok && k < 2; ++k) {
            float best = 1e30f;
            for (int r = 0; ok && r < 4; ++r) {
                ok = hipMemsetAsync(ctr, 0, 8, s) == hipSuccess && hipEventRecord(e0, s) == hipSuccess;
                if (k == 0)
                    hipLaunchKernelGGL(DEC_L, dim3(grid_for(kDecL, dev, kN[p])), dim3(384), 0, s, A);
                else
                    hipLaunchKernelGGL(DEC_T, dim3(grid_for(kDecT, dev, kN[p])), dim3(kDecTWaves * 64), 0, s, A, ctr);
                float ms = 0.f;
                ok = ok && hipGetLastError() == hipSuccess && hipEventRecord(e1, s) == hipSuccess &&
                     hipEventSynchronize(e1) == hipSuccess && hipEventElapsedTime(&ms, e0, e1) == hipSuccess;
                if (r > 0) best = std::min(best, ms);  // r == 0 warms up
            }
            u[k][p] = best / kN[p];
        }
    }
    bool sane = ok;
    if (ok) {
        for (int k = 0; k < 2; ++k) {
            const double b = (u[k][1] - u[k][0]) / (double)(kL[1] - kL[0]), a = u[k][0] - b * kL[0];
            fit[2 * k] = (float)(a * 1e9), fit[2 * k + 1] = (float)(b * 1e9);  // ms -> ps
        }
        for (int k = 0; k < 4; ++k) sane = sane && fit[k] > -50.0f && fit[k] < 5000.0f;
        sane = sane && fit[1] > 0.0f && fit[3] > 0.0f;
    }
    (void)hipGetLastError();  // a failed probe keeps the prices in effect and leaves no sticky error
    if (e0) (void)hipEventDestroy(e0);
    if (e1) (void)hipEventDestroy(e1);
    for (void* q : {(void*)in, (void*)out, (void*)st, (void*)off, (void*)olen, (void*)ctr})
        if (q) (void)hipFree(q);
    if (s) (void)hipStreamDestroy(s);
    if (sane) {
        std::lock_guard<std::mutex> g(g_price_mu);
        for (int k = 0; k < 4; ++k) g_prices[dev][k] = std::max(fit[k], 0.0f);
        g_price_set[dev] = true;
    }
}

int decode_prices_of(int device, float out[4], int calibrate) {
    for (int k = 0; k < 4; ++k) out[k] = kDefPrices[k];
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev || device >= 64) return -1;
    if (calibrate) {
        int cur = 0;
        if (hipGetDevice(&cur) != hipSuccess) return -1;
        if (device != cur && hipSetDevice(device) != hipSuccess) return -1;
        calibrate_prices(device);
        if (device != cur) (void)hipSetDevice(cur);
    }
    prices_in_effect(device, out);
    return 0;
}

int set_decode_prices(int device, const float* in4) {
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev || device >= 64) return -1;
    if (in4)
        for (int k = 0; k < 4; ++k)
            if (!(in4[k] >= 0.0f && in4[k] < 1e6f)) return -2;
    std::lock_guard<std::mutex> g(g_price_mu);
    for (int k = 0; k < 4; ++k) g_prices[device][k] = in4 ? in4[k] : kDefPrices[k];
    g_price_set[device] = in4 != nullptr;
    return 0;
}

#if HHUFF_AB_VARIANTS
#include "hhuff_ab_launch.h"
#else
// The segment decoder and the length-sorted decode chunks are A/B-only builds (tools/ab/hhuff_ab_*.h); here the
// contiguous-batch decode is always the staged / stream choice, and hhuff_set_decode_kernel takes mode 0 only.
int set_decode_kernel(int mode) { return mode == 0 ? 0 : -1; }
static bool use_seg(uint64_t, uint32_t, const uint32_t*, const uint32_t*) { return false; }
static hipError_t launch_seg(DecArgs, uint64_t, uint32_t, uint8_t*, hipStream_t) { return hipErrorInvalidValue; }
static bool sorted_decode_on() { return false; }
static hipError_t launch_sorted_decode(DecArgs, uint32_t, uint8_t*, hipStream_t) { return hipErrorInvalidValue; }
#endif

static hipError_t launch_decode_kernels(DecArgs A, uint64_t in_size, const uint32_t* in_len, uint32_t n, uint8_t* out,
                                        const uint32_t* out_off, hipStream_t stream, uint64_t sel_bytes) {
    A.claim = stream_claim(sel_bytes ? sel_bytes : in_size, n);
    if (use_seg(sel_bytes ? sel_bytes : in_size, n, in_len, out_off)) return launch_seg(A, in_size, n, out, stream);
    if (in_len == nullptr && out_off == nullptr && sorted_decode_on() &&
        pick_decode(sel_bytes ? sel_bytes : in_size, n) == kDecS)
        return launch_sorted_decode(A, n, out, stream);
#ifdef HHUFF_MIX_STREAM  // A/B builds: mixed lengths go to the stream kernel alone
    const int v = pick_decode(sel_bytes ? sel_bytes : in_size, n) == kDecL ? (int)kDecT : pick_decode(sel_bytes ? sel_bytes : in_size, n);
#else
    const int v = pick_decode(sel_bytes ? sel_bytes : in_size, n);
#endif
    const int grid = grid_for(v, current_device(), n);
    const bool defer = (v == kDecS || v == kDecL) && in_len == nullptr && out_off == nullptr && defer_edges(n);
    if (v == kDecL) {  // mixed lengths: the device picks staged or stream (see below)
        prices_in_effect(current_device(), A.price);  // no GPU work: see calibrate_prices
        uint64_t* sel = nullptr;  // [0, 3 kSelBlocks): partial sums; then the verdict and the work counter
        hipError_t e = pool_alloc((void**)&sel, (3 * kSelBlocks + 2) * sizeof(uint64_t), stream);
        if (e != hipSuccess) return e;
        A.sel = sel;
        A.gate = reinterpret_cast<uint32_t*>(sel + 3 * kSelBlocks);
        unsigned long long* ctr = reinterpret_cast<unsigned long long*>(sel + 3 * kSelBlocks + 1);
        hipLaunchKernelGGL(decode_select_kernel, dim3(kSelBlocks), dim3(64), 0, stream, A, sel, ctr);
        e = hipGetLastError();
        if (e == hipSuccess && defer) {
            e = alloc_edges(&A.edges, n, stream);
            if (e == hipSuccess) {
                hipLaunchKernelGGL(DEC_L, dim3(grid), dim3(384), 0, stream, A);
                e = finish_deferred(out, A.edges, n, stream, A.gate);
            }
        } else if (e == hipSuccess) {
            hipLaunchKernelGGL(DEC_L, dim3(grid), dim3(384), 0, stream, A);
            e = hipGetLastError();
        }
        if (e == hipSuccess) {
            A.edges = nullptr;
#if HHUFF_DEC_RUN
            if (in_len == nullptr && out_off == nullptr && A.n_dev == nullptr)
                hipLaunchKernelGGL(DEC_R, dim3(grid_for(kDecT, current_device(), n)), dim3(kDecTWaves * 64), 0, stream,
                                   A, ctr);
            else
#endif
                hipLaunchKernelGGL(DEC_T, dim3(grid_for(kDecT, current_device(), n)), dim3(kDecTWaves * 64), 0, stream,
                                   A, ctr);
            e = hipGetLastError();
        }
        const hipError_t f = hipFreeAsync(sel, stream);
        return e != hipSuccess ? e : f;
    }
    if (defer) {
        hipError_t e = alloc_edges(&A.edges, n, stream);
        if (e != hipSuccess) return e;
    }
    if (v == kDecT) {  // work counter for the waves' string batches
        unsigned long long* ctr = nullptr;
        hipError_t e = pool_alloc((void**)&ctr, sizeof(*ctr), stream);
        if (e == hipSuccess) e = hipMemsetAsync(ctr, 0, sizeof(*ctr), stream);
        if (e == hipSuccess) {
#if HHUFF_DEC_RUN
            if (in_len == nullptr && out_off == nullptr && A.n_dev == nullptr)
                hipLaunchKernelGGL(DEC_R, dim3(grid), dim3(kDecTWaves * 64), 0, stream, A, ctr);
            else
#endif
                hipLaunchKernelGGL(DEC_T, dim3(grid), dim3(kDecTWaves * 64), 0, stream, A, ctr);
            e = hipGetLastError();
        }
        if (ctr) {
            const hipError_t f = hipFreeAsync(ctr, stream);
            if (e == hipSuccess) e = f;
        }
        return e;
    }
#if HHUFF_DEC_SW
    if (v == kDecS && defer && A.n_dev == nullptr) {  // the store-wave variant (15 decode waves a block)
        hipLaunchKernelGGL(DEC_SW, dim3(grid), dim3(1024), 0, stream, A);
        return finish_deferred(out, A.edges, n, stream);
    }
#endif
    switch (v) {
        case kDecS: hipLaunchKernelGGL(DEC_S, dim3(grid), dim3(kDecSWaves * 64), 0, stream, A); break;
        case kDecL: hipLaunchKernelGGL(DEC_L, dim3(grid), dim3(384), 0, stream, A); break;
        default: hipLaunchKernelGGL(DEC_D, dim3(grid), dim3(256), 0, stream, A); break;
    }
    return defer ? finish_deferred(out, A.edges, n, stream) : hipGetLastError();
}

// Long strings (kSplitMin Huffman bytes or more) are listed by the decode kernels and decoded afterwards, one
// wave each, by split_decode_kernel (kSplitBig bytes or more: a block each, the second list and launch)
// -- in batches whose mean string is long (>= 128 B: QPACK values, cookies)
// and in tiny batches (kSplitMinFew: the per-string launch path for strings over the service's 768 B, where a
// lane would take the whole string's bits one after another).  Elsewhere the list
// would cost a memset and a launch on every call for strings that are almost never there, and a rare long
// string is decoded by one lane.
#ifndef HHUFF_SPLIT
#define HHUFF_SPLIT 1  // 0: no list (A/B builds: every long string decoded by one lane)
#endif
#ifndef HHUFF_SPLIT_WAVES
#define HHUFF_SPLIT_WAVES 4
#endif
#ifndef HHUFF_BIG_GRID  // most blocks of the block-list launch
#define HHUFF_BIG_GRID 128u
#endif
#ifndef HHUFF_SPLIT_BIG  // 0: no block list (every listed string on one wave)
#define HHUFF_SPLIT_BIG 1
#endif
constexpr int kSplitWaves = HHUFF_SPLIT_WAVES;  // one-wave list: 4-wave blocks (16 measured 8 % slower)
constexpr int kSplitBlockWaves = 16;             // block list: 1024 segments per string
// strings this long are decoded by a whole block (split_decode_block): 64 KB in batches, 4 KB in tiny ones
constexpr uint32_t kSplitBig = 65536, kSplitBigFew = 4096;
hipError_t launch_decode(const uint8_t* in, uint64_t in_size, const uint32_t* in_off, const uint32_t* in_len, uint32_t n,
                         const uint32_t* is_name_bits, uint8_t* out, const uint32_t* out_off, uint32_t* out_len,
                         uint8_t* status, hipStream_t stream, uint64_t sel_bytes) {
    if (n == 0) return hipSuccess;
    DecArgs A{in, in_size, in_off, in_len, n, is_name_bits, out, out_off, out_len, status, nullptr, nullptr, nullptr, nullptr, nullptr};
    const uint64_t bytes = sel_bytes ? sel_bytes : in_size;
    const uint32_t smin = n <= 16u ? kSplitMinFew : kSplitMin;
    const bool split = HHUFF_SPLIT && bytes >= smin && (bytes / n >= 128u || n <= 16u);
    uint32_t* sp = nullptr;
    if (split) {
        A.split_min = smin;
        A.split_cap = (uint32_t)std::min<uint64_t>(n, bytes / smin + 1);
        A.big_min = n <= 16u ? kSplitBigFew : kSplitBig;
        A.big_cap = HHUFF_SPLIT_BIG ? (uint32_t)std::min<uint64_t>(n, bytes / A.big_min) : 0u;
        hipError_t e = pool_alloc((void**)&sp, 4ull * (2 + A.split_cap + A.big_cap), stream);
        if (e == hipSuccess) e = hipMemsetAsync(sp, 0, 8, stream);
        if (e != hipSuccess) return e;
        A.split_n = sp;
        A.big_n = sp + 1;
        A.split_list = sp + 2;
        A.big_list = A.big_cap ? sp + 2 + A.split_cap : nullptr;
    }
    hipError_t e = launch_decode_kernels(A, in_size, in_len, n, out, out_off, stream, sel_bytes);
    if (split) {
        if (e == hipSuccess) {
            const int grid = (int)std::min<uint32_t>((A.split_cap + kSplitWaves - 1) / kSplitWaves, 512u);
            hipLaunchKernelGGL((split_decode_kernel<kSplitWaves, false>), dim3(grid), dim3(kSplitWaves * 64), 0, stream,
                               A);
            e = hipGetLastError();
        }
        if (e == hipSuccess && A.big_cap) {
            // (at most HHUFF_BIG_GRID blocks: the list is almost always empty, and a launch's blocks all start)
            hipLaunchKernelGGL((split_decode_kernel<kSplitBlockWaves, true>),
                               dim3(std::min<uint32_t>(A.big_cap, HHUFF_BIG_GRID)),
                               dim3(kSplitBlockWaves * 64), 0, stream, A);
            e = hipGetLastError();
        }
        const hipError_t f = hipFreeAsync(sp, stream);
        if (e == hipSuccess) e = f;
    }
    return e;
}

hipError_t launch_encode(const uint8_t* in, uint64_t in_size, const uint32_t* in_off, const uint32_t* in_len, uint32_t n,
                         uint8_t* out, const uint32_t* out_off, uint32_t* out_len, uint8_t* status, hipStream_t stream,
                         uint64_t sel_bytes) {
    if (n == 0) return hipSuccess;
    EncArgs A{in, in_size, in_off, in_len, n, out, out_off, out_len, status, nullptr, nullptr};
    if (sel_bytes) in_size = sel_bytes;  // variant selection only; A keeps the addressable size
    if (in_len == nullptr && out_off == nullptr && use_pl_encode(in_size, n)) {
        // contiguous wire layout: proportional-lane tiles of K strings (about 5/8 of a stage of bytes)
        const uint64_t mean = in_size / n;
        uint32_t K = (uint32_t)(mean ? kPlFill / mean : 64u);
        K = K < 1 ? 1u : (K > 64 ? 64u : K);
        K = 64u / ((64u + K - 1u) / K);  // down to 64 / m: m lanes per string, few idle
        const bool sample = K > kPlCand[5] && n >= 4096;
        const uint32_t kmin = sample ? kPlCand[5] : K;
        const uint64_t tiles = ((uint64_t)n + kmin - 1) / kmin;
        const int g = grid_for(kEncP, current_device(), 0xFFFFFFFFu);
        const uint64_t want = (tiles + 15) / 16;
        const int grid = (int)(want < (uint64_t)g ? (want ? want : 1) : g);
        const bool defer = defer_edges(n);  // else edges stored in the kernel, one launch
        const uint64_t recs = defer ? 2 * tiles : 0;  // deferred edges: 2 per tile of the smallest K the plan can pick
        hipError_t e = defer ? pool_alloc((void**)&A.edges, recs * sizeof(EdgeRec), stream) : hipSuccess;
        if (e != hipSuccess) return e;
        if (!sample) {
            hipLaunchKernelGGL(ENC_P, dim3(grid), dim3(1024), 0, stream, A, K, (const uint32_t*)nullptr, recs);
            return defer ? finish_deferred(out, A.edges, n, stream, nullptr, recs) : hipGetLastError();
        }
        uint32_t* part = nullptr;
        e = pool_alloc((void**)&part, 6 * kPlBlocks * sizeof(uint32_t), stream);
        if (e == hipSuccess) {
            // a tile fits when its 16-B aligned span does: raw span + 30 <= stage
            hipLaunchKernelGGL(encode_plan_kernel, dim3(kPlBlocks), dim3(64), 0, stream, in_off, n, K, kPlStage - 30u, part);
            e = hipGetLastError();
        }
        if (e == hipSuccess) {
            hipLaunchKernelGGL(ENC_P, dim3(grid), dim3(1024), 0, stream, A, K, (const uint32_t*)part, recs);
            e = hipGetLastError();
        }
        if (part) {
            const hipError_t f = hipFreeAsync(part, stream);
            if (e == hipSuccess) e = f;
        }
        if (e != hipSuccess) {
            if (defer) (void)hipFreeAsync(A.edges, stream);
            return e;
        }
        return defer ? finish_deferred(out, A.edges, n, stream, nullptr, recs) : hipSuccess;
    }
    int v = pick_encode(in_size, n);
#ifndef HHUFF_ENC_TILES  // contiguous layout: length-sorted chunks (A/B builds -DHHUFF_ENC_TILES: 64-string tiles)
    if (v == kEncS && in_len == nullptr && out_off == nullptr) v = kEncO;
#endif
    const int grid = grid_for(v, current_device(), n);
    const bool defer = v != kEncD && in_len == nullptr && out_off == nullptr && defer_edges(n);
    if (defer) {
        hipError_t e = alloc_edges(&A.edges, n, stream);
        if (e != hipSuccess) return e;
    }
    switch (v) {
        case kEncS: hipLaunchKernelGGL(ENC_S, dim3(grid), dim3(kEncSWaves * 64), 0, stream, A); break;
        case kEncO: hipLaunchKernelGGL(ENC_O, dim3(grid), dim3(kEncOThreads), 0, stream, A); break;
        case kEncL: hipLaunchKernelGGL(ENC_L, dim3(grid), dim3(512), 0, stream, A); break;
        default: hipLaunchKernelGGL(ENC_D, dim3(grid), dim3(256), 0, stream, A); break;
    }
    // the sorted encoder writes two records per chunk of kEncOStr strings, the tile kernels two per 64
    const uint64_t recs = v == kEncO ? 2 * (((uint64_t)n + kEncOStr - 1) / kEncOStr) : 0;
    return defer ? finish_deferred(out, A.edges, n, stream, nullptr, recs) : hipGetLastError();
}


// ------------------------------------------------------------------------------------------------
// Resident per-string service.  A launch per string costs ~18 us (launch + stream synchronisation); here
// one wave stays resident and polls kSvcSlots mailboxes in coherent host memory (one per calling thread):
// lane l watches slot l's request counter with system-scope loads.  A posted request is served by the
// whole wave: its header and input come over PCIe in one round of system-scope loads into LDS, the wave
// codes it (wave_encode / wave_decode, the tables staged once per launch), writes the output back with
// system-scope stores, waits for them, then stores the slot's `done` counter.  The wave exits when the host
// sets ctrl->stop, after idle_ticks of the real-time counter (100 MHz) without a request, or after
// max_ticks in all -- every exit is reached without the host, so the grid always drains -- and the host
// relaunches it on the next request it finds unserved.
// ------------------------------------------------------------------------------------------------
// ------------------------------------------------------------------------------------------------
// Wave-parallel codecs for one string (the per-string service; same results as encode_core / decode_core).
//   encode: 64 bytes per round, one per lane: table entry, wave prefix sum of the code lengths, each code
//           OR-ed into the MSB-first output stage at its bit (place_bits); the verdict from the total.
//   decode: the code stream is a chain of steps (each step: one window-LUT entry, 1-2 symbols, or a long
//           code).  Per round every lane takes the step that would start at bit W + lane (all 64 of them in
//           parallel, one LUT round trip), then the wave follows the chain through those 64 candidates with
//           scalar reads (v_readlane at the chain position: no memory round trip per step) until it leaves
//           the window; the lanes on the chain write their symbols at a wave prefix sum of their counts.
//           A lone lane decoding the string waits on one LUT read per step (~35 steps for 48 B).
// ------------------------------------------------------------------------------------------------
// encode s_in bytes [0, len) into out32 (LDS, MSB-first words); returns the code bits or kFailLen
__device__ __forceinline__ uint32_t wave_encode(const uint8_t* in, uint32_t len, uint32_t* out32, const uint2* s_enc,
                                                uint32_t lane, uint32_t cap = kSvcMax) {
    for (uint32_t k = lane; k < len / 4u + 4u; k += 64u) out32[k] = 0u;
    wave_lds_sync();
    const uint32_t obase = lds_addr(out32);
    const uint32_t lim = len ? 8u * len - 8u : 0u;  // hpack.c:799-800: ceil(bits / 8) < len
    uint32_t bits = 0;                               // wave-uniform
    bool fail = len == 0 || len > cap;
    for (uint32_t j0 = 0; j0 < len && !fail; j0 += 64u) {
        const uint32_t j = j0 + lane;
        const uint2 e = j < len ? s_enc[in[j]] : make_uint2(0u, 0u);
        const uint32_t incl = wave_incl_scan(e.y);
        const uint32_t tot = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
        if (bits + tot > lim) {
            fail = true;  // already longer than the input allows: the rest cannot shorten it
            break;
        }
        if (e.y) place_bits(obase, bits + incl - e.y, e.x, e.y);
        bits += tot;
    }
    if (fail) return kFailLen;
    const uint32_t p = (0u - bits) & 7u;  // fill the last byte with ones (EOS prefix, hpack.c:795-798)
    if (lane == 0 && p) place_bits(obase, bits, (1ull << p) - 1ull, p);
    wave_lds_sync();
    return bits;
}

// The same with the whole block (W waves) on one string (one_string_kernel): each wave takes a contiguous
// part of the input (64-byte multiples), a first pass sums its code lengths, a block prefix over the waves
// places the parts (and decides the verdict from the total, hpack.c:799-800), and a second pass ORs each
// wave's codes in at its place -- the parts meet inside shared words, hence the LDS OR.  All threads call it.
template <int W>
__device__ __forceinline__ uint32_t block_encode(const uint8_t* in, uint32_t len, uint32_t* out32, const uint2* s_enc,
                                                 uint32_t cap, uint32_t (&sx)[5][W]) {
    const uint32_t t = threadIdx.x, lane = t & 63u, wave = t >> 6;
    for (uint32_t k = t; k < len / 4u + 4u; k += 64u * W) out32[k] = 0u;
    const uint32_t per = ((len + 64u * W - 1u) / (64u * W)) * 64u;
    const uint32_t b0 = min(wave * per, len), b1 = min(b0 + per, len);
    uint32_t mine = 0;
    for (uint32_t j = b0 + lane; j < b1; j += 64u) mine += s_enc[in[j]].y;
    const uint32_t wsum = (uint32_t)__builtin_amdgcn_readlane((int)wave_incl_scan(mine), 63);
    if (lane == 0u) sx[0][wave] = wsum;
    __syncthreads();  // (also: the zeroed stage)
    uint32_t pos = 0, bits = 0;
#pragma unroll
    for (uint32_t k = 0; k < (uint32_t)W; ++k) {
        const uint32_t v = sx[0][k];
        pos += k < wave ? v : 0u;
        bits += v;
    }
    const uint32_t lim = len ? 8u * len - 8u : 0u;  // hpack.c:799-800: ceil(bits / 8) < len
    if (len == 0 || len > cap || bits > lim) return kFailLen;  // (block-uniform)
    const uint32_t obase = lds_addr(out32);
    for (uint32_t j0 = b0; j0 < b1; j0 += 64u) {
        const uint32_t j = j0 + lane;
        const uint2 e = j < b1 ? s_enc[in[j]] : make_uint2(0u, 0u);
        const uint32_t incl = wave_incl_scan(e.y);
        if (e.y) place_bits(obase, pos + incl - e.y, e.x, e.y);
        pos += (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
    }
    const uint32_t p = (0u - bits) & 7u;  // fill the last byte with ones (EOS prefix, hpack.c:795-798)
    if (t == 0u && p) place_bits(obase, bits, (1ull << p) - 1ull, p);
    __syncthreads();
    return bits;
}

// decode s_in bytes [0, len) into out (LDS bytes).  Two candidates per lane: bits W + lane and W + 64 + lane.
struct WaveStep {  // the step that would start at one candidate bit
    uint32_t nx;    // chain offset of the next step (offset + bits taken), or kStop
    uint32_t syms;  // 1-2 symbol bytes
    uint32_t ns;    // symbols (1-2; 0 at a chain end)
    uint32_t fl;    // invalid-char flags (decode_core's)
    uint32_t w, R;  // window at the candidate, string bits left there
    bool eos;       // EOS symbol (a chain end that fails)
};
constexpr uint32_t kStop = 0xFFFFu;  // past every window offset (up to 64 NC + 30)
__device__ __forceinline__ WaveStep wave_step(const uint8_t* in, uint32_t TB, uint32_t p, uint32_t off, const DecTables& T) {
    WaveStep s;
    const uint32_t q = (p >> 5) * 4u;  // the aligned dword holding bit p; bits past the string are don't-care
    const uint64_t x = (uint64_t)bswap32(*reinterpret_cast<const uint32_t*>(in + q)) << 32 |
                       bswap32(*reinterpret_cast<const uint32_t*>(in + q + 4u));
    s.w = (uint32_t)((x << (p & 31u)) >> 32);
    s.R = p < TB ? TB - p : 0u;
    const uint32_t e = T.lut[s.w >> (32 - HHUFF_LUT_BITS)];
    s.eos = false;
    if (e & kLong) {  // leading-ones table (as decode_core)
        const uint32_t k = min((uint32_t)__builtin_clz(~s.w | 1u), 30u);
        const uint32_t ki = T.kinfo[k];
        const uint32_t le = T.ones[(ki & 0xFFFFu) + (((s.w << (k + 1)) >> 1) >> (31 - (ki >> 16)))];
        const uint32_t L = (le >> 9) & 31u, sym = le & 0x1FFu;
        const bool stop = L > s.R || sym == kEos;
        s.eos = L <= s.R && sym == kEos;
        s.nx = stop ? kStop : off + L;
        s.ns = stop ? 0u : 1u;
        s.syms = sym;
        s.fl = (le >> 14) & 3u;
    } else {
        const uint32_t L1 = lut_l1(e), L12 = lut_l12(e);
        const bool two = (e & kHas2) && L12 <= s.R;
        const bool stop = L1 > s.R;
        s.nx = stop ? kStop : off + (two ? L12 : L1);
        s.ns = stop ? 0u : (two ? 2u : 1u);
        s.syms = lut_pair(e);
        s.fl = (e >> 24) & (two ? 15u : 3u);
    }
    return s;
}
// JUMP (NC = 1): every lane also holds the step after its own (one ds_bpermute per round), so the scalar walk
// reads two steps per chain link and the chain is half as long.
template <int NC, bool JUMP = false>
__device__ __forceinline__ DecResult wave_decode(const uint8_t* in, uint32_t len, uint8_t* out, const DecTables& T,
                                                 uint32_t lane) {
    static_assert(NC == 1 || NC == 2, "one or two candidates per lane");
    static_assert(!JUMP || NC == 1, "the jump table is for one candidate per lane");
    constexpr uint32_t kWin = 64u * NC;
    const uint32_t TB = 8u * len;
    uint32_t W = 0, opos = 0, flags = 0;
    DecResult r;
    r.ok = false;
    for (;;) {
        WaveStep s[NC];
#pragma unroll
        for (int j = 0; j < NC; ++j) s[j] = wave_step(in, TB, W + 64u * j + lane, 64u * j + lane, T);
        // follow the chain through this round's candidates (scalar: c is wave-uniform)
        uint64_t on[NC];
#pragma unroll
        for (int j = 0; j < NC; ++j) on[j] = 0;
        uint32_t c = 0;
        bool end = false;
        if constexpr (JUMP) {
            const uint32_t n1 = s[0].nx;  // < 64: the next step starts in this window (kStop is not)
            const uint32_t n2 = (uint32_t)__builtin_amdgcn_ds_bpermute((int)((n1 < 64u ? n1 : lane) << 2), (int)n1);
            while (c < 64u) {
                const uint32_t a = (uint32_t)__builtin_amdgcn_readlane((int)n1, (int)c);  // both reads hang on c only
                const uint32_t b = (uint32_t)__builtin_amdgcn_readlane((int)n2, (int)c);
                if (a == kStop) {
                    end = true;
                    break;
                }
                on[0] |= 1ull << c;
                if (a >= 64u) {
                    c = a;
                    break;
                }
                if (b == kStop) {
                    c = a;
                    end = true;
                    break;
                }
                on[0] |= 1ull << a;
                c = b;
            }
        }
        while (!JUMP && c < kWin) {
            const uint32_t nx = NC == 1 || c < 64u ? (uint32_t)__builtin_amdgcn_readlane((int)s[0].nx, (int)(c & 63u))
                                                   : (uint32_t)__builtin_amdgcn_readlane((int)s[NC - 1].nx, (int)(c & 63u));
            if (nx == kStop) {
                end = true;
                break;
            }
            if (NC == 1 || c < 64u) on[0] |= 1ull << (c & 63u);
            else on[NC - 1] |= 1ull << (c & 63u);
            c = nx;
        }
        uint32_t base = opos;
#pragma unroll
        for (int j = 0; j < NC; ++j) {
            const uint32_t n = ((on[j] >> lane) & 1u) ? s[j].ns : 0u;
            const uint32_t incl = wave_incl_scan(n);
            if (n) {
                out[base + incl - n] = (uint8_t)s[j].syms;
                if (n == 2u) out[base + incl - 1u] = (uint8_t)(s[j].syms >> 8);
                flags |= s[j].fl;
            }
            base += (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
        }
        opos = base;
        if (end) {
            // padding: at most 7 bits, all ones (mkhufftbl.py:374-381, hpack.c:132-133); EOS fails (hpack.c:88-89)
            const bool lo = NC == 1 || c < 64u;
            const uint32_t cl = c & 63u;
            const uint32_t wc = (uint32_t)__builtin_amdgcn_readlane((int)(lo ? s[0].w : s[NC - 1].w), (int)cl);
            const uint32_t Rc = (uint32_t)__builtin_amdgcn_readlane((int)(lo ? s[0].R : s[NC - 1].R), (int)cl);
            const uint32_t ec =
                (uint32_t)__builtin_amdgcn_readlane((int)((lo ? s[0].eos : s[NC - 1].eos) ? 1u : 0u), (int)cl);
            r.ok = ec == 0u && Rc <= 7u && ((wc >> 24) | (0xFFu >> Rc)) == 0xFFu;
            break;
        }
        W += c;
    }
    uint32_t fa = 0;  // OR over the wave (4 flag bits)
#pragma unroll
    for (uint32_t k = 0; k < 4; ++k) fa |= __builtin_amdgcn_ballot_w64(((flags >> k) & 1u) != 0u) != 0 ? 1u << k : 0u;
    r.len = opos;
    r.flags = (fa | (fa >> 2)) & 3u;
    r.status = 0;
    return r;
}

// The per-string service's decode (round 5): NC columns of 64 candidates per round (bits W .. W + 64 NC - 1), the
// table steps of all of them in one LDS phase (wave_step_bf: the long-code lookups done for every candidate, not
// behind a branch, so the columns' loads issue back to back: input dwords, then LUT and leading-ones info, then
// the long-code entry), then the chain walked column by column -- each column's next offsets read with v_readlane
// from that column's own register (a per-step column select made NC = 2 slower in round 3), two links a step
// through a per-column jump table (ds_bpermute).  A 48-B string is one round instead of six.
__device__ __forceinline__ WaveStep wave_step_bf(const uint8_t* in, uint32_t TB, uint32_t p, uint32_t off, const DecTables& T) {
    WaveStep s;
    const uint32_t q = (p >> 5) * 4u;
    const uint64_t x = (uint64_t)bswap32(*reinterpret_cast<const uint32_t*>(in + q)) << 32 |
                       bswap32(*reinterpret_cast<const uint32_t*>(in + q + 4u));
    s.w = (uint32_t)((x << (p & 31u)) >> 32);
    s.R = p < TB ? TB - p : 0u;
    const uint32_t e = T.lut[s.w >> (32 - HHUFF_LUT_BITS)];
    const uint32_t k = min((uint32_t)__builtin_clz(~s.w | 1u), 30u);
    const uint32_t ki = T.kinfo[k];
    const uint32_t le = T.ones[(ki & 0xFFFFu) + (((s.w << (k + 1)) >> 1) >> (31 - (ki >> 16)))];
    if (e & kLong) {
        const uint32_t L = (le >> 9) & 31u, sym = le & 0x1FFu;
        const bool stop = L > s.R || sym == kEos;
        s.eos = L <= s.R && sym == kEos;
        s.nx = stop ? kStop : off + L;
        s.ns = stop ? 0u : 1u;
        s.syms = sym;
        s.fl = (le >> 14) & 3u;
    } else {
        const uint32_t L1 = lut_l1(e), L12 = lut_l12(e);
        const bool two = (e & kHas2) && L12 <= s.R;
        const bool stop = L1 > s.R;
        s.eos = false;
        s.nx = stop ? kStop : off + (two ? L12 : L1);
        s.ns = stop ? 0u : (two ? 2u : 1u);
        s.syms = lut_pair(e);
        s.fl = (e >> 24) & (two ? 15u : 3u);
    }
    return s;
}
template <int NC>
__device__ __forceinline__ DecResult wave_decode_cols(const uint8_t* in, uint32_t len, uint8_t* out, const DecTables& T,
                                                      uint32_t lane) {
    constexpr uint32_t kWin = 64u * NC;
    const uint32_t TB = 8u * len;
    uint32_t W = 0, opos = 0, flags = 0;
    DecResult r;
    r.ok = false;
    for (;;) {
        WaveStep s[NC];
#pragma unroll
        for (int j = 0; j < NC; ++j) s[j] = wave_step_bf(in, TB, W + 64u * j + lane, 64u * j + lane, T);
        uint64_t on[NC];
        uint32_t c = 0, endj = 0;
        bool end = false;
#pragma unroll
        for (int j = 0; j < NC; ++j) {
            on[j] = 0;
            const uint32_t lo = 64u * j, hi = lo + 64u;
            const uint32_t n1 = s[j].nx;
            // the step after each candidate's, when it starts in this column (else the lane's own value, unused)
            const uint32_t n2 = (uint32_t)__builtin_amdgcn_ds_bpermute(
                (int)(((n1 >= lo && n1 < hi) ? n1 - lo : lane) << 2), (int)n1);
            while (!end && c < hi) {  // c >= lo: a link moves at most 30 bits, so no column is skipped
                const uint32_t a = (uint32_t)__builtin_amdgcn_readlane((int)n1, (int)(c - lo));
                const uint32_t b = (uint32_t)__builtin_amdgcn_readlane((int)n2, (int)(c - lo));
                if (a == kStop) {
                    end = true, endj = j;
                    break;
                }
                on[j] |= 1ull << (c - lo);
                if (a >= hi) {
                    c = a;
                    break;
                }
                if (b == kStop) {
                    c = a;
                    end = true, endj = j;
                    break;
                }
                on[j] |= 1ull << (a - lo);
                c = b;
            }
        }
        uint32_t base = opos;
#pragma unroll
        for (int j = 0; j < NC; ++j) {
            const uint32_t n = ((on[j] >> lane) & 1u) ? s[j].ns : 0u;
            const uint32_t incl = wave_incl_scan(n);
            if (n) {
                out[base + incl - n] = (uint8_t)s[j].syms;
                if (n == 2u) out[base + incl - 1u] = (uint8_t)(s[j].syms >> 8);
                flags |= s[j].fl;
            }
            base += (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
        }
        opos = base;
        if (end) {
            // padding: at most 7 bits, all ones (mkhufftbl.py:374-381, hpack.c:132-133); EOS fails (hpack.c:88-89)
            uint32_t wc = 0, Rc = 0, ec = 0;
#pragma unroll
            for (int j = 0; j < NC; ++j)
                if (endj == (uint32_t)j) {
                    const int cl = (int)(c - 64u * j);
                    wc = (uint32_t)__builtin_amdgcn_readlane((int)s[j].w, cl);
                    Rc = (uint32_t)__builtin_amdgcn_readlane((int)s[j].R, cl);
                    ec = (uint32_t)__builtin_amdgcn_readlane((int)(s[j].eos ? 1u : 0u), cl);
                }
            r.ok = ec == 0u && Rc <= 7u && ((wc >> 24) | (0xFFu >> Rc)) == 0xFFu;
            break;
        }
        W += c;  // c >= kWin: the chain left this round's window
        (void)kWin;
    }
    uint32_t fa = 0;  // OR over the wave (4 flag bits)
#pragma unroll
    for (uint32_t k = 0; k < 4; ++k) fa |= __builtin_amdgcn_ballot_w64(((flags >> k) & 1u) != 0u) != 0 ? 1u << k : 0u;
    r.len = opos;
    r.flags = (fa | (fa >> 2)) & 3u;
    r.status = 0;
    return r;
}

// ------------------------------------------------------------------------------------------------
// One string per launch: the h2o per-string symbols (h2o_hpack_{de,en}code_huffman).  The string sits in
// pinned, device-visible host memory, [meta 16 B][input][output]: one launch reads it across PCIe (the
// block's 16-B loads in one round trip) into LDS, wave 0 codes it from LDS into an LDS output buffer (encode:
// block_encode, the service's 64-bytes-a-round wave encoder on a quarter of the string per wave; decode:
// split_decode_block over the block's four waves, 256
// self-synchronising segments of at least 128 bits -- a lone lane took ~100 us for 1 KB), and the block writes the result and the meta words back -- no copies,
// one launch, one synchronisation.
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void one_string_kernel(uint8_t* __restrict__ h, uint32_t len, uint32_t in_cap,
                                                         uint32_t is_name, uint32_t encode) {
    __shared__ __attribute__((aligned(16))) uint32_t s_lut[1u << HHUFF_LUT_BITS];
    __shared__ uint32_t s_kinfo[32];
    __shared__ uint32_t s_ones[HHUFF_ONES_NENT];
    __shared__ __attribute__((aligned(16))) uint32_t s_in[kOneMax / 4 + 4];
    __shared__ __attribute__((aligned(16))) uint8_t s_out[(kOneMax * 8) / 5 + 64];
    __shared__ uint32_t s_win[256][kSplitNW + 1];    // decode: the split windows
    uint2* s_enc = reinterpret_cast<uint2*>(s_lut);  // encode: the table takes the LUT's place
    if (encode) {
        for (uint32_t k = threadIdx.x; k < 256; k += 256) s_enc[k] = make_uint2(g_enc_code[k], g_enc_nbits[k]);
    } else {
        load_dec_tables(s_lut, s_kinfo, s_ones, 256);
    }
    for (uint32_t k = 16u * threadIdx.x; k < len; k += 16u * 256u)
        *reinterpret_cast<uint4*>(reinterpret_cast<uint8_t*>(s_in) + k) = *reinterpret_cast<const uint4*>(h + 16 + k);
    __syncthreads();
    __shared__ uint32_t s_res[2];
    __shared__ uint32_t s_x[5][4];
    if (encode) {  // (launch-uniform) the block's four waves, a quarter of the string each
        uint32_t ol = block_encode<4>(reinterpret_cast<const uint8_t*>(s_in), len, reinterpret_cast<uint32_t*>(s_out),
                                      s_enc, kOneMax, s_x);
        const uint32_t st = ol == kFailLen ? kStatusFail : 0u;
        if (ol != kFailLen) ol = (ol + 7u) >> 3;
        if (threadIdx.x == 0) {
            s_res[0] = ol;
            s_res[1] = st;
        }
    } else {  // the block's four waves: the split decoder over the staged string, 256 segments
        const LdsSource src{s_in, len ? ((len + 3u) & ~3u) - 4u : 0u};
        uint32_t ol;
        uint8_t st8;
        split_decode_block<4>(src, 0u, len, is_name != 0, s_out, DecTables{s_lut, s_kinfo, s_ones},
                              s_win[threadIdx.x], s_x, ol, st8);
        if (threadIdx.x == 0) {
            s_res[0] = ol;
            s_res[1] = st8;
        }
    }
    __syncthreads();
    const uint32_t ol = s_res[0];
    const uint32_t n = ol == kFailLen ? 0u : ol;
    for (uint32_t k = 4u * threadIdx.x; k < n; k += 4u * 256u) {  // encode's stage holds MSB-first words
        const uint32_t v = *reinterpret_cast<const uint32_t*>(s_out + k);
        *reinterpret_cast<uint32_t*>(h + 16 + in_cap + k) = encode ? bswap32(v) : v;
    }
    // the result length last, after every output word (each thread's fence, then the barrier): the host
    // may take the result as soon as it sees the length, before the launch's completion signal
    __threadfence_system();
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t* meta = reinterpret_cast<uint32_t*>(h);
        __hip_atomic_store(&meta[3], s_res[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(&meta[2], ol, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

hipError_t launch_one(uint8_t* h, uint32_t len, uint32_t in_cap, bool is_name, bool encode, hipStream_t stream) {
    hipLaunchKernelGGL(one_string_kernel, dim3(1), dim3(256), 0, stream, h, len, in_cap, is_name ? 1u : 0u,
                       encode ? 1u : 0u);
    return hipGetLastError();
}

// ------------------------------------------------------------------------------------------------
// One string past kOneMax to encode (the per-string path's long values; a lone lane took 8 ms for 64 KB):
// one block of 1,024 threads walks the string in rounds of kLongChunk input bytes, 16 per thread.  Pass 1
// sums each thread's code bits, a block scan places the threads' codes, and the round total decides the
// verdict early (hpack.c:799-800: the bits only grow).  Pass 2 ORs each thread's codes into an LDS stage
// whose word 0 carries the previous round's partial word; the round's whole words go out byte-swapped and
// the partial one is carried.  The end: the EOS-prefix padding (hpack.c:795-798) and the last word.
// ------------------------------------------------------------------------------------------------
constexpr uint32_t kLongChunk = 16384;
__global__ __launch_bounds__(1024) void encode_long_kernel(const uint8_t* __restrict__ in, uint32_t len,
                                                          uint8_t* __restrict__ out, uint32_t* __restrict__ out_len) {
    __shared__ uint2 s_enc[256];
    __shared__ __attribute__((aligned(16))) uint32_t s_st[(kLongChunk * 30u) / 32u + 8u];
    __shared__ uint32_t s_w[16];
    constexpr uint32_t kSt = (kLongChunk * 30u) / 32u + 8u;
    const uint32_t t = threadIdx.x, lane = t & 63u, wave = t >> 6;
    if (t < 256) s_enc[t] = make_uint2(g_enc_code[t], g_enc_nbits[t]);
    for (uint32_t k = t; k < kSt; k += 1024u) s_st[k] = 0u;
    __syncthreads();
    const uint32_t sbase = lds_addr(s_st);
    uint32_t* out32 = reinterpret_cast<uint32_t*>(out);  // 4-byte aligned (the caller's device buffer)
    const uint64_t lim = len ? 8ull * len - 8ull : 0ull;
    bool fail = len == 0;
    uint64_t P = 0;      // bits placed so far (block-uniform)
    uint32_t carry = 0;  // the partial word holding bits [P & ~31, P), MSB-first
    for (uint32_t c0 = 0; c0 < len && !fail; c0 += kLongChunk) {
        const uint32_t cl = min(kLongChunk, len - c0);
        const uint32_t b0 = 16u * t, nb = b0 < cl ? min(16u, cl - b0) : 0u;
        const uint4 v = nb ? load16_bounded(in, len, (uint64_t)c0 + b0) : make_uint4(0u, 0u, 0u, 0u);
        const uint32_t w4[4] = {v.x, v.y, v.z, v.w};
        uint32_t bits = 0;
#pragma unroll
        for (uint32_t k = 0; k < 16; ++k)
            if (k < nb) bits += s_enc[(w4[k >> 2] >> (8u * (k & 3u))) & 0xFFu].y;
        const uint32_t incl = wave_incl_scan(bits);
        if (lane == 63u) s_w[wave] = incl;
        __syncthreads();
        uint32_t pre = 0, T = 0;
#pragma unroll
        for (uint32_t k = 0; k < 16; ++k) {
            const uint32_t x = s_w[k];
            pre += k < wave ? x : 0u;
            T += x;
        }
        if (P + T > lim) {  // (block-uniform)
            fail = true;
            break;
        }
        const uint32_t base = (uint32_t)(P & 31u);
        if (t == 0) s_st[0] = carry;  // (word 0 holds only zeros past bit `base`)
        __syncthreads();
        {  // this thread's codes from stage bit base + pre + incl - bits, a 64-bit accumulator, one OR a word
            const uint32_t pos = base + pre + incl - bits;
            uint32_t wp = pos >> 5, fill = pos & 31u;
            uint64_t acc = 0;
#pragma unroll
            for (uint32_t k = 0; k < 16; ++k) {
                if (k < nb) {
                    const uint2 e = s_enc[(w4[k >> 2] >> (8u * (k & 3u))) & 0xFFu];
                    acc |= (uint64_t)e.x << (64u - fill - e.y);
                    fill += e.y;
                    if (fill >= 32u) {
                        lds_or32(sbase + 4u * wp, (uint32_t)(acc >> 32));
                        ++wp;
                        acc <<= 32;
                        fill -= 32u;
                    }
                }
            }
            if (fill) lds_or32(sbase + 4u * wp, (uint32_t)(acc >> 32));
        }
        __syncthreads();
        const uint32_t nfull = (base + T) >> 5;
        const uint64_t ow = P >> 5;
        for (uint32_t k = t; k < nfull; k += 1024u) {
            out32[ow + k] = bswap32(s_st[k]);
            s_st[k] = 0u;
        }
        __syncthreads();
        carry = s_st[nfull];
        __syncthreads();
        if (t < 3) s_st[nfull + t] = 0u;  // the partial word and what the last ORs may have reached
        P += T;
    }
    if (fail) {
        if (t == 0) *out_len = kFailLen;
        return;
    }
    if (t == 0) {
        const uint32_t p = (uint32_t)((0u - (uint32_t)P) & 7u);  // ones to the byte's end (EOS prefix)
        const uint32_t sh = (uint32_t)(P & 31u);
        uint32_t w = carry;
        if (p) w |= (0xFFFFFFFFu >> sh) & ~(sh + p >= 32u ? 0u : 0xFFFFFFFFu >> (sh + p));
        if (sh) out32[P >> 5] = bswap32(w);  // the last (partial) word
        *out_len = (uint32_t)((P + 7u) >> 3);
    }
}

hipError_t launch_encode_long(const uint8_t* in, uint32_t len, uint8_t* out, uint32_t* out_len, hipStream_t stream) {
    hipLaunchKernelGGL(encode_long_kernel, dim3(1), dim3(1024), 0, stream, in, len, out, out_len);
    return hipGetLastError();
}

__device__ __forceinline__ uint32_t sys_load(const uint32_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void sys_store(uint32_t* p, uint32_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// one 16-B system-scope store (seen whole by the host: old or new, see SvcSlot)
__device__ __forceinline__ void sys_store16(void* p, uint32_t a, uint32_t b, uint32_t c, uint32_t d) {
    typedef uint32_t v4 __attribute__((ext_vector_type(4)));
    const v4 v = {a, b, c, d};
    __asm__ volatile("global_store_dwordx4 %0, %1, off sc0 sc1" : : "v"(p), "v"(v) : "memory");
}

// two 16-B system-scope loads (each is seen whole: old or new, see SvcSlot), waited for here
__device__ __forceinline__ void sys_load16x2(const void* pa, const void* pb, uint4& a, uint4& b) {
    __asm__ volatile(
        "global_load_dwordx4 %0, %2, off sc0 sc1\n\t"
        "global_load_dwordx4 %1, %3, off sc0 sc1\n\t"
        "s_waitcnt vmcnt(0)"
        : "=&v"(a), "=&v"(b)
        : "v"(pa), "v"(pb)
        : "memory");
}

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
// A poll's two 16-B system-scope loads on the lanes of two masks only (exec narrowed inside the asm and
// restored before the wait), so an idle poll moves only the headers, the control words and the chunks the hot
// mailbox is expected to need over PCIe -- not 2 KiB per wave per poll.  Lanes outside a mask read zeros (a
// chunk numbered 0 never matches a request: mailbox request numbers start at 1).  (Pointing those lanes at one
// device-memory line instead made every poll slower: 16 waves' uncached reads of the same line.)
__device__ __forceinline__ void sys_poll(const void* pa, uint64_t ma, const void* pb, uint64_t mb, uint4& ra, uint4& rb) {
    uint64_t save;
    u32x4 a = {0u, 0u, 0u, 0u}, b = {0u, 0u, 0u, 0u};
    __asm__ volatile(
        "s_mov_b64 %2, exec\n\t"
        "s_and_b64 exec, exec, %5\n\t"
        "global_load_dwordx4 %0, %3, off sc0 sc1\n\t"
        "s_mov_b64 exec, %2\n\t"
        "s_and_b64 exec, exec, %6\n\t"
        "global_load_dwordx4 %1, %4, off sc0 sc1\n\t"
        "s_mov_b64 exec, %2\n\t"
        "s_waitcnt vmcnt(0)"
        : "+&v"(a), "+&v"(b), "=&s"(save)
        : "v"(pa), "v"(pb), "s"(ma), "s"(mb)
        : "memory", "scc");
    ra = make_uint4(a.x, a.y, a.z, a.w);
    rb = make_uint4(b.x, b.y, b.z, b.w);
}

// (The service's strings measured faster on the candidate chain than on split_decode_wave: 48 B, 3.0 against
// 7.6 us from input to coded, profiles/r04pq_per_string_ab.jsonl; and than lane 0 alone running the staged
// kernels' lane decoder: 8,284 against 7,280 shader cycles at the full 2.4 GHz clock, HHUFF_SVC_CLK stamps,
// profiles/r05as_per_string_clk.jsonl.)
template <int NC, bool JUMP = false>
__global__ __launch_bounds__(64) void service_kernel(SvcSlot* __restrict__ slots, SvcCtrl* __restrict__ ctrl,
                                                     uint64_t idle_ticks, uint64_t max_ticks) {
    __shared__ __attribute__((aligned(16))) uint32_t s_lut[1u << HHUFF_LUT_BITS];
    __shared__ uint32_t s_kinfo[32];
    __shared__ uint32_t s_ones[HHUFF_ONES_NENT];
    __shared__ __attribute__((aligned(16))) uint2 s_enc[256];
    __shared__ __attribute__((aligned(16))) uint32_t s_in[kSvcMax / 4 + 24];  // [input][slack: a round reads 384 bits past W]
    __shared__ __attribute__((aligned(16))) uint8_t s_out[(kSvcMax * 8) / 5 + 64];
    const uint32_t lane = threadIdx.x;
    const uint32_t G = gridDim.x, g = blockIdx.x;  // G divides kSvcSlots (launch_service)
    const uint32_t M = kSvcSlots / G;              // mailboxes of this wave: lane j < M polls mailbox g + G j
    const bool mine = lane < M;
    SvcSlot* const my = slots + (g + G * (mine ? lane : 0u));
    load_dec_tables(s_lut, s_kinfo, s_ones, 64);
    for (uint32_t k = lane; k < 256; k += 64) s_enc[k] = make_uint2(g_enc_code[k], g_enc_nbits[k]);
    __syncthreads();
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    if (lane == 0) {
        sys_store(&ctrl->last[g], (uint32_t)t0);
        if (g == 0) sys_store(&ctrl->alive, 1u);
    }
    uint32_t handled = sys_load(&my->done);  // lane j keeps its mailbox's last served request
    // hot: the lane whose mailbox was served last; every poll reads its chunks too, as many as its last
    // request needed plus one (hot_ck)
    uint32_t hot = 0, hot_ck = 1, polls = 0;
    const uint64_t mhdr = (2ull << M) - 1ull;  // lanes 0 .. M
    // one round: lane j < M reads its mailbox's header, lane M the control words {stop, alive, quit, G},
    // lane l < hot_ck chunk l of the hot mailbox; the other lanes read nothing.  step() handles one round's
    // reads: true when the wave is to exit.
    auto step = [&](uint4 hdr, uint4 ck) -> bool {
        const uint32_t req = hdr.x;
        const uint32_t ctl_stop = (uint32_t)__shfl((int)hdr.x, (int)M), ctl_quit = (uint32_t)__shfl((int)hdr.z, (int)M);
        // newer than the last served (a poll that left before that request was served may still show it)
        uint64_t pend = __builtin_amdgcn_ballot_w64(mine && (int32_t)(req - handled) > 0);
        const uint64_t now = __builtin_amdgcn_s_memrealtime();
        if (pend == 0) {
            if (ctl_quit != 0 || ctl_stop != 0) return true;
            if (g == 0 && (++polls & 15u) == 0u) {
                // wave 0: the grid's idle time is the youngest of the waves' last requests
                const uint32_t l = lane < G ? sys_load(&ctrl->last[lane]) : (uint32_t)t0;
                const uint32_t idle = wave_min_u32((uint32_t)now - l);
                if (idle > (uint32_t)idle_ticks || now - t0 > max_ticks) {
                    if (lane == 0) sys_store(&ctrl->quit, 1u);
                    return true;
                }
            }
            return false;  // each poll is a PCIe round trip already: no sleep between them
        }
        int ck_slot = (int)hot;  // the lane whose mailbox's chunks `ck` holds
        while (pend) {
            const uint32_t s = (uint32_t)__builtin_ctzll(pend);
            pend &= pend - 1;
            SvcSlot* sl = slots + (g + G * s);
            const uint32_t r = (uint32_t)__shfl((int)req, (int)s);
            const uint32_t op = (uint32_t)__shfl((int)hdr.y, (int)s);
            const uint32_t len = min((uint32_t)__shfl((int)hdr.z, (int)s), kSvcMax);
            const uint32_t is_name = (uint32_t)__shfl((int)hdr.w, (int)s);
            const uint32_t t_seen = (uint32_t)now;
            const bool need = 12u * lane < len;
            // the chunks read with the headers serve if every one needed carries this request's number;
            // else read them now: the header was stored after them, so this read sees them all
            if ((int)s != ck_slot || __builtin_amdgcn_ballot_w64(need && ck.x != r) != 0) {
                uint4 unused;
                sys_load16x2(sl->chunk[lane], &sl->req, ck, unused);
            }
            ck_slot = -1;
            if (need) {
                uint32_t* d = s_in + 3u * lane;
                d[0] = ck.y;
                d[1] = ck.z;
                d[2] = ck.w;
            }
            wave_lds_sync();
            const uint32_t t_data = (uint32_t)__builtin_amdgcn_s_memrealtime();
#ifdef HHUFF_SVC_CLK
            const uint64_t c_data = __builtin_amdgcn_s_memtime();
#endif
            const uint8_t* in = reinterpret_cast<const uint8_t*>(s_in);
            uint32_t ol, st = 0;
            if (op == 1u) {
                ol = wave_encode(in, len, reinterpret_cast<uint32_t*>(s_out), s_enc, lane);
                st = ol == kFailLen ? kStatusFail : 0u;
                if (ol != kFailLen) ol = (ol + 7u) >> 3;
            } else {
                const DecResult d = NC >= 3 ? wave_decode_cols<NC>(in, len, s_out, DecTables{s_lut, s_kinfo, s_ones}, lane)
                                            : wave_decode<NC < 3 ? NC : 1, JUMP>(in, len, s_out,
                                                                                 DecTables{s_lut, s_kinfo, s_ones}, lane);
                wave_lds_sync();
                ol = d.ok ? d.len : kFailLen;
                st = d.ok ? soft_bits(is_name != 0, d.len, d.flags, d.len ? s_out[0] : 0u, d.len ? s_out[d.len - 1] : 0u)
                          : kStatusFail;
            }
            const uint32_t t_coded = (uint32_t)__builtin_amdgcn_s_memrealtime();
#ifdef HHUFF_SVC_CLK
            const uint64_t c_coded = __builtin_amdgcn_s_memtime();
#endif
            const uint32_t n = ol == kFailLen ? 0u : ol;
            // the output as tagged 16-B chunks and then the result chunk, no wait between them (SvcSlot)
            for (uint32_t k = lane; 12u * k < n; k += 64u) {  // encode's stage holds MSB-first words
                const uint32_t* w = reinterpret_cast<const uint32_t*>(s_out) + 3u * k;
                const uint32_t a = w[0], b = w[1], c = w[2];
                sys_store16(sl->outc[k], r, op == 1u ? bswap32(a) : a, op == 1u ? bswap32(b) : b,
                            op == 1u ? bswap32(c) : c);
            }
            if (lane == 0) {
#ifdef HHUFF_SVC_CLK  // diagnostic builds: the 4th stamp is t_coded + the shader-clock cycles of the coding
                sys_store16(&sl->t_seen, t_seen, t_data, t_coded, t_coded + (uint32_t)(c_coded - c_data));
#else
                sys_store16(&sl->t_seen, t_seen, t_data, t_coded, (uint32_t)__builtin_amdgcn_s_memrealtime());
#endif
                sys_store(&ctrl->last[g], t_seen);
                sys_store16(&sl->done, r, ol, st, 0u);
            }
            __asm__ volatile("s_waitcnt vmcnt(0)" ::: "memory");  // nothing of this request left in flight
            if (lane == s) handled = r;
            hot = s;
            hot_ck = min(len / 12u + 2u, 64u);
            wave_lds_sync();
        }
            return false;
    };
    const void* hp = mine ? (const void*)&my->req : (const void*)ctrl;
    auto ck_mask = [&]() {
        const uint32_t hk = (uint32_t)__builtin_amdgcn_readfirstlane((int)hot_ck);  // wave-uniform
        return hk >= 64u ? ~0ull : (1ull << hk) - 1ull;
    };
    for (;;) {
        uint4 hdr, ck;
        sys_poll(hp, mhdr, slots[g + G * hot].chunk[lane], ck_mask(), hdr, ck);
        if (step(hdr, ck)) break;
    }
    if (lane == 0) sys_store(&ctrl->gone[g], 1u);
    if (g == 0) {  // the grid is over for the host once every wave has left (bounded: 1 s)
        const uint64_t tq = __builtin_amdgcn_s_memrealtime();
        for (;;) {
            const uint32_t gone = lane < G ? sys_load(&ctrl->gone[lane]) : 1u;
            if (__builtin_amdgcn_ballot_w64(gone == 0u) == 0 || __builtin_amdgcn_s_memrealtime() - tq > 100000000ull) break;
            __builtin_amdgcn_s_sleep(8);
        }
        if (lane == 0) {
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
            sys_store(&ctrl->alive, 0u);
        }
    }
}

hipError_t launch_service(SvcSlot* slots, SvcCtrl* ctrl, uint64_t idle_ticks, uint64_t max_ticks, hipStream_t stream) {
    // decode walk (A/B knob HHUFF_SVC_NC): 1 = one candidate per lane, one step per chain link; 2 = two
    // candidates per lane; default: one candidate per lane, two steps per link (the jump table)
    // ("6" / "4": six / four columns of 64 candidates per round walked column by column, wave_decode_cols -- measured
    // slower per call than the jump table, 9.2 vs 8.5 us median through bench.py's ctypes call,
    // profiles/r05i_per_string_ab.jsonl)
    static const int nc = [] {
        const char* e = getenv("HHUFF_SVC_NC");
        return e && *e == '2' ? 2 : e && *e == '1' ? 1 : e && *e == '6' ? 6 : e && *e == '4' ? 4 : 3;
    }();
    const uint32_t G = service_waves();
    if (nc == 6)
        hipLaunchKernelGGL(service_kernel<6>, dim3(G), dim3(64), 0, stream, slots, ctrl, idle_ticks, max_ticks);
    else if (nc == 4)
        hipLaunchKernelGGL(service_kernel<4>, dim3(G), dim3(64), 0, stream, slots, ctrl, idle_ticks, max_ticks);
    else if (nc == 2)
        hipLaunchKernelGGL(service_kernel<2>, dim3(G), dim3(64), 0, stream, slots, ctrl, idle_ticks, max_ticks);
    else if (nc == 1)
        hipLaunchKernelGGL(service_kernel<1>, dim3(G), dim3(64), 0, stream, slots, ctrl, idle_ticks, max_ticks);
    else
        hipLaunchKernelGGL((service_kernel<1, true>), dim3(G), dim3(64), 0, stream, slots, ctrl, idle_ticks, max_ticks);
    return hipGetLastError();
}

// waves of the per-string service (HHUFF_SVC_WAVES, a divisor of kSvcSlots from 2 on -- a wave's lane M reads
// the control words --; default 16): caller threads are spread over the mailboxes (thread number mod
// kSvcSlots), mailbox m over wave m mod G, so up to G threads' strings are coded at once
uint32_t service_waves() {
    static const uint32_t G = [] {
        const char* e = getenv("HHUFF_SVC_WAVES");
        const uint32_t w = e && *e ? (uint32_t)atoi(e) : 16u;
        return (w >= 2 && w <= kSvcSlots && kSvcSlots % w == 0) ? w : 16u;
    }();
    return G;
}

// ------------------------------------------------------------------------------------------------
// Packed output for the variants without a native packed mode (long strings: stream / direct decode,
// proportional-lane encode): the kernel writes the slot layout into a stream-ordered scratch buffer,
// then pack_tiles_kernel moves each 64-string tile's outputs to their places (one wave per tile: wave
// prefix sum of the kept lengths, then byte copies by all 64 lanes, string after string).  Same places
// as the native packed kernels; the extra pass costs a read and a write of the output.
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void pack_tiles_kernel(const uint8_t* __restrict__ tmp, const uint32_t* __restrict__ in_off,
                                                         uint32_t n, bool dec, const uint32_t* __restrict__ out_len,
                                                         uint8_t* __restrict__ out, uint32_t* __restrict__ pk_off) {
    const int lane = threadIdx.x & 63;
    const uint64_t ntiles = ((uint64_t)n + 63) / 64;
    for (uint64_t t = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) / 64; t < ntiles;
         t += (uint64_t)gridDim.x * blockDim.x / 64) {
        const uint64_t i = t * 64 + lane;
        const bool valid = i < n;
        const uint32_t ol = valid ? out_len[i] : 0u;
        const uint32_t keep = ol != kFailLen ? ol : 0u;
        const uint32_t place = wave_excl_scan(keep, lane);
        const uint32_t s = valid ? in_off[i] : 0u;
        const uint64_t G = dec ? dec_slot(in_off[t * 64]) : (uint64_t)in_off[t * 64];
        const uint64_t src = dec ? dec_slot(s) : (uint64_t)s;
        if (valid) {
            pk_off[i] = (uint32_t)(G + place);
            if (i == n - 1) pk_off[n] = (uint32_t)(G + place + keep);
        }
        for (int j = 0; j < 64; ++j) {
            const uint32_t kj = (uint32_t)__shfl((int)keep, j, 64);
            if (kj == 0) continue;
            const uint64_t sj = ((uint64_t)(uint32_t)__shfl((int)(src >> 32), j, 64) << 32) | (uint32_t)__shfl((int)(uint32_t)src, j, 64);
            const uint64_t dj = G + (uint32_t)__shfl((int)place, j, 64);
            for (uint32_t b = (uint32_t)lane; b < kj; b += 64u) out[dj + b] = tmp[sj + b];
        }
    }
}

static hipError_t pack_via_scratch(bool dec, const uint8_t* in, uint64_t in_size, const uint32_t* in_off, uint32_t n,
                                   const uint32_t* is_name_bits, uint8_t* out, uint32_t* pk_off, uint32_t* out_len,
                                   uint8_t* status, hipStream_t stream);

hipError_t launch_decode_packed(const uint8_t* in, uint64_t in_size, const uint32_t* in_off, uint32_t n,
                                const uint32_t* is_name_bits, uint8_t* out, uint32_t* pk_off, uint32_t* out_len,
                                uint8_t* status, hipStream_t stream) {
    if (n == 0) return hipMemsetAsync(pk_off, 0, sizeof(uint32_t), stream);
    const uint64_t mean = in_size / n;
    if (mean > 128) return pack_via_scratch(true, in, in_size, in_off, n, is_name_bits, out, pk_off, out_len, status, stream);
    DecArgs A{in, in_size, in_off, nullptr, n, is_name_bits, out, nullptr, out_len, status, nullptr, nullptr, nullptr, pk_off, nullptr};
    const int v = mean <= 40 ? kDecSP : kDecLP;
    const bool defer = defer_edges(n);
    hipError_t e = defer ? alloc_edges(&A.edges, n, stream) : hipSuccess;
    if (e != hipSuccess) return e;
    const int grid = grid_for(v, current_device(), n);
    if (v == kDecSP)
        hipLaunchKernelGGL(DEC_SP, dim3(grid), dim3(kDecSWaves * 64), 0, stream, A);
    else
        hipLaunchKernelGGL(DEC_LP, dim3(grid), dim3(384), 0, stream, A);
    return defer ? finish_deferred(out, A.edges, n, stream) : hipGetLastError();
}

hipError_t launch_encode_packed(const uint8_t* in, uint64_t in_size, const uint32_t* in_off, uint32_t n, uint8_t* out,
                                uint32_t* pk_off, uint32_t* out_len, uint8_t* status, hipStream_t stream) {
    if (n == 0) return hipMemsetAsync(pk_off, 0, sizeof(uint32_t), stream);
    const uint64_t mean = in_size / n;
    if (mean > 120) return pack_via_scratch(false, in, in_size, in_off, n, nullptr, out, pk_off, out_len, status, stream);
    EncArgs A{in, in_size, in_off, nullptr, n, out, nullptr, out_len, status, nullptr, pk_off};
    const int v = mean <= 52 ? kEncSP : kEncLP;
    const bool defer = defer_edges(n);
    hipError_t e = defer ? alloc_edges(&A.edges, n, stream) : hipSuccess;
    if (e != hipSuccess) return e;
    const int grid = grid_for(v, current_device(), n);
    if (v == kEncSP)
        hipLaunchKernelGGL(ENC_SP, dim3(grid), dim3(kEncSWaves * 64), 0, stream, A);
    else
        hipLaunchKernelGGL(ENC_LP, dim3(grid), dim3(512), 0, stream, A);
    return defer ? finish_deferred(out, A.edges, n, stream) : hipGetLastError();
}

static hipError_t pack_via_scratch(bool dec, const uint8_t* in, uint64_t in_size, const uint32_t* in_off, uint32_t n,
                                   const uint32_t* is_name_bits, uint8_t* out, uint32_t* pk_off, uint32_t* out_len,
                                   uint8_t* status, hipStream_t stream) {
    uint8_t* tmp = nullptr;
    const uint64_t bytes = (dec ? (in_size * 8) / 5 : in_size) + 64;
    hipError_t e = pool_alloc((void**)&tmp, bytes, stream);
    if (e != hipSuccess) return e;
    e = dec ? launch_decode(in, in_size, in_off, nullptr, n, is_name_bits, tmp, nullptr, out_len, status, stream)
            : launch_encode(in, in_size, in_off, nullptr, n, tmp, nullptr, out_len, status, stream);
    if (e == hipSuccess) {
        const uint32_t blocks = (uint32_t)min(((uint64_t)n + 255) / 256, (uint64_t)65535);
        hipLaunchKernelGGL(pack_tiles_kernel, dim3(blocks), dim3(256), 0, stream, tmp, in_off, n, dec, out_len, out, pk_off);
        e = hipGetLastError();
    }
    const hipError_t f = hipFreeAsync(tmp, stream);
    return e != hipSuccess ? e : f;
}

hipError_t launch_flatten(const uint8_t* in, uint64_t in_size, const uint32_t* in_off, const uint32_t* in_len, uint32_t n,
                          const uint8_t* first_bytes, uint32_t prefix_bits, const uint32_t* raw_bits, uint8_t* out,
                          const uint32_t* out_off, uint32_t* out_len, hipStream_t stream) {
    if (n == 0) return hipSuccess;
    FlatArgs A{in, in_size, in_off, in_len, n, first_bytes, prefix_bits, raw_bits, out, out_off, out_len};
    if (in_len == nullptr && out_off == nullptr) {  // contiguous layout, implicit slots: proportional lanes
        const uint64_t mean = in_size / n;
        uint32_t K = (uint32_t)(mean ? kPlFill / mean : 64u);  // as launch_encode
        K = K < 1 ? 1u : (K > 64 ? 64u : K);
        K = 64u / ((64u + K - 1u) / K);
        const bool sample = K > kPlCand[5] && n >= 4096;
        const uint32_t kmin = sample ? kPlCand[5] : K;
        const uint64_t tiles = ((uint64_t)n + kmin - 1) / kmin;
        const int g = grid_for(kFlatP, current_device(), 0xFFFFFFFFu);
        const uint64_t want = (tiles + FLAT_P_THREADS / 64 - 1) / (FLAT_P_THREADS / 64);
        const int grid = (int)(want < (uint64_t)g ? (want ? want : 1) : g);
        const bool defer = defer_edges(n);  // else edges stored in the kernel, one launch
        const uint64_t recs = defer ? 2 * tiles : 0;  // deferred edges (see encode_pl_kernel)
        hipError_t e = defer ? pool_alloc((void**)&A.edges, recs * sizeof(EdgeRec), stream) : hipSuccess;
        if (e != hipSuccess) return e;
        if (!sample) {
            hipLaunchKernelGGL(FLAT_P, dim3(grid), dim3(FLAT_P_THREADS), 0, stream, A, K, (const uint32_t*)nullptr, recs);
            return defer ? finish_deferred(out, A.edges, n, stream, nullptr, recs) : hipGetLastError();
        }
        uint32_t* part = nullptr;
        e = pool_alloc((void**)&part, 6 * kPlBlocks * sizeof(uint32_t), stream);
        if (e == hipSuccess) {
            hipLaunchKernelGGL(encode_plan_kernel, dim3(kPlBlocks), dim3(64), 0, stream, in_off, n, K, kPlStage - 30u, part);
            e = hipGetLastError();
        }
        if (e == hipSuccess) {
            hipLaunchKernelGGL(FLAT_P, dim3(grid), dim3(FLAT_P_THREADS), 0, stream, A, K, (const uint32_t*)part, recs);
            e = hipGetLastError();
        }
        if (part) {
            const hipError_t f = hipFreeAsync(part, stream);
            if (e == hipSuccess) e = f;
        }
        if (e != hipSuccess) {
            if (defer) (void)hipFreeAsync(A.edges, stream);
            return e;
        }
        return defer ? finish_deferred(out, A.edges, n, stream, nullptr, recs) : hipSuccess;
    }
    const int grid = grid_for(kFlatD, current_device(), n);
    hipLaunchKernelGGL(FLAT_D, dim3(grid), dim3(256), 0, stream, A);
    return hipGetLastError();
}

hipError_t launch_literals(const uint8_t* in, uint64_t in_size, const uint32_t* lit_off, const uint32_t* lit_end, uint32_t n,
                           uint32_t prefix_bits, uint32_t flags, const uint32_t* is_name_bits, uint8_t* out,
                           uint32_t* out_len, uint32_t* pay_off, uint32_t* consumed, uint8_t* status, uint32_t* huff_len,
                           hipStream_t stream) {
    if (n == 0) return hipSuccess;
    LitArgs A{in, in_size, lit_off, lit_end, n, prefix_bits, flags, is_name_bits, out, out_len, pay_off, consumed, status,
              huff_len, reinterpret_cast<uint8_t*>(huff_len + n), nullptr, nullptr, nullptr, nullptr};
    const uint32_t blocks = min((n + 255u) / 256u, 4096u);
    hipLaunchKernelGGL(literal_parse_kernel, dim3(blocks), dim3(256), 0, stream, A);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    e = launch_decode(in, in_size, pay_off, huff_len, n, is_name_bits, out, nullptr, out_len, status, stream);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(literal_fix_kernel, dim3(blocks), dim3(256), 0, stream, A);
    return hipGetLastError();
}

// Literals whose count is only known on the device (the header-block pipeline, hhuff_blocks.hip): n_max
// bounds the arrays, *n_dev is the count.  Huffman payloads go through the stream kernel, which takes its
// strings from a work counter and so needs no host-side count.  ws: 5 n_max bytes + 16.
hipError_t launch_literals_dev(const uint8_t* in, uint64_t in_size, const uint32_t* lit_off, uint32_t n_max,
                               const uint32_t* n_dev, uint32_t prefix_bits, uint32_t flags, const uint32_t* is_name_bits,
                               uint8_t* out, uint32_t* out_len, uint32_t* pay_off, uint32_t* consumed, uint8_t* status,
                               uint8_t* ws, hipStream_t stream, const uint8_t* prefix_of) {
    if (n_max == 0) return hipSuccess;
    // ws: huff_len u32[n_max], code u8[n_max], then (8-aligned) the stream counter u64, the long-literal
    // count u32 (+ pad) and list u32[in_size / kLongRaw + 1]
    uint32_t* huff_len = reinterpret_cast<uint32_t*>(ws);
    uint8_t* tail = ws + 5ull * n_max + ((8 - (5ull * n_max) % 8) % 8);
    unsigned long long* ctr = reinterpret_cast<unsigned long long*>(tail);
    uint32_t* long_count = reinterpret_cast<uint32_t*>(tail + 8);
    uint32_t* long_list = reinterpret_cast<uint32_t*>(tail + 16);
    LitArgs A{in, in_size, lit_off, nullptr, n_max, prefix_bits, flags, is_name_bits, out, out_len, pay_off, consumed,
              status, huff_len, reinterpret_cast<uint8_t*>(huff_len + n_max), n_dev, long_list, long_count, prefix_of};
    const int dev = current_device();
    const uint32_t blocks = min((n_max + 255u) / 256u, 8192u);
    hipError_t e = hipMemsetAsync(tail, 0, 16, stream);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(literal_parse_kernel, dim3(blocks), dim3(256), 0, stream, A);
    hipLaunchKernelGGL(literal_long_kernel, dim3(1024), dim3(256), 0, stream, A);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    DecArgs D{in, in_size, pay_off, huff_len, n_max, is_name_bits, out, nullptr, out_len, status, nullptr, nullptr, nullptr,
              nullptr, n_dev};
    // header literals are short: the staged kernel (tiles of 64 consecutive literals, their span staged in
    // LDS; a tile whose span exceeds the stage decodes lane by lane from global memory).  Measured against
    // the stream kernel on the f4 benches: blocks 1.685 -> 1.485 ms, qpack 1.25 -> 1.08 ms.
    (void)ctr;
    hipLaunchKernelGGL(DEC_S, dim3(grid_for(kDecS, dev, n_max)), dim3(kDecSWaves * 64), 0, stream, D);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    hipLaunchKernelGGL(literal_fix_kernel, dim3(blocks), dim3(256), 0, stream, A);
    return hipGetLastError();
}

uint64_t literals_dev_ws(uint32_t n_max, uint64_t in_size) { return 5ull * n_max + 8 + 16 + 4 * (in_size / kLongRaw + 1); }

hipError_t work_alloc(void** p, uint64_t bytes, hipStream_t stream) { return pool_alloc(p, bytes, stream); }

hipError_t pool_trim() {
    const int dev = current_device();
    if (dev < 0 || dev >= 64) return hipErrorInvalidDevice;
    std::lock_guard<std::mutex> g(g_pool_mu);
    if (!g_pools[dev]) return hipSuccess;
    hipError_t e = hipDeviceSynchronize();  // memory freed on a stream returns to the pool once the stream passes it
    return e == hipSuccess ? hipMemPoolTrimTo(g_pools[dev], 0) : e;
}

int grid_size(int device, int which) { return grid_for(which == 0 ? kDecS : kEncS, device, 0xFFFFFFFFu); }

}  // namespace hhuff

#ifdef HHUFF_PROFILE
namespace hhuff {
hipError_t read_prof(unsigned long long* out16, bool reset) {
    hipError_t e = hipMemcpyFromSymbol(out16, HIP_SYMBOL(g_prof), sizeof(g_prof));
    if (e == hipSuccess && reset) {
        static const unsigned long long z[16] = {};
        e = hipMemcpyToSymbol(HIP_SYMBOL(g_prof), z, sizeof(g_prof));
    }
    return e;
}
}  // namespace hhuff
#endif
