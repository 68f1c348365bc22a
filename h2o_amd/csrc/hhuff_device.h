// Device-side building blocks of the hhuff kernels (gfx950 / CDNA4, wave64).
//
// Semantics restated from the reference (file:line under /root/reference):
//   decode  lib/http2/hpack.c:85-156   (nibble FSM; accept rule misc/mkhufftbl.py:374-381)
//   encode  lib/http2/hpack.c:774-804  (40-bit accumulator; SIZE_MAX unless strictly shorter)
// The MI355X formulation differs from the reference's (same results, bit for bit):
//   * decode peeks a 13-bit window per step through an 8192-entry LUT in LDS that yields up to two
//     symbols.  Codes longer than 13 bits (and EOS) go through the leading-ones table: every RFC 7541
//     code is k leading ones, a zero, and at most 5 more bits, so k = clz(~window) plus <= 5 bits index
//     a 348-entry table.  A symbol is taken only when its whole code lies inside the string, so bits
//     past the end never matter; the string is accepted iff no EOS was decoded and the R <= 7 unused
//     bits are all ones (the reference's ACCEPTED state, mkhufftbl.py:374-381).
//   * encode packs codes MSB-first into a 64-bit accumulator and emits 32 bits at a time; a string
//     fails as soon as its Huffman length can no longer be shorter than its input (hpack.c:789-800).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "hhuff_tables.h"

namespace hhuff {


constexpr uint32_t kLong = 1u << 31;  // window LUT bits: tools/gen_tables.py:window_lut
constexpr uint32_t kHas2 = 1u << 30;
// window LUT entry fields: [7:0] sym1, [11:8] L1, [15:12] L12, [23:16] sym2 (stored by a byte store of the
// entry's high half, no shift), [27:24] validity flags, [29:28] symbol count
__host__ __device__ __forceinline__ uint32_t lut_l1(uint32_t e) { return (e >> 8) & 15u; }
__host__ __device__ __forceinline__ uint32_t lut_l12(uint32_t e) { return (e >> 12) & 15u; }
__host__ __device__ __forceinline__ uint32_t lut_sym2(uint32_t e) { return e >> 16; }  // low byte: the symbol
__host__ __device__ __forceinline__ uint32_t lut_pair(uint32_t e) { return (e & 0xFFu) | ((e >> 8) & 0xFF00u); }
constexpr uint32_t kEos = 256;
constexpr uint32_t kFailLen = 0xFFFFFFFFu;
constexpr uint8_t kStatusFail = 0x80;
constexpr uint8_t kStatusTooLong = 0xC0;
constexpr uint32_t kMaxStrLen = (1u << 29) - 1;
constexpr uint64_t kArenaLimit = 1ull << 32;  // header-block arenas: field offsets are u32

__device__ __forceinline__ uint32_t bswap32(uint32_t x) { return __builtin_bswap32(x); }

// decode slot of an input offset: floor(8 * x / 5), the tight output bound (shortest code = 5 bits)
__device__ __forceinline__ uint64_t dec_slot(uint32_t x) { return ((uint64_t)x * 8u) / 5u; }

// ---------------------------------------------------------------------------------------------------
// wave helpers
// ---------------------------------------------------------------------------------------------------
// Wave-wide reductions and scan with DPP (row shifts within 16-lane rows, then row broadcasts across
// them): no LDS / ds_bpermute traffic and no per-lane address registers.  The results of the
// reductions are read from lane 63, so they are wave-uniform (SGPR) values.
template <int CTRL, int ROW_MASK = 0xF>
__device__ __forceinline__ uint32_t dpp(uint32_t old, uint32_t x) {
    return (uint32_t)__builtin_amdgcn_update_dpp((int)old, (int)x, CTRL, ROW_MASK, 0xF, false);
}
__device__ __forceinline__ uint32_t wave_min_u32(uint32_t v) {
    v = min(v, dpp<0x111>(v, v));  // row_shr:1 (lanes without a source keep their own value)
    v = min(v, dpp<0x112>(v, v));  // row_shr:2
    v = min(v, dpp<0x114>(v, v));  // row_shr:4
    v = min(v, dpp<0x118>(v, v));  // row_shr:8: lane 15 of each row holds the row's minimum
    v = min(v, dpp<0x142, 0xA>(v, v));  // row_bcast:15
    v = min(v, dpp<0x143, 0xC>(v, v));  // row_bcast:31: lane 63 holds the wave's minimum
    return (uint32_t)__builtin_amdgcn_readlane((int)v, 63);
}
__device__ __forceinline__ uint32_t wave_max_u32(uint32_t v) {
    v = max(v, dpp<0x111>(v, v));
    v = max(v, dpp<0x112>(v, v));
    v = max(v, dpp<0x114>(v, v));
    v = max(v, dpp<0x118>(v, v));
    v = max(v, dpp<0x142, 0xA>(v, v));
    v = max(v, dpp<0x143, 0xC>(v, v));
    return (uint32_t)__builtin_amdgcn_readlane((int)v, 63);
}
// inclusive prefix sum over the wave (lane 63 holds the total)
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v) {
    v += dpp<0x111>(0u, v);
    v += dpp<0x112>(0u, v);
    v += dpp<0x114>(0u, v);
    v += dpp<0x118>(0u, v);
    v += dpp<0x142, 0xA>(0u, v);
    v += dpp<0x143, 0xC>(0u, v);
    return v;
}
// exclusive prefix sum over the wave
__device__ __forceinline__ uint32_t wave_excl_scan(uint32_t v, int lane) {
    (void)lane;
    return wave_incl_scan(v) - v;
}

__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}


// ---------------------------------------------------------------------------------------------------
// Byte sources.  word(a) returns the little-endian dword at 4-aligned position a.
// ---------------------------------------------------------------------------------------------------
struct LdsSource {  // a wave's staged input span; positions relative to the 16-aligned span start
    const uint32_t* base;
    uint32_t last;  // last readable dword position (reads are clamped: bits past a string are don't-care)
    __device__ __forceinline__ uint32_t word(uint32_t a) const { return base[min(a, last) >> 2]; }
};

struct GlobalSource {  // absolute offsets into `in`; never reads at or past in_size
    const uint8_t* in;
    uint64_t in_size;
    __device__ __forceinline__ uint32_t word(uint32_t a) const {
        if ((uint64_t)a + 4 <= in_size) return *reinterpret_cast<const uint32_t*>(in + a);
        uint32_t v = 0;
        for (uint32_t k = 0; k < 4; ++k)
            if ((uint64_t)a + k < in_size) v |= (uint32_t)in[a + k] << (8 * k);
        return v;
    }
};

// ---------------------------------------------------------------------------------------------------
// Byte sinks.
// LdsSink: bytes go to the wave's LDS output stage (copied out coalesced afterwards).
// RegSink: lane-private byte stream straight to global memory, dword stores once 4-aligned.
// ---------------------------------------------------------------------------------------------------
struct LdsSink {
    uint8_t* base;  // LDS
    uint32_t op;    // next byte position
    uint32_t start;
    uint32_t trash;  // lane-private scratch byte for predicated-off second writes
    __device__ __forceinline__ void put1(uint32_t b) { base[op] = (uint8_t)b; op += 1; }
    __device__ __forceinline__ void put12(uint32_t syms, bool two) {
        base[op] = (uint8_t)syms;
        base[two ? op + 1 : trash] = (uint8_t)(syms >> 8);
        op += two ? 2u : 1u;
    }
    __device__ __forceinline__ void put4(uint32_t w) {  // w: 4 bytes in output order, first in bits 0..7
        base[op] = (uint8_t)w;
        base[op + 1] = (uint8_t)(w >> 8);
        base[op + 2] = (uint8_t)(w >> 16);
        base[op + 3] = (uint8_t)(w >> 24);
        op += 4;
    }
    __device__ __forceinline__ void putn(uint32_t w, uint32_t n) {
        for (uint32_t k = 0; k < n; ++k) base[op + k] = (uint8_t)(w >> (8 * k));
        op += n;
    }
    __device__ __forceinline__ uint32_t count() const { return op - start; }
    __device__ __forceinline__ void finish() {}
};

struct RegSink {
    uint8_t* p;
    uint64_t acc;  // pending bytes, first byte in bits 0..7
    uint32_t pending, cnt;
    __device__ __forceinline__ void init(uint8_t* dst) { p = dst; acc = 0; pending = 0; cnt = 0; }
    __device__ __forceinline__ void push(uint32_t bytes, uint32_t k) {  // k in 1..4
        acc |= (uint64_t)(bytes & (0xFFFFFFFFu >> (32 - 8 * k))) << (8 * pending);
        pending += k;
        cnt += k;
        if (__builtin_expect(((uintptr_t)p & 3) != 0, 0)) {
            while (pending > 0 && ((uintptr_t)p & 3) != 0) {
                *p++ = (uint8_t)acc;
                acc >>= 8;
                --pending;
            }
        }
        if (pending >= 4) {
            *reinterpret_cast<uint32_t*>(p) = (uint32_t)acc;
            p += 4;
            acc >>= 32;
            pending -= 4;
        }
    }
    __device__ __forceinline__ void put1(uint32_t b) { push(b & 0xFFu, 1); }
    __device__ __forceinline__ void put12(uint32_t syms, bool two) { push(two ? (syms & 0xFFFFu) : (syms & 0xFFu), two ? 2u : 1u); }
    __device__ __forceinline__ void put4(uint32_t w) { push(w, 4); }
    __device__ __forceinline__ void putn(uint32_t w, uint32_t n) { push(w, n); }
    __device__ __forceinline__ uint32_t count() const { return cnt; }
    __device__ __forceinline__ void finish() {
        while (pending > 0) {
            *p++ = (uint8_t)acc;
            acc >>= 8;
            --pending;
        }
    }
};

// CountSink: counts the bytes and remembers the first and last one, writes nothing (first pass of the
// packed-output direct path: the lengths fix every string's place before the second pass writes).
struct CountSink {
    uint32_t cnt, first, last;
    __device__ __forceinline__ void init() { cnt = first = last = 0; }
    __device__ __forceinline__ void put1(uint32_t b) {
        first = cnt == 0 ? (b & 0xFFu) : first;
        last = b & 0xFFu;
        cnt += 1;
    }
    __device__ __forceinline__ void put12(uint32_t syms, bool two) {
        first = cnt == 0 ? (syms & 0xFFu) : first;
        last = (two ? (syms >> 8) : syms) & 0xFFu;
        cnt += two ? 2u : 1u;
    }
    __device__ __forceinline__ uint32_t count() const { return cnt; }
    __device__ __forceinline__ void finish() {}
};

// ---------------------------------------------------------------------------------------------------
// Huffman bit reader: 64-bit MSB-aligned window; invariant at the top of a step: nb >= 33.
// ---------------------------------------------------------------------------------------------------
template <class Src>
struct BitReader {
    uint64_t buf;  // next bits, MSB first; bits below the valid count are zero
    uint32_t nb;   // valid bits in buf
    uint32_t a;    // position of the next dword to load (4-aligned)

    __device__ __forceinline__ void init(const Src& src, uint32_t start) {
        a = start & ~3u;
        uint32_t skip = start & 3u;
        buf = (uint64_t)(bswap32(src.word(a)) << (8 * skip)) << 32;
        nb = 32 - 8 * skip;
        a += 4;
        refill(src);
    }
    __device__ __forceinline__ void refill(const Src& src) {
        buf |= (uint64_t)bswap32(src.word(a)) << (32 - nb);
        nb += 32;
        a += 4;
    }
    __device__ __forceinline__ void consume(uint32_t n, const Src& src) {
        buf <<= n;
        nb -= n;
        if (nb <= 32) refill(src);
    }
    __device__ __forceinline__ uint32_t hi() const { return (uint32_t)(buf >> 32); }
};

struct DecTables {  // LDS copies
    const uint32_t* lut;    // 2^HHUFF_LUT_BITS window entries
    const uint32_t* kinfo;  // 31 leading-ones entries
    const uint32_t* ones;   // HHUFF_ONES_NENT symbol entries
};

struct DecResult {
    uint32_t len;
    uint8_t status;
    uint32_t flags;
    bool ok;
};

// ---------------------------------------------------------------------------------------------------
// decode one string (h2o_hpack_decode_huffman semantics) from `src` [start, start+len) into `sink`.
// Returns ok / decoded count / accumulated invalid-char flags (bit0 name, bit1 value); the caller
// derives the status from the first and last decoded bytes.
// ---------------------------------------------------------------------------------------------------
template <class Src, class Sink>
__device__ __forceinline__ DecResult decode_core(const Src& src, uint32_t start, uint32_t len, Sink& sink,
                                                 const DecTables& T) {
    BitReader<Src> br;
    br.init(src, start);
    uint32_t R = 8 * len;  // string bits not yet consumed
    uint32_t flags = 0;
    bool fail = false;
    for (;;) {
        const uint32_t w = br.hi();
        const uint32_t e = T.lut[w >> (32 - HHUFF_LUT_BITS)];
        if (__builtin_expect((e & kLong) != 0, 0)) {
            // code longer than the window (or EOS): leading-ones table
            const uint32_t k = min((uint32_t)__builtin_clz(~w | 1u), 30u);  // ~w | 1: 32 ones -> 31, capped
            const uint32_t ki = T.kinfo[k];
            const uint32_t idx = (ki & 0xFFFFu) + (((w << (k + 1)) >> 1) >> (31 - (ki >> 16)));
            const uint32_t le = T.ones[idx];
            const uint32_t L = (le >> 9) & 31u;
            if (L > R) break;  // incomplete code: padding
            const uint32_t sym = le & 0x1FFu;
            if (sym == kEos) {  // EOS inside the string (hpack.c:88-89)
                fail = true;
                break;
            }
            sink.put1(sym);
            flags |= (le >> 14) & 3u;
            R -= L;
            br.consume(L, src);
        } else {
            const uint32_t L1 = lut_l1(e);
            if (L1 > R) break;  // fewer bits left than the next code: padding
            const uint32_t L12 = lut_l12(e);
            const bool two = (e & kHas2) && L12 <= R;
            const uint32_t cons = two ? L12 : L1;
            sink.put12(lut_pair(e), two);
            flags |= (e >> 24) & (two ? 15u : 3u);
            R -= cons;
            br.consume(cons, src);
        }
    }
    DecResult r;
    // accept iff no EOS and the padding is <= 7 bits of ones (mkhufftbl.py:374-381, hpack.c:132-133)
    r.ok = !fail && R <= 7 && ((br.hi() >> 24) | (0xFFu >> R)) == 0xFFu;
    r.len = sink.count();
    r.flags = (flags | (flags >> 2)) & 3u;
    r.status = 0;
    return r;
}

typedef __attribute__((address_space(3))) uint8_t lds_u8;
typedef __attribute__((address_space(3))) uint32_t lds_u32;

__device__ __forceinline__ uint32_t lds_addr(const void* p) { return (uint32_t)(size_t)(const lds_u8*)p; }
__device__ __forceinline__ void lds_st8(uint32_t addr, uint32_t v) { *(lds_u8*)(size_t)addr = (uint8_t)v; }
__device__ __forceinline__ uint32_t sel_bits(uint32_t m, uint32_t a, uint32_t b) { return (m & a) | (~m & b); }
__device__ __forceinline__ void lds_or32(uint32_t addr, uint32_t v) {
    __hip_atomic_fetch_or((lds_u32*)(size_t)addr, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ uint32_t lds_ld8(uint32_t addr) { return *(const lds_u8*)(size_t)addr; }
__device__ __forceinline__ uint32_t lds_ld32(uint32_t addr) { return *(const lds_u32*)(size_t)addr; }
__device__ __forceinline__ void lds_st32(uint32_t addr, uint32_t v) { *(lds_u32*)(size_t)addr = v; }

// Move n bytes from LDS byte address src to LDS byte address dst: one lane's string in a packed-output
// compaction (the wave's prefix sum of the lengths gives dst).  The destination range must be zero: every
// destination dword the string touches is OR-ed in (ds_or_b32), bytes outside [dst, dst + n) as zeros, so
// the dwords a string shares with its neighbours need no byte stores and no ordering between lanes.  The
// source is read as aligned dwords from 3 bytes before src on (those bytes are masked out) and shifted to
// the destination's phase with v_alignbyte.  SWAP: the source holds MSB-first words (the encode stage),
// byte-swapped on the way.
template <bool SWAP = false>
__device__ __forceinline__ void lds_move_or(uint32_t src, uint32_t dst, uint32_t n) {
    if (n == 0) return;
    const uint32_t ph = dst & 3u;
    const uint32_t s0 = src - ph;  // source byte of the first destination dword's byte 0
    const uint32_t q = s0 & ~3u, sh = s0 & 3u;
    const uint32_t nd = (ph + n + 3u) >> 2;  // destination dwords
    const uint32_t d4 = dst & ~3u;
    const uint32_t hi_last = ph + n - 4u * (nd - 1u);  // bytes of the last dword that are ours (1..4)
    auto rd = [&](uint32_t a) { const uint32_t w = lds_ld32(a); return SWAP ? bswap32(w) : w; };
    // four destination dwords per round: the five source reads are issued back to back, one wait per round
    for (uint32_t k = 0; k < nd; k += 4u) {
        uint32_t w[5];
#pragma unroll
        for (uint32_t j = 0; j < 5; ++j) w[j] = rd(q + 4u * (k + j));
#pragma unroll
        for (uint32_t j = 0; j < 4; ++j) {
            const uint32_t kk = k + j;
            uint32_t m = kk == 0 ? 0xFFFFFFFFu << (8u * ph) : 0xFFFFFFFFu;
            m &= kk + 1u == nd ? 0xFFFFFFFFu >> (32u - 8u * hi_last) : 0xFFFFFFFFu;
            if (kk < nd) lds_or32(d4 + 4u * kk, __builtin_amdgcn_alignbyte(w[j + 1], w[j], sh) & m);
        }
    }
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

// The wave copies 64 byte segments at once (lane i holds segment i: src, dst, len; len 0 = none) in 16-byte
// pieces spread over all lanes (whole pieces as unaligned 16-B accesses, tails bytewise), so a long segment does not serialise one lane: every 64 pieces cost one
// round trip.  Piece t belongs to the last lane k whose piece prefix excl[k] <= t (binary search by lanes).
__device__ void wave_copy64(const uint8_t* src, uint8_t* dst, uint32_t len, int lane) {
    const uint32_t chunks = (len + 15u) >> 4;
    const uint32_t excl = wave_excl_scan(chunks, lane);
    const uint32_t total = (uint32_t)__builtin_amdgcn_readlane((int)(excl + chunks), 63);
    for (uint32_t t0 = 0; t0 < total; t0 += 64) {
        const uint32_t t = t0 + (uint32_t)lane;
        int k = 0;
#pragma unroll
        for (int step = 32; step > 0; step >>= 1) {
            const uint32_t e = (uint32_t)__shfl((int)excl, k + step);
            k += e <= t ? step : 0;
        }
        const uint32_t c = t - (uint32_t)__shfl((int)excl, k);
        const uint8_t* s = (const uint8_t*)__shfl((long long)(uintptr_t)src, k);
        uint8_t* d = (uint8_t*)__shfl((long long)(uintptr_t)dst, k);
        const uint32_t n = (uint32_t)__shfl((int)len, k);
        if (t < total) {
            const uint32_t a = 16u * c, m = min(16u, n - a);
            if (m == 16) {  // a whole piece: one unaligned 16-B load and store (inside both strings)
                uint4 w;
                __builtin_memcpy(&w, s + a, 16);
                __builtin_memcpy(d + a, &w, 16);
            } else {  // the tail: bytes, so nothing outside the two strings is touched
                uint8_t v[16];
#pragma unroll
                for (uint32_t j = 0; j < 15; ++j)
                    if (j < m) v[j] = s[a + j];
#pragma unroll
                for (uint32_t j = 0; j < 15; ++j)
                    if (j < m) d[a + j] = v[j];
            }
        }
    }
}

// Field copies of up to 64 consecutive field lists (header blocks / sections) per wave: lane j holds list
// j's first field slot s0 and field count nf (0 for no list); the lists' 2 nf name / value segments are
// numbered back to back and handed to wave_copy64 64 at a time, so a wave stays full however few fields a
// list has.  seg(slot, val, src, dst, len) describes one segment (len 0: nothing to copy).
template <class Seg>
__device__ __forceinline__ void wave_copy_fields(uint32_t s0, uint32_t nf, int lane, Seg seg) {
    const uint32_t cnt = 2u * nf;
    const uint32_t excl = wave_excl_scan(cnt, lane);
    const uint32_t total = (uint32_t)__builtin_amdgcn_readlane((int)(excl + cnt), 63);
    for (uint32_t r0 = 0; r0 < total; r0 += 64) {
        const uint32_t t = r0 + (uint32_t)lane;
        int k = 0;  // the last lane whose segment prefix is <= t
#pragma unroll
        for (int step = 32; step > 0; step >>= 1) {
            const uint32_t e = (uint32_t)__shfl((int)excl, k + step);
            k += e <= t ? step : 0;
        }
        const uint32_t w = t - (uint32_t)__shfl((int)excl, k);
        const uint32_t slot = (uint32_t)__shfl((int)s0, k) + (w >> 1);
        const uint8_t* src = nullptr;
        uint8_t* dst = nullptr;
        uint32_t len = 0;
        if (t < total) seg(slot, (w & 1u) != 0, src, dst, len);
        wave_copy64(src, dst, len, lane);
    }
}

// Zero LDS bytes [a, b) of a wave's buffer (a, b multiples of 16), 16-B stores by the whole wave.
__device__ __forceinline__ void lds_zero(uint8_t* base, uint32_t a, uint32_t b, int lane) {
    for (uint32_t k = a + 16u * (uint32_t)lane; k < b; k += 1024u)
        *reinterpret_cast<uint4*>(base + k) = make_uint4(0u, 0u, 0u, 0u);
}

// A bulk step's two symbol bytes (decode_staged_lane_v7, the stream kernels): both bytes at o and o + 1 as they
// are, whatever the entry holds -- with >= 27 string bits left the bytes past the symbols taken are rewritten by
// the lane's next symbols or lie past its decoded length inside its slot (5 symbols' room), so the stores need
// no redirection of untaken bytes to a trash byte (c4 decode -7 % against that; one unaligned ds_write_b16 for
// both bytes was measured too: 0.66 -> 0.98 ms).
#ifndef HHUFF_DEC_READ_FIRST  // 1 (default): a bulk step's second LUT read goes to the LDS ahead of the first entry's
#define HHUFF_DEC_READ_FIRST 1   // byte stores: c4 decode -0.6 %, c3 -0.9 % (profiles/r06m_decode_read_first_ab.jsonl)
#endif
__device__ __forceinline__ void bulk_put2(uint32_t o, uint32_t e, uint32_t trash) {
    (void)trash;
    lds_st8(o, e);
    lds_st8(o + 1u, lut_sym2(e));
}

// ---------------------------------------------------------------------------------------------------
// Staged decode, v7: a BULK phase and a TAIL phase (same results as decode_core).
// Bulk steps run only for lanes with >= 27 string bits left (pm < lim = end - 26; inactive and parked
// lanes have lim = INT_MIN), so everything both lookups of a step hold lies inside the string: there are
// no end-of-string take-masks, the entry says what to take -- [29:28] symbol count, L12 bits (none for
// LONG) -- and flag bits of absent symbols are zero, so `accb |= e` collects them.  Lanes below lim are
// switched off (exec mask) until the bulk loop drains; then the checked tail step finishes every lane
// (<= 26 bits, at most ~3 steps).  Bulk VALU per step is about half of the checked step's.  Codes longer than the
// window take the same wave-uniform detour (fit checked against `end`; EOS or a code that cannot fit
// parks the lane, which then fails).
// ---------------------------------------------------------------------------------------------------
__device__ __forceinline__ DecResult decode_staged_lane_v7(const uint32_t* stage, uint32_t start, uint32_t len,
                                                           bool active, uint8_t* obuf, uint32_t op0, uint32_t trash_off,
                                                           const DecTables& T) {
    const lds_u32* st = (const lds_u32*)stage;
    int32_t pm = (int32_t)(8u * start) - 1;
    const int32_t end = (int32_t)(8u * (start + len));
    int32_t q = pm >> 5;
    uint32_t x0 = st[q], x1 = st[q + 1], x2 = st[q + 2];
    const uint32_t o0 = lds_addr(obuf) + op0, trash = lds_addr(obuf) + trash_off;  // trash: 4 lane-private bytes
    uint32_t o = o0, accb = 0, acc1 = 0, acc2 = 0, accl = 0, fail = 0, parked = active ? 0u : 1u;
    int32_t lim = active ? end - 26 : (int32_t)0x80000000;

    auto advance = [&](int32_t cons) {
        pm += cons;
        const int32_t qn = pm >> 5;
        const bool adv = qn != q;
        x0 = adv ? x1 : x0;
        x1 = adv ? x2 : x1;
        q = qn;
        x2 = st[q + 2];
    };
    auto bstep = [&](bool longchk) {
        if (pm < lim) {
            const uint32_t w = __builtin_amdgcn_alignbit(x0, x1, ~(uint32_t)pm);
            const uint32_t e = T.lut[w >> (32 - HHUFF_LUT_BITS)];
            const uint32_t sl = (uint32_t)((int32_t)e >> 31);  // LONG: nothing taken from the window
            uint32_t cons = lut_l12(e);  // LONG entries carry L12 = 0
#if HHUFF_DEC_READ_FIRST
            {  // the second lookup goes to the LDS ahead of the first entry's byte stores (in-order LDS queue)
                const uint32_t wb = w << cons;
                const uint32_t eb = T.lut[wb >> (32 - HHUFF_LUT_BITS)];
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
                const uint32_t wb = w << cons;
                const uint32_t eb = T.lut[wb >> (32 - HHUFF_LUT_BITS)];
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

    // ---- tail: the checked step.  c = p - end - 1 is negative while bits remain, so "a code of L bits
    // fits" is the sign of L + c; with LONG / HAS2 in the LUT's top bits the take-masks m1 (first symbol)
    // and m2 (second symbol) are sign bits of one AND each.  Switched-off writes go to the lane-private
    // trash byte; a lane whose next code can never fit is parked by pushing c positive. ----
    int32_t c = parked ? 0x40000000 : pm - end;
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
            const uint32_t wb = w << cons;
            const uint32_t eb = T.lut[wb >> (32 - HHUFF_LUT_BITS)];
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
    for (;;) {  // the vote follows a long-code step: a lane with no progress there is finished
        step(false);
        step(true);
        if (!__any(prog != 0)) break;
    }
    DecResult r;
    const uint32_t R = ~(uint32_t)c;
    const uint32_t w = __builtin_amdgcn_alignbit(x0, x1, ~(uint32_t)pm);
    r.ok = active && !fail && R <= 7 && (w | (0xFFFFFFFFu >> (R & 31u))) == 0xFFFFFFFFu;
    r.len = o - o0;
    r.flags = ((accb >> 24) | (accb >> 26) | (acc1 >> 24) | (acc2 >> 26) | (accl >> 14)) & 3u;
    r.status = 0;
    return r;
}

// hpack.c:136-152: soft-error bits from the accumulated flags and the first / last decoded bytes
__device__ __forceinline__ uint8_t soft_bits(bool is_name, uint32_t cnt, uint32_t flags, uint32_t first, uint32_t last) {
    if (is_name)  // ':'-prefixed names are not validated; upper case is only soft (hpack.c:136-147)
        return (cnt == 0 || ((flags & 1u) && first != ':')) ? 0x1 : 0x0;
    const bool ws = cnt != 0 && (first == ' ' || first == '\t' || last == ' ' || last == '\t');  // :110-115
    return ((flags & 2u) || ws) ? 0x2 : 0x0;
}

// ---------------------------------------------------------------------------------------------------
// encode one string (h2o_hpack_encode_huffman semantics).  enc = 256 x {code, nbits} in LDS.
// Emits at most len - 1 bytes into `sink`; returns the Huffman length or kFailLen.
// ---------------------------------------------------------------------------------------------------
template <class Src, class Sink>
__device__ __forceinline__ uint32_t encode_core(const Src& src, uint32_t start, uint32_t len, Sink& sink,
                                                const uint2* __restrict__ enc) {
    uint64_t acc = 0;  // code bits, MSB-aligned
    uint32_t an = 0;   // bits in acc (< 32 between symbols)
    uint32_t emitted = 0;
    bool fail = false;
    const uint32_t end = start + len;
    for (uint32_t a = start & ~3u; a < end; a += 4) {
        const uint32_t w = src.word(a);
#pragma unroll
        for (uint32_t k = 0; k < 4; ++k) {
            const uint32_t pos = a + k;
            const bool valid = pos >= start && pos < end;
            const uint2 ent = enc[(w >> (8 * k)) & 0xFFu];
            const uint32_t nb = valid ? ent.y : 0u;
            const uint64_t code = valid ? (uint64_t)ent.x : 0ull;
            acc |= code << (64 - an - nb);
            an += nb;
            if (an >= 32) {
                if (emitted + 4 >= len) {  // can no longer end up shorter than the input
                    fail = true;
                    break;
                }
                sink.put4(bswap32((uint32_t)(acc >> 32)));
                emitted += 4;
                acc <<= 32;
                an -= 32;
            }
        }
        if (fail) break;
    }
    const uint32_t tail = (an + 7) >> 3;
    if (fail || emitted + tail >= len) return kFailLen;  // hpack.c:789-791, :799-800
    if (an != 0) acc |= ~0ull >> an;                        // pad with the EOS prefix (hpack.c:795-798)
    if (tail) sink.putn(bswap32((uint32_t)(acc >> 32)), tail);
    sink.finish();
    return emitted + tail;
}

// Fused encode path of encode_chunk: the four codes of a dword enter the accumulator as two 32-bit pairs
// when every code is <= 16 bits; a longer code takes a wave-uniform byte-by-byte detour.
constexpr uint32_t kFusedMaxBits = 16u;

// Encode the stage bytes [start, start + len) with the first code bit landing at bit `startbit` of the
// LDS output stage (MSB-first dwords, OR-ed in, so neighbouring chunks may share a dword).  The trip
// count jmax is wave-uniform (>= this lane's dword count).  `limit`: fail as soon as the code bits
// reach it (8 * len - 7 for a whole string: ceil(bits / 8) >= len; ~0 for a chunk of a longer string
// whose verdict is already known).  `pad`: this chunk ends the string, so fill its last byte with
// ones (EOS prefix, hpack.c:795-798).  Returns the code bits, or kFailLen.
__device__ __forceinline__ uint32_t encode_chunk(const uint32_t* stage, uint32_t last, uint32_t start, uint32_t len,
                                                 bool active, uint32_t* obuf32, uint32_t startbit,
                                                 const uint2* __restrict__ enc, uint32_t jmax, uint32_t limit, bool pad) {
    const uint32_t end = start + len;
    const uint32_t a0 = start & ~3u;
    const uint32_t ndw = active ? (end - a0 + 3u) >> 2 : 0u;
    const uint32_t mfirst = 0xFFFFFFFFu << (8u * (start & 3u));
    const uint32_t mlast = (uint32_t)(0xFFFFFFFFull >> ((32u - 8u * (end & 3u)) & 31u));
    uint64_t acc = 0;
    uint32_t an = startbit & 31u;
    uint32_t opw = startbit >> 5;
    uint32_t tb = 0;
    bool live = active, fail = false;
    for (uint32_t j = 0; j < jmax; ++j) {
        const uint32_t w = stage[min(a0 + 4u * j, last) >> 2];
        uint32_t vm = j == 0 ? mfirst : 0xFFFFFFFFu;
        vm &= (j + 1 == ndw) ? mlast : 0xFFFFFFFFu;
        vm = (live && j < ndw) ? vm : 0u;
        const uint32_t iw = ~vm & 0x01010101u;
        const uint2 e0 = enc[__builtin_amdgcn_perm(iw, w, 0x0C0C0400u)];
        const uint2 e1 = enc[__builtin_amdgcn_perm(iw, w, 0x0C0C0501u)];
        const uint2 e2 = enc[__builtin_amdgcn_perm(iw, w, 0x0C0C0602u)];
        const uint2 e3 = enc[__builtin_amdgcn_perm(iw, w, 0x0C0C0703u)];
        const bool lng = max(max(e0.y, e1.y), max(e2.y, e3.y)) > kFusedMaxBits;
        const uint32_t n = e0.y + e1.y + e2.y + e3.y;
        const bool over = tb + n >= limit;
        if (__any(lng && !over)) {  // a code too long for the fused path: byte by byte (wave-uniform detour)
            if (lng && !over) {
                const uint2 ek[4] = {e0, e1, e2, e3};
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    const uint32_t nk = ek[k].y;
                    acc |= (uint64_t)ek[k].x << ((64u - an - nk) & 63u);
                    an += nk;
                    tb += nk;
                    const uint32_t e = an >= 32 ? 1u : 0u;
                    atomicOr(&obuf32[opw], e ? bswap32((uint32_t)(acc >> 32)) : 0u);
                    acc <<= 32u * e;
                    an -= 32u * e;
                    opw += e;
                }
            }
        }
        fail = fail || over;
        live = live && !over;
        const bool put = live && !lng;
        // codes <= 16 bits: two 32-bit pairs, each inserted and (at most one word) emitted in turn
        const uint32_t p01 = put ? (e0.x << e1.y | e1.x) : 0u, n01 = put ? e0.y + e1.y : 0u;
        const uint32_t p23 = put ? (e2.x << e3.y | e3.x) : 0u, n23 = put ? e2.y + e3.y : 0u;
        {
            acc |= (uint64_t)p01 << ((64u - an - n01) & 63u);
            an += n01;
            const uint32_t e = an >= 32 ? 1u : 0u;
            atomicOr(&obuf32[opw], e ? bswap32((uint32_t)(acc >> 32)) : 0u);
            acc <<= 32u * e;
            an -= 32u * e;
            opw += e;
        }
        acc |= (uint64_t)p23 << ((64u - an - n23) & 63u);
        an += n23;
        tb += n01 + n23;
        const uint32_t e = an >= 32 ? 1u : 0u;
        atomicOr(&obuf32[opw], e ? bswap32((uint32_t)(acc >> 32)) : 0u);
        acc <<= 32u * e;
        an -= 32u * e;
        opw += e;
    }
    if (fail || !active) return kFailLen;
    if (pad) {
        const uint32_t an8 = (an + 7) & ~7u;
        acc |= (~0ull >> an) & ~(~0ull >> an8);
    }
    if (an) atomicOr(&obuf32[opw], bswap32((uint32_t)(acc >> 32)));
    return tb;
}

// ---------------------------------------------------------------------------------------------------
// Encode v2: stateless bit placement + a bulk phase (same results as encode_core).
// The output stage holds the code stream as MSB-first u32 words (bit 31 of word k = stream bit 32k), so
// n <= 64 code bits land at absolute stage bit tb with at most three ds_or_b32 and no accumulator:
// left-align them in 64 bits, shift right by tb % 32 for words k, k+1, and the bits shifted out go to
// word k+2 (only when tb % 32 + n > 64).  OR is order-free, so there is no emit state to carry and no
// per-step flush; the caller byte-swaps the stage's words once before copying out.
// A lane's dwords split into a head (the first dword, when the string does not start on it), whole
// dwords (bulk: no byte masks, one placement of all four codes when each is <= 16 bits), and a tail (the
// last, partial dword).  Head and tail use the masked lookups (entries 256..511 are zero); bulk steps
// run for lanes inside their whole-dword range with the others switched off (exec mask).
// ---------------------------------------------------------------------------------------------------
// The output stage is addressed either by its LDS byte address (uint32_t) or by a word pointer derived from the
// __shared__ array itself (uint32_t*): with the pointer the compiler can tell the stage from other LDS objects
// (an LDS-DMA in flight into another buffer then needs no wait before an OR; round 6's double-buffered framing
// kernel used it, and lost: profiles/r06h_flatten_double_buffer_ab.jsonl).
__device__ __forceinline__ void or_word(uint32_t obase, uint32_t wi, uint32_t v) { lds_or32(obase + 4u * wi, v); }
__device__ __forceinline__ void or_word(uint32_t* o32, uint32_t wi, uint32_t v) {
    __hip_atomic_fetch_or(o32 + wi, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
template <class O>
__device__ __forceinline__ void place_bits(O obase, uint32_t tb, uint64_t c, uint32_t n) {
    const uint64_t t = c << ((64u - n) & 63u);  // left-aligned (n == 0 needs c == 0)
    const uint32_t sh = tb & 31u;
    const uint64_t u = t >> sh;
    const uint32_t a = tb >> 5;
    or_word(obase, a, (uint32_t)(u >> 32));
    or_word(obase, a + 1u, (uint32_t)u);
    if (sh + n > 64u) or_word(obase, a + 2u, (uint32_t)t << (32u - sh));  // sh > 0 here
}

#ifndef HHUFF_ENC_HEAD_REUSE  // encode_chunk_v2: the head's stage word seeds the bulk loop (no second read of it)
#define HHUFF_ENC_HEAD_REUSE 0
#endif
#ifndef HHUFF_ENC_OR3  // encode_chunk_v2's bulk step: the third output word ORed on every step (see put4m)
#define HHUFF_ENC_OR3 0
#endif

template <class O>
struct EncV2 {
    const uint2* enc;
    O obase;  // the MSB-first output stage: LDS byte address or word pointer (see or_word)
    uint32_t tb;     // next stage bit
    uint32_t tlim;   // stage bit at which the string fails (~0: no limit)
    bool live, fail;
    // four table entries of one input dword; `on`: this lane has these bytes
    __device__ __forceinline__ void put4(uint2 e0, uint2 e1, uint2 e2, uint2 e3, bool on) {
        const uint32_t n01 = e0.y + e1.y, n23 = e2.y + e3.y, n = n01 + n23;
        const bool lng = max(max(e0.y, e1.y), max(e2.y, e3.y)) > 16u;
        const bool over = on && live && tb + n >= tlim;
        fail = fail || over;
        live = live && !over;
        const bool put = on && live;
        if (__any(put && lng)) {  // a code longer than 16 bits: two placements of 64-bit pairs
            if (put && lng) {
                place_bits(obase, tb, (uint64_t)e0.x << e1.y | e1.x, n01);
                place_bits(obase, tb + n01, (uint64_t)e2.x << e3.y | e3.x, n23);
            }
        }
        const bool f = put && !lng;
        const uint32_t p01 = e0.x << e1.y | e1.x, p23 = e2.x << e3.y | e3.x;
        const uint64_t cc = f ? ((uint64_t)p01 << n23 | p23) : 0ull;
        place_bits(obase, tb, cc, f ? n : 0u);
        tb += put ? n : 0u;
    }
    // Same with every per-lane predicate an all-ones / zero mask in a VGPR (no exec-mask juggling on
    // the SALU): `onm` = this lane has these four bytes.
    __device__ __forceinline__ void put4m(uint2 e0, uint2 e1, uint2 e2, uint2 e3, uint32_t onm) {
        const uint32_t n01 = e0.y + e1.y, n23 = e2.y + e3.y, n = n01 + n23;
        const uint32_t mx = max(max(e0.y, e1.y), max(e2.y, e3.y));
        const uint32_t lngm = (uint32_t)((int32_t)(16u - mx) >> 31);                 // a code > 16 bits
        // the running bit count grows with every byte of the lane, placed or not: once a dword would reach
        // tlim every later one does too, so "tb + n < tlim" alone says whether this dword is placed (the
        // verdict is tb >= tlim after the loop; -4 % c4 encode against masks carried from dword to dword)
        const uint32_t nm = n & onm;
        const uint32_t putm = onm & (uint32_t)((int32_t)(tb + nm - tlim) >> 31);
        if (__builtin_amdgcn_ballot_w64((putm & lngm) != 0u) != 0) {
            if (putm & lngm) {
                place_bits(obase, tb, (uint64_t)e0.x << e1.y | e1.x, n01);
                place_bits(obase, tb + n01, (uint64_t)e2.x << e3.y | e3.x, n23);
            }
        }
        const uint32_t fm = putm & ~lngm;
        const uint32_t p01 = e0.x << e1.y | e1.x, p23 = e2.x << e3.y | e3.x;
        const uint64_t cc = ((uint64_t)p01 << n23 | p23) & ((uint64_t)fm << 32 | fm);
        const uint32_t nf = n & fm;
        const uint64_t t = cc << ((64u - nf) & 63u);
        const uint32_t sh = tb & 31u;
        const uint64_t u = t >> sh;
        const uint32_t a = tb >> 5;
#if defined(HHUFF_X_ENC_NOOR)  // ablation (output wrong by design): no placement (one OR keeps the values live)
        if (__builtin_amdgcn_ballot_w64((uint32_t)u == 0x12345u) != 0) or_word(obase, a, (uint32_t)(u >> 32));
#else
        or_word(obase, a, (uint32_t)(u >> 32));
        or_word(obase, a + 1u, (uint32_t)u);
#endif
#if HHUFF_ENC_OR3  // the third word's OR on every step (0 where nothing spills into it): no vote, no branch
        or_word(obase, a + 2u, sh + nf > 64u ? (uint32_t)t << ((32u - sh) & 31u) : 0u);
#else
        if (__builtin_amdgcn_ballot_w64(sh + nf > 64u) != 0) {
            if (sh + nf > 64u) or_word(obase, a + 2u, (uint32_t)t << (32u - sh));
        }
#endif
        tb += nm;
    }
};

// Encode stage bytes [start, start + len) to stage bit `startbit` of the MSB-first output stage at LDS
// byte address `obase`.  `limit`, `pad`: as encode_chunk.  Returns the code bits or kFailLen.
#ifndef HHUFF_ENC_SORTED_U  // whole dwords a bulk-loop trip (encode_chunk_v2's U) in the sorted encoder
#define HHUFF_ENC_SORTED_U 1
#endif
#ifndef HHUFF_ENC_OTHER_U   // ... and in the staged / proportional-lane encoders and the framing kernel
#define HHUFF_ENC_OTHER_U 1
#endif
// U: whole dwords a trip of the bulk loop (1 or 2; the loop's ballots keep the compiler from unrolling it)
template <int U = 1, class O>
__device__ __forceinline__ uint32_t encode_chunk_v2(const uint32_t* stage, uint32_t last, uint32_t start, uint32_t len,
                                                    bool active, O obase, uint32_t startbit,
                                                    const uint2* __restrict__ enc, uint32_t limit, bool pad) {
    const uint32_t end = start + len;
    const uint32_t a0 = start & ~3u;
    const uint32_t ndw = active ? (end - a0 + 3u) >> 2 : 0u;
    const uint32_t jf = (start & 3u) ? 1u : 0u;            // whole dwords: [jf, jl)
    const uint32_t jl = active ? (end - a0) >> 2 : 0u;
    const uint32_t mfirst = 0xFFFFFFFFu << (8u * (start & 3u));
    const uint32_t mlast = (uint32_t)(0xFFFFFFFFull >> ((32u - 8u * (end & 3u)) & 31u));
    // tlim < 2^31 keeps tb + n - tlim a signed quantity (stage bits are < 2^20)
    EncV2<O> E{enc, obase, startbit, limit >= 0x40000000u ? 0x7FFFFFFFu : startbit + limit, active, false};
    auto masked = [&](uint32_t j, bool on, uint32_t w) {  // one dword with byte masks (head / tail); w: its word
        uint32_t vm = j == 0 ? mfirst : 0xFFFFFFFFu;
        vm &= (j + 1 == ndw) ? mlast : 0xFFFFFFFFu;
        vm = on ? vm : 0u;
        const uint32_t iw = ~vm & 0x01010101u;
        E.put4(enc[__builtin_amdgcn_perm(iw, w, 0x0C0C0400u)], enc[__builtin_amdgcn_perm(iw, w, 0x0C0C0501u)],
               enc[__builtin_amdgcn_perm(iw, w, 0x0C0C0602u)], enc[__builtin_amdgcn_perm(iw, w, 0x0C0C0703u)], on);
    };
    // the head's word is the bulk loop's first word too (an active lane has a0 <= last; an inactive lane's words
    // are never placed): one LDS read, issued before the head's lookups and ORs
    const uint32_t w0 = stage[min(a0, last) >> 2];
    masked(0, active && jf != 0, w0);  // head
    const uint32_t* sw = stage + (a0 >> 2);
    const uint32_t jlast = (last >> 2) - (a0 >> 2);  // stage reads are clamped to the span
    {
        const uint32_t jlv = E.live ? jl : 0u;  // a lane that failed in its head places nothing more
        const uint32_t jend = wave_max_u32(jlv);  // uniform trip count: no vote per step
#if HHUFF_ENC_HEAD_REUSE
        uint32_t wn = w0;
#else
        uint32_t wn = sw[min(0u, jlast)];
#endif
        // U == 2: the extra dword past jend has onm == 0 (jlv <= jend) and a clamped read
        if constexpr (U == 2) for (uint32_t j = 0; j < jend; j += 2) {
            const uint32_t w0 = wn, w1 = sw[min(j + 1u, jlast)];
            wn = sw[min(j + 2u, jlast)];
            const uint32_t m0 = ~(uint32_t)((int32_t)((j - jf) | (jlv - 1u - j)) >> 31);
            const uint32_t m1 = ~(uint32_t)((int32_t)((j + 1u - jf) | (jlv - 2u - j)) >> 31);
            const uint2 a0 = enc[w0 & 0xFFu], a1 = enc[(w0 >> 8) & 0xFFu], a2 = enc[(w0 >> 16) & 0xFFu], a3 = enc[w0 >> 24];
            const uint2 b0 = enc[w1 & 0xFFu], b1 = enc[(w1 >> 8) & 0xFFu], b2 = enc[(w1 >> 16) & 0xFFu], b3 = enc[w1 >> 24];
            E.put4m(a0, a1, a2, a3, m0);
            E.put4m(b0, b1, b2, b3, m1);
        }
        else for (uint32_t j = 0; j < jend; ++j) {  // bulk
            const uint32_t w = wn;
            wn = sw[min(j + 1u, jlast)];
            const uint32_t onm = ~(uint32_t)((int32_t)((j - jf) | (jlv - 1u - j)) >> 31);  // jf <= j < jlv
#if defined(HHUFF_X_ENC_TABCF)  // ablation (output wrong by design): conflict-free table reads (entry = lane % 32 + 32)
            const uint32_t lq = (uint32_t)(__lane_id() & 31) + 32u + (w & 0u);
            E.put4m(enc[lq], enc[lq ^ 1u], enc[lq ^ 2u], enc[lq ^ 3u], onm);
#elif defined(HHUFF_X_ENC_TABDEP) || defined(HHUFF_X_ENC_TABBC)
            // ablations: the same conflict-free (TABDEP) / single-entry broadcast (TABBC) reads, still dependent on the
            // input word (an opaque zero from it), so the input reads and the chain stay
            uint32_t z;
            __asm__ volatile("v_and_b32 %0, 0, %1" : "=v"(z) : "v"(w));
#if defined(HHUFF_X_ENC_TABDEP)
            const uint32_t lq = (uint32_t)(__lane_id() & 31) + 32u + z;
#else
            const uint32_t lq = 0x61u + z;
#endif
            E.put4m(enc[lq], enc[lq ^ 1u], enc[lq ^ 2u], enc[lq ^ 3u], onm);
#else
            E.put4m(enc[w & 0xFFu], enc[(w >> 8) & 0xFFu], enc[(w >> 16) & 0xFFu], enc[w >> 24], onm);
#endif
        }
    }
    E.fail = E.fail || (E.live && E.tb >= E.tlim);
    E.live = E.live && !E.fail;
    masked(jl, active && (end & 3u) != 0 && jl >= jf, stage[min(a0 + 4u * jl, last) >> 2]);  // tail
    if (E.fail || !active) return kFailLen;
    const uint32_t tbits = E.tb - startbit;
    if (pad) {  // fill the last byte with ones (EOS prefix, hpack.c:795-798); strings start on a byte, so the
                // padding is the absolute stage bit's (a share of a longer string starts mid-byte)
        const uint32_t p = (0u - E.tb) & 7u;
        place_bits(obase, E.tb, (1ull << p) - 1ull, p);
    }
    return tbits;
}

// Byte-swap the words of an MSB-first output stage [0, bytes) in place (one wave; bytes % 16 == 0).
__device__ __forceinline__ void stage_bswap(uint32_t* obuf32, uint32_t bytes, int lane) {
    for (uint32_t k = (uint32_t)lane * 16u; k < bytes; k += 64u * 16u) {
        uint4 v = *reinterpret_cast<uint4*>(reinterpret_cast<uint8_t*>(obuf32) + k);
        v = make_uint4(bswap32(v.x), bswap32(v.y), bswap32(v.z), bswap32(v.w));
        *reinterpret_cast<uint4*>(reinterpret_cast<uint8_t*>(obuf32) + k) = v;
    }
}

// Code bits of the stage bytes [start, start + len), as encode_chunk_v2 walks them: a masked head dword, whole
// dwords with no byte masks (one code-length read per byte; the trip count is wave-uniform and lanes outside
// their range add nothing), a masked tail dword (pass 1 of the proportional-lane kernels).
__device__ __forceinline__ uint32_t chunk_code_bits_v2(const uint32_t* stage, uint32_t last, uint32_t start, uint32_t len,
                                                       bool active, const uint2* __restrict__ enc) {
    const uint32_t end = start + len;
    const uint32_t a0 = start & ~3u;
    const uint32_t ndw = active ? (end - a0 + 3u) >> 2 : 0u;
    const uint32_t jf = (start & 3u) ? 1u : 0u;  // whole dwords: [jf, jl)
    const uint32_t jl = active ? (end - a0) >> 2 : 0u;
    const uint32_t mfirst = 0xFFFFFFFFu << (8u * (start & 3u));
    const uint32_t mlast = (uint32_t)(0xFFFFFFFFull >> ((32u - 8u * (end & 3u)) & 31u));
    auto masked = [&](uint32_t j, bool on) {
        const uint32_t w = stage[min(a0 + 4u * j, last) >> 2];
        uint32_t vm = j == 0 ? mfirst : 0xFFFFFFFFu;
        vm &= (j + 1 == ndw) ? mlast : 0xFFFFFFFFu;
        vm = on ? vm : 0u;
        const uint32_t iw = ~vm & 0x01010101u;
        return enc[__builtin_amdgcn_perm(iw, w, 0x0C0C0400u)].y + enc[__builtin_amdgcn_perm(iw, w, 0x0C0C0501u)].y +
               enc[__builtin_amdgcn_perm(iw, w, 0x0C0C0602u)].y + enc[__builtin_amdgcn_perm(iw, w, 0x0C0C0703u)].y;
    };
    uint32_t tb = masked(0, active && jf != 0);  // head
    const uint32_t* sw = stage + (a0 >> 2);
    const uint32_t jlast = (last >> 2) - (a0 >> 2);
    const uint32_t jend = wave_max_u32(jl);
    uint32_t bulk = 0;
    for (uint32_t j = 0; j < jend; ++j) {
        const uint32_t w = sw[min(j, jlast)];
        const uint32_t n = enc[w & 0xFFu].y + enc[(w >> 8) & 0xFFu].y + enc[(w >> 16) & 0xFFu].y + enc[w >> 24].y;
        bulk += (j >= jf && j < jl) ? n : 0u;
    }
    return tb + bulk + masked(jl, active && (end & 3u) != 0 && jl >= jf);  // + tail
}

// The same count from a byte table of code lengths (nb[0..255]; nb[256] = 0 for the bytes outside the string):
// an ASCII byte's entry sits in LDS dwords 8..31, each on its own bank, so a wave's lookups meet no bank
// conflict (the .y word of the {code, nbits} table puts 96 ASCII entries on 16 banks: ~3.5 cycles a lane group).
__device__ __forceinline__ uint32_t chunk_code_bits_nb(const uint32_t* stage, uint32_t last, uint32_t start, uint32_t len,
                                                       bool active, const uint8_t* __restrict__ nb) {
    const uint32_t end = start + len;
    const uint32_t a0 = start & ~3u;
    const uint32_t ndw = active ? (end - a0 + 3u) >> 2 : 0u;
    const uint32_t jf = (start & 3u) ? 1u : 0u;  // whole dwords: [jf, jl)
    const uint32_t jl = active ? (end - a0) >> 2 : 0u;
    const uint32_t mfirst = 0xFFFFFFFFu << (8u * (start & 3u));
    const uint32_t mlast = (uint32_t)(0xFFFFFFFFull >> ((32u - 8u * (end & 3u)) & 31u));
    auto masked = [&](uint32_t j, bool on) {
        uint32_t vm = j == 0 ? mfirst : 0xFFFFFFFFu;
        vm &= (j + 1 == ndw) ? mlast : 0xFFFFFFFFu;
        vm = on ? vm : 0u;
        const uint32_t w = stage[min(a0 + 4u * j, last) >> 2] & vm;  // bytes outside: index 256 (one entry)
        const uint32_t iw = ~vm & 0x01010101u;
        return (uint32_t)nb[__builtin_amdgcn_perm(iw, w, 0x0C0C0400u)] + nb[__builtin_amdgcn_perm(iw, w, 0x0C0C0501u)] +
               nb[__builtin_amdgcn_perm(iw, w, 0x0C0C0602u)] + nb[__builtin_amdgcn_perm(iw, w, 0x0C0C0703u)];
    };
    uint32_t tb = masked(0, active && jf != 0);  // head
    const uint32_t* sw = stage + (a0 >> 2);
    const uint32_t jlast = (last >> 2) - (a0 >> 2);
    const uint32_t jend = wave_max_u32(jl);
    uint32_t bulk = 0;
    for (uint32_t j = 0; j < jend; ++j) {
        const uint32_t w = sw[min(j, jlast)];
        const uint32_t n = (uint32_t)nb[w & 0xFFu] + nb[(w >> 8) & 0xFFu] + nb[(w >> 16) & 0xFFu] + nb[w >> 24];
        bulk += (j >= jf && j < jl) ? n : 0u;
    }
    return tb + bulk + masked(jl, active && (end & 3u) != 0 && jl >= jf);  // + tail
}

// Code bits of the stage bytes [start, start + len) (pass 1 of the proportional-lane encode).
__device__ __forceinline__ uint32_t chunk_code_bits(const uint32_t* stage, uint32_t last, uint32_t start, uint32_t len,
                                                    bool active, const uint2* __restrict__ enc, uint32_t jmax) {
    const uint32_t end = start + len;
    const uint32_t a0 = start & ~3u;
    const uint32_t ndw = active ? (end - a0 + 3u) >> 2 : 0u;
    const uint32_t mfirst = 0xFFFFFFFFu << (8u * (start & 3u));
    const uint32_t mlast = (uint32_t)(0xFFFFFFFFull >> ((32u - 8u * (end & 3u)) & 31u));
    uint32_t tb = 0;
    for (uint32_t j = 0; j < jmax; ++j) {
        const uint32_t w = stage[min(a0 + 4u * j, last) >> 2];
        uint32_t vm = j == 0 ? mfirst : 0xFFFFFFFFu;
        vm &= (j + 1 == ndw) ? mlast : 0xFFFFFFFFu;
        vm = j < ndw ? vm : 0u;
        const uint32_t iw = ~vm & 0x01010101u;
        tb += enc[__builtin_amdgcn_perm(iw, w, 0x0C0C0400u)].y + enc[__builtin_amdgcn_perm(iw, w, 0x0C0C0501u)].y +
              enc[__builtin_amdgcn_perm(iw, w, 0x0C0C0602u)].y + enc[__builtin_amdgcn_perm(iw, w, 0x0C0C0703u)].y;
    }
    return tb;
}

}  // namespace hhuff
