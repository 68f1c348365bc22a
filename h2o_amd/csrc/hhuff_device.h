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
constexpr uint32_t kEos = 256;
constexpr uint32_t kFailLen = 0xFFFFFFFFu;
constexpr uint8_t kStatusFail = 0x80;
constexpr uint8_t kStatusTooLong = 0xC0;
constexpr uint32_t kMaxStrLen = (1u << 29) - 1;

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
#ifdef HHUFF_SHFL_REDUCE  // A/B knob: ds_bpermute (__shfl_xor / __shfl_up) reductions and scan
__device__ __forceinline__ uint32_t wave_min_u32(uint32_t v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = min(v, (uint32_t)__shfl_xor((int)v, o, 64));
    return v;
}
__device__ __forceinline__ uint32_t wave_max_u32(uint32_t v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = max(v, (uint32_t)__shfl_xor((int)v, o, 64));
    return v;
}
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v) {
    const int lane = (int)__lane_id();
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = (uint32_t)__shfl_up((int)v, o, 64);
        if (lane >= o) v += y;
    }
    return v;
}
#else
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
#endif
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
            const uint32_t L1 = (e >> 16) & 15u;
            if (L1 > R) break;  // fewer bits left than the next code: padding
            const uint32_t L12 = (e >> 20) & 15u;
            const bool two = (e & kHas2) && L12 <= R;
            const uint32_t cons = two ? L12 : L1;
            sink.put12(e, two);
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

// ---------------------------------------------------------------------------------------------------
// Staged decode of one string per lane, all 64 lanes in lock step (same results as decode_core).
// Every per-lane predicate is a 0/1 integer in a VGPR (no lane masks, no SALU mask algebra): selects
// become multiply-adds, R is kept complemented (nR = ~R) so that "L <= R" is the sign bit of L + nR.
// Up to two symbols per step are written to the LDS output stage (writes that are switched off go to a
// lane-private trash byte); the 64-bit window is refilled without a branch; codes longer than the
// window take a wave-uniform detour through the leading-ones table.  Two steps per vote.
// ---------------------------------------------------------------------------------------------------
__device__ __forceinline__ DecResult decode_staged_lane_i(const uint32_t* stage, uint32_t last, uint32_t start, uint32_t len,
                                                          bool active, uint8_t* obuf, uint32_t op0, uint32_t trash,
                                                          const DecTables& T) {
    uint32_t a = start & ~3u;
    const uint32_t skip = start & 3u;
    uint64_t buf = (uint64_t)(bswap32(stage[min(a, last) >> 2]) << (8 * skip)) << 32;
    uint32_t nb = 32 - 8 * skip;
    a += 4;
    buf |= (uint64_t)bswap32(stage[min(a, last) >> 2]) << (32 - nb);
    nb += 32;
    a += 4;
    uint32_t nR = ~(active ? 8 * len : 0u);  // ~(string bits not yet consumed)
    uint32_t act = active ? 1u : 0u;
    uint32_t op = op0, flags = 0, fail = 0;
    auto step = [&]() {
        const uint32_t w = (uint32_t)(buf >> 32);
        const uint32_t e = T.lut[w >> (32 - HHUFF_LUT_BITS)];
        const uint32_t word = stage[min(a, last) >> 2];
        const uint32_t isl = e >> 31;
        const uint32_t L1 = (e >> 16) & 15u, L12 = (e >> 20) & 15u;
        const uint32_t ok1 = act & (isl ^ 1u) & ((L1 + nR) >> 31);                 // L1 <= R
        const uint32_t two = ok1 & (e >> 30) & ((L12 + nR) >> 31);                 // bit 30 = second symbol
        uint32_t cons = __umul24(ok1, L1) + __umul24(two, L12 - L1);
#ifndef HHUFF_ABL_NOWRITE
        obuf[trash - __umul24(ok1, trash - op)] = (uint8_t)e;  // trash > op: both mul24 operands < 2^24
        obuf[trash - __umul24(two, trash - op - 1u)] = (uint8_t)(e >> 8);
#endif
        op += ok1 + two;
        flags |= (e >> 24) & (3u * ok1 + 12u * two);
        uint32_t nact = ok1;
        const uint32_t lact = act & isl;
        if (__any(lact != 0u)) {  // wave-uniform: codes longer than the window, EOS
            if (lact) {
                const uint32_t k = min((uint32_t)__builtin_clz(~w | 1u), 30u);
                const uint32_t ki = T.kinfo[k];
                const uint32_t le = T.ones[(ki & 0xFFFFu) + (((w << (k + 1)) >> 1) >> (31 - (ki >> 16)))];
                const uint32_t L = (le >> 9) & 31u;
                const uint32_t okL = (L + nR) >> 31;
                const uint32_t eos = (le & 0x1FFu) == kEos ? 1u : 0u;
                const uint32_t ok = okL & (eos ^ 1u);
                fail |= okL & eos;  // EOS inside the string (hpack.c:88-89)
                obuf[trash - __umul24(ok, trash - op)] = (uint8_t)le;
                op += ok;
                flags |= ((le >> 14) & 3u) * ok;
                cons = __umul24(ok, L);
                nact = ok;
            }
        }
        act = nact;
        nR += cons;
        buf <<= cons;
        nb -= cons;
        const uint32_t need = (nb - 33u) >> 31;  // nb <= 32
        buf |= (uint64_t)(bswap32(word) & (0u - need)) << ((32u - nb) & 63u);
        nb += need << 5;
        a += need << 2;
    };
    for (;;) {
        step();
        step();
        if (!__any(act != 0u)) break;
    }
    const uint32_t R = ~nR;
    DecResult r;
    r.ok = !fail && R <= 7 && ((uint32_t)(buf >> 56) | (0xFFu >> R)) == 0xFFu;
    r.len = op - op0;
    r.flags = (flags | (flags >> 2)) & 3u;
    r.status = 0;
    return r;
}

// ---------------------------------------------------------------------------------------------------
// Staged decode, v5 step.  Same results as decode_core; the stage holds big-endian (byte-swapped)
// dwords so that the 32-bit window at any bit is one v_alignbit of two of them:
//   pm = p - 1 (p = next unread bit, MSB first), q = pm >> 5 (arithmetic), x0 = stage[q], x1 = stage[q+1]
//   window = alignbit(x0, x1, ~pm)                      (bits p .. p+31; x0 unused when p % 32 == 0)
// c = p - end - 1 is negative while bits remain, so "a code of L bits fits" is the sign of L + c; with
// LONG / HAS2 in the LUT's top bits the take-masks m1 (first symbol) and m2 (second symbol) are sign
// bits of one AND each.  Switched-off writes are steered to a lane-private trash byte with v_bfi, so no
// byte outside [op0, op0 + count) is ever written.  A lane whose next code can never fit is parked by
// pushing c positive.  x2 = stage[q+2] is fetched one step ahead, so only the LUT read is on the
// step's dependency chain.  Two steps per vote.
// ---------------------------------------------------------------------------------------------------
#ifndef HHUFF_DEC_LONG2  // A/B knob: look for long codes every other decode step only
#define HHUFF_DEC_LONG2 1
#endif
#ifndef HHUFF_DEC_X2  // A/B knob: two dependent LUT lookups per decode step (up to 4 symbols)
#define HHUFF_DEC_X2 1
#endif
#ifndef HHUFF_DEC_B16  // A/B knob: one 2-byte output store per decode step instead of two byte stores.
#define HHUFF_DEC_B16 0  // Off: correct, but odd-address ds_write_b16 is slow on gfx950 (c4 decode 1.01 -> 1.48 ms)
#endif
typedef __attribute__((address_space(3))) uint8_t lds_u8;
typedef __attribute__((address_space(3))) uint32_t lds_u32;
typedef __attribute__((address_space(3))) uint16_t lds_u16;

__device__ __forceinline__ uint32_t lds_addr(const void* p) { return (uint32_t)(size_t)(const lds_u8*)p; }
__device__ __forceinline__ void lds_st8(uint32_t addr, uint32_t v) { *(lds_u8*)(size_t)addr = (uint8_t)v; }
// 2-byte store at any byte address (gfx950 LDS honours unaligned ds_write_b16: tools/probe/lds_unaligned.hip)
__device__ __forceinline__ void lds_st16(uint32_t addr, uint32_t v) { *(lds_u16*)(size_t)addr = (uint16_t)v; }
__device__ __forceinline__ uint32_t sel_bits(uint32_t m, uint32_t a, uint32_t b) { return (m & a) | (~m & b); }

__device__ __forceinline__ DecResult decode_staged_lane_v5(const uint32_t* stage, uint32_t start, uint32_t len,
                                                           bool active, uint8_t* obuf, uint32_t op0, uint32_t trash_off,
                                                           const DecTables& T) {
    const lds_u32* st = (const lds_u32*)stage;
    int32_t pm = (int32_t)(8u * start) - 1;
    const int32_t end = (int32_t)(8u * (start + len));
    int32_t c = active ? pm - end : 0x40000000;
    int32_t q = pm >> 5;
    uint32_t x0 = st[q], x1 = st[q + 1], x2 = st[q + 2];
    const uint32_t o0 = lds_addr(obuf) + op0, trash = lds_addr(obuf) + trash_off;
    uint32_t o = o0, acc1 = 0, acc2 = 0, accl = 0, fail = 0;
    int32_t prog = 0;
    uint32_t first = 0;  // first decoded byte, kept in a register (HHUFF_DEC_B16 fix-up below)
    auto step = [&](bool cap, bool longchk) {
        const uint32_t w = __builtin_amdgcn_alignbit(x0, x1, ~(uint32_t)pm);
        const uint32_t e = T.lut[w >> (32 - HHUFF_LUT_BITS)];
        const int32_t L1 = (e >> 16) & 15u, L12 = (e >> 20) & 15u;
        const int32_t s1 = L1 + c, s2 = L12 + c;
        const uint32_t m1 = (uint32_t)((s1 & ~(int32_t)e) >> 31);         // first code fits, not LONG
        const uint32_t m2 = (uint32_t)((s2 & (int32_t)(e << 1)) >> 31);  // HAS2 and both fit
        int32_t cons = (int32_t)sel_bits(m2, (uint32_t)L12, m1 & (uint32_t)L1);
#if HHUFF_DEC_B16
        // both symbol bytes in one store; with one symbol taken the second byte is garbage one past it,
        // overwritten by the next step -- or, at the string's end, possibly on the next string's first
        // byte, which every lane restores from `first` after the loop
        lds_st16(sel_bits(m1, o, trash), e);
#elif !defined(HHUFF_ABL_V5_NOWRITE)  // ablation: drop the output stores (wrong output, timing only)
        lds_st8(sel_bits(m1, o - m2, trash), e >> 8);  // second symbol, or onto the first one's byte
        lds_st8(sel_bits(m1, o, trash), e);
#endif
        if (cap) first = m1 ? (e & 0xFFu) : first;
        o = o - m1 - m2;
        acc1 |= e & m1;
        acc2 |= e & m2;
#if HHUFF_DEC_X2
        {  // second lookup on the same 32-bit window, after what the first one took (<= 13 bits): up to
           // 4 symbols per step.  Nothing taken first -> same window, same entry, nothing taken again.
            const uint32_t wb = w << cons;
            const uint32_t eb = T.lut[wb >> (32 - HHUFF_LUT_BITS)];
            const int32_t cb = c + cons;
            const int32_t L1b = (eb >> 16) & 15u, L12b = (eb >> 20) & 15u;
            const uint32_t m1b = (uint32_t)(((L1b + cb) & ~(int32_t)eb) >> 31);
            const uint32_t m2b = (uint32_t)(((L12b + cb) & (int32_t)(eb << 1)) >> 31);
#ifndef HHUFF_ABL_V5_NOWRITE
            lds_st8(sel_bits(m1b, o - m2b, trash), eb >> 8);
            lds_st8(sel_bits(m1b, o, trash), eb);
#endif
            o = o - m1b - m2b;
            acc1 |= eb & m1b;
            acc2 |= eb & m2b;
            cons += (int32_t)sel_bits(m2b, (uint32_t)L12b, m1b & (uint32_t)L1b);
        }
#endif
        const bool lact = (s1 & (int32_t)e) < 0;  // LONG entry and >= LUT_BITS + 1 bits left
        uint32_t consl = 0;
        // wave-uniform detour for codes longer than the window and EOS; with HHUFF_DEC_LONG2 only every
        // other step looks (a lane parked on a long code for one step retries it on the next)
        if ((!HHUFF_DEC_LONG2 || longchk) && __builtin_amdgcn_ballot_w64(lact) != 0) {
            if (lact) {
                const uint32_t k = min((uint32_t)__builtin_clz(~w | 1u), 30u);
                const uint32_t ki = T.kinfo[k];
                const uint32_t le = T.ones[(ki & 0xFFFFu) + (((w << (k + 1)) >> 1) >> (31 - (ki >> 16)))];
                const int32_t L = (le >> 9) & 31u;
                const uint32_t fits = (uint32_t)((L + c) >> 31);
                const uint32_t eos = (le & 0x1FFu) == kEos ? 0xFFFFFFFFu : 0u;
                const uint32_t okm = fits & ~eos;
                fail |= fits & eos & 1u;  // EOS inside the string (hpack.c:88-89)
                lds_st8(sel_bits(okm, o, trash), le);
                if (cap) first = okm ? (le & 0xFFu) : first;
                o -= okm;
                accl |= le & okm;
                consl = okm & (uint32_t)L;
                c = (int32_t)sel_bits(okm, (uint32_t)c, 0x40000000u);  // park: EOS, or a code that cannot fit
            }
        }
        cons |= (int32_t)consl;  // LONG lanes took no window symbol, so cons was 0 there
        c += cons;
        pm += cons;
        const int32_t qn = pm >> 5;
        const bool adv = qn != q;
        x0 = adv ? x1 : x0;
        x1 = adv ? x2 : x1;
        q = qn;
        x2 = st[q + 2];
        prog = cons;
    };
    step(true, true);
    for (;;) {
        step(false, false);
        step(false, true);
        if (!__any(prog != 0)) break;
    }
#if HHUFF_DEC_B16
    lds_st8(o != o0 ? o0 : trash, first);  // every lane's garbage byte is down by now (lock step)
#endif
    DecResult r;
    const uint32_t R = ~(uint32_t)c;  // string bits left (meaningless for parked lanes, which fail)
    const uint32_t w = __builtin_amdgcn_alignbit(x0, x1, ~(uint32_t)pm);
    r.ok = active && !fail && R <= 7 && (w | (0xFFFFFFFFu >> (R & 31u))) == 0xFFFFFFFFu;
    r.len = o - o0;
    r.flags = ((acc1 >> 24) | (acc2 >> 26) | (accl >> 14)) & 3u;
    r.status = 0;
    return r;
}

// ---------------------------------------------------------------------------------------------------
// Staged decode, v6 step: v5's window, LUT and take-masks, but the decoded bytes collect in a register
// accumulator (lo:hi, `pend` bytes pending, pend <= 3 between steps) and leave as ONE ds_or_b32 per step
// into the zeroed output stage at dword granularity, instead of four predicated ds_write_b8 (two per
// lookup).  The accumulator starts `op0 & 3` bytes into its dword, so a lane only ever ORs non-zero
// bits into its own bytes [op0, op0 + count): neighbouring slots that share a dword do not interfere.
// LDS instructions per step: 2 LUT reads + 1 stage read + 1 OR (v5: 2 + 1 + 4 byte stores).
// The caller zeroes the stage bytes the lanes may touch before the call.
// ---------------------------------------------------------------------------------------------------
#ifndef HHUFF_DEC_ACC  // A/B knob: 1 = v6 register-accumulated output, 0 = v5 byte stores
#define HHUFF_DEC_ACC 0
#endif
typedef __attribute__((address_space(3))) uint32_t lds_u32w;

__device__ __forceinline__ void lds_or32(uint32_t addr, uint32_t v) {
    __hip_atomic_fetch_or((lds_u32w*)(size_t)addr, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

struct OutAcc {  // pending output bytes, first byte in bits 0..7 of lo
    uint32_t lo, hi, pend, addr;
    // insert n <= 4 bytes (b, first byte in bits 0..7, bits above 8n zero), then emit one dword if >= 4 pend
    __device__ __forceinline__ void put(uint32_t b, uint32_t n) {
        const uint64_t v = (uint64_t)b << (8u * pend);  // pend <= 3
        lo |= (uint32_t)v;
        hi |= (uint32_t)(v >> 32);
        pend += n;
        const uint32_t em = 0u - (pend >> 2);  // pend >= 4 (pend <= 7)
#ifndef HHUFF_ABL_V6_NOOR
        lds_or32(addr, lo & em);
#else
        asm volatile("" ::"v"(lo & em), "v"(addr));
#endif
        lo = sel_bits(em, hi, lo);
        hi &= ~em;
        pend -= em & 4u;
        addr += em & 4u;
    }
    __device__ __forceinline__ void flush() {
        if (pend) lds_or32(addr, lo);
    }
};

__device__ __forceinline__ DecResult decode_staged_lane_v6(const uint32_t* stage, uint32_t start, uint32_t len,
                                                           bool active, uint8_t* obuf, uint32_t op0, const DecTables& T) {
    const lds_u32* st = (const lds_u32*)stage;
    int32_t pm = (int32_t)(8u * start) - 1;
    const int32_t end = (int32_t)(8u * (start + len));
    int32_t c = active ? pm - end : 0x40000000;
    int32_t q = pm >> 5;
    uint32_t x0 = st[q], x1 = st[q + 1], x2 = st[q + 2];
    const uint32_t ob = lds_addr(obuf) + op0;
    OutAcc acc{0u, 0u, ob & 3u, ob & ~3u};
    uint32_t acc1 = 0, acc2 = 0, accl = 0, fail = 0, cnt = 0;
    int32_t prog = 0;
    auto step = [&](bool longchk) {
        const uint32_t w = __builtin_amdgcn_alignbit(x0, x1, ~(uint32_t)pm);
        const uint32_t e = T.lut[w >> (32 - HHUFF_LUT_BITS)];
        const int32_t L1 = (e >> 16) & 15u, L12 = (e >> 20) & 15u;
        const int32_t s1 = L1 + c, s2 = L12 + c;
        const uint32_t m1 = (uint32_t)((s1 & ~(int32_t)e) >> 31);         // first code fits, not LONG
        const uint32_t m2 = (uint32_t)((s2 & (int32_t)(e << 1)) >> 31);  // HAS2 and both fit
        int32_t cons = (int32_t)sel_bits(m2, (uint32_t)L12, m1 & (uint32_t)L1);
        acc1 |= e & m1;
        acc2 |= e & m2;
        const uint32_t n1 = (m1 & 1u) + (m2 & 1u);
        uint32_t bytes = e & ((m1 & 0xFFu) | (m2 & 0xFF00u));
        uint32_t n = n1;
#if HHUFF_DEC_X2
        {  // second lookup on the same 32-bit window, after what the first one took (<= 13 bits)
            const uint32_t wb = w << cons;
            const uint32_t eb = T.lut[wb >> (32 - HHUFF_LUT_BITS)];
            const int32_t cb = c + cons;
            const int32_t L1b = (eb >> 16) & 15u, L12b = (eb >> 20) & 15u;
            const uint32_t m1b = (uint32_t)(((L1b + cb) & ~(int32_t)eb) >> 31);
            const uint32_t m2b = (uint32_t)(((L12b + cb) & (int32_t)(eb << 1)) >> 31);
            acc1 |= eb & m1b;
            acc2 |= eb & m2b;
            bytes |= (eb & ((m1b & 0xFFu) | (m2b & 0xFF00u))) << (8u * n1);
            n += (m1b & 1u) + (m2b & 1u);
            cons += (int32_t)sel_bits(m2b, (uint32_t)L12b, m1b & (uint32_t)L1b);
        }
#endif
        acc.put(bytes, n);
        cnt += n;
        const bool lact = (s1 & (int32_t)e) < 0;  // LONG entry and >= LUT_BITS + 1 bits left
        uint32_t consl = 0;
        if ((!HHUFF_DEC_LONG2 || longchk) && __builtin_amdgcn_ballot_w64(lact) != 0) {
            if (lact) {
                const uint32_t k = min((uint32_t)__builtin_clz(~w | 1u), 30u);
                const uint32_t ki = T.kinfo[k];
                const uint32_t le = T.ones[(ki & 0xFFFFu) + (((w << (k + 1)) >> 1) >> (31 - (ki >> 16)))];
                const int32_t L = (le >> 9) & 31u;
                const uint32_t fits = (uint32_t)((L + c) >> 31);
                const uint32_t eos = (le & 0x1FFu) == kEos ? 0xFFFFFFFFu : 0u;
                const uint32_t okm = fits & ~eos;
                fail |= fits & eos & 1u;  // EOS inside the string (hpack.c:88-89)
                acc.put(le & okm & 0xFFu, okm & 1u);
                cnt += okm & 1u;
                accl |= le & okm;
                consl = okm & (uint32_t)L;
                c = (int32_t)sel_bits(okm, (uint32_t)c, 0x40000000u);  // park: EOS, or a code that cannot fit
            }
        }
        cons |= (int32_t)consl;  // LONG lanes took no window symbol, so cons was 0 there
        c += cons;
        pm += cons;
        const int32_t qn = pm >> 5;
        const bool adv = qn != q;
        x0 = adv ? x1 : x0;
        x1 = adv ? x2 : x1;
        q = qn;
        x2 = st[q + 2];
        prog = cons;
    };
    step(true);
    for (;;) {
        step(false);
        step(true);
        if (!__any(prog != 0)) break;
    }
    acc.flush();
    DecResult r;
    const uint32_t R = ~(uint32_t)c;
    const uint32_t w = __builtin_amdgcn_alignbit(x0, x1, ~(uint32_t)pm);
    r.ok = active && !fail && R <= 7 && (w | (0xFFFFFFFFu >> (R & 31u))) == 0xFFFFFFFFu;
    r.len = cnt;
    r.flags = ((acc1 >> 24) | (acc2 >> 26) | (accl >> 14)) & 3u;
    r.status = 0;
    return r;
}

// ---------------------------------------------------------------------------------------------------
// Staged decode, v7: a BULK phase and a TAIL phase (same results as decode_core).
// Bulk steps run only for lanes with >= 27 string bits left (pm < lim = end - 26; inactive and parked
// lanes have lim = INT_MIN), so everything both lookups of a step hold lies inside the string: there are
// no end-of-string take-masks, the entry says what to take -- [29:28] symbol count, L12 bits (none for
// LONG) -- and flag bits of absent symbols are zero, so `accb |= e` collects them.  Lanes below lim are
// switched off (exec mask) until the bulk loop drains; then v5's checked step finishes every lane
// (<= 26 bits, at most ~3 steps).  Bulk VALU per step is about half of v5's.  Codes longer than the
// window take the same wave-uniform detour (fit checked against `end`; EOS or a code that cannot fit
// parks the lane, which then fails).
// ---------------------------------------------------------------------------------------------------
#ifndef HHUFF_DEC_BULK  // A/B knob: 1 = v7 bulk + tail decode, 0 = v5 / v6
#define HHUFF_DEC_BULK 1
#endif

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
#ifdef HHUFF_ABL_DEC_NOSTEP  // ablation: no decoding at all (wrong output, timing of the tile overhead)
    {
        DecResult r0;
        r0.ok = active;
        r0.len = len;
        r0.flags = 0;
        r0.status = 0;
        if (__any(active)) return r0;
    }
#endif

    // ---- bulk ----
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
            const uint32_t sl = (uint32_t)((int32_t)e >> 31);         // LONG: nothing taken from the window
            const uint32_t h2 = (uint32_t)((int32_t)(e << 1) >> 31);  // HAS2
            lds_st8(sel_bits(sl, trash, o), e);
            lds_st8(sel_bits(h2, o, trash - 1u) + 1u, e >> 8);
            o += (e >> 28) & 3u;
            accb |= e;
            uint32_t cons = ((e >> 20) & 15u) & ~sl;
            {
                const uint32_t wb = w << cons;
                const uint32_t eb = T.lut[wb >> (32 - HHUFF_LUT_BITS)];
                const uint32_t slb = (uint32_t)((int32_t)eb >> 31);
                const uint32_t h2b = (uint32_t)((int32_t)(eb << 1) >> 31);
                lds_st8(sel_bits(slb, trash, o), eb);
                lds_st8(sel_bits(h2b, o, trash - 1u) + 1u, eb >> 8);
                o += (eb >> 28) & 3u;
                accb |= eb;
                cons += ((eb >> 20) & 15u) & ~slb;
            }
            if ((!HHUFF_DEC_LONG2 || longchk) && __builtin_amdgcn_ballot_w64(sl != 0u) != 0) {
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

    // ---- tail: v5's checked step ----
    int32_t c = parked ? 0x40000000 : pm - end;
    int32_t prog = 0;
    auto step = [&](bool longchk) {
        const uint32_t w = __builtin_amdgcn_alignbit(x0, x1, ~(uint32_t)pm);
        const uint32_t e = T.lut[w >> (32 - HHUFF_LUT_BITS)];
        const int32_t L1 = (e >> 16) & 15u, L12 = (e >> 20) & 15u;
        const int32_t s1 = L1 + c, s2 = L12 + c;
        const uint32_t m1 = (uint32_t)((s1 & ~(int32_t)e) >> 31);
        const uint32_t m2 = (uint32_t)((s2 & (int32_t)(e << 1)) >> 31);
        int32_t cons = (int32_t)sel_bits(m2, (uint32_t)L12, m1 & (uint32_t)L1);
        lds_st8(sel_bits(m1, o - m2, trash), e >> 8);
        lds_st8(sel_bits(m1, o, trash), e);
        o = o - m1 - m2;
        acc1 |= e & m1;
        acc2 |= e & m2;
        {
            const uint32_t wb = w << cons;
            const uint32_t eb = T.lut[wb >> (32 - HHUFF_LUT_BITS)];
            const int32_t cb = c + cons;
            const int32_t L1b = (eb >> 16) & 15u, L12b = (eb >> 20) & 15u;
            const uint32_t m1b = (uint32_t)(((L1b + cb) & ~(int32_t)eb) >> 31);
            const uint32_t m2b = (uint32_t)(((L12b + cb) & (int32_t)(eb << 1)) >> 31);
            lds_st8(sel_bits(m1b, o - m2b, trash), eb >> 8);
            lds_st8(sel_bits(m1b, o, trash), eb);
            o = o - m1b - m2b;
            acc1 |= eb & m1b;
            acc2 |= eb & m2b;
            cons += (int32_t)sel_bits(m2b, (uint32_t)L12b, m1b & (uint32_t)L1b);
        }
        const bool lact = (s1 & (int32_t)e) < 0;
        uint32_t consl = 0;
        if ((!HHUFF_DEC_LONG2 || longchk) && __builtin_amdgcn_ballot_w64(lact) != 0) {
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

// ---------------------------------------------------------------------------------------------------
// Staged encode of one string per lane, all lanes in lock step, one input dword per step (same results
// as encode_core).  `enc` = 512 x {code, nbits} in LDS; entries 256..511 are {0, 0} and stand for bytes
// outside the string, selected with one v_perm per byte.  Fast path: the dword's four codes are all
// <= 8 bits, so they combine into one 32-bit chunk, enter the 64-bit accumulator at once and leave at
// most one 32-bit word.  Output words are OR-ed (ds_or_b32) into a zeroed LDS stage at dword
// granularity: the stream is pre-shifted by the slot's byte offset within its dword, so lanes whose
// slots share a dword never overwrite each other.  Other dwords (a code longer than 8 bits) take a
// wave-uniform per-byte detour.  Returns the Huffman length or kFailLen; `active` = len in 1..limit.
// ---------------------------------------------------------------------------------------------------
__device__ __forceinline__ void enc_put(uint32_t* obuf32, uint64_t& acc, uint32_t& an, uint32_t& opw, bool on) {
    const bool emit = on && an >= 32;
    atomicOr(&obuf32[opw], emit ? bswap32((uint32_t)(acc >> 32)) : 0u);
    acc = emit ? acc << 32 : acc;
    an -= emit ? 32u : 0u;
    opw += emit ? 1u : 0u;
}

__device__ __forceinline__ uint32_t encode_staged_lane(const uint32_t* stage, uint32_t last, uint32_t start, uint32_t len,
                                                       bool active, uint32_t* obuf32, uint32_t opb,
                                                       const uint2* __restrict__ enc) {
    const uint32_t end = start + len;
    const uint32_t limit = 8 * len - 7;  // fail as soon as the code bits reach it: ceil(bits/8) >= len
    uint64_t acc = 0;                     // code bits, MSB-aligned, after (opb & 3) zero bytes
    uint32_t an = 8 * (opb & 3u);         // bits in acc
    uint32_t opw = opb >> 2;              // next LDS output dword
    uint32_t tb = 0;                      // code bits of the string so far
    bool fail = false;
    for (uint32_t a = start & ~3u;; a += 4) {
        const uint32_t w = stage[min(a, last) >> 2];
        const int32_t dlo = (int32_t)(start - a), dhi = (int32_t)(end - a);
        const uint32_t nlo = (uint32_t)min(max(dlo, 0), 4), nhi = active ? (uint32_t)min(max(dhi, 0), 4) : 0u;
        const uint32_t vm = (uint32_t)(0xFFFFFFFFull >> (8 * (4 - nhi))) & (uint32_t)(0xFFFFFFFFull << (8 * nlo));
        const uint32_t iw = ~vm & 0x01010101u;  // 1 in every byte outside the string
        const uint2 e0 = enc[__builtin_amdgcn_perm(iw, w, 0x0C0C0400u)];
        const uint2 e1 = enc[__builtin_amdgcn_perm(iw, w, 0x0C0C0501u)];
        const uint2 e2 = enc[__builtin_amdgcn_perm(iw, w, 0x0C0C0602u)];
        const uint2 e3 = enc[__builtin_amdgcn_perm(iw, w, 0x0C0C0703u)];
        const bool lng = max(max(e0.y, e1.y), max(e2.y, e3.y)) > 8;
        const bool fast = active && !lng;
        const uint32_t n = e0.y + e1.y + e2.y + e3.y;
        uint32_t c = (((e0.x << e1.y | e1.x) << e2.y | e2.x) << e3.y) | e3.x;
        const bool over = fast && tb + n >= limit;
        fail = fail || over;
        const bool put = fast && !over;
        c = put ? c : 0u;
        const uint32_t nn = put ? n : 0u;
        acc |= (uint64_t)c << ((64 - an - nn) & 63u);
        an += nn;
        tb += nn;
        enc_put(obuf32, acc, an, opw, put);
        bool stay = put;
        if (__any(active && lng)) {  // a code longer than 8 bits in this dword: byte by byte
            if (active && lng) {
                bool ok = true;
                const uint2 ek[4] = {e0, e1, e2, e3};
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    const bool ov = ok && tb + ek[k].y >= limit;
                    fail = fail || ov;
                    ok = ok && !ov;
                    const uint32_t nk = ok ? ek[k].y : 0u;
                    acc |= (uint64_t)(ok ? ek[k].x : 0u) << ((64 - an - nk) & 63u);
                    an += nk;
                    tb += nk;
                    enc_put(obuf32, acc, an, opw, ok);
                }
                stay = ok;
            }
        }
        active = active && stay && dhi > 4;  // more bytes after this dword
        if (!__any(active)) break;
    }
    if (fail || len == 0 || len > kMaxStrLen) return kFailLen;
    // pad the partial byte with ones (EOS prefix, hpack.c:795-798) and flush the last <= 4 bytes
    const uint32_t an8 = (an + 7) & ~7u;
    acc |= (~0ull >> an) & ~(~0ull >> an8);
    if (an) atomicOr(&obuf32[opw], bswap32((uint32_t)(acc >> 32)));
    return (tb + 7) >> 3;
}

// Same contract as encode_staged_lane, with a wave-uniform trip count: `jmax` = the largest number of
// input dwords over the wave's lanes, so the loop needs no vote; lanes that finished or failed run with
// every byte masked out (their table entries are {0, 0}).  The first / last dword masks are precomputed.
#ifndef HHUFF_ENC_PAIRS  // A/B knob: fused encode path for codes <= 16 bits as two 32-bit pairs (else <= 8 bits)
#define HHUFF_ENC_PAIRS 1
#endif
constexpr uint32_t kFusedMaxBits = HHUFF_ENC_PAIRS ? 16u : 8u;

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
#if HHUFF_ENC_PAIRS
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
#else
        const uint32_t c = put ? ((((e0.x << e1.y | e1.x) << e2.y | e2.x) << e3.y) | e3.x) : 0u;
        const uint32_t nn = put ? n : 0u;
        acc |= (uint64_t)c << ((64u - an - nn) & 63u);
        an += nn;
        tb += nn;
#endif
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

// Whole string at byte `opb` of the output stage: returns the Huffman length in bytes or kFailLen.
__device__ __forceinline__ uint32_t encode_staged_lane_u(const uint32_t* stage, uint32_t last, uint32_t start, uint32_t len,
                                                         bool active, uint32_t* obuf32, uint32_t opb,
                                                         const uint2* __restrict__ enc, uint32_t jmax) {
    const uint32_t tb = encode_chunk(stage, last, start, len, active, obuf32, 8u * opb, enc, jmax,
                                     active ? 8 * len - 7 : 0xFFFFFFFFu, true);
    return tb == kFailLen ? kFailLen : (tb + 7) >> 3;
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
#ifndef HHUFF_ENC_V2  // A/B knob: 1 = encode v2 (stateless placement, bulk phase), 0 = encode_chunk
#define HHUFF_ENC_V2 1
#endif

__device__ __forceinline__ void place_bits(uint32_t obase, uint32_t tb, uint64_t c, uint32_t n) {
    const uint64_t t = c << ((64u - n) & 63u);  // left-aligned (n == 0 needs c == 0)
    const uint32_t sh = tb & 31u;
    const uint64_t u = t >> sh;
    const uint32_t a = obase + ((tb >> 3) & ~3u);
#ifdef HHUFF_ABL_ENC_NOOR  // ablation: no output (wrong output, timing only)
    asm volatile("" ::"v"(a), "v"((uint32_t)(u >> 32)), "v"((uint32_t)u), "v"((uint32_t)t << (32u - sh)));
#else
    lds_or32(a, (uint32_t)(u >> 32));
    lds_or32(a + 4u, (uint32_t)u);
    if (sh + n > 64u) lds_or32(a + 8u, (uint32_t)t << (32u - sh));  // sh > 0 here
#endif
}

struct EncV2 {
    const uint2* enc;
    uint32_t obase;  // LDS byte address of the MSB-first output stage
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
    // the SALU): `onm` = this lane has these four bytes; `livem` mirrors `live`.
    uint32_t livem, failm;
    __device__ __forceinline__ void put4m(uint2 e0, uint2 e1, uint2 e2, uint2 e3, uint32_t onm) {
        const uint32_t n01 = e0.y + e1.y, n23 = e2.y + e3.y, n = n01 + n23;
        const uint32_t mx = max(max(e0.y, e1.y), max(e2.y, e3.y));
        const uint32_t lngm = (uint32_t)((int32_t)(16u - mx) >> 31);                 // a code > 16 bits
        const uint32_t overm = onm & livem & ~(uint32_t)((int32_t)(tb + n - tlim) >> 31);  // tb + n >= tlim
        failm |= overm;
        livem &= ~overm;
        const uint32_t putm = onm & livem;
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
        const uint32_t a = obase + ((tb >> 3) & ~3u);
        lds_or32(a, (uint32_t)(u >> 32));
        lds_or32(a + 4u, (uint32_t)u);
        if (__builtin_amdgcn_ballot_w64(sh + nf > 64u) != 0) {
            if (sh + nf > 64u) lds_or32(a + 8u, (uint32_t)t << (32u - sh));
        }
        tb += n & putm;
    }
};

#ifndef HHUFF_ENC_PRED  // A/B knob: 1 = predicated bulk loop with a uniform trip count, 0 = exec-masked
#define HHUFF_ENC_PRED 1
#endif

// Encode stage bytes [start, start + len) to stage bit `startbit` of the MSB-first output stage at LDS
// byte address `obase`.  `limit`, `pad`: as encode_chunk.  Returns the code bits or kFailLen.
__device__ __forceinline__ uint32_t encode_chunk_v2(const uint32_t* stage, uint32_t last, uint32_t start, uint32_t len,
                                                    bool active, uint32_t obase, uint32_t startbit,
                                                    const uint2* __restrict__ enc, uint32_t limit, bool pad) {
    const uint32_t end = start + len;
    const uint32_t a0 = start & ~3u;
    const uint32_t ndw = active ? (end - a0 + 3u) >> 2 : 0u;
    const uint32_t jf = (start & 3u) ? 1u : 0u;            // whole dwords: [jf, jl)
    const uint32_t jl = active ? (end - a0) >> 2 : 0u;
    const uint32_t mfirst = 0xFFFFFFFFu << (8u * (start & 3u));
    const uint32_t mlast = (uint32_t)(0xFFFFFFFFull >> ((32u - 8u * (end & 3u)) & 31u));
    // tlim < 2^31 keeps tb + n - tlim a signed quantity (stage bits are < 2^20)
    EncV2 E{enc, obase, startbit, limit >= 0x40000000u ? 0x7FFFFFFFu : startbit + limit, active, false,
            active ? 0xFFFFFFFFu : 0u, 0u};
    auto masked = [&](uint32_t j, bool on) {  // one dword with byte masks (head / tail)
        const uint32_t w = stage[min(a0 + 4u * j, last) >> 2];
        uint32_t vm = j == 0 ? mfirst : 0xFFFFFFFFu;
        vm &= (j + 1 == ndw) ? mlast : 0xFFFFFFFFu;
        vm = on ? vm : 0u;
        const uint32_t iw = ~vm & 0x01010101u;
        E.put4(enc[__builtin_amdgcn_perm(iw, w, 0x0C0C0400u)], enc[__builtin_amdgcn_perm(iw, w, 0x0C0C0501u)],
               enc[__builtin_amdgcn_perm(iw, w, 0x0C0C0602u)], enc[__builtin_amdgcn_perm(iw, w, 0x0C0C0703u)], on);
    };
#ifdef HHUFF_ABL_ENC_NOSTEP  // ablation: no encoding at all (wrong output, timing of the tile overhead)
    if (active) return len;
#endif
    masked(0, active && jf != 0);  // head
    const uint32_t* sw = stage + (a0 >> 2);
    const uint32_t jlast = (last >> 2) - (a0 >> 2);  // stage reads are clamped to the span
#if HHUFF_ENC_PRED
    E.livem = E.live ? 0xFFFFFFFFu : 0u;
    {
        const uint32_t jend = wave_max_u32(E.live ? jl : 0u);  // uniform trip count: no vote per step
        uint32_t wn = sw[min(0u, jlast)];
        for (uint32_t j = 0; j < jend; ++j) {  // bulk
            const uint32_t w = wn;
            wn = sw[min(j + 1u, jlast)];
            const uint32_t onm = ~(uint32_t)((int32_t)((j - jf) | (jl - 1u - j)) >> 31);  // jf <= j < jl
#ifdef HHUFF_ABL_ENC_NOTAB
            E.put4m(make_uint2(w & 0x3Fu, 6u), make_uint2((w >> 8) & 0x1Fu, 5u), make_uint2((w >> 16) & 0x3Fu, 6u),
                    make_uint2((w >> 24) & 0x7Fu, 7u), onm);
#else
            E.put4m(enc[w & 0xFFu], enc[(w >> 8) & 0xFFu], enc[(w >> 16) & 0xFFu], enc[w >> 24], onm);
#endif
        }
    }
    E.live = E.livem != 0u;
    E.fail = E.fail || E.failm != 0u;
#else
    uint32_t wn = sw[min(jf, jlast)];                 // next whole dword, read one step ahead
    for (uint32_t j = 0;; ++j) {                      // bulk
        if (!__any(E.live && j < jl)) break;
        if (E.live && j >= jf && j < jl) {
            const uint32_t w = wn;
            wn = sw[min(j + 1u, jlast)];
#ifdef HHUFF_ABL_ENC_NOTAB  // ablation: table entries from registers (wrong output, timing only)
            E.put4(make_uint2(w & 0x3Fu, 6u), make_uint2((w >> 8) & 0x1Fu, 5u), make_uint2((w >> 16) & 0x3Fu, 6u),
                   make_uint2((w >> 24) & 0x7Fu, 7u), true);
#else
            E.put4(enc[w & 0xFFu], enc[(w >> 8) & 0xFFu], enc[(w >> 16) & 0xFFu], enc[w >> 24], true);
#endif
        }
    }
#endif
    masked(jl, active && (end & 3u) != 0 && jl >= jf);  // tail
    if (E.fail || !active) return kFailLen;
    const uint32_t tbits = E.tb - startbit;
    if (pad) {  // fill the last byte with ones (EOS prefix, hpack.c:795-798)
        const uint32_t p = (0u - tbits) & 7u;
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
