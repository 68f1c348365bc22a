// Device-side building blocks of the hhuff kernels (gfx950 / CDNA4, wave64).
//
// Semantics restated from the reference (file:line under /root/reference):
//   decode  lib/http2/hpack.c:85-156   (nibble FSM; accept rule misc/mkhufftbl.py:374-381)
//   encode  lib/http2/hpack.c:774-804  (40-bit accumulator; SIZE_MAX unless strictly shorter)
// The MI355X formulation is different from the reference's (same results, bit for bit):
//   * decode consumes a 12-bit window per step through a 4096-entry LUT staged in LDS that yields up to
//     two symbols; codes longer than 12 bits (and EOS) take a canonical-code path.  The bit stream is
//     padded with ones past the end of the string, so "at most 7 padding bits, all ones" becomes
//     "remaining bits <= 7 and the next 8 bits of the window are 0xFF".
//   * encode packs codes MSB-first into a 64-bit accumulator and emits whole 32-bit words; a string
//     fails as soon as its Huffman length can no longer be shorter than its input.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "hhuff_tables.h"

namespace hhuff {

constexpr uint32_t kLong = 1u << 29;
constexpr uint32_t kEos = 256;
constexpr uint32_t kFailLen = 0xFFFFFFFFu;
constexpr uint8_t kStatusFail = 0x80;
constexpr uint8_t kStatusTooLong = 0xC0;
constexpr uint32_t kMaxStrLen = (1u << 29) - 1;

constexpr uint32_t c_len[HHUFF_NUM_LENGTHS] = HHUFF_LEN_INIT;
constexpr uint32_t c_lim1[HHUFF_NUM_LENGTHS] = HHUFF_LIM1_INIT;
constexpr uint32_t c_first[HHUFF_NUM_LENGTHS] = HHUFF_FIRST_INIT;
constexpr uint32_t c_base[HHUFF_NUM_LENGTHS] = HHUFF_BASE_INIT;

__device__ __forceinline__ uint32_t bswap32(uint32_t x) { return __builtin_bswap32(x); }

// ---------------------------------------------------------------------------------------------------
// Byte sources.  word(a) returns the little-endian dword at 4-aligned byte position a.
// ---------------------------------------------------------------------------------------------------
struct LdsSource {  // a wave's staged input span; positions are relative to the 16-aligned span start
    const uint32_t* base;
    __device__ __forceinline__ uint32_t word(uint32_t a) const { return base[a >> 2]; }
};

struct GlobalSource {  // positions are absolute offsets into `in`; never reads at or past in_size
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
// Output writer: lane-private byte stream into global memory with dword stores.  Bytes before the first
// 4-aligned address are stored singly (the destination region may start at any byte, and its
// neighbours belong to other lanes).  Invariant after flush(): pending <= 3.
// ---------------------------------------------------------------------------------------------------
struct Writer {
    uint8_t* p;
    uint64_t acc;  // pending bytes, first byte in bits 0..7
    uint32_t pending;

    __device__ __forceinline__ void init(uint8_t* dst) { p = dst; acc = 0; pending = 0; }
    // append k (<= 4) bytes packed little-endian in `bytes`
    __device__ __forceinline__ void push(uint32_t bytes, uint32_t k) {
        acc |= (uint64_t)bytes << (8 * pending);
        pending += k;
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
    __device__ __forceinline__ void finish() {
        if (pending >= 2 && ((uintptr_t)p & 1) == 0) {
            *reinterpret_cast<uint16_t*>(p) = (uint16_t)acc;
            p += 2;
            acc >>= 16;
            pending -= 2;
        }
        while (pending > 0) {
            *p++ = (uint8_t)acc;
            acc >>= 8;
            --pending;
        }
    }
};

// ---------------------------------------------------------------------------------------------------
// Huffman bit reader: 64-bit MSB-aligned window over the string's bytes, ones past the end.
// ---------------------------------------------------------------------------------------------------
template <class Src>
struct BitReader {
    uint64_t buf;  // next bits of the stream, MSB first; bits below the valid count are zero
    uint32_t nb;   // valid bits in buf
    uint32_t a;    // position of the next dword to load (4-aligned)
    uint32_t end;  // string end position

    __device__ __forceinline__ uint32_t fetch(const Src& src, uint32_t pos) const {
        // big-endian word of the 4 bytes at pos; bytes at or past `end` read as 0xFF
        int32_t rem = (int32_t)(end - pos);
        uint32_t raw = 0xFFFFFFFFu;
        if (rem > 0) raw = src.word(pos);
        uint32_t w = bswap32(raw);
        uint32_t ones = rem >= 4 ? 0u : (rem <= 0 ? 0xFFFFFFFFu : (0xFFFFFFFFu >> (8 * rem)));
        return w | ones;
    }
    __device__ __forceinline__ void init(const Src& src, uint32_t start, uint32_t len) {
        end = start + len;
        a = start & ~3u;
        uint32_t skip = start & 3u;
        uint32_t w = fetch(src, a) << (8 * skip);
        buf = (uint64_t)w << 32;
        nb = 32 - 8 * skip;
        a += 4;
    }
    __device__ __forceinline__ void refill(const Src& src) {
        uint32_t w = fetch(src, a);
        buf |= (uint64_t)w << (32 - nb);
        nb += 32;
        a += 4;
    }
};

// ---------------------------------------------------------------------------------------------------
// decode one string (h2o_hpack_decode_huffman semantics).  lut = the 4096-entry window table in LDS.
// ---------------------------------------------------------------------------------------------------
template <class Src>
__device__ __forceinline__ void decode_string(const Src& src, uint32_t start, uint32_t len, bool is_name, uint8_t* dst,
                                              const uint32_t* __restrict__ lut, const uint16_t* __restrict__ sorted_syms,
                                              const uint32_t* __restrict__ inv_maps, uint32_t& out_len,
                                              uint8_t& status) {
    if (len > kMaxStrLen) {
        out_len = kFailLen;
        status = kStatusTooLong;
        return;
    }
    BitReader<Src> br;
    br.init(src, start, len);
    Writer wr;
    wr.init(dst);
    uint32_t R = 8 * len;  // string bits not yet consumed
    uint32_t cnt = 0, first = 0, last = 0, flags = 0;
    bool fail = false;
    for (;;) {
        if (br.nb <= 32) br.refill(src);
        uint32_t e = lut[(uint32_t)(br.buf >> (64 - HHUFF_LUT_BITS))];
        uint32_t consumed, syms, nsym, fl;
        if (__builtin_expect((e & kLong) != 0, 0)) {
            // canonical decode of a code longer than the window (hpack.c:85-99 walks the same tree)
            uint32_t t = (uint32_t)(br.buf >> 32);
            uint32_t j = HHUFF_FIRST_LONG_IDX;
#pragma unroll
            for (int k = HHUFF_FIRST_LONG_IDX; k < HHUFF_NUM_LENGTHS - 1; ++k) j += (t > c_lim1[k]) ? 1u : 0u;
            uint32_t L = 0, f = 0, b = 0;
#pragma unroll
            for (int k = HHUFF_FIRST_LONG_IDX; k < HHUFF_NUM_LENGTHS; ++k)
                if (j == (uint32_t)k) { L = c_len[k]; f = c_first[k]; b = c_base[k]; }
            if (L > R) break;  // incomplete code: padding
            uint32_t sym = sorted_syms[b + (t >> (32 - L)) - f];
            if (sym == kEos) { fail = true; break; }  // EOS inside the string (hpack.c:88-89)
            consumed = L;
            syms = sym;
            nsym = 1;
            fl = ((inv_maps[sym >> 5] >> (sym & 31)) & 1u) | (((inv_maps[8 + (sym >> 5)] >> (sym & 31)) & 1u) << 1);
        } else {
            uint32_t L1 = (e >> 16) & 15u, L12 = (e >> 20) & 15u;
            if (L1 > R) break;  // fewer bits left than the next code: padding
            bool take2 = ((e >> 24) & 1u) && L12 <= R;
            consumed = take2 ? L12 : L1;
            nsym = take2 ? 2u : 1u;
            syms = take2 ? (e & 0xFFFFu) : (e & 0xFFu);
            uint32_t f4 = (e >> 25) & (take2 ? 15u : 3u);
            fl = (f4 | (f4 >> 2)) & 3u;
        }
        flags |= fl;
        first = cnt == 0 ? (syms & 0xFFu) : first;
        last = (syms >> (8 * (nsym - 1))) & 0xFFu;
        wr.push(syms, nsym);
        cnt += nsym;
        br.buf <<= consumed;
        br.nb -= consumed;
        R -= consumed;
    }
    // accept iff no EOS and the padding is <= 7 bits of ones (mkhufftbl.py:374-381, hpack.c:132-133)
    if (fail || R > 7 || (uint32_t)(br.buf >> 56) != 0xFFu) {
        out_len = kFailLen;
        status = kStatusFail;
        return;
    }
    wr.finish();
    out_len = cnt;
    uint8_t st;
    if (is_name) {  // hpack.c:136-147 (':'-prefixed names are not validated; upper case is only soft)
        st = (cnt == 0 || ((flags & 1u) && first != ':')) ? 0x1 : 0x0;
    } else {  // hpack.c:150-152 + header_value_valid_as_whole :110-115
        bool ws = cnt != 0 && (first == ' ' || first == '\t' || last == ' ' || last == '\t');
        st = ((flags & 2u) || ws) ? 0x2 : 0x0;
    }
    status = st;
}

// ---------------------------------------------------------------------------------------------------
// encode one string (h2o_hpack_encode_huffman semantics).  enc = 256 x {code, nbits} in LDS.
// Writes at most len - 1 bytes at dst.
// ---------------------------------------------------------------------------------------------------
template <class Src>
__device__ __forceinline__ void encode_string(const Src& src, uint32_t start, uint32_t len, uint8_t* dst,
                                              const uint2* __restrict__ enc, uint32_t& out_len) {
    if (len > kMaxStrLen) {
        out_len = kFailLen;
        return;
    }
    Writer wr;
    wr.init(dst);
    uint64_t acc = 0;   // code bits, MSB-aligned
    uint32_t an = 0;    // bits in acc (< 32 between symbols)
    uint32_t emitted = 0;
    bool fail = false;
    const uint32_t end = start + len;
    for (uint32_t a = start & ~3u; a < end; a += 4) {
        uint32_t w = src.word(a);
#pragma unroll
        for (uint32_t k = 0; k < 4; ++k) {
            uint32_t pos = a + k;
            bool valid = pos >= start && pos < end;
            uint2 ent = enc[(w >> (8 * k)) & 0xFFu];
            uint32_t nb = valid ? ent.y : 0u;
            uint64_t code = valid ? (uint64_t)ent.x : 0ull;
            acc |= code << (64 - an - nb);
            an += nb;
            if (an >= 32) {
                if (emitted + 4 >= len) { fail = true; break; }  // cannot end up shorter than the input
                wr.push(bswap32((uint32_t)(acc >> 32)), 4);
                emitted += 4;
                acc <<= 32;
                an -= 32;
            }
        }
        if (fail) break;
    }
    uint32_t tail = (an + 7) >> 3;
    if (fail || emitted + tail >= len) {  // hpack.c:789-791, :799-800
        out_len = kFailLen;
        return;
    }
    if (an != 0) acc |= ~0ull >> an;  // pad with the EOS prefix (hpack.c:795-798)
    if (tail) wr.push(bswap32((uint32_t)(acc >> 32)) & (0xFFFFFFFFu >> (8 * (4 - tail))), tail);
    wr.finish();
    out_len = emitted + tail;
}

// ---------------------------------------------------------------------------------------------------
// wave helpers
// ---------------------------------------------------------------------------------------------------
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

}  // namespace hhuff
