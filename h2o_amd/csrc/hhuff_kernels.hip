// hhuff HIP kernels for gfx950 (MI355X) and their launchers.
//
// Work decomposition (both directions): one lane per string, 64 consecutive strings per wave, waves
// grid-stride over the batch.  Each wave stages the contiguous input span of its 64 strings into LDS
// with 16-byte coalesced loads (1 KiB per wave instruction); lanes then read their own string from
// LDS.  Spans larger than the stage fall back to direct global loads for that wave (wave-uniform
// branch).  The decode LUT (16 KiB) / encode table (2 KiB) is staged in LDS once per workgroup.
//
// Reference semantics: lib/http2/hpack.c:117-156 (decode), :774-804 (encode); see hhuff_device.h.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "hhuff_device.h"
#include "hhuff_launch.h"

namespace hhuff {

__device__ const uint32_t g_dec_lut[1u << HHUFF_LUT_BITS] = HHUFF_DEC_LUT_INIT;
__device__ const uint16_t g_sorted_syms[257] = HHUFF_SORTED_SYMS_INIT;
__device__ const uint32_t g_name_inv[8] = HHUFF_NAME_INVALID_INIT;
__device__ const uint32_t g_value_inv[8] = HHUFF_VALUE_INVALID_INIT;
__device__ const uint32_t g_enc_code[256] = HHUFF_ENC_CODE_INIT;
__device__ const uint8_t g_enc_nbits[256] = HHUFF_ENC_NBITS_INIT;

// Stage the wave's input span [a0, a0 + span) into LDS (16-byte loads; bytes past in_size read 0).
__device__ __forceinline__ void stage_span(uint32_t* stage, const uint8_t* __restrict__ in, uint64_t in_size, uint32_t a0,
                                           uint32_t span, int lane) {
    for (uint32_t k = (uint32_t)lane * 16u; k < span; k += 64u * 16u) {
        uint64_t g = (uint64_t)a0 + k;
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

__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

template <int WAVES, int STAGE>
__global__ __launch_bounds__(WAVES * 64) void decode_kernel(const uint8_t* __restrict__ in, uint64_t in_size,
                                                            const uint32_t* __restrict__ in_off,
                                                            const uint32_t* __restrict__ in_len, uint32_t n,
                                                            const uint32_t* __restrict__ is_name_bits,
                                                            uint8_t* __restrict__ out, const uint32_t* __restrict__ out_off,
                                                            uint32_t* __restrict__ out_len, uint8_t* __restrict__ status) {
    __shared__ __attribute__((aligned(16))) uint32_t s_lut[1u << HHUFF_LUT_BITS];
    __shared__ __attribute__((aligned(16))) uint32_t s_stage[WAVES][STAGE / 4];
    __shared__ uint32_t s_inv[16];
    __shared__ uint16_t s_sorted[257];
    for (uint32_t k = threadIdx.x; k < (1u << HHUFF_LUT_BITS) / 4; k += WAVES * 64)
        reinterpret_cast<uint4*>(s_lut)[k] = reinterpret_cast<const uint4*>(g_dec_lut)[k];
    for (uint32_t k = threadIdx.x; k < 257; k += WAVES * 64) s_sorted[k] = g_sorted_syms[k];
    if (threadIdx.x < 16) s_inv[threadIdx.x] = threadIdx.x < 8 ? g_name_inv[threadIdx.x] : g_value_inv[threadIdx.x - 8];
    __syncthreads();

    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint32_t* stage = s_stage[wave];
    const uint64_t stride = (uint64_t)gridDim.x * WAVES * 64;
    for (uint64_t base = ((uint64_t)blockIdx.x * WAVES + wave) * 64; base < n; base += stride) {
        const uint32_t i = (uint32_t)base + lane;
        const bool valid = i < n;
        uint32_t s = 0, len = 0;
        if (valid) {
            s = in_off[i];
            len = in_len ? in_len[i] : in_off[i + 1] - s;
        }
        const bool has = valid && len != 0;
        const uint32_t lo = wave_min_u32(has ? s : 0xFFFFFFFFu);
        const uint32_t hi = wave_max_u32(has ? s + len : 0u);
        const uint32_t a0 = lo & ~15u;
        const uint32_t span = hi > lo ? ((hi + 15u) & ~15u) - a0 : 0u;
        uint32_t ol = 0;
        uint8_t st = 0;
        const bool is_name = valid && is_name_bits ? ((is_name_bits[i >> 5] >> (i & 31)) & 1u) : false;
        uint8_t* dst = out + (out_off ? (uint64_t)(valid ? out_off[i] : 0u) : ((uint64_t)s * 8u) / 5u);
        if (span <= STAGE) {
            stage_span(stage, in, in_size, a0, span, lane);
            wave_lds_sync();
            if (valid) decode_string(LdsSource{stage}, s - (has ? a0 : s), len, is_name, dst, s_lut, s_sorted, s_inv, ol, st);
            wave_lds_sync();
        } else {
            if (valid) decode_string(GlobalSource{in, in_size}, s, len, is_name, dst, s_lut, s_sorted, s_inv, ol, st);
        }
        if (valid) {
            out_len[i] = ol;
            status[i] = st;
        }
    }
}

template <int WAVES, int STAGE>
__global__ __launch_bounds__(WAVES * 64) void encode_kernel(const uint8_t* __restrict__ in, uint64_t in_size,
                                                            const uint32_t* __restrict__ in_off,
                                                            const uint32_t* __restrict__ in_len, uint32_t n,
                                                            uint8_t* __restrict__ out, const uint32_t* __restrict__ out_off,
                                                            uint32_t* __restrict__ out_len, uint8_t* __restrict__ status) {
    __shared__ __attribute__((aligned(16))) uint2 s_enc[256];
    __shared__ __attribute__((aligned(16))) uint32_t s_stage[WAVES][STAGE / 4];
    for (uint32_t k = threadIdx.x; k < 256; k += WAVES * 64) s_enc[k] = make_uint2(g_enc_code[k], g_enc_nbits[k]);
    __syncthreads();

    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint32_t* stage = s_stage[wave];
    const uint64_t stride = (uint64_t)gridDim.x * WAVES * 64;
    for (uint64_t base = ((uint64_t)blockIdx.x * WAVES + wave) * 64; base < n; base += stride) {
        const uint32_t i = (uint32_t)base + lane;
        const bool valid = i < n;
        uint32_t s = 0, len = 0;
        if (valid) {
            s = in_off[i];
            len = in_len ? in_len[i] : in_off[i + 1] - s;
        }
        const bool has = valid && len != 0;
        const uint32_t lo = wave_min_u32(has ? s : 0xFFFFFFFFu);
        const uint32_t hi = wave_max_u32(has ? s + len : 0u);
        const uint32_t a0 = lo & ~15u;
        const uint32_t span = hi > lo ? ((hi + 15u) & ~15u) - a0 : 0u;
        uint32_t ol = kFailLen;
        uint8_t* dst = out + (out_off ? (uint64_t)(valid ? out_off[i] : 0u) : (uint64_t)s);
        if (span <= STAGE) {
            stage_span(stage, in, in_size, a0, span, lane);
            wave_lds_sync();
            if (valid) encode_string(LdsSource{stage}, s - (has ? a0 : s), len, dst, s_enc, ol);
            wave_lds_sync();
        } else {
            if (valid) encode_string(GlobalSource{in, in_size}, s, len, dst, s_enc, ol);
        }
        if (valid) {
            out_len[i] = ol;
            if (status) status[i] = ol == kFailLen ? (len > kMaxStrLen ? kStatusTooLong : kStatusFail) : 0;
        }
    }
}

// ------------------------------------------------------------------------------------------------
// launch configuration
// ------------------------------------------------------------------------------------------------
constexpr int kDecWaves = 4, kDecStage = 6144;
constexpr int kEncWaves = 4, kEncStage = 8192;

static int grid_for(const void* fn, int threads, int device, uint32_t n) {
    static int cache[64][2] = {};
    int which = fn == (const void*)decode_kernel<kDecWaves, kDecStage> ? 0 : 1;
    if (device < 0 || device >= 64) device = 0;
    if (cache[device][which] == 0) {
        int per_cu = 0, cus = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, threads, 0) != hipSuccess || per_cu < 1) per_cu = 1;
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess || cus < 1) cus = 256;
        cache[device][which] = per_cu * cus;
    }
    uint64_t tiles = ((uint64_t)n + threads - 1) / threads;
    int g = cache[device][which];
    return (int)(tiles < (uint64_t)g ? (tiles ? tiles : 1) : g);
}

hipError_t launch_decode(const uint8_t* in, uint64_t in_size, const uint32_t* in_off, const uint32_t* in_len, uint32_t n,
                         const uint32_t* is_name_bits, uint8_t* out, const uint32_t* out_off, uint32_t* out_len,
                         uint8_t* status, hipStream_t stream) {
    if (n == 0) return hipSuccess;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) dev = 0;
    const void* fn = (const void*)decode_kernel<kDecWaves, kDecStage>;
    int grid = grid_for(fn, kDecWaves * 64, dev, n);
    hipLaunchKernelGGL((decode_kernel<kDecWaves, kDecStage>), dim3(grid), dim3(kDecWaves * 64), 0, stream, in, in_size,
                       in_off, in_len, n, is_name_bits, out, out_off, out_len, status);
    return hipGetLastError();
}

hipError_t launch_encode(const uint8_t* in, uint64_t in_size, const uint32_t* in_off, const uint32_t* in_len, uint32_t n,
                         uint8_t* out, const uint32_t* out_off, uint32_t* out_len, uint8_t* status, hipStream_t stream) {
    if (n == 0) return hipSuccess;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) dev = 0;
    const void* fn = (const void*)encode_kernel<kEncWaves, kEncStage>;
    int grid = grid_for(fn, kEncWaves * 64, dev, n);
    hipLaunchKernelGGL((encode_kernel<kEncWaves, kEncStage>), dim3(grid), dim3(kEncWaves * 64), 0, stream, in, in_size,
                       in_off, in_len, n, out, out_off, out_len, status);
    return hipGetLastError();
}

int grid_size(int device, int which) {
    if (which == 0) return grid_for((const void*)decode_kernel<kDecWaves, kDecStage>, kDecWaves * 64, device, 0xFFFFFFFFu);
    return grid_for((const void*)encode_kernel<kEncWaves, kEncStage>, kEncWaves * 64, device, 0xFFFFFFFFu);
}

}  // namespace hhuff
