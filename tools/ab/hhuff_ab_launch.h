// A/B-only launch code of the decoders in hhuff_ab_decoders.h (HHUFF_AB_VARIANTS builds only).
#pragma once

// Segment decode (decode_seg_kernel) is a selectable alternative, not the default: measured against the stream kernel
// in one process on c3 (1M Zipf strings) 0.343 vs 0.290 ms and on c5 0.65 vs 0.45 ms (profiles/r05*_dec_ab.jsonl,
// DESIGN (e)).  Modes (hhuff_set_decode_kernel / HHUFF_DEC_SEG): 0 (default) the staged / stream choice, 1 the
// segment kernel for contiguous batches with a mean string above kSegMean bytes, 2 for every contiguous batch.
#ifndef HHUFF_SEG_CAP  // A/B builds: stage bytes per tile, tile budget, waves per CU
#define HHUFF_SEG_CAP 2560
#define HHUFF_SEG_TB 1920
#define HHUFF_SEG_WAVES 12
#endif
constexpr uint32_t kSegCap = HHUFF_SEG_CAP, kSegTB = HHUFF_SEG_TB;  // stage bytes per tile; tile budget (longest kept
                                                                   // last string: CAP - TB = 640)
constexpr int kSegWaves = HHUFF_SEG_WAVES;                         // 12 x 10.3 KiB + 33.5 KiB of tables per CU
constexpr uint64_t kSegMean = 40;
#define DEC_G decode_seg_kernel<kSegWaves, kSegCap, kSegTB>
static std::atomic<int> g_seg_mode{-1};
static int seg_mode() {
    int m = g_seg_mode.load(std::memory_order_relaxed);
    if (m < 0) {
        const char* v = getenv("HHUFF_DEC_SEG");
        const int env = v && *v ? (v[0] == '2' ? 2 : (v[0] == '1' ? 1 : 0)) : 0;
        int expect = -1;
        g_seg_mode.compare_exchange_strong(expect, env);
        m = g_seg_mode.load(std::memory_order_relaxed);
    }
    return m;
}
int set_decode_kernel(int mode) {
    if (mode < 0 || mode > 2) return -1;
    const int prev = seg_mode();
    g_seg_mode.store(mode);
    return prev;
}
static bool use_seg(uint64_t bytes, uint32_t n, const uint32_t* in_len, const uint32_t* out_off) {
    const int m = seg_mode();
    if (m == 0 || in_len != nullptr || out_off != nullptr || n == 0) return false;
    return m == 2 || bytes / n > kSegMean;
}
static hipError_t launch_seg(DecArgs A, uint64_t in_size, uint32_t n, uint8_t* out, hipStream_t stream) {
    const uint64_t tmax64 = in_size / kSegTB + 2u;  // tiles + 1 (the plan needs tf[T], T <= in_size / TB + 1)
    if (tmax64 >= (1ull << 31)) return hipErrorInvalidValue;
    const uint32_t tmax = (uint32_t)tmax64;
    uint32_t* tf = nullptr;
    hipError_t e = pool_alloc((void**)&tf, 4ull * tmax, stream);
    if (e != hipSuccess) return e;
    e = pool_alloc((void**)&A.edges, 2ull * tmax * sizeof(EdgeRec), stream);
    if (e != hipSuccess) {
        (void)hipFreeAsync(tf, stream);
        return e;
    }
    const uint32_t pblocks = (uint32_t)std::min<uint64_t>(((uint64_t)n + 256u) / 256u, 4096u);
    hipLaunchKernelGGL(seg_plan_kernel, dim3(pblocks), dim3(256), 0, stream, A.in_off, n, kSegTB, tmax, tf, A.edges);
    e = hipGetLastError();
    if (e == hipSuccess) {
        static int cus[64] = {};
        const int dev = current_device();
        int& c = cus[dev >= 0 && dev < 64 ? dev : 0];
        if (c == 0 && (hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || c < 1)) c = 256;
        const uint64_t want = (tmax64 + kSegWaves - 1) / kSegWaves;
        const uint32_t grid = (uint32_t)std::min<uint64_t>(want, (uint64_t)c);
        hipLaunchKernelGGL(DEC_G, dim3(grid), dim3(kSegWaves * 64), 0, stream, A, (const uint32_t*)tf, tmax);
        e = finish_deferred(out, A.edges, n, stream, nullptr, 2ull * tmax);
    } else {
        (void)hipFreeAsync(A.edges, stream);
    }
    const hipError_t f = hipFreeAsync(tf, stream);
    return e != hipSuccess ? e : f;
}

// Length-sorted decode chunks (decode_sorted_kernel) for the short-string contiguous layout, HHUFF_DEC_SORTED=1 (A/B;
// off by default: c4 decode 0.588 -> 0.606 ms in two alternating runs each, profiles/r05i_sorted_decode_ab.jsonl --
// the waves of a group that wait for its longest-string wave leave their SIMD fewer waves to hide the LUT chain's
// latency, which the balanced lanes do not win back)
#ifndef HHUFF_DS_CH
#define HHUFF_DS_CH 10240
#endif
static bool sorted_decode_on() {
    static const bool on = [] {
        const char* v = getenv("HHUFF_DEC_SORTED");
        return v && v[0] == '1';
    }();
    return on;
}
static hipError_t launch_sorted_decode(DecArgs A, uint32_t n, uint8_t* out, hipStream_t stream) {
    const uint64_t nch = ((uint64_t)n + kDsStr - 1) / kDsStr;
    hipError_t e = pool_alloc((void**)&A.edges, 2ull * nch * sizeof(EdgeRec), stream);
    if (e != hipSuccess) return e;
    static int cus[64] = {};
    const int dev = current_device();
    int& cu = cus[dev >= 0 && dev < 64 ? dev : 0];
    if (cu == 0 && (hipDeviceGetAttribute(&cu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cu < 1)) cu = 256;
    const uint32_t grid = (uint32_t)std::min<uint64_t>((nch + 3) / 4, (uint64_t)cu);
    hipLaunchKernelGGL(decode_sorted_kernel<HHUFF_DS_CH>, dim3(grid), dim3(1024), 0, stream, A);
    return finish_deferred(out, A.edges, n, stream, nullptr, 2ull * nch);
}
