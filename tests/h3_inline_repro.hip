// Reduction attempt for the gfx950 code-generation fault behind the `__noinline__` on the HTTP/3 request rules
// (h2o_amd/csrc/hhuff_qpack.hip, req_field_h3).  The rules (h2o_amd/csrc/hhuff_request.h) run over the same
// field sequences in two kernels that differ only in whether req_field<true> is inlined into the per-section
// loop; the host compares every record word.  tests/test_rules_host.py shows the rules' source is free of
// undefined behaviour (ASan + UBSan, equal to the oracle); the full sections kernel inlined loses err_desc
// codes (profiles/r04_h3_inline_tests.log).  Whether this small kernel shows it too is what the run records.
//   hipcc -O3 --offload-arch=gfx950 -Iinclude -Ih2o_amd/csrc tests/h3_inline_repro.hip -o build/h3_inline_repro
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <random>
#include <vector>

#include "hhuff_request.h"

namespace {
struct Field {
    uint32_t cls, voff, vlen, soft;
};

__device__ __noinline__ int32_t rule_call(hhuff::ReqState& r, uint32_t cls, const uint8_t* v, uint32_t vl, uint32_t soft,
                                          int32_t k, bool& header) {
    return hhuff::req_field<true>(r, cls, v, vl, soft, k, header);
}

template <bool INLINE>
__global__ void sections(const Field* __restrict__ f, const uint32_t* __restrict__ sec, uint32_t nsec,
                         const uint8_t* __restrict__ vals, hhuff_request_t* __restrict__ out, uint32_t* __restrict__ nhdr) {
    for (uint32_t k = blockIdx.x * blockDim.x + threadIdx.x; k < nsec; k += gridDim.x * blockDim.x) {
        hhuff::ReqState rq;
        rq.reset();
        uint32_t nh = 0;
        for (uint32_t j = sec[k]; j < sec[k + 1]; ++j) {
            const Field x = f[j];
            bool header = false;
            const int32_t rr = INLINE ? hhuff::req_field<true>(rq, x.cls, vals + x.voff, x.vlen, x.soft, (int32_t)(j - sec[k]), header)
                                      : rule_call(rq, x.cls, vals + x.voff, x.vlen, x.soft, (int32_t)(j - sec[k]), header);
            nh += header ? 1u : 0u;
            if (rr != 0) break;
        }
        hhuff::req_store(out + k, rq);
        nhdr[k] = nh;
    }
}
}  // namespace

#define CK(x)                                                                            \
    do {                                                                                 \
        hipError_t e_ = (x);                                                             \
        if (e_ != hipSuccess) {                                                          \
            printf("{\"error\": \"%s: %s\"}\n", #x, hipGetErrorString(e_));              \
            return 2;                                                                    \
        }                                                                                \
    } while (0)

int main() {
    const char* vals_txt[] = {"", "trailers", "TRAILERS", "gzip", "0", "123", "12a", "https", "masque", "http", "/",
                              "100-continue", "websocket", "99999999999999999999"};
    std::string vals;
    std::vector<uint32_t> voff, vlen;
    for (const char* v : vals_txt) {
        voff.push_back((uint32_t)vals.size());
        vlen.push_back((uint32_t)strlen(v));
        vals += v;
    }
    std::mt19937_64 rng(7);
    std::vector<Field> f;
    std::vector<uint32_t> sec{0};
    const uint32_t nsec = 200000;
    for (uint32_t k = 0; k < nsec; ++k) {
        // a request: pseudo-headers first (sometimes), then regular and special fields
        const uint32_t n = 1 + (uint32_t)(rng() % 14);
        for (uint32_t j = 0; j < n; ++j) {
            uint32_t cls = (uint32_t)(rng() % 15);  // the name classes of hhuff_request.h
            if (j < 3 && rng() % 2) cls = hhuff::kNMethod + (uint32_t)(rng() % 2);
            const uint32_t v = (uint32_t)(rng() % voff.size());
            f.push_back(Field{cls, voff[v], vlen[v], rng() % 9 == 0 ? 1u + (uint32_t)(rng() % 2) : 0u});
        }
        sec.push_back((uint32_t)f.size());
    }
    Field* df;
    uint32_t *dsec, *dnh[2];
    uint8_t* dv;
    hhuff_request_t* dout[2];
    CK(hipMalloc(&df, f.size() * sizeof(Field)));
    CK(hipMalloc(&dsec, sec.size() * 4));
    CK(hipMalloc(&dv, vals.size() + 16));
    for (int m = 0; m < 2; ++m) {
        CK(hipMalloc(&dout[m], nsec * sizeof(hhuff_request_t)));
        CK(hipMalloc(&dnh[m], nsec * 4));
    }
    CK(hipMemcpy(df, f.data(), f.size() * sizeof(Field), hipMemcpyHostToDevice));
    CK(hipMemcpy(dsec, sec.data(), sec.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(dv, vals.data(), vals.size(), hipMemcpyHostToDevice));
    hipLaunchKernelGGL(sections<true>, dim3(512), dim3(256), 0, 0, df, dsec, nsec, dv, dout[0], dnh[0]);
    hipLaunchKernelGGL(sections<false>, dim3(512), dim3(256), 0, 0, df, dsec, nsec, dv, dout[1], dnh[1]);
    CK(hipDeviceSynchronize());
    std::vector<hhuff_request_t> r[2];
    std::vector<uint32_t> nh[2];
    for (int m = 0; m < 2; ++m) {
        r[m].resize(nsec);
        nh[m].resize(nsec);
        CK(hipMemcpy(r[m].data(), dout[m], nsec * sizeof(hhuff_request_t), hipMemcpyDeviceToHost));
        CK(hipMemcpy(nh[m].data(), dnh[m], nsec * 4, hipMemcpyDeviceToHost));
    }
    uint32_t bad = 0, bad_err = 0;
    for (uint32_t k = 0; k < nsec; ++k) {
        if (memcmp(&r[0][k], &r[1][k], sizeof(hhuff_request_t)) != 0 || nh[0][k] != nh[1][k]) {
            ++bad;
            bad_err += r[0][k].err != r[1][k].err;
        }
    }
    printf("{\"sections\": %u, \"records_differing\": %u, \"err_differing\": %u}\n", nsec, bad, bad_err);
    return 0;
}
