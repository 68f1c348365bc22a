// Probe: does gfx950 LDS honour 2-byte stores at odd addresses (unaligned access mode)?
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

__global__ void k(uint8_t* out) {
    __shared__ __attribute__((aligned(16))) uint8_t s[256];
    const int t = threadIdx.x;
    for (int i = t; i < 256; i += 64) s[i] = 0;
    __syncthreads();
    // lane t writes 0xAB,0xCD at byte 3*t+1 (odd and even addresses)
    uint16_t* p = reinterpret_cast<uint16_t*>(s + 3 * t + 1);
    *p = (uint16_t)(0xCDAB);
    __syncthreads();
    for (int i = t; i < 256; i += 64) out[i] = s[i];
}

int main() {
    uint8_t* d;
    (void)hipMalloc(&d, 256);
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
    uint8_t h[256];
    (void)hipMemcpy(h, d, 256, hipMemcpyDeviceToHost);
    int bad = 0;
    for (int t = 0; t < 64; ++t) {
        if (h[3 * t + 1] != 0xAB || h[3 * t + 2] != 0xCD) ++bad;
    }
    printf("unaligned ds_write_b16: %s (%d lanes wrong); bytes 0..8: %02x %02x %02x %02x %02x %02x %02x %02x\n",
           bad ? "NOT honoured" : "honoured", bad, h[0], h[1], h[2], h[3], h[4], h[5], h[6], h[7]);
    return 0;
}
