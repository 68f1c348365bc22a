// Probe: can the host write device memory directly (a mailbox in VRAM for the per-string service)?
// Allocates fine-grained and uncached device memory, asks HIP for a host pointer, writes through it from the
// host and has a kernel read the words back (vector loads), timing a host-write -> device-see round trip.
//   hipcc --offload-arch=gfx950 -O2 tools/vram_probe.hip -o tools/vram_probe && ./tools/vram_probe
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>

__global__ void read_back(const volatile unsigned* p, unsigned* out) {
    if (threadIdx.x == 0) out[0] = p[0];
}

// spins (bounded) until the word changes from `old`; reports the iterations it took
__global__ void spin_see(const unsigned* p, unsigned old, unsigned* out, unsigned max_iter) {
    if (threadIdx.x != 0) return;
    unsigned it = 0, v = old;
    for (; it < max_iter; ++it) {
        v = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        if (v != old) break;
        __builtin_amdgcn_s_sleep(1);
    }
    out[0] = v;
    out[1] = it;
}

static void probe(const char* name, unsigned flags) {
    void* d = nullptr;
    hipError_t e = hipExtMallocWithFlags(&d, 4096, flags);
    printf("{\"alloc\": \"%s\", \"rc\": %d", name, (int)e);
    if (e != hipSuccess) {
        printf("}\n");
        return;
    }
    hipPointerAttribute_t a;
    e = hipPointerGetAttributes(&a, d);
    printf(", \"attr_rc\": %d, \"type\": %d, \"host_ptr\": %s", (int)e, (int)a.type, a.hostPointer ? "true" : "false");
    unsigned* out = nullptr;
    (void)hipHostMalloc((void**)&out, 64, hipHostMallocCoherent);
    volatile unsigned* hp = static_cast<volatile unsigned*>(a.hostPointer);
    if (hp) {
        hp[0] = 0x1234u;  // host write through the pointer HIP gave
        hipLaunchKernelGGL(read_back, dim3(1), dim3(64), 0, 0, static_cast<const volatile unsigned*>(d), out);
        (void)hipDeviceSynchronize();
        printf(", \"device_read\": %u", out[0]);
        // a spinning kernel sees a later host write: the host-to-device hand-over time
        hp[0] = 7u;
        hipLaunchKernelGGL(spin_see, dim3(1), dim3(64), 0, 0, static_cast<const unsigned*>(d), 7u, out, 2000000u);
        auto t0 = std::chrono::steady_clock::now();
        while (std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count() < 200.0) {
        }
        hp[0] = 8u;
        (void)hipDeviceSynchronize();
        printf(", \"spin_saw\": %u, \"spin_iters\": %u", out[0], out[1]);
    }
    printf("}\n");
    (void)hipHostFree(out);
    (void)hipFree(d);
}

int main() {
    probe("finegrained", hipDeviceMallocFinegrained);
    probe("uncached", hipDeviceMallocUncached);
    probe("default", hipDeviceMallocDefault);
    return 0;
}
