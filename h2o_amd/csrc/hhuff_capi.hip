// hhuff C-ABI shim (include/hhuff.h): argument checks, stream plumbing, the per-string h2o symbols
// and the host-array batch entry points.  All compute goes through the HIP kernels in
// hhuff_kernels.hip; there is no CPU codec in this library.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "hhuff.h"
#include "hhuff_launch.h"

#define HHUFF_API extern "C" __attribute__((visibility("default")))

namespace {

thread_local char t_err[256] = "";

int hip_fail(hipError_t e, const char* where) {
    snprintf(t_err, sizeof(t_err), "%s: %s (%d)", where, hipGetErrorString(e), (int)e);
    return HHUFF_EHIP;
}

int arg_fail(const char* what) {
    snprintf(t_err, sizeof(t_err), "invalid argument: %s", what);
    return HHUFF_EINVAL;
}

#define HIP_TRY(call, where)                         \
    do {                                             \
        hipError_t e_ = (call);                      \
        if (e_ != hipSuccess) return hip_fail(e_, where); \
    } while (0)

// Per-thread device context: a stream on the chosen device plus growable device / pinned buffers.
struct Ctx {
    int dev = -1;
    hipStream_t stream = nullptr;
    uint8_t* d = nullptr;
    size_t dcap = 0;
    uint8_t* h = nullptr;
    size_t hcap = 0;
    ~Ctx() {
        // thread exit: release what this thread allocated (ignore errors at process teardown)
        if (d) (void)hipFree(d);
        if (h) (void)hipHostFree(h);
        if (stream) (void)hipStreamDestroy(stream);
    }
    int bind(int device) {
        if (device < 0) HIP_TRY(hipGetDevice(&device), "hipGetDevice");
        if (dev != device) {
            if (d) (void)hipFree(d), d = nullptr, dcap = 0;
            if (stream) (void)hipStreamDestroy(stream), stream = nullptr;
            HIP_TRY(hipSetDevice(device), "hipSetDevice");
            HIP_TRY(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking), "hipStreamCreate");
            dev = device;
        } else {
            HIP_TRY(hipSetDevice(device), "hipSetDevice");
        }
        return HHUFF_OK;
    }
    int reserve(size_t dneed, size_t hneed) {
        if (dneed > dcap) {
            if (d) (void)hipFree(d), d = nullptr, dcap = 0;
            size_t cap = dneed < (1u << 20) ? (1u << 20) : dneed + dneed / 4;
            HIP_TRY(hipMalloc(&d, cap), "hipMalloc");
            dcap = cap;
        }
        if (hneed > hcap) {
            if (h) (void)hipHostFree(h), h = nullptr, hcap = 0;
            size_t cap = hneed < (1u << 16) ? (1u << 16) : hneed + hneed / 4;
            HIP_TRY(hipHostMalloc(&h, cap, hipHostMallocDefault), "hipHostMalloc");
            hcap = cap;
        }
        return HHUFF_OK;
    }
};

thread_local Ctx t_ctx;

inline size_t up16(size_t x) { return (x + 15) & ~(size_t)15; }

[[noreturn]] void die(const char* fn) {
    fprintf(stderr, "hhuff: %s failed: %s\n", fn, t_err);
    abort();
}

int check_batch(const uint8_t* in, const uint32_t* in_off, uint32_t n, const uint8_t* out, const uint32_t* out_len) {
    if (n == 0) return HHUFF_OK;
    if (!in || !in_off || !out || !out_len) return arg_fail("NULL array");
    if (((uintptr_t)in & 15) != 0) return arg_fail("`in` must be 16-byte aligned");
    if (((uintptr_t)out & 15) != 0) return arg_fail("`out` must be 16-byte aligned");
    if (n > 0xFFFFFFFEu) return arg_fail("n too large");
    return HHUFF_OK;
}

}  // namespace

// ---------------------------------------------------------------------------------------------------
// (2) device batch API
// ---------------------------------------------------------------------------------------------------
HHUFF_API int hhuff_decode_batch(const uint8_t* in, uint64_t in_size, const uint32_t* in_off, const uint32_t* in_len,
                                 uint32_t n, const uint32_t* is_name_bits, uint8_t* out, const uint32_t* out_off,
                                 uint32_t* out_len, uint8_t* status, void* stream) {
    int rc = check_batch(in, in_off, n, out, out_len);
    if (rc) return rc;
    if (n && !status) return arg_fail("NULL status");
    hipError_t e = hhuff::launch_decode(in, in_size, in_off, in_len, n, is_name_bits, out, out_off, out_len, status,
                                        (hipStream_t)stream);
    return e == hipSuccess ? HHUFF_OK : hip_fail(e, "decode launch");
}

HHUFF_API int hhuff_encode_batch(const uint8_t* in, uint64_t in_size, const uint32_t* in_off, const uint32_t* in_len,
                                 uint32_t n, uint8_t* out, const uint32_t* out_off, uint32_t* out_len, uint8_t* status,
                                 void* stream) {
    int rc = check_batch(in, in_off, n, out, out_len);
    if (rc) return rc;
    hipError_t e = hhuff::launch_encode(in, in_size, in_off, in_len, n, out, out_off, out_len, status, (hipStream_t)stream);
    return e == hipSuccess ? HHUFF_OK : hip_fail(e, "encode launch");
}

HHUFF_API int hhuff_flatten_batch(const uint8_t* in, uint64_t in_size, const uint32_t* in_off, const uint32_t* in_len,
                                  uint32_t n, const uint8_t* first_bytes, unsigned prefix_bits, const uint32_t* raw_bits,
                                  uint8_t* out, const uint32_t* out_off, uint32_t* out_len, void* stream) {
    int rc = check_batch(in, in_off, n, out, out_len);
    if (rc) return rc;
    if (prefix_bits < 1 || prefix_bits > 7) return arg_fail("prefix_bits must be in 1..7");
    hipError_t e = hhuff::launch_flatten(in, in_size, in_off, in_len, n, first_bytes, prefix_bits, raw_bits, out, out_off,
                                         out_len, (hipStream_t)stream);
    return e == hipSuccess ? HHUFF_OK : hip_fail(e, "flatten launch");
}

// ---------------------------------------------------------------------------------------------------
// (1) h2o per-string symbols: a batch of one on the thread's stream, synchronously
// device/pinned layout: [meta 32 B: u32 in_off[2], out_len, is_name word, u8 status][input][output]
// ---------------------------------------------------------------------------------------------------
namespace {
constexpr size_t kMeta = 32;
}

HHUFF_API size_t h2o_hpack_decode_huffman(char* dst, unsigned* soft_errors, const uint8_t* src, size_t len, int is_name,
                                          const char** err_desc) {
    (void)err_desc;  // never written, as in the reference (hpack.c:142-144 is unreachable)
    Ctx& c = t_ctx;
    if (len > 0x1FFFFFFFu) {
        snprintf(t_err, sizeof(t_err), "string of %zu bytes exceeds the per-string limit", len);
        die("h2o_hpack_decode_huffman");
    }
    const size_t in_cap = up16(len ? len : 1), out_cap = up16(len * 8 / 5 + 4);
    if (c.bind(-1) || c.reserve(kMeta + in_cap + out_cap, kMeta + in_cap + out_cap)) die("h2o_hpack_decode_huffman");
    uint32_t* meta = reinterpret_cast<uint32_t*>(c.h);
    meta[0] = 0;
    meta[1] = (uint32_t)len;
    meta[2] = 0;
    meta[3] = is_name ? 1u : 0u;
    memcpy(c.h + kMeta, src, len);
    uint32_t* d_meta = reinterpret_cast<uint32_t*>(c.d);
    uint8_t* d_in = c.d + kMeta;
    uint8_t* d_out = c.d + kMeta + in_cap;
    hipError_t e = hipMemcpyAsync(c.d, c.h, kMeta + len, hipMemcpyHostToDevice, c.stream);
    if (e != hipSuccess) hip_fail(e, "H2D"), die("h2o_hpack_decode_huffman");
    e = hhuff::launch_decode(d_in, len, d_meta, nullptr, 1, d_meta + 3, d_out, nullptr, d_meta + 2,
                             reinterpret_cast<uint8_t*>(d_meta + 4), c.stream);
    if (e != hipSuccess) hip_fail(e, "decode launch"), die("h2o_hpack_decode_huffman");
    uint8_t* h_out = c.h + kMeta + in_cap;
    e = hipMemcpyAsync(c.h, c.d, kMeta, hipMemcpyDeviceToHost, c.stream);
    if (e == hipSuccess) e = hipMemcpyAsync(h_out, d_out, out_cap, hipMemcpyDeviceToHost, c.stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c.stream);
    if (e != hipSuccess) hip_fail(e, "D2H"), die("h2o_hpack_decode_huffman");
    const uint32_t r = meta[2];
    if (r == HHUFF_FAIL_LEN) return SIZE_MAX;
    memcpy(dst, h_out, r);
    *soft_errors |= *reinterpret_cast<const uint8_t*>(meta + 4);
    return r;
}

HHUFF_API size_t h2o_hpack_encode_huffman(uint8_t* dst, const uint8_t* src, size_t len) {
    Ctx& c = t_ctx;
    if (len > 0x1FFFFFFFu) {
        snprintf(t_err, sizeof(t_err), "string of %zu bytes exceeds the per-string limit", len);
        die("h2o_hpack_encode_huffman");
    }
    const size_t in_cap = up16(len ? len : 1), out_cap = up16(len + 4);
    if (c.bind(-1) || c.reserve(kMeta + in_cap + out_cap, kMeta + in_cap + out_cap)) die("h2o_hpack_encode_huffman");
    uint32_t* meta = reinterpret_cast<uint32_t*>(c.h);
    meta[0] = 0;
    meta[1] = (uint32_t)len;
    meta[2] = 0;
    meta[3] = 0;
    memcpy(c.h + kMeta, src, len);
    uint8_t* d_in = c.d + kMeta;
    uint8_t* d_out = c.d + kMeta + in_cap;
    uint32_t* d_meta = reinterpret_cast<uint32_t*>(c.d);
    hipError_t e = hipMemcpyAsync(c.d, c.h, kMeta + len, hipMemcpyHostToDevice, c.stream);
    if (e != hipSuccess) hip_fail(e, "H2D"), die("h2o_hpack_encode_huffman");
    e = hhuff::launch_encode(d_in, len, d_meta, nullptr, 1, d_out, nullptr, d_meta + 2, nullptr, c.stream);
    if (e != hipSuccess) hip_fail(e, "encode launch"), die("h2o_hpack_encode_huffman");
    uint8_t* h_out = c.h + kMeta + in_cap;
    e = hipMemcpyAsync(c.h, c.d, kMeta, hipMemcpyDeviceToHost, c.stream);
    if (e == hipSuccess && len) e = hipMemcpyAsync(h_out, d_out, len, hipMemcpyDeviceToHost, c.stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c.stream);
    if (e != hipSuccess) hip_fail(e, "D2H"), die("h2o_hpack_encode_huffman");
    uint32_t r = meta[2];
    if (r == HHUFF_FAIL_LEN) return SIZE_MAX;
    memcpy(dst, h_out, r);
    return r;
}

// ---------------------------------------------------------------------------------------------------
// (3) host batch API: copy in, run, copy out (synchronous)
// ---------------------------------------------------------------------------------------------------
namespace {

struct Carve {
    uint8_t* base;
    size_t off = 0;
    template <class T>
    T* take(size_t count) {
        T* p = reinterpret_cast<T*>(base + off);
        off += up16(count * sizeof(T));
        return p;
    }
};

size_t in_off_count(const uint32_t* in_len, uint32_t n) { return in_len ? n : (size_t)n + 1; }

int host_batch(bool decode, const uint8_t* in, uint64_t in_size, const uint32_t* in_off, const uint32_t* in_len,
               uint32_t n, const uint32_t* is_name_bits, uint8_t* out, uint64_t out_size, const uint32_t* out_off,
               uint32_t* out_len, uint8_t* status, int device) {
    if (n == 0) return HHUFF_OK;
    if (!in || !in_off || !out || !out_len || (decode && !status)) return arg_fail("NULL array");
    Ctx& c = t_ctx;
    int rc = c.bind(device);
    if (rc) return rc;
    const size_t noff = in_off_count(in_len, n), nw = ((size_t)n + 31) / 32;
    size_t need = up16(in_size ? in_size : 1) + up16(noff * 4) + (in_len ? up16((size_t)n * 4) : 0) +
                  (is_name_bits ? up16(nw * 4) : 0) + (out_off ? up16((size_t)n * 4) : 0) + up16(out_size ? out_size : 1) +
                  up16((size_t)n * 4) + up16(n);
    rc = c.reserve(need, 0);
    if (rc) return rc;
    Carve cv{c.d};
    uint8_t* d_in = cv.take<uint8_t>(in_size ? in_size : 1);
    uint32_t* d_in_off = cv.take<uint32_t>(noff);
    uint32_t* d_in_len = in_len ? cv.take<uint32_t>(n) : nullptr;
    uint32_t* d_name = is_name_bits ? cv.take<uint32_t>(nw) : nullptr;
    uint32_t* d_out_off = out_off ? cv.take<uint32_t>(n) : nullptr;
    uint8_t* d_out = cv.take<uint8_t>(out_size ? out_size : 1);
    uint32_t* d_out_len = cv.take<uint32_t>(n);
    uint8_t* d_status = cv.take<uint8_t>(n);
    hipStream_t s = c.stream;
    HIP_TRY(hipMemcpyAsync(d_in, in, in_size, hipMemcpyHostToDevice, s), "H2D in");
    HIP_TRY(hipMemcpyAsync(d_in_off, in_off, noff * 4, hipMemcpyHostToDevice, s), "H2D in_off");
    if (in_len) HIP_TRY(hipMemcpyAsync(d_in_len, in_len, (size_t)n * 4, hipMemcpyHostToDevice, s), "H2D in_len");
    if (is_name_bits) HIP_TRY(hipMemcpyAsync(d_name, is_name_bits, nw * 4, hipMemcpyHostToDevice, s), "H2D is_name");
    if (out_off) HIP_TRY(hipMemcpyAsync(d_out_off, out_off, (size_t)n * 4, hipMemcpyHostToDevice, s), "H2D out_off");
    hipError_t e = decode ? hhuff::launch_decode(d_in, in_size, d_in_off, d_in_len, n, d_name, d_out, d_out_off, d_out_len,
                                                 d_status, s)
                          : hhuff::launch_encode(d_in, in_size, d_in_off, d_in_len, n, d_out, d_out_off, d_out_len,
                                                 status ? d_status : nullptr, s);
    if (e != hipSuccess) return hip_fail(e, decode ? "decode launch" : "encode launch");
    HIP_TRY(hipMemcpyAsync(out, d_out, out_size, hipMemcpyDeviceToHost, s), "D2H out");
    HIP_TRY(hipMemcpyAsync(out_len, d_out_len, (size_t)n * 4, hipMemcpyDeviceToHost, s), "D2H out_len");
    if (status) HIP_TRY(hipMemcpyAsync(status, d_status, n, hipMemcpyDeviceToHost, s), "D2H status");
    HIP_TRY(hipStreamSynchronize(s), "sync");
    return HHUFF_OK;
}

}  // namespace

HHUFF_API int hhuff_decode_batch_host(const uint8_t* in, uint64_t in_size, const uint32_t* in_off, const uint32_t* in_len,
                                      uint32_t n, const uint32_t* is_name_bits, uint8_t* out, uint64_t out_size,
                                      const uint32_t* out_off, uint32_t* out_len, uint8_t* status, int device) {
    return host_batch(true, in, in_size, in_off, in_len, n, is_name_bits, out, out_size, out_off, out_len, status, device);
}

HHUFF_API int hhuff_encode_batch_host(const uint8_t* in, uint64_t in_size, const uint32_t* in_off, const uint32_t* in_len,
                                      uint32_t n, uint8_t* out, uint64_t out_size, const uint32_t* out_off,
                                      uint32_t* out_len, uint8_t* status, int device) {
    return host_batch(false, in, in_size, in_off, in_len, n, nullptr, out, out_size, out_off, out_len, status, device);
}

// ---------------------------------------------------------------------------------------------------
// (4) info
// ---------------------------------------------------------------------------------------------------
HHUFF_API const char* hhuff_version(void) { return "hhuff 0.1.0 (gfx950)"; }
HHUFF_API const char* hhuff_last_error_string(void) { return t_err; }
HHUFF_API int hhuff_grid_size(int device, int which) {
    if (hipSetDevice(device) != hipSuccess) return -1;
    return hhuff::grid_size(device, which);
}
