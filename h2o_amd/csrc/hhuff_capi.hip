// hhuff C-ABI shim (include/hhuff.h): argument checks, stream plumbing, the per-string h2o symbols
// and the host-array batch entry points.  All compute goes through the HIP kernels in
// hhuff_kernels.hip; there is no CPU codec in this library.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <functional>
#include <string>
#include <immintrin.h>
#include <mutex>
#include <thread>
#include <vector>

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
// bind() never changes the calling thread's current device for good: the per-string symbols run on the
// thread's current device (h2o's worker threads may have set one), the host batch calls on their `device`
// argument with the caller's current device restored on return (DeviceGuard).
struct Ctx {
    int dev = -1;
    hipStream_t stream = nullptr;
    uint8_t* d = nullptr;
    size_t dcap = 0;
    uint8_t* h = nullptr;  // pinned, device-visible (the per-string kernel reads and writes it in place)
    size_t hcap = 0;
    ~Ctx() {
        // thread exit: release what this thread allocated (ignore errors at process teardown); a one-string
        // kernel whose result was taken early (wait_one) may still be retiring
        if (stream) (void)hipStreamSynchronize(stream);
        if (d) (void)hipFree(d);
        if (h) (void)hipHostFree(h);
        if (stream) (void)hipStreamDestroy(stream);
    }
    // make `device` (-1: the thread's current device) this context's device; the caller's current device is
    // the one left current (the stream of a device can be used with another device current)
    int bind(int device) {
        int cur = 0;
        HIP_TRY(hipGetDevice(&cur), "hipGetDevice");
        if (device < 0) device = cur;
        if (dev != device) {
            if (stream) (void)hipStreamSynchronize(stream);
            if (d) (void)hipFree(d), d = nullptr, dcap = 0;
            if (h) (void)hipHostFree(h), h = nullptr, hcap = 0;
            if (stream) (void)hipStreamDestroy(stream), stream = nullptr;
            if (device != cur) HIP_TRY(hipSetDevice(device), "hipSetDevice");
            const hipError_t e = hipStreamCreateWithFlags(&stream, hipStreamNonBlocking);
            if (device != cur) (void)hipSetDevice(cur);
            if (e != hipSuccess) return hip_fail(e, "hipStreamCreate");
            dev = device;
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
            if (h) (void)hipStreamSynchronize(stream), (void)hipHostFree(h), h = nullptr, hcap = 0;  // (wait_one)
            size_t cap = hneed < (1u << 16) ? (1u << 16) : hneed + hneed / 4;
            // coherent (fine-grained): the per-string kernel reads and writes it in place across PCIe
            HIP_TRY(hipHostMalloc(&h, cap, hipHostMallocMapped | hipHostMallocCoherent), "hipHostMalloc");
            hcap = cap;
        }
        return HHUFF_OK;
    }
};

// Makes `device` current for the scope of a host batch call, restoring the caller's device on exit.
struct DeviceGuard {
    int prev = -1;
    hipError_t err = hipSuccess;
    explicit DeviceGuard(int device) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        if (device >= 0 && device != prev) err = hipSetDevice(device);
    }
    ~DeviceGuard() {
        int cur = -1;
        if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
    }
};

thread_local Ctx t_ctx;

inline size_t up16(size_t x) { return (x + 15) & ~(size_t)15; }

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

HHUFF_API int hhuff_decode_batch_packed(const uint8_t* in, uint64_t in_size, const uint32_t* in_off, uint32_t n,
                                        const uint32_t* is_name_bits, uint8_t* out, uint32_t* out_off, uint32_t* out_len,
                                        uint8_t* status, void* stream) {
    if (!out_off) return arg_fail("NULL out_off");
    int rc = check_batch(in, in_off, n, out, out_len);
    if (rc) return rc;
    if (n && !status) return arg_fail("NULL status");
    if ((in_size * 8) / 5 >= 0xFFFFFFFFull) return arg_fail("in_size too large for u32 packed offsets");
    hipError_t e = hhuff::launch_decode_packed(in, in_size, in_off, n, is_name_bits, out, out_off, out_len, status,
                                               (hipStream_t)stream);
    return e == hipSuccess ? HHUFF_OK : hip_fail(e, "packed decode launch");
}

HHUFF_API int hhuff_encode_batch_packed(const uint8_t* in, uint64_t in_size, const uint32_t* in_off, uint32_t n,
                                        uint8_t* out, uint32_t* out_off, uint32_t* out_len, uint8_t* status, void* stream) {
    if (!out_off) return arg_fail("NULL out_off");
    int rc = check_batch(in, in_off, n, out, out_len);
    if (rc) return rc;
    if (in_size >= 0xFFFFFFFFull) return arg_fail("in_size too large for u32 packed offsets");
    hipError_t e = hhuff::launch_encode_packed(in, in_size, in_off, n, out, out_off, out_len, status, (hipStream_t)stream);
    return e == hipSuccess ? HHUFF_OK : hip_fail(e, "packed encode launch");
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

HHUFF_API int hhuff_decode_literals(const uint8_t* in, uint64_t in_size, const uint32_t* lit_off, const uint32_t* lit_end,
                                    uint32_t n, unsigned prefix_bits, unsigned flags, const uint32_t* is_name_bits,
                                    uint8_t* out, uint32_t* out_len, uint32_t* pay_off, uint32_t* consumed,
                                    uint8_t* status, void* stream) {
    int rc = check_batch(in, lit_off, n, out, out_len);
    if (rc) return rc;
    if (n && (!lit_end || !pay_off || !consumed || !status)) return arg_fail("NULL array");
    if (prefix_bits < 1 || prefix_bits > 7) return arg_fail("prefix_bits must be in 1..7");
    if (n == 0) return HHUFF_OK;
    hipStream_t s = (hipStream_t)stream;
    void* ws = nullptr;  // Huffman payload lengths + per-literal verdict bytes, stream-ordered scratch
    HIP_TRY(hipMallocAsync(&ws, (size_t)n * 5, s), "hipMallocAsync");
    hipError_t e = hhuff::launch_literals(in, in_size, lit_off, lit_end, n, prefix_bits, flags & HHUFF_LIT_QPACK, is_name_bits, out, out_len,
                                          pay_off, consumed, status, (uint32_t*)ws, s);
    hipError_t f = hipFreeAsync(ws, s);
    if (e != hipSuccess) return hip_fail(e, "literal launch");
    return f == hipSuccess ? HHUFF_OK : hip_fail(f, "hipFreeAsync");
}

HHUFF_API uint64_t hhuff_hpack_scratch_size(uint32_t nconn, uint32_t table_size) {
    return (uint64_t)nconn * hhuff::hpack_conn_scratch(table_size);
}

namespace {
int hpack_blocks(const uint8_t* in, uint64_t in_size, const uint32_t* blk_off, const uint32_t* conn_first, uint32_t nconn,
                 uint32_t table_size, uint8_t* arena, const uint64_t* arena_off, uint32_t* name_off, uint32_t* name_len,
                 uint32_t* value_off, uint32_t* value_len, uint8_t* fflags, uint32_t* nfields, int32_t* bstatus,
                 hhuff_request_t* req, hhuff_response_t* res, const uint8_t* trailers, void* scratch,
                 uint64_t scratch_size, unsigned flags, void* stream) {
    if (nconn == 0) return HHUFF_OK;
    if (!in || !blk_off || !conn_first || !arena || !arena_off || !name_off || !name_len || !value_off || !value_len ||
        !fflags || !nfields || !bstatus || !scratch)
        return arg_fail("NULL array");
    if (scratch_size < hhuff_hpack_scratch_size(nconn, table_size)) return arg_fail("scratch smaller than hhuff_hpack_scratch_size");
    if (((uintptr_t)scratch & 15u) != 0) return arg_fail("scratch must be 16-byte aligned");
    if (((uintptr_t)req & 7u) != 0) return arg_fail("req must be 8-byte aligned");
    if (((uintptr_t)res & 3u) != 0) return arg_fail("res must be 4-byte aligned");
    hipError_t e = hhuff::launch_hpack_blocks(in, in_size, blk_off, conn_first, nconn, table_size, arena, arena_off, name_off,
                                              name_len, value_off, value_len, fflags, nfields, bstatus, req, res, trailers,
                                              (uint8_t*)scratch, flags, (hipStream_t)stream);
    return e == hipSuccess ? HHUFF_OK : hip_fail(e, "hpack block launch");
}
}  // namespace

HHUFF_API int hhuff_hpack_decode_blocks(const uint8_t* in, uint64_t in_size, const uint32_t* blk_off,
                                        const uint32_t* conn_first, uint32_t nconn, uint32_t table_size, uint8_t* arena,
                                        const uint64_t* arena_off, uint32_t* name_off, uint32_t* name_len,
                                        uint32_t* value_off, uint32_t* value_len, uint8_t* fflags, uint32_t* nfields,
                                        int32_t* bstatus, void* scratch, uint64_t scratch_size, unsigned flags,
                                        void* stream) {
    return hpack_blocks(in, in_size, blk_off, conn_first, nconn, table_size, arena, arena_off, name_off, name_len,
                        value_off, value_len, fflags, nfields, bstatus, nullptr, nullptr, nullptr, scratch, scratch_size,
                        flags, stream);
}

HHUFF_API int hhuff_hpack_parse_requests(const uint8_t* in, uint64_t in_size, const uint32_t* blk_off,
                                         const uint32_t* conn_first, uint32_t nconn, uint32_t table_size, uint8_t* arena,
                                         const uint64_t* arena_off, uint32_t* name_off, uint32_t* name_len,
                                         uint32_t* value_off, uint32_t* value_len, uint8_t* fflags, uint32_t* nfields,
                                         int32_t* bstatus, hhuff_request_t* req, void* scratch, uint64_t scratch_size,
                                         unsigned flags, void* stream) {
    if (nconn != 0 && !req) return arg_fail("NULL array");
    return hpack_blocks(in, in_size, blk_off, conn_first, nconn, table_size, arena, arena_off, name_off, name_len,
                        value_off, value_len, fflags, nfields, bstatus, req, nullptr, nullptr, scratch, scratch_size,
                        flags, stream);
}

HHUFF_API int hhuff_hpack_parse_responses(const uint8_t* in, uint64_t in_size, const uint32_t* blk_off,
                                          const uint32_t* conn_first, uint32_t nconn, uint32_t table_size,
                                          const uint8_t* trailers, uint8_t* arena, const uint64_t* arena_off,
                                          uint32_t* name_off, uint32_t* name_len, uint32_t* value_off, uint32_t* value_len,
                                          uint8_t* fflags, uint32_t* nfields, int32_t* bstatus, hhuff_response_t* res,
                                          void* scratch, uint64_t scratch_size, unsigned flags, void* stream) {
    if (nconn != 0 && !res) return arg_fail("NULL array");
    return hpack_blocks(in, in_size, blk_off, conn_first, nconn, table_size, arena, arena_off, name_off, name_len,
                        value_off, value_len, fflags, nfields, bstatus, nullptr, res, trailers, scratch, scratch_size,
                        flags, stream);
}

HHUFF_API uint64_t hhuff_hpack_enc_scratch_size(uint32_t nconn) { return (uint64_t)nconn * hhuff::hpenc_conn_scratch(); }

HHUFF_API int hhuff_hpack_flatten_responses(const uint8_t* in, uint64_t in_size, const hhuff_hpack_header_t* hdr,
                                            uint32_t nhdr, const hhuff_hpack_response_t* res, const uint32_t* conn_first,
                                            uint32_t nconn, uint32_t nres, uint32_t server_off, uint32_t server_len,
                                            uint8_t* out, const uint64_t* out_off, uint32_t* out_len,
                                            uint32_t* headers_size, int32_t* rstatus, void* scratch, uint64_t scratch_size,
                                            unsigned flags, void* stream) {
    if (nconn == 0) return HHUFF_OK;
    if (!conn_first || !scratch || (nres && (!res || !out || !out_off || !out_len || !headers_size || !rstatus)) ||
        (nhdr && (!hdr || !in)))
        return arg_fail("NULL array");
    if (in_size >= (1ull << 32)) return arg_fail("in_size must stay below 2^32 (u32 offsets)");
    if (scratch_size < hhuff_hpack_enc_scratch_size(nconn)) return arg_fail("scratch smaller than hhuff_hpack_enc_scratch_size");
    if (((uintptr_t)scratch & 15u) != 0) return arg_fail("scratch must be 16-byte aligned");
    if (((uintptr_t)res & 7u) != 0 || ((uintptr_t)hdr & 3u) != 0 || ((uintptr_t)out_off & 7u) != 0)
        return arg_fail("misaligned hdr / res / out_off");
    hipError_t e = hhuff::launch_hpack_flatten(in, in_size, hdr, nhdr, res, conn_first, nconn, nres, server_off, server_len,
                                               out, out_off, out_len, headers_size, rstatus, (uint8_t*)scratch, flags,
                                               (hipStream_t)stream);
    return e == hipSuccess ? HHUFF_OK : hip_fail(e, "hpack flatten launch");
}

HHUFF_API int hhuff_qpack_flatten_responses(const uint8_t* in, uint64_t in_size, const hhuff_hpack_header_t* hdr,
                                            uint32_t nhdr, const hhuff_qpack_response_t* res, uint32_t nres,
                                            uint32_t server_off, uint32_t server_len, uint8_t* out, const uint64_t* out_off,
                                            uint32_t* out_len, uint32_t* header_len, int32_t* rstatus, void* stream) {
    if (nres == 0) return HHUFF_OK;
    if (!res || !out || !out_off || !out_len || !header_len || !rstatus || (nhdr && !hdr) || !in) return arg_fail("NULL array");
    if (in_size >= (1ull << 32)) return arg_fail("in_size must stay below 2^32 (u32 offsets)");
    if (((uintptr_t)res & 7u) != 0 || ((uintptr_t)hdr & 3u) != 0 || ((uintptr_t)out_off & 7u) != 0)
        return arg_fail("misaligned hdr / res / out_off");
    hipError_t e = hhuff::launch_qpack_flatten(in, in_size, hdr, nhdr, res, nres, server_off, server_len, out, out_off, out_len,
                                               header_len, rstatus, (hipStream_t)stream);
    return e == hipSuccess ? HHUFF_OK : hip_fail(e, "qpack flatten launch");
}

HHUFF_API uint64_t hhuff_qpack_scratch_size(uint32_t nconn, uint32_t header_table_size) {
    return (uint64_t)nconn * hhuff::qpack_conn_scratch(header_table_size);
}

namespace {
int qpack_step(const uint8_t* in, uint64_t in_size, const uint32_t* enc_off, const uint32_t* enc_len,
               const uint32_t* sec_off, const uint32_t* conn_first, uint32_t nconn, uint32_t nsec,
               uint32_t header_table_size, uint64_t max_blocked, const uint32_t* num_blocked, uint8_t* arena,
               const uint64_t* arena_off, uint32_t* name_off, uint32_t* name_len, uint32_t* value_off,
               uint32_t* value_len, uint8_t* fflags, uint32_t* nfields, int32_t* sstatus, uint64_t* req_insert_count,
               int32_t* enc_status, uint32_t* enc_consumed, uint64_t* insert_count, const uint64_t* stream_id,
               hhuff_qpack_request_t* req, hhuff_qpack_response_head_t* res, void* scratch, uint64_t scratch_size,
               unsigned flags, void* stream) {
    if (nconn == 0) return HHUFF_OK;
    if (!in || !enc_off || !enc_len || !sec_off || !conn_first || !enc_status || !enc_consumed || !insert_count ||
        !scratch)
        return arg_fail("NULL array");
    if (nsec && (!arena || !arena_off || !name_off || !name_len || !value_off || !value_len || !fflags || !nfields ||
                 !sstatus || !req_insert_count))
        return arg_fail("NULL array");
    if (header_table_size > (1u << 30)) return arg_fail("header_table_size above 2^30");
    // u32 offsets, and the literal workspace is sized for in_size + 2 literals in 32 bits
    if (in_size > (1ull << 32) - 3) return arg_fail("in_size must be at most 2^32 - 3 (u32 offsets)");
    if (scratch_size < hhuff_qpack_scratch_size(nconn, header_table_size))
        return arg_fail("scratch smaller than hhuff_qpack_scratch_size");
    if (((uintptr_t)scratch & 15u) != 0) return arg_fail("scratch must be 16-byte aligned");
    hipError_t e = hhuff::launch_qpack(in, in_size, enc_off, enc_len, sec_off, conn_first, nconn, nsec,
                                       header_table_size, max_blocked, num_blocked, arena, arena_off, name_off, name_len,
                                       value_off, value_len, fflags, nfields, sstatus, req_insert_count, enc_status,
                                       enc_consumed, insert_count, (uint8_t*)scratch, flags, (hipStream_t)stream,
                                       stream_id, req, res);
    return e == hipSuccess ? HHUFF_OK : hip_fail(e, "qpack launch");
}
}  // namespace

HHUFF_API int hhuff_qpack_decode(const uint8_t* in, uint64_t in_size, const uint32_t* enc_off, const uint32_t* enc_len,
                                 const uint32_t* sec_off, const uint32_t* conn_first, uint32_t nconn, uint32_t nsec,
                                 uint32_t header_table_size, uint64_t max_blocked, const uint32_t* num_blocked,
                                 uint8_t* arena, const uint64_t* arena_off, uint32_t* name_off, uint32_t* name_len,
                                 uint32_t* value_off, uint32_t* value_len, uint8_t* fflags, uint32_t* nfields,
                                 int32_t* sstatus, uint64_t* req_insert_count, int32_t* enc_status,
                                 uint32_t* enc_consumed, uint64_t* insert_count, void* scratch, uint64_t scratch_size,
                                 unsigned flags, void* stream) {
    return qpack_step(in, in_size, enc_off, enc_len, sec_off, conn_first, nconn, nsec, header_table_size, max_blocked,
                      num_blocked, arena, arena_off, name_off, name_len, value_off, value_len, fflags, nfields, sstatus,
                      req_insert_count, enc_status, enc_consumed, insert_count, nullptr, nullptr, nullptr, scratch,
                      scratch_size, flags, stream);
}

HHUFF_API int hhuff_qpack_parse_requests(const uint8_t* in, uint64_t in_size, const uint32_t* enc_off,
                                         const uint32_t* enc_len, const uint32_t* sec_off, const uint32_t* conn_first,
                                         uint32_t nconn, uint32_t nsec, uint32_t header_table_size, uint64_t max_blocked,
                                         const uint32_t* num_blocked, uint8_t* arena, const uint64_t* arena_off,
                                         uint32_t* name_off, uint32_t* name_len, uint32_t* value_off, uint32_t* value_len,
                                         uint8_t* fflags, uint32_t* nfields, int32_t* sstatus, uint64_t* req_insert_count,
                                         int32_t* enc_status, uint32_t* enc_consumed, uint64_t* insert_count,
                                         const uint64_t* stream_id, hhuff_qpack_request_t* req, void* scratch,
                                         uint64_t scratch_size, unsigned flags, void* stream) {
    if (nconn != 0 && nsec != 0 && (!stream_id || !req)) return arg_fail("NULL array");
    if (((uintptr_t)req & 7u) != 0) return arg_fail("req must be 8-byte aligned");
    return qpack_step(in, in_size, enc_off, enc_len, sec_off, conn_first, nconn, nsec, header_table_size, max_blocked,
                      num_blocked, arena, arena_off, name_off, name_len, value_off, value_len, fflags, nfields, sstatus,
                      req_insert_count, enc_status, enc_consumed, insert_count, stream_id, req, nullptr, scratch,
                      scratch_size, flags, stream);
}

HHUFF_API int hhuff_qpack_parse_responses(const uint8_t* in, uint64_t in_size, const uint32_t* enc_off,
                                          const uint32_t* enc_len, const uint32_t* sec_off, const uint32_t* conn_first,
                                          uint32_t nconn, uint32_t nsec, uint32_t header_table_size, uint64_t max_blocked,
                                          const uint32_t* num_blocked, uint8_t* arena, const uint64_t* arena_off,
                                          uint32_t* name_off, uint32_t* name_len, uint32_t* value_off, uint32_t* value_len,
                                          uint8_t* fflags, uint32_t* nfields, int32_t* sstatus, uint64_t* req_insert_count,
                                          int32_t* enc_status, uint32_t* enc_consumed, uint64_t* insert_count,
                                          const uint64_t* stream_id, hhuff_qpack_response_head_t* res, void* scratch,
                                          uint64_t scratch_size, unsigned flags, void* stream) {
    if (nconn != 0 && nsec != 0 && (!stream_id || !res)) return arg_fail("NULL array");
    if (((uintptr_t)res & 7u) != 0) return arg_fail("res must be 8-byte aligned");
    return qpack_step(in, in_size, enc_off, enc_len, sec_off, conn_first, nconn, nsec, header_table_size, max_blocked,
                      num_blocked, arena, arena_off, name_off, name_len, value_off, value_len, fflags, nfields, sstatus,
                      req_insert_count, enc_status, enc_consumed, insert_count, stream_id, nullptr, res, scratch,
                      scratch_size, flags, stream);
}

// ---------------------------------------------------------------------------------------------------
// (1) h2o per-string symbols: one string per launch on the thread's stream, synchronously.
// Strings up to kOneMax bytes go through one_string_kernel on a pinned, device-visible buffer
// [u32 len, is_name, result, status][input][output] (no copies: one launch, one synchronisation); longer
// ones through the batch kernels with device copies.  A HIP failure (no GPU, a lost device) never aborts
// the caller: decode returns SIZE_MAX -- h2o's decode_string then reports H2O_HTTP2_ERROR_COMPRESSION for
// that literal (hpack.c:241-242) and the connection closes --, encode returns SIZE_MAX -- every caller then
// emits the string raw (hpack.c:836, qpack.c:1046-1051), which is a correct encoding; the reason is in
// hhuff_last_error_string().
// ---------------------------------------------------------------------------------------------------
namespace {
constexpr size_t kMeta = 32;
#ifndef HHUFF_LONG_ENC_DEFAULT
#define HHUFF_LONG_ENC_DEFAULT 1
#endif
uint64_t g_per_string_calls = 0;  // process-wide, atomic adds (hhuff_per_string_calls)

// ---- the resident per-string service (service_kernel, hhuff_kernels.hip), one grid per device ----
// A call posts its string in its thread's mailbox (slot = thread number mod kSvcSlots, a mutex per slot for
// more threads than slots), raises the slot's request counter and spins on the slot's done counter.  The
// grid has service_waves() waves (default 16), wave g serving mailboxes g, g + G, ..., so calls from up to G
// threads are coded at once.  It exits after kSvcIdle without a request to any wave; a call that finds its
// request unserved and the grid gone (ctrl->alive 0, the service stream idle) launches it again.  atexit stops every service before the HIP
// runtime goes away.  HHUFF_NO_SERVICE=1 in the environment keeps the launch-per-string path.
constexpr uint64_t kSvcIdle = 200000;      // real-time counter ticks (100 MHz): 2 ms without a request
constexpr uint64_t kSvcLife = 1000000000;  // 10 s in all, then a fresh launch
struct Service {
    std::mutex mu;
    bool ready = false, broken = false;
    hipStream_t stream = nullptr;
    hhuff::SvcSlot* slots = nullptr;  // host view (pinned, mapped, coherent)
    hhuff::SvcSlot* d_slots = nullptr;
    hhuff::SvcCtrl* ctrl = nullptr;
    hhuff::SvcCtrl* d_ctrl = nullptr;
    uint32_t seq[hhuff::kSvcSlots] = {};
    std::mutex slot_mu[hhuff::kSvcSlots];
};
Service g_svc[64];
std::atomic<uint32_t> g_svc_threads{0};
thread_local int t_svc_slot = -1;

void svc_shutdown() {
    for (auto& S : g_svc) {
        std::lock_guard<std::mutex> g(S.mu);
        if (!S.ready) continue;
        __atomic_store_n(&S.ctrl->stop, 1u, __ATOMIC_RELEASE);
        (void)hipStreamSynchronize(S.stream);  // the wave polls stop: it exits within a poll
        S.ready = false;
    }
}

bool svc_enabled() {
    static const bool on = [] {
        const char* e = getenv("HHUFF_NO_SERVICE");
        return !(e && *e && *e != '0');
    }();
    return on;
}

// make sure device dev's service is set up and running (stream idle -> launch); caller holds nothing
int svc_kick(Service& S, int dev) {
    std::lock_guard<std::mutex> g(S.mu);
    if (S.broken) return HHUFF_EHIP;
    if (!S.ready) {
        int cur = 0;
        HIP_TRY(hipGetDevice(&cur), "hipGetDevice");
        if (cur != dev) HIP_TRY(hipSetDevice(dev), "hipSetDevice");
        hipError_t e = hipStreamCreateWithFlags(&S.stream, hipStreamNonBlocking);
        void* h = nullptr;
        const size_t bytes = sizeof(hhuff::SvcSlot) * hhuff::kSvcSlots + sizeof(hhuff::SvcCtrl);
        if (e == hipSuccess) e = hipHostMalloc(&h, bytes, hipHostMallocMapped | hipHostMallocCoherent);
        void* d = nullptr;
        if (e == hipSuccess) {
            memset(h, 0, bytes);
            e = hipHostGetDevicePointer(&d, h, 0);
        }
        if (cur != dev) (void)hipSetDevice(cur);
        if (e != hipSuccess) {
            S.broken = true;
            return hip_fail(e, "per-string service setup");
        }
        S.slots = static_cast<hhuff::SvcSlot*>(h);
        S.d_slots = static_cast<hhuff::SvcSlot*>(d);
        S.ctrl = reinterpret_cast<hhuff::SvcCtrl*>(S.slots + hhuff::kSvcSlots);
        S.d_ctrl = reinterpret_cast<hhuff::SvcCtrl*>(S.d_slots + hhuff::kSvcSlots);
        static std::once_flag once;
        std::call_once(once, [] { atexit(svc_shutdown); });
        S.ready = true;
    }
    const hipError_t q = hipStreamQuery(S.stream);
    if (q == hipErrorNotReady) return HHUFF_OK;  // running (or starting)
    if (q != hipSuccess) return hip_fail(q, "per-string service query");
    // a fresh grid: no quit, no wave gone yet, alive from the launch on (the stream tells a finished grid)
    for (uint32_t g = 0; g < hhuff::kSvcMaxWaves; ++g) S.ctrl->gone[g] = 0u;
    S.ctrl->quit = 0u;
    S.ctrl->waves = hhuff::service_waves();
    __atomic_store_n(&S.ctrl->stop, 0u, __ATOMIC_RELEASE);
    __atomic_store_n(&S.ctrl->alive, 1u, __ATOMIC_RELEASE);
    const hipError_t e = hhuff::launch_service(S.d_slots, S.d_ctrl, kSvcIdle, kSvcLife, S.stream);
    return e == hipSuccess ? HHUFF_OK : hip_fail(e, "per-string service launch");
}

// 1: served (result in *res), 0: not taken (the caller uses the launch path), -1: HIP failure
int svc_call(int dev, bool encode, const uint8_t* src, size_t len, int is_name, uint8_t* dst, uint32_t* res,
             uint32_t* status) {
    if (dev < 0 || dev >= 64 || len > hhuff::kSvcMax || !svc_enabled()) return 0;
    Service& S = g_svc[dev];
    if (S.broken) return 0;
    if (!S.ready && svc_kick(S, dev) != HHUFF_OK) return S.broken ? 0 : -1;
    if (t_svc_slot < 0) t_svc_slot = (int)(g_svc_threads.fetch_add(1) % hhuff::kSvcSlots);
    const int k = t_svc_slot;
    std::lock_guard<std::mutex> g(S.slot_mu[k]);
    hhuff::SvcSlot* sl = S.slots + k;
    const uint32_t n = ++S.seq[k];
    // chunks first, each one 16-B store {n, 12 bytes}; then the header, one 16-B store (see SvcSlot)
    for (size_t i = 0; 12 * i < len; ++i) {
        uint32_t w[4] = {n, 0u, 0u, 0u};
        memcpy(&w[1], src + 12 * i, len - 12 * i < 12 ? len - 12 * i : 12);
        _mm_store_si128(reinterpret_cast<__m128i*>(sl->chunk[i]), _mm_loadu_si128(reinterpret_cast<const __m128i*>(w)));
    }
    __atomic_thread_fence(__ATOMIC_RELEASE);
    const uint32_t h[4] = {n, encode ? 1u : 0u, (uint32_t)len, is_name ? 1u : 0u};
    _mm_store_si128(reinterpret_cast<__m128i*>(&sl->req), _mm_loadu_si128(reinterpret_cast<const __m128i*>(h)));
    // spin for the result.  While the wave is alive nothing else is done; a wave that is gone (idle exit,
    // or exiting just as this request arrived) is launched again -- checked every 64 spins, so a wave that
    // is still starting up is not launched twice (svc_kick sees its stream busy)
    // a grid that is gone is launched again; once the service is broken (another thread's 5-s timeout, a
    // failed setup) this call is not a Huffman error but a request for the launch path
    auto revive = [&]() -> int {
        if (__atomic_load_n(&S.ctrl->alive, __ATOMIC_ACQUIRE) != 0u) return 1;
        if (svc_kick(S, dev) == HHUFF_OK) return 1;
        return S.broken ? 0 : -1;
    };
    if (const int rv = revive(); rv <= 0) return rv;
    uint64_t spins = 0;
    const auto t0 = std::chrono::steady_clock::now();
    // {done, result, status} arrive as one 16-B store: one 16-B load sees them together
    auto load16 = [](const void* q, uint32_t (&w)[4]) {
        __asm__ volatile("" ::: "memory");  // re-read the device-written line on every try
        _mm_storeu_si128(reinterpret_cast<__m128i*>(w), _mm_load_si128(reinterpret_cast<const __m128i*>(q)));
    };
    uint32_t res4[4];
    for (load16(&sl->done, res4); res4[0] != n; load16(&sl->done, res4)) {
        ++spins;
        if ((spins & 63u) == 0u) {
            if (const int rv = revive(); rv <= 0) return rv;
            if ((spins & 4095u) == 0u && std::chrono::steady_clock::now() - t0 > std::chrono::seconds(5)) {
                // a busy device (a long batch kernel ahead of the wave) is not a HIP failure: this call and
                // the later ones take the launch path, so a valid string is still coded
                snprintf(t_err, sizeof(t_err), "per-string service: no answer in 5 s (launch path from now on)");
                std::lock_guard<std::mutex> gg(S.mu);
                S.broken = true;
                return 0;
            }
        }
        __builtin_ia32_pause();
    }
    const uint32_t r = res4[1];
    *res = r;
    *status = res4[2];
    if (r != HHUFF_FAIL_LEN) {
        for (uint32_t i = 0; 12u * i < r; ++i) {  // each chunk once it carries this request's number
            uint32_t c4[4];
            for (uint64_t k = 0;; ++k) {  // stored with the result: here within microseconds
                load16(sl->outc[i], c4);
                if (c4[0] == n) break;
                if ((k & 4095u) == 4095u && std::chrono::steady_clock::now() - t0 > std::chrono::seconds(5)) {
                    snprintf(t_err, sizeof(t_err), "per-string service: output chunk %u never arrived", i);
                    return -1;
                }
                __builtin_ia32_pause();
            }
            memcpy(dst + 12u * i, &c4[1], r - 12u * i < 12u ? r - 12u * i : 12u);
        }
    }
    return 1;
}

// The one-string kernel stores its result length last (system scope, after every output word): spin on it
// instead of waiting for the launch's completion signal, for up to 2 ms, then synchronise the stream as before
// (which also reports a failed launch).  HHUFF_ONE_SYNC=1: always synchronise.
// A result taken early is complete (every output word precedes the length's release store), but an error the
// kernel raises after that store -- nothing in it runs after the store but the exit -- would surface at the
// next synchronisation of this thread's stream, i.e. be reported against the thread's next call.
constexpr uint32_t kOnePending = 0xFFFFFFFEu;  // never a result: lengths stay below 2^16, failures are ~0u
static hipError_t wait_one(Ctx& c, const uint32_t* meta) {
    static const bool sync_only = [] {
        const char* v = getenv("HHUFF_ONE_SYNC");
        return v && v[0] == '1';
    }();
    if (!sync_only) {
        const auto t0 = std::chrono::steady_clock::now();
        for (uint64_t k = 0;; ++k) {
            if (__atomic_load_n(&meta[2], __ATOMIC_ACQUIRE) != kOnePending) return hipSuccess;
            if ((k & 1023u) == 1023u && std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(2)) break;
            __builtin_ia32_pause();
        }
    }
    return hipStreamSynchronize(c.stream);
}

// Per-string encode past kOneMax: one block over the string (encode_long_kernel) with HHUFF_LONG_ENC=1 (or a
// build default of 1), else the batch kernels on a batch of one (one lane: ~8 ms for 64 KB)
static bool long_encode_block() {
    static const bool on = [] {
        const char* v = getenv("HHUFF_LONG_ENC");
        return v ? v[0] != '0' : HHUFF_LONG_ENC_DEFAULT != 0;
    }();
    return on;
}

size_t per_string(bool encode, uint8_t* dst, const uint8_t* src, size_t len, int is_name, unsigned* soft_errors) {
    __atomic_fetch_add(&g_per_string_calls, 1, __ATOMIC_RELAXED);
    Ctx& c = t_ctx;
    if (len > 0x1FFFFFFFu) {
        snprintf(t_err, sizeof(t_err), "string of %zu bytes exceeds the per-string limit", len);
        return SIZE_MAX;
    }
    if (c.bind(-1)) return SIZE_MAX;
    {
        uint32_t r = 0, st = 0;
        const int sv = svc_call(c.dev, encode, src, len, is_name, dst, &r, &st);
        if (sv < 0) return SIZE_MAX;
        if (sv > 0) {
            if (r == HHUFF_FAIL_LEN) return SIZE_MAX;
            if (!encode) *soft_errors |= st & 3u;
            return r;
        }
    }
    const size_t in_cap = up16(len ? len : 1);
    if (len <= hhuff::kOneMax) {
        const size_t out_cap = up16(len * 8 / 5 + 4);
        if (c.reserve(0, 16 + in_cap + out_cap)) return SIZE_MAX;
        uint32_t* meta = reinterpret_cast<uint32_t*>(c.h);
        meta[0] = (uint32_t)len;
        meta[1] = is_name ? 1u : 0u;
        __atomic_store_n(&meta[2], kOnePending, __ATOMIC_RELAXED);
        memcpy(c.h + 16, src, len);
        hipError_t e = hhuff::launch_one(c.h, (uint32_t)len, (uint32_t)in_cap, is_name != 0, encode, c.stream);
        if (e == hipSuccess) e = wait_one(c, meta);
        if (e != hipSuccess) return hip_fail(e, encode ? "encode (one string)" : "decode (one string)"), SIZE_MAX;
        const uint32_t r = __atomic_load_n(&meta[2], __ATOMIC_ACQUIRE);
        if (r == HHUFF_FAIL_LEN) return SIZE_MAX;
        memcpy(dst, c.h + 16 + in_cap, r);
        if (!encode) *soft_errors |= meta[3] & 3u;
        return r;
    }
    // long strings: the batch kernels on a batch of one, device copies
    const size_t out_cap = up16(len * 8 / 5 + 4);
    if (c.reserve(kMeta + in_cap + out_cap, kMeta + in_cap + out_cap)) return SIZE_MAX;
    uint32_t* meta = reinterpret_cast<uint32_t*>(c.h);
    meta[0] = 0;
    meta[1] = (uint32_t)len;
    meta[2] = 0;
    meta[3] = is_name ? 1u : 0u;
    memcpy(c.h + kMeta, src, len);
    uint32_t* d_meta = reinterpret_cast<uint32_t*>(c.d);
    uint8_t* d_in = c.d + kMeta;
    uint8_t* d_out = c.d + kMeta + in_cap;
    uint8_t* h_out = c.h + kMeta + in_cap;
    hipError_t e = hipMemcpyAsync(c.d, c.h, kMeta + len, hipMemcpyHostToDevice, c.stream);
    if (e == hipSuccess)
        e = encode ? (long_encode_block()
                          ? hhuff::launch_encode_long(d_in, (uint32_t)len, d_out, d_meta + 2, c.stream)
                          : hhuff::launch_encode(d_in, len, d_meta, nullptr, 1, d_out, nullptr, d_meta + 2, nullptr,
                                                 c.stream))
                   : hhuff::launch_decode(d_in, len, d_meta, nullptr, 1, d_meta + 3, d_out, nullptr, d_meta + 2,
                                          reinterpret_cast<uint8_t*>(d_meta + 4), c.stream);
    if (e == hipSuccess) e = hipMemcpyAsync(c.h, c.d, kMeta, hipMemcpyDeviceToHost, c.stream);
    if (e == hipSuccess) e = hipMemcpyAsync(h_out, d_out, out_cap, hipMemcpyDeviceToHost, c.stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c.stream);
    if (e != hipSuccess) return hip_fail(e, encode ? "encode (long string)" : "decode (long string)"), SIZE_MAX;
    const uint32_t r = meta[2];
    if (r == HHUFF_FAIL_LEN) return SIZE_MAX;
    memcpy(dst, h_out, r);
    if (!encode) *soft_errors |= *reinterpret_cast<const uint8_t*>(meta + 4);
    return r;
}
}  // namespace

HHUFF_API size_t h2o_hpack_decode_huffman(char* dst, unsigned* soft_errors, const uint8_t* src, size_t len, int is_name,
                                          const char** err_desc) {
    (void)err_desc;  // never written, as in the reference (hpack.c:142-144 is unreachable)
    return per_string(false, reinterpret_cast<uint8_t*>(dst), src, len, is_name, soft_errors);
}

HHUFF_API size_t h2o_hpack_encode_huffman(uint8_t* dst, const uint8_t* src, size_t len) {
    return per_string(true, dst, src, len, 0, nullptr);
}

HHUFF_API uint64_t hhuff_per_string_calls(void) { return __atomic_load_n(&g_per_string_calls, __ATOMIC_RELAXED); }

HHUFF_API int hhuff_service_stamps(uint32_t* out4) {
    int dev = 0;
    if (!out4 || hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return HHUFF_EINVAL;
    const Service& S = g_svc[dev];
    if (!S.ready || t_svc_slot < 0) return HHUFF_EINVAL;
    const hhuff::SvcSlot* sl = S.slots + t_svc_slot;
    out4[0] = sl->t_seen, out4[1] = sl->t_data, out4[2] = sl->t_coded, out4[3] = sl->t_out;
    return HHUFF_OK;
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

constexpr uint64_t kDefaultChunk = 64ull << 20;  // pipelined host path: input bytes per chunk
int pipelined(bool decode, const uint8_t* in, uint64_t in_size, const uint32_t* in_off, uint32_t n,
              const uint32_t* is_name_bits, uint8_t* out, uint64_t out_size, uint32_t* out_len, uint8_t* status,
              int device, uint64_t chunk_bytes);

int host_batch(bool decode, const uint8_t* in, uint64_t in_size, const uint32_t* in_off, const uint32_t* in_len,
               uint32_t n, const uint32_t* is_name_bits, uint8_t* out, uint64_t out_size, const uint32_t* out_off,
               uint32_t* out_len, uint8_t* status, int device) {
    if (n == 0) return HHUFF_OK;
    if (!in || !in_off || !out || !out_len || (decode && !status)) return arg_fail("NULL array");
    if (!in_len && !out_off && in_size >= 2 * kDefaultChunk && in_off[n] <= in_size)  // large contiguous batch
        return pipelined(decode, in, in_size, in_off, n, is_name_bits, out, out_size, out_len, status, device, 0);
    DeviceGuard guard(device);
    if (guard.err != hipSuccess) return hip_fail(guard.err, "hipSetDevice");
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

// ---------------------------------------------------------------------------------------------------
// (3b) pipelined host path: pageable -> pinned -> device -> pinned -> pageable, chunk by chunk
//
// The batch (contiguous layout, implicit output slots) is cut at multiples of 32 strings into chunks
// of about `chunk_bytes` input bytes.  Chunk k runs on stream k % depth: H2D of its input bytes,
// offsets and is-name words, the kernel, D2H of its output slots, lengths and statuses.  While the GPU
// works on chunks k-1 and k-2 the calling thread (plus helper threads) copies chunk k's input into its
// pinned slot and chunk k-depth's results out of theirs, so host copies, both DMA directions and the
// kernels overlap.  Caller buffers that are already pinned are used by the DMA engines directly.
// The kernel sees absolute offsets: `in` and `out` are passed shifted back by the chunk base (a
// multiple of 80 bytes, so the decode slot floor(8 base / 5) stays 16-byte aligned).
// ---------------------------------------------------------------------------------------------------
constexpr int kDepth = 3;

bool is_pinned(const void* p) {
    if (!p) return true;
    hipPointerAttribute_t a;
    if (hipPointerGetAttributes(&a, p) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    return a.type == hipMemoryTypeHost;
}

// memcpy split over a few threads for large copies (the host staging copies bound the host path)
void par_copy(void* dst, const void* src, size_t n) {
    const size_t kMin = 4u << 20;
    unsigned t = std::thread::hardware_concurrency();
    t = t == 0 ? 1 : (t > 8 ? 8 : t);
    if (n < kMin || t == 1) {
        memcpy(dst, src, n);
        return;
    }
    const size_t per = ((n / t) + 4095) & ~(size_t)4095;
    std::vector<std::thread> th;
    for (unsigned k = 1; k < t && k * per < n; ++k)
        th.emplace_back([=] { memcpy((uint8_t*)dst + k * per, (const uint8_t*)src + k * per, std::min(per, n - k * per)); });
    memcpy(dst, src, std::min(per, n));
    for (auto& x : th) x.join();
}

struct Slot {
    hipStream_t s = nullptr;
    uint8_t *d = nullptr, *h = nullptr;
    size_t dcap = 0, hcap = 0;
    bool busy = false;
    // chunk bookkeeping for the host-side unstaging
    uint64_t i0 = 0, m = 0, out_lo = 0, out_n = 0;
    size_t h_out = 0, h_len = 0, h_st = 0;
};

struct Pipe {
    int dev = -1;
    Slot slot[kDepth];
    ~Pipe() {
        for (auto& x : slot) {
            if (x.d) (void)hipFree(x.d);
            if (x.h) (void)hipHostFree(x.h);
            if (x.s) (void)hipStreamDestroy(x.s);
        }
    }
    int bind(int device) {
        if (dev == device) return HHUFF_OK;
        for (auto& x : slot) {
            if (x.d) (void)hipFree(x.d), x.d = nullptr, x.dcap = 0;
            if (x.s) (void)hipStreamDestroy(x.s), x.s = nullptr;
            HIP_TRY(hipStreamCreateWithFlags(&x.s, hipStreamNonBlocking), "hipStreamCreate");
        }
        dev = device;
        return HHUFF_OK;
    }
};
thread_local Pipe t_pipe;

int grow(Slot& x, size_t dneed, size_t hneed) {
    if (dneed > x.dcap) {
        if (x.d) (void)hipFree(x.d), x.d = nullptr, x.dcap = 0;
        HIP_TRY(hipMalloc(&x.d, dneed + dneed / 8), "hipMalloc");
        x.dcap = dneed + dneed / 8;
    }
    if (hneed > x.hcap) {
        if (x.h) (void)hipHostFree(x.h), x.h = nullptr, x.hcap = 0;
        HIP_TRY(hipHostMalloc(&x.h, hneed + hneed / 8, hipHostMallocDefault), "hipHostMalloc");
        x.hcap = hneed + hneed / 8;
    }
    return HHUFF_OK;
}

int pipelined(bool decode, const uint8_t* in, uint64_t in_size, const uint32_t* in_off, uint32_t n,
              const uint32_t* is_name_bits, uint8_t* out, uint64_t out_size, uint32_t* out_len, uint8_t* status,
              int device, uint64_t chunk_bytes) {
    if (chunk_bytes == 0) chunk_bytes = kDefaultChunk;
    DeviceGuard guard(device);
    if (guard.err != hipSuccess) return hip_fail(guard.err, "hipSetDevice");
    Ctx& c = t_ctx;
    int rc = c.bind(device);
    if (rc) return rc;
    Pipe& P = t_pipe;
    rc = P.bind(c.dev);
    if (rc) return rc;
    const bool pin_in = is_pinned(in), pin_out = is_pinned(out);
    const bool pin_meta = is_pinned(in_off) && is_pinned(out_len) && (!status || is_pinned(status)) &&
                          (!is_name_bits || is_pinned(is_name_bits));  // offsets/lengths DMA'd in place
    auto slot_of = [&](uint64_t pos) { return decode ? (pos * 8) / 5 : pos; };  // implicit output slot
    // Zero copy: with every caller array pinned (so device-visible) the kernels read the input and write the
    // output across PCIe themselves, one launch, no DMA staging -- both link directions in use at once (the
    // chunked DMA pipeline below moved ~55 GB/s in all).  HHUFF_HOST_COPY=1 keeps the pipeline.
    const char* hc = getenv("HHUFF_HOST_COPY");
    if (pin_in && pin_out && pin_meta && !(hc && *hc && *hc != '0') && out_size >= slot_of(in_off[n])) {
        auto dev_ptr = [](const void* p) -> void* {
            if (!p) return nullptr;
            hipPointerAttribute_t a;
            if (hipPointerGetAttributes(&a, p) != hipSuccess) {
                (void)hipGetLastError();
                return nullptr;
            }
            return a.devicePointer;
        };
        const uint8_t* d_in = static_cast<const uint8_t*>(dev_ptr(in));
        const uint32_t* d_off = static_cast<const uint32_t*>(dev_ptr(in_off));
        const uint32_t* d_nm = static_cast<const uint32_t*>(dev_ptr(is_name_bits));
        uint8_t* d_out = static_cast<uint8_t*>(dev_ptr(out));
        uint32_t* d_len = static_cast<uint32_t*>(dev_ptr(out_len));
        uint8_t* d_st = static_cast<uint8_t*>(dev_ptr(status));
        // the kernels' 16-B staging loads / stores and dword offset loads need the device API's alignment
        // (hhuff.h: in / out 16-B aligned, arrays 4-B aligned): an offset view of a registered socket buffer
        // or a numpy slice takes the chunked pipeline instead, whose staged buffers are aligned
        auto al = [](const void* p, uintptr_t a) { return ((uintptr_t)p & (a - 1)) == 0; };
        const bool aligned = al(d_in, 16) && al(d_out, 16) && al(d_off, 4) && al(d_len, 4) && al(d_nm, 4);
        if (aligned && d_in && d_off && d_out && d_len && (!status || d_st) && (!is_name_bits || d_nm)) {
            // (the kernel variant follows the batch's own bytes: a shard of a larger buffer passes in_off + lo)
            const uint64_t sel = (uint64_t)in_off[n] - in_off[0];
            hipError_t e = decode ? hhuff::launch_decode(d_in, in_size, d_off, nullptr, n, d_nm, d_out, nullptr, d_len, d_st,
                                                         c.stream, sel)
                                  : hhuff::launch_encode(d_in, in_size, d_off, nullptr, n, d_out, nullptr, d_len, d_st, c.stream,
                                                         sel);
            if (e != hipSuccess) return hip_fail(e, decode ? "decode launch (zero copy)" : "encode launch (zero copy)");
            HIP_TRY(hipStreamSynchronize(c.stream), "sync");
            return HHUFF_OK;
        }
    }
    // chunk boundaries: multiples of 32 strings, about chunk_bytes of input each
    std::vector<uint64_t> cut{0};
    while (cut.back() < n) {
        const uint64_t a = cut.back();
        const uint64_t target = (uint64_t)in_off[a] + chunk_bytes;
        uint64_t b = (uint64_t)(std::upper_bound(in_off + a, in_off + n + 1, (uint32_t)std::min<uint64_t>(target, 0xFFFFFFFFull)) -
                                in_off);  // first string starting past the target
        b = b > a + 32 ? ((b - a) / 32) * 32 + a : a + 32;
        cut.push_back(std::min<uint64_t>(b, n));
    }
    auto drain = [&](Slot& x) -> int {
        if (!x.busy) return HHUFF_OK;
        HIP_TRY(hipStreamSynchronize(x.s), "sync");
        if (!pin_out && x.out_n) par_copy(out + x.out_lo, x.h + x.h_out, x.out_n);
        if (!pin_meta) {
            par_copy(out_len + x.i0, x.h + x.h_len, x.m * 4);
            if (status) par_copy(status + x.i0, x.h + x.h_st, x.m);
        }
        x.busy = false;
        return HHUFF_OK;
    };
    for (size_t k = 0; k + 1 < cut.size(); ++k) {
        Slot& x = P.slot[k % kDepth];
        rc = drain(x);
        if (rc) return rc;
        const uint64_t i0 = cut[k], i1 = cut[k + 1], m = i1 - i0;
        const uint64_t s0 = in_off[i0], e0 = in_off[i1];
        const uint64_t base = (s0 / 80) * 80;
        const uint64_t nbytes = e0 - base;
        const uint64_t olo = slot_of(s0), ohi = std::min<uint64_t>(slot_of(e0), out_size);
        const uint64_t obase = slot_of(base);
        const uint64_t ocap = slot_of(e0) - obase + 16;
        const size_t nw = decode && is_name_bits ? (size_t)(m + 31) / 32 : 0;
        // device slot layout: [in bytes][in_off m+1][names][out][out_len m][status m]
        const size_t o_in = 0, o_off = up16(nbytes + 16), o_nm = o_off + up16((m + 1) * 4), o_out = o_nm + up16(nw * 4),
                     o_len = o_out + up16(ocap), o_st = o_len + up16(m * 4), dneed = o_st + up16(m);
        // pinned slot layout: [in bytes][in_off][names] | [out][out_len][status]
        const size_t hneed = dneed;
        rc = grow(x, dneed, hneed);
        if (rc) return rc;
        if (pin_in) {
            HIP_TRY(hipMemcpyAsync(x.d + o_in, in + base, nbytes, hipMemcpyHostToDevice, x.s), "H2D in");
        } else {
            par_copy(x.h + o_in, in + base, nbytes);
            HIP_TRY(hipMemcpyAsync(x.d + o_in, x.h + o_in, nbytes, hipMemcpyHostToDevice, x.s), "H2D in");
        }
        if (pin_meta) {
            HIP_TRY(hipMemcpyAsync(x.d + o_off, in_off + i0, (m + 1) * 4, hipMemcpyHostToDevice, x.s), "H2D offsets");
            if (nw)
                HIP_TRY(hipMemcpyAsync(x.d + o_nm, is_name_bits + i0 / 32, nw * 4, hipMemcpyHostToDevice, x.s),
                        "H2D names");
        } else {
            par_copy(x.h + o_off, in_off + i0, (m + 1) * 4);
            if (nw) memcpy(x.h + o_nm, is_name_bits + i0 / 32, nw * 4);
            HIP_TRY(hipMemcpyAsync(x.d + o_off, x.h + o_off, (o_nm - o_off) + nw * 4, hipMemcpyHostToDevice, x.s),
                    "H2D offsets");
        }
        const uint8_t* d_in = x.d + o_in - base;  // absolute offsets address the chunk
        uint8_t* d_out = x.d + o_out - obase;
        const uint32_t* d_off = reinterpret_cast<const uint32_t*>(x.d + o_off);
        uint32_t* d_len = reinterpret_cast<uint32_t*>(x.d + o_len);
        uint8_t* d_st = x.d + o_st;
        hipError_t e = decode ? hhuff::launch_decode(d_in, e0, d_off, nullptr, (uint32_t)m,
                                                     nw ? reinterpret_cast<const uint32_t*>(x.d + o_nm) : nullptr, d_out,
                                                     nullptr, d_len, d_st, x.s, nbytes)
                              : hhuff::launch_encode(d_in, e0, d_off, nullptr, (uint32_t)m, d_out, nullptr, d_len,
                                                     status ? d_st : nullptr, x.s, nbytes);
        if (e != hipSuccess) return hip_fail(e, decode ? "decode launch" : "encode launch");
        x.i0 = i0;
        x.m = m;
        x.out_lo = olo;
        x.out_n = ohi > olo ? ohi - olo : 0;
        x.h_out = o_out;
        x.h_len = o_len;
        x.h_st = o_st;
        if (x.out_n) {
            if (pin_out)
                HIP_TRY(hipMemcpyAsync(out + olo, d_out + olo, x.out_n, hipMemcpyDeviceToHost, x.s), "D2H out");
            else
                HIP_TRY(hipMemcpyAsync(x.h + o_out, d_out + olo, x.out_n, hipMemcpyDeviceToHost, x.s), "D2H out");
        }
        if (pin_meta) {
            HIP_TRY(hipMemcpyAsync(out_len + i0, x.d + o_len, m * 4, hipMemcpyDeviceToHost, x.s), "D2H len");
            if (status) HIP_TRY(hipMemcpyAsync(status + i0, x.d + o_st, m, hipMemcpyDeviceToHost, x.s), "D2H status");
        } else {
            HIP_TRY(hipMemcpyAsync(x.h + o_len, x.d + o_len, o_st + m - o_len, hipMemcpyDeviceToHost, x.s), "D2H len");
        }
        x.busy = true;
    }
    for (auto& x : P.slot) {
        rc = drain(x);
        if (rc) return rc;
    }
    return HHUFF_OK;
}

// (3c) packed host path: the packed kernels (hhuff_*_batch_packed) on host buffers.  With every caller array pinned
// and aligned the kernels read the strings and write only the outputs' bytes, out_off, out_len and status across
// PCIe (zero copy; the slot layout's tails, ~45 % of a decode slot and ~25 % of an encode slot on header text,
// never cross the link); otherwise one staged round trip through device memory.  out_off may be NULL (the caller
// places string i at its tile's position plus the kept lengths before it in the tile) and so may an encode's
// status (out_len says HHUFF_FAIL_LEN): 4 and 1 bytes a string fewer across the link.
int host_packed(bool decode, const uint8_t* in, uint64_t in_size, const uint32_t* in_off, uint32_t n,
                const uint32_t* is_name_bits, uint8_t* out, uint64_t out_size, uint32_t* out_off, uint32_t* out_len,
                uint8_t* status, int device) {
    if (n == 0) return HHUFF_OK;
    if (!in || !in_off || !out || !out_len || (decode && !status)) return arg_fail("NULL array");
    if (in_off[n] > in_size) return arg_fail("in_off[n] > in_size");
    const uint64_t slot_end = decode ? ((uint64_t)in_off[n] * 8) / 5 : in_off[n];
    if (out_size < slot_end) return arg_fail("out_size below the output slots of the batch");
    if ((decode ? (in_size * 8) / 5 : in_size) >= 0xFFFFFFFFull) return arg_fail("in_size too large for u32 packed offsets");
    DeviceGuard guard(device);
    if (guard.err != hipSuccess) return hip_fail(guard.err, "hipSetDevice");
    Ctx& c = t_ctx;
    int rc = c.bind(device);
    if (rc) return rc;
    auto dev_ptr = [](const void* p) -> void* {
        if (!p) return nullptr;
        hipPointerAttribute_t a;
        if (hipPointerGetAttributes(&a, p) != hipSuccess) {
            (void)hipGetLastError();
            return nullptr;
        }
        return a.type == hipMemoryTypeHost ? a.devicePointer : nullptr;
    };
    auto al = [](const void* p, uintptr_t a) { return ((uintptr_t)p & (a - 1)) == 0; };
    const uint8_t* z_in = static_cast<const uint8_t*>(dev_ptr(in));
    const uint32_t* z_off = static_cast<const uint32_t*>(dev_ptr(in_off));
    const uint32_t* z_nm = static_cast<const uint32_t*>(dev_ptr(is_name_bits));
    uint8_t* z_out = static_cast<uint8_t*>(dev_ptr(out));
    uint32_t* z_ooff = static_cast<uint32_t*>(dev_ptr(out_off));
    uint32_t* z_len = static_cast<uint32_t*>(dev_ptr(out_len));
    uint8_t* z_st = static_cast<uint8_t*>(dev_ptr(status));
    const bool zero = z_in && z_off && (!is_name_bits || z_nm) && z_out && (!out_off || z_ooff) && z_len &&
                      (!status || z_st) && al(z_in, 16) && al(z_out, 16) && al(z_off, 4) && al(z_nm, 4) &&
                      al(z_ooff, 4) && al(z_len, 4);
    hipStream_t s = c.stream;
    if (zero) {
        if (!out_off) {  // not returned: the kernels' offsets stay in device scratch and never cross the link
            rc = c.reserve(up16(((size_t)n + 1) * 4), 0);
            if (rc) return rc;
            z_ooff = reinterpret_cast<uint32_t*>(c.d);
        }
        hipError_t e = decode ? hhuff::launch_decode_packed(z_in, in_size, z_off, n, z_nm, z_out, z_ooff, z_len, z_st, s)
                              : hhuff::launch_encode_packed(z_in, in_size, z_off, n, z_out, z_ooff, z_len, z_st, s);
        if (e != hipSuccess) return hip_fail(e, decode ? "packed decode launch (zero copy)" : "packed encode launch (zero copy)");
        HIP_TRY(hipStreamSynchronize(s), "sync");
        return HHUFF_OK;
    }
    const size_t nw = ((size_t)n + 31) / 32;
    const size_t need = up16(in_size ? in_size : 1) + up16(((size_t)n + 1) * 4) + (is_name_bits ? up16(nw * 4) : 0) +
                        up16(slot_end + 16) + up16(((size_t)n + 1) * 4) + up16((size_t)n * 4) + up16(n);
    rc = c.reserve(need, 0);
    if (rc) return rc;
    Carve cv{c.d};
    uint8_t* d_in = cv.take<uint8_t>(in_size ? in_size : 1);
    uint32_t* d_off = cv.take<uint32_t>((size_t)n + 1);
    uint32_t* d_nm = is_name_bits ? cv.take<uint32_t>(nw) : nullptr;
    uint8_t* d_out = cv.take<uint8_t>(slot_end + 16);
    uint32_t* d_ooff = cv.take<uint32_t>((size_t)n + 1);
    uint32_t* d_len = cv.take<uint32_t>(n);
    uint8_t* d_st = cv.take<uint8_t>(n);
    HIP_TRY(hipMemcpyAsync(d_in, in, in_size, hipMemcpyHostToDevice, s), "H2D in");
    HIP_TRY(hipMemcpyAsync(d_off, in_off, ((size_t)n + 1) * 4, hipMemcpyHostToDevice, s), "H2D in_off");
    if (is_name_bits) HIP_TRY(hipMemcpyAsync(d_nm, is_name_bits, nw * 4, hipMemcpyHostToDevice, s), "H2D is_name");
    hipError_t e = decode ? hhuff::launch_decode_packed(d_in, in_size, d_off, n, d_nm, d_out, d_ooff, d_len, d_st, s)
                          : hhuff::launch_encode_packed(d_in, in_size, d_off, n, d_out, d_ooff, d_len, status ? d_st : nullptr, s);
    if (e != hipSuccess) return hip_fail(e, decode ? "packed decode launch" : "packed encode launch");
    // the metadata first: the tiles' runs follow from out_off / out_len, and only the runs go back to the caller
    // (the gaps between them were never written by the kernels; the caller's bytes there stay untouched, as on
    // the zero-copy path: hhuff.h's packed contract)
    std::vector<uint32_t> tmp_off(out_off ? 0 : (size_t)n + 1);
    uint32_t* h_ooff = out_off ? out_off : tmp_off.data();
    HIP_TRY(hipMemcpyAsync(h_ooff, d_ooff, ((size_t)n + 1) * 4, hipMemcpyDeviceToHost, s), "D2H out_off");
    HIP_TRY(hipMemcpyAsync(out_len, d_len, (size_t)n * 4, hipMemcpyDeviceToHost, s), "D2H out_len");
    if (status) HIP_TRY(hipMemcpyAsync(status, d_st, n, hipMemcpyDeviceToHost, s), "D2H status");
    HIP_TRY(hipStreamSynchronize(s), "sync");
    // run of tile t: [its slot position, end of its last kept string); chunks of the device output go through the
    // context's pinned buffer and each run's part of a chunk is copied out of it
    const uint32_t ntiles = (n + 63) / 64;
    auto run_lo = [&](uint32_t t) -> uint64_t {
        const uint64_t o = in_off[(size_t)t * 64];
        return decode ? (o * 8) / 5 : o;
    };
    auto run_hi = [&](uint32_t t) -> uint64_t {
        const uint32_t last = (t + 1) * 64 < n ? (t + 1) * 64 - 1 : n - 1;
        return (uint64_t)h_ooff[last] + (out_len[last] != HHUFF_FAIL_LEN ? out_len[last] : 0);
    };
    const size_t chunk = (size_t)64 << 20;
    rc = c.reserve(need, std::min<size_t>(chunk, up16(slot_end + 16)));
    if (rc) return rc;
    uint32_t t = 0;
    for (uint64_t lo = 0; lo < slot_end && t < ntiles; lo += chunk) {
        const uint64_t hi = std::min<uint64_t>(slot_end, lo + chunk);
        while (t < ntiles && run_hi(t) <= lo) ++t;  // runs ending before this chunk (empty runs included)
        if (t >= ntiles || run_lo(t) >= hi) continue;  // nothing of any run in this chunk
        HIP_TRY(hipMemcpyAsync(c.h, d_out + lo, hi - lo, hipMemcpyDeviceToHost, s), "D2H out");
        HIP_TRY(hipStreamSynchronize(s), "sync");
        for (uint32_t u = t; u < ntiles; ++u) {
            const uint64_t a = std::max(run_lo(u), lo), b = std::min(run_hi(u), hi);
            if (run_lo(u) >= hi) break;
            if (b > a) memcpy(out + a, c.h + (a - lo), b - a);
        }
    }
    return HHUFF_OK;
}

}  // namespace

HHUFF_API int hhuff_decode_batch_host_packed(const uint8_t* in, uint64_t in_size, const uint32_t* in_off, uint32_t n,
                                             const uint32_t* is_name_bits, uint8_t* out, uint64_t out_size, uint32_t* out_off,
                                             uint32_t* out_len, uint8_t* status, int device) {
    return host_packed(true, in, in_size, in_off, n, is_name_bits, out, out_size, out_off, out_len, status, device);
}

HHUFF_API int hhuff_encode_batch_host_packed(const uint8_t* in, uint64_t in_size, const uint32_t* in_off, uint32_t n,
                                             uint8_t* out, uint64_t out_size, uint32_t* out_off, uint32_t* out_len,
                                             uint8_t* status, int device) {
    return host_packed(false, in, in_size, in_off, n, nullptr, out, out_size, out_off, out_len, status, device);
}

HHUFF_API int hhuff_decode_batch_host_pipelined(const uint8_t* in, uint64_t in_size, const uint32_t* in_off, uint32_t n,
                                                const uint32_t* is_name_bits, uint8_t* out, uint64_t out_size,
                                                uint32_t* out_len, uint8_t* status, int device, uint64_t chunk_bytes) {
    if (n == 0) return HHUFF_OK;
    if (!in || !in_off || !out || !out_len || !status) return arg_fail("NULL array");
    if (in_off[n] > in_size) return arg_fail("in_off[n] > in_size");
    return pipelined(true, in, in_size, in_off, n, is_name_bits, out, out_size, out_len, status, device, chunk_bytes);
}

HHUFF_API int hhuff_encode_batch_host_pipelined(const uint8_t* in, uint64_t in_size, const uint32_t* in_off, uint32_t n,
                                                uint8_t* out, uint64_t out_size, uint32_t* out_len, uint8_t* status,
                                                int device, uint64_t chunk_bytes) {
    if (n == 0) return HHUFF_OK;
    if (!in || !in_off || !out || !out_len) return arg_fail("NULL array");
    if (in_off[n] > in_size) return arg_fail("in_off[n] > in_size");
    return pipelined(false, in, in_size, in_off, n, nullptr, out, out_size, out_len, status, device, chunk_bytes);
}

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
// (3d) multi-device batch: one batch over several GPUs of this process (include/hhuff.h (3d)).  Offsets stay
// absolute, so a shard is just a sub-range of in_off with `in` / `out` (and, for a shard copied to another
// device, its scratch shifted back by the shard's base) -- the same addressing as the chunked host pipeline.
// ---------------------------------------------------------------------------------------------------
namespace {

// the byte-balanced cut (hhuff_shard_bounds): the first string at or past the k/ns quantile of the bytes, rounded
// down to a multiple of align -- a lower_bound over in_off[0 .. n], the same search as dist.byte_balanced_bounds
__host__ __device__ inline uint32_t shard_bound(const uint32_t* in_off, uint32_t n, uint32_t k, uint32_t ns,
                                                uint32_t align) {
    if (k == 0) return 0;
    if (k >= ns) return n;
    const uint64_t base = in_off[0];
    const uint64_t end = in_off[n];
    const uint64_t target = base + (end > base ? ((uint64_t)k * (end - base)) / ns : 0);
    uint32_t lo = 0, hi = n;
    while (lo < hi) {
        const uint32_t mid = lo + (hi - lo) / 2;
        if ((uint64_t)in_off[mid] < target)
            lo = mid + 1;
        else
            hi = mid;
    }
    return align > 1 ? lo - lo % align : lo;
}

// device-resident batches: the cut and the byte offsets at the cut, into mapped host memory (b[0 .. ns], then
// in_off[b[k]] at b[ns + 1 + k])
__global__ void shard_bounds_kernel(const uint32_t* in_off, uint32_t n, uint32_t ns, uint32_t align, uint32_t* b) {
    const uint32_t k = threadIdx.x;
    if (k <= ns) {
        const uint32_t i = shard_bound(in_off, n, k, ns, align);
        b[k] = i;
        b[ns + 1 + k] = in_off[i];
    }
}

constexpr int kMaxDev = 64;
// HHUFF_MULTI_COPY=1: shards on the source device go through the copy path too (a device-to-device copy there):
// the peer path's addressing, tested on a one-GPU box
bool force_copy() {
    const char* v = getenv("HHUFF_MULTI_COPY");  // read per call (tests switch it within one process)
    return v && v[0] == '1';
}
constexpr uint32_t kShardAlign = 64;  // a shard starts on a tile (and on an is-name word)

int check_devices(int ndev, const int* devices, int* dv) {
    if (ndev < 1 || ndev > kMaxDev) return arg_fail("ndev must be in [1, 64]");
    int count = 0;
    HIP_TRY(hipGetDeviceCount(&count), "hipGetDeviceCount");
    for (int k = 0; k < ndev; ++k) {
        dv[k] = devices ? devices[k] : k;
        if (dv[k] < 0 || dv[k] >= count) return arg_fail("device id out of range");
    }
    return HHUFF_OK;
}

// host arrays: one persistent library thread per device (its thread-local stream, scratch and pinned staging
// persist across calls), each running its shard through the host path
struct DevWorker {
    std::mutex mu;
    std::condition_variable cv;
    std::function<void()> job;
    bool has = false, done = false;
    DevWorker() {
        std::thread([this] {
            for (;;) {
                std::function<void()> j;
                {
                    std::unique_lock<std::mutex> l(mu);
                    cv.wait(l, [this] { return has; });
                    j = std::move(job);
                    has = false;
                }
                j();
                {
                    std::lock_guard<std::mutex> l(mu);
                    done = true;
                }
                cv.notify_all();
            }
        }).detach();
    }
    void post(std::function<void()> f) {
        {
            std::lock_guard<std::mutex> l(mu);
            job = std::move(f);
            has = true;
            done = false;
        }
        cv.notify_all();
    }
    void wait() {
        std::unique_lock<std::mutex> l(mu);
        cv.wait(l, [this] { return done; });
    }
};
std::mutex g_multi_mu;                       // one multi-device host call at a time (each uses every device)
DevWorker* g_workers[kMaxDev] = {};          // created on first use, never destroyed (detached threads)

int multi_host(bool decode, int ndev, const int* dv, const uint8_t* in, uint64_t in_size, const uint32_t* in_off,
               uint32_t n, const uint32_t* names, uint8_t* out, uint64_t out_size, uint32_t* out_len, uint8_t* status) {
    if (in_off[n] > in_size) return arg_fail("in_off[n] > in_size");
    std::vector<uint32_t> b(ndev + 1);
    for (int k = 0; k <= ndev; ++k) b[k] = shard_bound(in_off, n, (uint32_t)k, (uint32_t)ndev, kShardAlign);
    std::lock_guard<std::mutex> g(g_multi_mu);
    std::vector<int> rc(ndev, HHUFF_OK);
    std::vector<std::string> err(ndev);
    std::vector<int> posted;
    for (int k = 0; k < ndev; ++k) {
        const uint32_t lo = b[k], m = b[k + 1] - b[k];
        if (m == 0) continue;
        DevWorker*& w = g_workers[k];
        if (!w) w = new DevWorker();
        const int dev = dv[k];
        w->post([=, &rc, &err] {
            rc[k] = pipelined(decode, in, in_size, in_off + lo, m, names ? names + lo / 32 : nullptr, out, out_size,
                              out_len + lo, status ? status + lo : nullptr, dev, 0);
            if (rc[k]) err[k] = t_err;
        });
        posted.push_back(k);
    }
    for (int k : posted) g_workers[k]->wait();
    for (int k = 0; k < ndev; ++k)
        if (rc[k]) {
            snprintf(t_err, sizeof(t_err), "shard %d (device %d): %s", k, dv[k], err[k].c_str());
            return rc[k];
        }
    return HHUFF_OK;
}

// device arrays on src: per calling thread, one stream per device and the mapped words the cut comes back in
struct MultiCtx {
    hipStream_t s[kMaxDev] = {};
    uint32_t* hb = nullptr;  // mapped host memory: 2 (kMaxDev + 1) words
    bool peer[kMaxDev][kMaxDev] = {};
    ~MultiCtx() {
        for (auto& x : s)
            if (x) (void)hipStreamDestroy(x);
        if (hb) (void)hipHostFree(hb);
    }
};
thread_local MultiCtx t_multi;

int multi_device(bool decode, int ndev, const int* dv, int src, const uint8_t* in, uint64_t in_size,
                 const uint32_t* in_off, uint32_t n, const uint32_t* names, uint8_t* out, uint64_t out_size,
                 uint32_t* out_len, uint8_t* status, hipStream_t stream) {
    DeviceGuard guard(src);
    if (guard.err != hipSuccess) return hip_fail(guard.err, "hipSetDevice");
    MultiCtx& X = t_multi;
    if (!X.hb) HIP_TRY(hipHostMalloc(&X.hb, 8 * (kMaxDev + 1), hipHostMallocMapped | hipHostMallocCoherent), "hipHostMalloc");
    uint32_t* d_hb = nullptr;
    HIP_TRY(hipHostGetDevicePointer((void**)&d_hb, X.hb, 0), "hipHostGetDevicePointer");
    hipLaunchKernelGGL(shard_bounds_kernel, dim3(1), dim3(kMaxDev + 1), 0, stream, in_off,
                       n, (uint32_t)ndev, kShardAlign, d_hb);
    HIP_TRY(hipGetLastError(), "shard bounds launch");
    HIP_TRY(hipStreamSynchronize(stream), "sync (the cut)");
    std::vector<uint32_t> b(X.hb, X.hb + ndev + 1), boff(X.hb + ndev + 1, X.hb + 2 * ndev + 2);
    auto slot_of = [&](uint64_t pos) { return decode ? (pos * 8) / 5 : pos; };
    if (boff[ndev] > in_size) return arg_fail("in_off[n] > in_size");
    if (out_size < slot_of(boff[ndev])) return arg_fail("out_size below the output slots of the batch");
    hipEvent_t ready;
    HIP_TRY(hipEventCreateWithFlags(&ready, hipEventDisableTiming), "hipEventCreate");
    std::vector<hipEvent_t> fin;
    int rc = HHUFF_OK;
    auto fail = [&](hipError_t e, const char* where) {
        if (rc == HHUFF_OK) rc = hip_fail(e, where);
    };
    hipError_t e = hipEventRecord(ready, stream);
    if (e != hipSuccess) fail(e, "hipEventRecord");
    for (int k = 0; k < ndev && rc == HHUFF_OK; ++k) {
        const uint32_t lo = b[k], m = b[k + 1] - b[k];
        if (m == 0) continue;
        const int dev = dv[k];
        const uint64_t s0 = boff[k], e0 = boff[k + 1];
        if (dev == src && !force_copy()) {  // in place, on the caller's stream
            e = decode ? hhuff::launch_decode(in, in_size, in_off + lo, nullptr, m, names ? names + lo / 32 : nullptr, out,
                                              nullptr, out_len + lo, status + lo, stream, e0 - s0)
                       : hhuff::launch_encode(in, in_size, in_off + lo, nullptr, m, out, nullptr, out_len + lo,
                                              status ? status + lo : nullptr, stream, e0 - s0);
            if (e != hipSuccess) fail(e, "shard launch (source device)");
            continue;
        }
        if ((e = hipSetDevice(dev)) != hipSuccess) {
            fail(e, "hipSetDevice");
            break;
        }
        if (!X.s[dev] && (e = hipStreamCreateWithFlags(&X.s[dev], hipStreamNonBlocking)) != hipSuccess) {
            fail(e, "hipStreamCreate");
            break;
        }
        if (dev != src && !X.peer[dev][src]) {  // direct xGMI reads / writes of src's memory where the link allows it
            int can = 0;
            if (hipDeviceCanAccessPeer(&can, dev, src) == hipSuccess && can) {
                const hipError_t pe = hipDeviceEnablePeerAccess(src, 0);
                if (pe != hipSuccess && pe != hipErrorPeerAccessAlreadyEnabled) {
                    fail(pe, "hipDeviceEnablePeerAccess");
                    break;
                }
                (void)hipGetLastError();
            }
            X.peer[dev][src] = true;
        }
        hipStream_t ms = X.s[dev];
        // the shard's layout on its device (as one chunk of the host pipeline): [in bytes from base][in_off m + 1]
        // [names][out slots from slot_of(base)][out_len m][status m]; base a multiple of 80 keeps the decode slot
        // floor(8 base / 5) 16-byte aligned
        const uint64_t base = (s0 / 80) * 80, nbytes = e0 - base;
        const uint64_t olo = slot_of(s0), ohi = std::min<uint64_t>(slot_of(e0), out_size), obase = slot_of(base);
        const uint64_t ocap = slot_of(e0) - obase + 16;
        const size_t nw = names ? ((size_t)m + 31) / 32 : 0;
        const size_t o_off = up16(nbytes + 16), o_nm = o_off + up16(((size_t)m + 1) * 4), o_out = o_nm + up16(nw * 4),
                     o_len = o_out + up16(ocap), o_st = o_len + up16((size_t)m * 4), need = o_st + up16(m);
        uint8_t* d = nullptr;
        if ((e = hipStreamWaitEvent(ms, ready, 0)) != hipSuccess || (e = hhuff::work_alloc((void**)&d, need, ms)) != hipSuccess) {
            fail(e, "shard scratch");
            break;
        }
        uint32_t* d_off = reinterpret_cast<uint32_t*>(d + o_off);
        uint32_t* d_nm = nw ? reinterpret_cast<uint32_t*>(d + o_nm) : nullptr;
        uint32_t* d_len = reinterpret_cast<uint32_t*>(d + o_len);
        uint8_t* d_st = d + o_st;
        if ((e = hipMemcpyPeerAsync(d, dev, in + base, src, nbytes, ms)) != hipSuccess ||
            (e = hipMemcpyPeerAsync(d_off, dev, in_off + lo, src, ((size_t)m + 1) * 4, ms)) != hipSuccess ||
            (nw && (e = hipMemcpyPeerAsync(d_nm, dev, names + lo / 32, src, nw * 4, ms)) != hipSuccess)) {
            fail(e, "peer copy in");
            break;
        }
        e = decode ? hhuff::launch_decode(d - base, e0, d_off, nullptr, m, d_nm, d + o_out - obase, nullptr, d_len, d_st,
                                          ms, e0 - s0)
                   : hhuff::launch_encode(d - base, e0, d_off, nullptr, m, d + o_out - obase, nullptr, d_len,
                                          status ? d_st : nullptr, ms, e0 - s0);
        if (e != hipSuccess) {
            fail(e, "shard launch (peer device)");
            break;
        }
        if ((ohi > olo && (e = hipMemcpyPeerAsync(out + olo, src, d + o_out + (olo - obase), dev, ohi - olo, ms)) != hipSuccess) ||
            (e = hipMemcpyPeerAsync(out_len + lo, src, d_len, dev, (size_t)m * 4, ms)) != hipSuccess ||
            (status && (e = hipMemcpyPeerAsync(status + lo, src, d_st, dev, m, ms)) != hipSuccess)) {
            fail(e, "peer copy out");
            break;
        }
        if ((e = hipFreeAsync(d, ms)) != hipSuccess) {
            fail(e, "hipFreeAsync");
            break;
        }
        hipEvent_t f;
        if ((e = hipEventCreateWithFlags(&f, hipEventDisableTiming)) != hipSuccess || (e = hipEventRecord(f, ms)) != hipSuccess) {
            fail(e, "hipEventRecord");
            break;
        }
        fin.push_back(f);
    }
    (void)hipSetDevice(src);
    for (hipEvent_t f : fin) {  // the caller's stream goes on once every shard is back
        e = hipStreamWaitEvent(stream, f, 0);
        if (e != hipSuccess) fail(e, "hipStreamWaitEvent");
        (void)hipEventDestroy(f);  // released once it completes
    }
    (void)hipEventDestroy(ready);
    return rc;
}

int batch_multi(bool decode, int ndev, const int* devices, int src, const uint8_t* in, uint64_t in_size,
                const uint32_t* in_off, uint32_t n, const uint32_t* names, uint8_t* out, uint64_t out_size, uint32_t* out_len,
                uint8_t* status, void* stream) {
    int dv[kMaxDev];
    int rc = check_devices(ndev, devices, dv);
    if (rc) return rc;
    if (n == 0) return HHUFF_OK;
    if (!in || !in_off || !out || !out_len || (decode && !status)) return arg_fail("NULL array");
    if (src == HHUFF_HOST_MEMORY)
        return multi_host(decode, ndev, dv, in, in_size, in_off, n, names, out, out_size, out_len, status);
    int count = 0;
    HIP_TRY(hipGetDeviceCount(&count), "hipGetDeviceCount");
    if (src < 0 || src >= count) return arg_fail("src_device out of range");
    return multi_device(decode, ndev, dv, src, in, in_size, in_off, n, names, out, out_size, out_len, status,
                        static_cast<hipStream_t>(stream));
}

}  // namespace

HHUFF_API int hhuff_decode_batch_multi(int ndev, const int* devices, int src_device, const uint8_t* in, uint64_t in_size,
                                       const uint32_t* in_off, uint32_t n, const uint32_t* is_name_bits, uint8_t* out,
                                       uint64_t out_size, uint32_t* out_len, uint8_t* status, void* stream) {
    return batch_multi(true, ndev, devices, src_device, in, in_size, in_off, n, is_name_bits, out, out_size, out_len,
                       status, stream);
}

HHUFF_API int hhuff_encode_batch_multi(int ndev, const int* devices, int src_device, const uint8_t* in, uint64_t in_size,
                                       const uint32_t* in_off, uint32_t n, uint8_t* out, uint64_t out_size, uint32_t* out_len,
                                       uint8_t* status, void* stream) {
    return batch_multi(false, ndev, devices, src_device, in, in_size, in_off, n, nullptr, out, out_size, out_len, status,
                       stream);
}

HHUFF_API int hhuff_shard_bounds(const uint32_t* in_off, uint32_t n, uint32_t nshards, uint32_t align, uint32_t* bounds) {
    if (!in_off || !bounds) return arg_fail("NULL array");
    if (nshards < 1) return arg_fail("nshards must be >= 1");
    for (uint32_t k = 0; k <= nshards; ++k) bounds[k] = shard_bound(in_off, n, k, nshards, align);
    return HHUFF_OK;
}

// ---------------------------------------------------------------------------------------------------
// (4) info
// ---------------------------------------------------------------------------------------------------
#ifdef HHUFF_PROFILE  // profile builds: per-phase cycle sums of the staged kernels (tools/ab.py prof)
namespace hhuff {
hipError_t read_prof(unsigned long long* out16, bool reset);
}
HHUFF_API int hhuff_debug_prof(unsigned long long* out16, int reset) {
    return hhuff::read_prof(out16, reset != 0) == hipSuccess ? 0 : -1;
}
#endif
HHUFF_API const char* hhuff_version(void) { return "hhuff 0.1.0 (gfx950)"; }
HHUFF_API const char* hhuff_last_error_string(void) { return t_err; }
HHUFF_API int hhuff_pool_trim(void) {
    // pool_trim synchronises the device (memory freed on any stream returns to the pool once that stream
    // passes the free), which would also wait for the resident per-string wave: it is stopped first, with
    // its lock held so no per-string call relaunches it meanwhile (the next call after the trim does)
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return hip_fail(hipErrorInvalidDevice, "pool trim");
    Service& S = g_svc[dev];
    std::lock_guard<std::mutex> g(S.mu);
    if (S.ready) {
        __atomic_store_n(&S.ctrl->stop, 1u, __ATOMIC_RELEASE);
        (void)hipStreamSynchronize(S.stream);  // the wave polls stop: it exits within a poll
    }
    hipError_t e = hhuff::pool_trim();
    return e == hipSuccess ? HHUFF_OK : hip_fail(e, "pool trim");
}
HHUFF_API int hhuff_decode_prices(int device, float* out4) {
    if (!out4) return arg_fail("NULL out4");
    return hhuff::decode_prices_of(device, out4, 0) == 0 ? HHUFF_OK : hip_fail(hipErrorInvalidDevice, "hhuff_decode_prices");
}
HHUFF_API int hhuff_calibrate_decode_prices(int device, float* out4) {
    float tmp[4];
    return hhuff::decode_prices_of(device, out4 ? out4 : tmp, 1) == 0
               ? HHUFF_OK
               : hip_fail(hipErrorInvalidDevice, "hhuff_calibrate_decode_prices");
}
HHUFF_API int hhuff_set_decode_prices(int device, const float* in4) {
    const int r = hhuff::set_decode_prices(device, in4);
    if (r == -2) return arg_fail("decode prices must be finite and >= 0");
    return r == 0 ? HHUFF_OK : hip_fail(hipErrorInvalidDevice, "hhuff_set_decode_prices");
}

HHUFF_API int hhuff_set_decode_kernel(int mode) {
    const int r = hhuff::set_decode_kernel(mode);
    return r < 0 ? arg_fail("decode kernel mode must be 0, 1 or 2") : r;
}

HHUFF_API uint32_t hhuff_set_edge_defer_min(uint32_t n) { return hhuff::set_edge_defer_min(n); }

HHUFF_API int hhuff_grid_size(int device, int which) {
    DeviceGuard guard(device);
    if (guard.err != hipSuccess) return -1;
    return hhuff::grid_size(device, which);
}
