// Internal launch interface between the C-ABI shim (hhuff_capi.hip) and the kernels (hhuff_kernels.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "hhuff.h"

namespace hhuff {
hipError_t launch_decode(const uint8_t* in, uint64_t in_size, const uint32_t* in_off, const uint32_t* in_len, uint32_t n,
                         const uint32_t* is_name_bits, uint8_t* out, const uint32_t* out_off, uint32_t* out_len,
                         uint8_t* status, hipStream_t stream, uint64_t sel_bytes = 0);
hipError_t launch_encode(const uint8_t* in, uint64_t in_size, const uint32_t* in_off, const uint32_t* in_len, uint32_t n,
                         uint8_t* out, const uint32_t* out_off, uint32_t* out_len, uint8_t* status, hipStream_t stream,
                         uint64_t sel_bytes = 0);
// One string per launch (the per-string h2o symbols): h = device-visible pinned host buffer
// [u32 len, is_name, result len, status][input, in_cap bytes (16-aligned)][output]; len <= kOneMax
constexpr uint32_t kOneMax = 32768;  // LDS: 32 KB input + 52 KB output beside the 32-KB table
hipError_t launch_one(uint8_t* h, uint32_t len, uint32_t in_cap, bool is_name, bool encode, hipStream_t stream);
// One device-resident string past kOneMax, encoded by one block (out: 4-byte aligned, at least 4 ceil(8 len / 32)
// bytes; out_len: the code bytes or kFailLen)
hipError_t launch_encode_long(const uint8_t* in, uint32_t len, uint8_t* out, uint32_t* out_len, hipStream_t stream);
// Resident per-string service (hhuff_capi.hip per_string): one wave polls kSvcSlots mailboxes in pinned,
// device-visible, coherent host memory and codes each posted string in place; it exits when `stop` is set,
// after idle_ticks of the 100 MHz real-time counter without a request, or after max_ticks in all.
constexpr uint32_t kSvcSlots = 64;
constexpr uint32_t kSvcMax = 768;  // longest string a mailbox takes (longer ones: launch_one / batch kernels):
                                   // 64 chunks of 12 input bytes, one 16-B load per lane
// One mailbox.  The host writes the input as 16-B chunks {request number, 12 bytes} with single 16-B stores,
// then the header {req, op, len, is_name} as one 16-B store.  A device load of a chunk sees it whole, old or
// new, so a chunk is current iff it carries the request number: the service wave can read the data of the
// mailbox it served last in the same round as the headers it polls, and use it when every chunk it needs
// is current (else it reads the chunks again, after the header -- then they are all current).
struct alignas(16) SvcSlot {
    uint32_t req, op, len, is_name;       // host, one 16-B store after the chunks; op: 0 decode, 1 encode
    uint32_t done, result, status, pad;   // device: done after the result
    uint32_t t_seen, t_data, t_coded, t_out;  // the wave's real-time stamps (100 MHz, low 32 bits): profiling
    uint32_t pad2[4];
    uint32_t chunk[64][4];                // {req, input bytes [12 i, 12 i + 12)}
    uint32_t outc[104][4];                // device: {req, output bytes [12 i, 12 i + 12)}, each one 16-B store
};
// The device writes the output chunks and then {done, result, status} with single 16-B system-scope stores and
// no wait between them: the host takes a chunk when it carries the request number, as the device does with
// the input chunks.
static_assert(sizeof(SvcSlot) % 16 == 0 && sizeof(SvcSlot) == 64 + 1024 + 1664, "mailbox layout");
static_assert(12 * 64 == kSvcMax && (kSvcMax * 8) / 5 <= 12 * 104, "mailbox sizes");
// Several service waves (one per block, launch_service's grid): wave g serves mailboxes g, g + G, g + 2G, ...
// Wave 0 decides when the grid ends (no request to any wave for idle_ticks, max_ticks in all, or `stop`) and
// raises `quit`; every wave polls it with its mailboxes, stores gone[g] as it leaves, and wave 0 clears
// `alive` once all have left, so the host relaunches only a finished grid.
constexpr uint32_t kSvcMaxWaves = 64;
struct SvcCtrl {
    uint32_t stop, alive, quit, waves;  // host: stop; wave 0: alive, quit; waves = G (read by the host)
    uint32_t last[kSvcMaxWaves];        // wave g: low 32 bits of the real-time counter at its last request
    uint32_t gone[kSvcMaxWaves];        // wave g: 1 once it has left its loop
};
hipError_t launch_service(SvcSlot* slots, SvcCtrl* ctrl, uint64_t idle_ticks, uint64_t max_ticks, hipStream_t stream);
uint32_t service_waves();
// Packed output (include/hhuff.h hhuff_{de,en}code_batch_packed): contiguous layout, pk_off u32[n + 1]
hipError_t launch_decode_packed(const uint8_t* in, uint64_t in_size, const uint32_t* in_off, uint32_t n,
                                const uint32_t* is_name_bits, uint8_t* out, uint32_t* pk_off, uint32_t* out_len,
                                uint8_t* status, hipStream_t stream);
hipError_t launch_encode_packed(const uint8_t* in, uint64_t in_size, const uint32_t* in_off, uint32_t n, uint8_t* out,
                                uint32_t* pk_off, uint32_t* out_len, uint8_t* status, hipStream_t stream);
// sel_bytes: bytes the batch's strings span, used only to pick the kernel variant from the mean string
// length (0 = in_size).  Chunked callers pass `in` shifted back by the chunk base so that absolute
// offsets address the chunk; in_size is then absolute and sel_bytes carries the chunk's own span.
hipError_t launch_flatten(const uint8_t* in, uint64_t in_size, const uint32_t* in_off, const uint32_t* in_len, uint32_t n,
                          const uint8_t* first_bytes, uint32_t prefix_bits, const uint32_t* raw_bits, uint8_t* out,
                          const uint32_t* out_off, uint32_t* out_len, hipStream_t stream);
hipError_t launch_literals(const uint8_t* in, uint64_t in_size, const uint32_t* lit_off, const uint32_t* lit_end, uint32_t n,
                           uint32_t prefix_bits, uint32_t flags, const uint32_t* is_name_bits, uint8_t* out,
                           uint32_t* out_len, uint32_t* pay_off, uint32_t* consumed, uint8_t* status, uint32_t* huff_len,
                           hipStream_t stream);
// literals whose count lives in device memory (*n_dev <= n_max); ws: literals_dev_ws bytes.  flags: the
// HHUFF_LIT_* flags, plus kLitNoRawCopy: raw payloads are validated but not copied to out
constexpr uint32_t kLitNoRawCopy = 0x100u;
hipError_t launch_literals_dev(const uint8_t* in, uint64_t in_size, const uint32_t* lit_off, uint32_t n_max,
                               const uint32_t* n_dev, uint32_t prefix_bits, uint32_t flags, const uint32_t* is_name_bits,
                               uint8_t* out, uint32_t* out_len, uint32_t* pay_off, uint32_t* consumed, uint8_t* status,
                               uint8_t* ws, hipStream_t stream, const uint8_t* prefix_of = nullptr);
uint64_t literals_dev_ws(uint32_t n_max, uint64_t in_size);
// The literal list of marked input bytes (hhuff_blocks.hip): bit p of lit_bits marks a literal at byte p.
// Writes word_pre (marks before each bitmap word), list (positions in order), lnames (bit r set when the
// literal's name_bits bit is), prefix_of[r] (when given) = pfx_alt if its pfx_bits bit is set, else pfx_name for
// a name, else 7, and *n_lit = chunk[nchunks]; chunk: u32[literal_list_chunks(nwords) + 1] of workspace.
uint64_t literal_list_chunks(uint64_t nwords);
hipError_t launch_literal_list(const uint32_t* lit_bits, const uint32_t* name_bits, const uint32_t* pfx_bits, uint32_t pfx_alt,
                               uint32_t pfx_name, uint64_t nwords, uint32_t* chunk, uint32_t* word_pre, uint32_t* list, uint32_t* lnames,
                               uint8_t* prefix_of, hipStream_t stream);
// stream-ordered device memory from the library's pool (free with hipFreeAsync on the same stream)
hipError_t work_alloc(void** p, uint64_t bytes, hipStream_t stream);
// hand the pool's kept memory on the current device back to the driver (hhuff_pool_trim)
hipError_t pool_trim();

// HTTP/2 response header blocks, encode side (hhuff_hpenc.hip): include/hhuff.h hhuff_hpack_flatten_responses;
// scratch = nconn x hpenc_conn_scratch() bytes
uint64_t hpenc_conn_scratch();
hipError_t launch_hpack_flatten(const uint8_t* in, uint64_t in_size, const hhuff_hpack_header_t* hdr, uint32_t nhdr,
                                const hhuff_hpack_response_t* res, const uint32_t* conn_first, uint32_t nconn, uint32_t nres,
                                uint32_t server_off, uint32_t server_len, uint8_t* out, const uint64_t* out_off,
                                uint32_t* out_len, uint32_t* headers_size, int32_t* rstatus, uint8_t* scratch,
                                uint32_t flags, hipStream_t stream);

// HTTP/3 response HEADERS frames (hhuff_hpenc.hip): include/hhuff.h hhuff_qpack_flatten_responses
hipError_t launch_qpack_flatten(const uint8_t* in, uint64_t in_size, const hhuff_hpack_header_t* hdr, uint32_t nhdr,
                                const hhuff_qpack_response_t* res, uint32_t nres, uint32_t server_off, uint32_t server_len,
                                uint8_t* out, const uint64_t* out_off, uint32_t* out_len, uint32_t* header_len,
                                int32_t* rstatus, hipStream_t stream);

// HPACK header blocks (f4): see include/hhuff.h hhuff_hpack_decode_blocks; scratch = nconn x
// hpack_conn_scratch(table_size) bytes of device memory
uint64_t hpack_conn_scratch(uint32_t table_size);
hipError_t launch_hpack_blocks(const uint8_t* in, uint64_t in_size, const uint32_t* blk_off, const uint32_t* conn_first,
                               uint32_t nconn, uint32_t table_size, uint8_t* arena, const uint64_t* arena_off,
                               uint32_t* name_off, uint32_t* name_len, uint32_t* value_off, uint32_t* value_len,
                               uint8_t* fflags, uint32_t* nfields, int32_t* bstatus, hhuff_request_t* req,
                               hhuff_response_t* res, const uint8_t* trailers, uint8_t* scratch, uint32_t flags,
                               hipStream_t stream);
// QPACK decoder (f4): see include/hhuff.h hhuff_qpack_decode; scratch = nconn x
// qpack_conn_scratch(header_table_size) bytes of device memory
uint64_t qpack_conn_scratch(uint32_t header_table_size);
hipError_t launch_qpack(const uint8_t* in, uint64_t in_size, const uint32_t* enc_off, const uint32_t* enc_len,
                        const uint32_t* sec_off, const uint32_t* conn_first, uint32_t nconn, uint32_t nsec,
                        uint32_t header_table_size, uint64_t max_blocked, const uint32_t* num_blocked, uint8_t* arena,
                        const uint64_t* arena_off, uint32_t* name_off, uint32_t* name_len, uint32_t* value_off,
                        uint32_t* value_len, uint8_t* fflags, uint32_t* nfields, int32_t* sstatus,
                        uint64_t* req_insert_count, int32_t* enc_status, uint32_t* enc_consumed, uint64_t* insert_count,
                        uint8_t* scratch, uint32_t flags, hipStream_t stream, const uint64_t* stream_id = nullptr,
                        hhuff_qpack_request_t* qreq = nullptr, hhuff_qpack_response_head_t* qres = nullptr);
int grid_size(int device, int which);
// the staged / stream prices (ps per string, per byte) a mixed-length decode on `device` uses: the fitted
// defaults, pinned values, or (calibrate != 0: measured now, synchronously) this device's own
// (hhuff_kernels.hip calibrate_prices); 0, or -1 when the device cannot be selected
int decode_prices_of(int device, float out[4], int calibrate);
// pin the prices of `device` (in4 NULL: back to the fitted defaults); 0, -1 bad device, -2 bad value
int set_decode_prices(int device, const float* in4);
int set_decode_kernel(int mode);  // hhuff_set_decode_kernel: previous mode, -1 for a bad one
uint32_t set_edge_defer_min(uint32_t n);  // hhuff_set_edge_defer_min: the previous threshold
}  // namespace hhuff
