/*
 * hhuff -- MI355X-native HPACK/QPACK Huffman codec: the drop-in C-ABI boundary.
 *
 * Library: h2o_amd/libhhuff.so (HIP kernels for gfx950 + host shim).  Plain C types only: no HIP,
 * torch or C++ types appear in these signatures; streams are passed as `void *` (a hipStream_t, or
 * NULL for the legacy default stream).
 *
 * 1. Per-string symbols with h2o's exact signatures and semantics.  A maintainer links libhhuff in
 *    place of the definitions in lib/http2/hpack.c.  Each call runs one HIP launch
 *    on the string, synchronously, on a per-thread stream of the calling thread's current device (which
 *    the call leaves as it was).  About 20 us per call on MI355X (bench.py per_string_latency_us) makes
 *    this the compatibility path; throughput comes from the batch API.  A HIP failure never aborts: the
 *    call returns SIZE_MAX (decode: h2o reports the literal as a COMPRESSION error; encode: h2o sends the
 *    string raw, a correct encoding) and hhuff_last_error_string() says why.
 * 2. Batch entry points on device-resident arrays (the hot path) and on host arrays (pinned staging,
 *    H2D/D2H included).  Element i of a batch has exactly the per-string semantics of (1).
 *
 * Batch array contract (all offsets/lengths u32; a batch addresses < 4 GiB of input):
 *   string i      in[in_off[i] .. in_off[i] + len_i)
 *                 len_i = in_len ? in_len[i] : in_off[i+1] - in_off[i]   (in_off has n+1 entries then)
 *   in_size       bytes readable at `in` (the kernels never read past it)
 *   is_name_bits  u32[(n+31)/32]; bit (i & 31) of word (i >> 5) set => string i is a header name
 *                 (NULL => every string is a header value)
 *   device `in` and `out` must be 16-byte aligned (hipMalloc / torch allocations are);
 *   strings may start at any byte.
 *   Per-string length limit: 2^29 - 1 bytes (status HHUFF_STATUS_TOO_LONG above it).
 */
#ifndef HHUFF_H
#define HHUFF_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define HHUFF_FAIL_LEN 0xFFFFFFFFu   /* out_len of a string whose per-string call returns SIZE_MAX */
#define HHUFF_SOFT_NAME 0x01u        /* H2O_HPACK_SOFT_ERROR_BIT_INVALID_NAME  (include/h2o/hpack.h:50) */
#define HHUFF_SOFT_VALUE 0x02u       /* H2O_HPACK_SOFT_ERROR_BIT_INVALID_VALUE (include/h2o/hpack.h:51) */
#define HHUFF_STATUS_FAIL 0x80u      /* hard failure: the per-string call returns SIZE_MAX */
#define HHUFF_STATUS_TOO_LONG 0xC0u  /* string longer than the per-string limit (never produced by h2o) */

#define HHUFF_OK 0
#define HHUFF_EINVAL (-1) /* bad argument (NULL array, misaligned base, n too large) */
#define HHUFF_EHIP (-2)   /* a HIP runtime call failed; see hhuff_last_error_string() */
#define HHUFF_ENODEV (-3) /* no gfx950 device / code object not loadable */

/* ---------------------------------------------------------------------------------------------
 * (1) h2o per-string symbols
 * ------------------------------------------------------------------------------------------- */

/* Replaces lib/http2/hpack.c:117 (declared include/h2o/hpack.h:69-70).
 * Returns the decoded length, or SIZE_MAX on a hard error (EOS symbol, padding longer than 7 bits or not
 * all ones).  On success ORs HHUFF_SOFT_NAME / HHUFF_SOFT_VALUE into *soft_errors (never clears it).
 * `dst` must hold at least 2 * len bytes (h2o's contract; floor(8 * len / 5) suffices).  *err_desc is
 * never written (the reference's upper-case hard error at hpack.c:142-144 is unreachable). */
size_t h2o_hpack_decode_huffman(char *dst, unsigned *soft_errors, const uint8_t *src, size_t len, int is_name,
                                const char **err_desc);

/* Replaces lib/http2/hpack.c:774 (declared include/h2o/hpack.h:60).
 * Returns the Huffman length when it is strictly shorter than `len`, else SIZE_MAX (also for len == 0).
 * `dst` must hold `len` bytes; its contents are unspecified on SIZE_MAX. */
size_t h2o_hpack_encode_huffman(uint8_t *dst, const uint8_t *src, size_t len);

/* Number of calls the two symbols above have taken in this process (both, any outcome).  An integration
 * check: after linking h2o against this library, a non-zero count after decoding a Huffman literal shows
 * h2o's callers (decode_string, h2o_hpack_encode_string, QPACK's flatten_string ...) bound here. */
uint64_t hhuff_per_string_calls(void);
/* Profiling: the resident per-string service's real-time stamps (100 MHz counter, low 32 bits) of the calling
 * thread's last served call on its current device: request seen, input in LDS, coded, output written.
 * HHUFF_OK, or HHUFF_EINVAL when this thread has no served call. */
int hhuff_service_stamps(uint32_t *out4);

/* ---------------------------------------------------------------------------------------------
 * (2) batch API, device-resident arrays (hot path).  Asynchronous on `stream`.
 * ------------------------------------------------------------------------------------------- */

/* Batched h2o_hpack_decode_huffman (hpack.c:117-156; callers hpack.c:241, qpack.c:228/370/579).
 *   out       decoded string i at out + (out_off ? out_off[i] : floor(8 * in_off[i] / 5)); the region
 *             must hold floor(8 * len_i / 5) bytes (the implicit layout is valid whenever the input
 *             strings do not overlap).  Bytes of the region past out_len[i] are unspecified.
 *   out_len   u32[n]: decoded length, or HHUFF_FAIL_LEN
 *   status    u8[n]:  soft-error bits on success, HHUFF_STATUS_FAIL on a hard error */
int hhuff_decode_batch(const uint8_t *in, uint64_t in_size, const uint32_t *in_off, const uint32_t *in_len, uint32_t n,
                       const uint32_t *is_name_bits, uint8_t *out, const uint32_t *out_off, uint32_t *out_len,
                       uint8_t *status, void *stream);

/* Batched h2o_hpack_encode_huffman (hpack.c:774-804; callers hpack.c:820, qpack.c:1046).
 *   out       Huffman string i at out + (out_off ? out_off[i] : in_off[i]); the region must hold len_i
 *             bytes.  Contents unspecified where out_len[i] == HHUFF_FAIL_LEN.
 *   out_len   u32[n]: Huffman length (< len_i), or HHUFF_FAIL_LEN when not shorter (SIZE_MAX)
 *   status    u8[n] or NULL: 0, or HHUFF_STATUS_FAIL */
int hhuff_encode_batch(const uint8_t *in, uint64_t in_size, const uint32_t *in_off, const uint32_t *in_len, uint32_t n,
                       uint8_t *out, const uint32_t *out_off, uint32_t *out_len, uint8_t *status, void *stream);

/* Packed output (wave-prefix compaction).  Contiguous layout only: string i = in[in_off[i] .. in_off[i+1]).
 * The strings are cut into tiles of 64 consecutive strings (string i is in tile i / 64).  Within a tile the
 * outputs are packed back to back in string order -- each wavefront lane owns one string and a wave-wide
 * prefix sum of the output lengths places them -- and tile t's run starts at its bound position
 *     decode: floor(8 * in_off[64 t] / 5)        encode: in_off[64 t]
 * (the first string's slot of the implicit layouts above), so runs of different tiles never overlap and
 * no byte outside the outputs is written: HBM traffic is exactly the output bytes.  Failed strings
 * (HHUFF_FAIL_LEN) take no bytes.
 *   out        decode: floor(8 * in_off[n] / 5) bytes; encode: in_off[n] bytes (16-byte aligned)
 *   out_off    u32[n + 1], written: string i at out + out_off[i], out_len[i] bytes; out_off[n] = the end of
 *              the last tile's run.  Inside a tile out_off[i + 1] = out_off[i] + string i's kept length, so
 *              tile t's run is the one range from out_off[64 t] to the end of its last string.
 *   out_len, status   as hhuff_decode_batch / hhuff_encode_batch
 * Device arrays, asynchronous on `stream`; in_size must stay below 2^32 * 5 / 8 (u32 offsets). */
int hhuff_decode_batch_packed(const uint8_t *in, uint64_t in_size, const uint32_t *in_off, uint32_t n,
                              const uint32_t *is_name_bits, uint8_t *out, uint32_t *out_off, uint32_t *out_len,
                              uint8_t *status, void *stream);
int hhuff_encode_batch_packed(const uint8_t *in, uint64_t in_size, const uint32_t *in_off, uint32_t n, uint8_t *out,
                              uint32_t *out_off, uint32_t *out_len, uint8_t *status, void *stream);

/* Batched string-literal framing: QPACK flatten_string (lib/http3/qpack.c:1042-1066) and, with
 * first_bytes == NULL and prefix_bits == 7, HPACK h2o_hpack_encode_string (lib/http2/hpack.c:816-837).
 * Per string: Huffman when not flagged in raw_bits (QPACK's dont_compress) and strictly shorter, i.e.
 *   [first & ~(2^p - 1) | 2^p, prefix-int(hufflen)] [Huffman bytes]
 * else raw:
 *   [first & ~(2^(p+1) - 1), prefix-int(len)] [the bytes]
 *   first_bytes  u8[n]: the caller's first byte (bits above the H bit are kept), NULL => 0
 *   prefix_bits  length-prefix width p in 1..7 (QPACK: 7 values, 5 encoder-stream names, 3 literal names)
 *   raw_bits     bitmask, NULL => all eligible for Huffman
 *   out          string i at out + (out_off ? out_off[i] : in_off[i] + 11 * i); region of len_i + 11 bytes
 *   out_len      u32[n]: framed length */
int hhuff_flatten_batch(const uint8_t *in, uint64_t in_size, const uint32_t *in_off, const uint32_t *in_len, uint32_t n,
                        const uint8_t *first_bytes, unsigned prefix_bits, const uint32_t *raw_bits, uint8_t *out,
                        const uint32_t *out_off, uint32_t *out_len, void *stream);

/* ---------------------------------------------------------------------------------------------
 * (3) batch API, host arrays: pinned staging + H2D, kernels, D2H on an internal stream of `device`.
 *     Synchronous.  Same array contract; `out` is a host buffer sized for the implicit layout
 *     (decode: floor(8 * in_size / 5) bytes, encode: in_size bytes) when out_off is NULL.
 * ------------------------------------------------------------------------------------------- */
int hhuff_decode_batch_host(const uint8_t *in, uint64_t in_size, const uint32_t *in_off, const uint32_t *in_len,
                            uint32_t n, const uint32_t *is_name_bits, uint8_t *out, uint64_t out_size,
                            const uint32_t *out_off, uint32_t *out_len, uint8_t *status, int device);
int hhuff_encode_batch_host(const uint8_t *in, uint64_t in_size, const uint32_t *in_off, const uint32_t *in_len,
                            uint32_t n, uint8_t *out, uint64_t out_size, const uint32_t *out_off, uint32_t *out_len,
                            uint8_t *status, int device);

/* (2b) Batched string-literal decode: HPACK decode_string (lib/http2/hpack.c:223-261) and
 *      QPACK decode_header_value_literal / decode_header_name_literal (lib/http3/qpack.c:559-629),
 *      minus the memory pool.  Literal i starts at in[lit_off[i]] -- its first byte carries the H flag
 *      at bit prefix_bits and the length as a prefix_bits-bit prefix integer (h2o_hpack_decode_int,
 *      hpack.c:52-83) -- and must end by in[lit_end[i]] (the walker's src_end).  Huffman payloads are
 *      decoded as h2o_hpack_decode_huffman does; raw payloads are copied and validated with
 *      h2o_hpack_validate_header_name / _value (hpack.c:163-221).  Raw names skip validation when they
 *      start with ':' (HPACK) or, with HHUFF_LIT_QPACK, when h2o_lookup_token knows them (qpack.c:585).
 *      Outputs: pay_off[i] = offset of the payload in `in`; decoded bytes at out + floor(8 pay_off[i] / 5)
 *      (out sized floor(8 in_size / 5) + 16); out_len[i] (HHUFF_FAIL_LEN on failure); consumed[i] =
 *      header + payload bytes, how far the walker's cursor advances (0 on failure); status[i] = soft
 *      bits (0x1 name, 0x2 value) | on failure HHUFF_STATUS_FAIL | verdict << 2 (HHUFF_LIT_*).
 *      Device arrays, asynchronous on `stream`; uses stream-ordered scratch (5 n bytes). */
#define HHUFF_LIT_QPACK 1u
#define HHUFF_LIT_INCOMPLETE 1 /* no byte, or the length integer runs past lit_end (H2O_HTTP2_ERROR_INCOMPLETE) */
#define HHUFF_LIT_BAD_INT 2    /* length integer overflow (H2O_HTTP2_ERROR_COMPRESSION from decode_int) */
#define HHUFF_LIT_TRUNCATED 3  /* length > bytes left before lit_end */
#define HHUFF_LIT_HUFFMAN 4    /* h2o_hpack_decode_huffman returned SIZE_MAX */
#define HHUFF_LIT_UPPERCASE 5  /* raw name with an upper-case letter (validate_header_name returned 0) */
#define HHUFF_LIT_TOO_LONG 6   /* payload of 2^29 bytes or more (this library's per-string limit) */
int hhuff_decode_literals(const uint8_t *in, uint64_t in_size, const uint32_t *lit_off, const uint32_t *lit_end,
                          uint32_t n, unsigned prefix_bits, unsigned flags, const uint32_t *is_name_bits, uint8_t *out,
                          uint32_t *out_len, uint32_t *pay_off, uint32_t *consumed, uint8_t *status, void *stream);

/* (2c) HPACK header blocks: h2o_hpack_decode_header (lib/http2/hpack.c:319-435) applied field
 *      after field over each block, as h2o_hpack_parse_request loops over a block (hpack.c:513-527), with
 *      one dynamic table per connection whose blocks are decoded in order.  One GPU lane per connection.
 *        block b        in[blk_off[b] .. blk_off[b+1])      (blocks packed back to back; blk_off has nblk+1)
 *        connection c   blocks conn_first[c] .. conn_first[c+1]-1   (conn_first has nconn+1 entries)
 *        table_size     SETTINGS_HEADER_TABLE_SIZE of every connection: the table's initial and maximum
 *                       capacity (hpack_capacity = hpack_max_capacity, lib/http2/connection.c:1844;
 *                       h2o's default 4096)
 *        arena          decoded names and values; block b writes arena[arena_off[b] .. arena_off[b+1])
 *                       (u64 offsets); every field's name is written, then its value.  Field offsets
 *                       are u32: arena bytes at or past 2^32 are out of reach (HHUFF_BLK_ARENA there)
 *      Per field f of block b (f in blk_off[b] .. blk_off[b] + nfields[b] - 1: a block of L bytes holds at
 *      most L fields, so field slots reuse the block's byte offsets): name_off/name_len/value_off/
 *      value_len (arena offsets, u32) and fflags = its soft-error bits (HHUFF_SOFT_NAME / _VALUE: the
 *      field's H2O_HTTP2_ERROR_INVALID_HEADER_CHAR).  Per block: nfields[b] and bstatus[b] = 0, or the
 *      hard error that stopped it: -9 H2O_HTTP2_ERROR_COMPRESSION, -1 H2O_HTTP2_ERROR_PROTOCOL (upper-case
 *      raw name), HHUFF_BLK_ARENA (a string does not fit the block's arena slice: a Huffman literal needs
 *      floor(8 len / 5) bytes free, a raw one len, an indexed one its size), or HHUFF_BLK_SKIPPED (an
 *      earlier block of the connection failed: h2o drops the connection).  Fields before the error stand.
 *      Device arrays; scratch = device memory of hhuff_hpack_scratch_size(nconn, table_size) bytes (the
 *      dynamic tables, 16-byte aligned), kept by the caller between calls for HHUFF_BLK_CONTINUE;
 *      asynchronous on `stream`.  The call also takes a stream-ordered workspace from the library's device
 *      memory pool: 16 bytes per input byte of field sources plus, for inputs below 4 GiB, the literal
 *      pre-pass -- 22 bytes per possible literal (up to 2/3 of the input bytes) plus 1.6 per input byte of
 *      decoded output -- about 33 bytes per input byte in all.  It is released on the stream; the pool
 *      keeps released memory for the next call (it never returns it to the driver by itself):
 *      hhuff_pool_trim() hands it back. */
#define HHUFF_BLK_CONTINUE 1u /* flags: the tables (and failed state) the previous call left in scratch
                                 carry over -- connection c of this call is connection c of that one; without
                                 it every connection starts with an empty table */
#define HHUFF_BLK_ARENA (-300)
#define HHUFF_BLK_SKIPPED (-301)
uint64_t hhuff_hpack_scratch_size(uint32_t nconn, uint32_t table_size);
int hhuff_hpack_decode_blocks(const uint8_t *in, uint64_t in_size, const uint32_t *blk_off, const uint32_t *conn_first,
                              uint32_t nconn, uint32_t table_size, uint8_t *arena, const uint64_t *arena_off,
                              uint32_t *name_off, uint32_t *name_len, uint32_t *value_off, uint32_t *value_len,
                              uint8_t *fflags, uint32_t *nfields, int32_t *bstatus, void *scratch, uint64_t scratch_size,
                              unsigned flags, void *stream);

/* (2c') HTTP/2 request header blocks: the same pass with h2o_hpack_parse_request's own rules applied to each
 *      field as it is decoded (lib/http2/hpack.c:502-637), called as h2o's HTTP/2 server calls it
 *      (lib/http2/connection.c:626-629: every out-pointer given, cache digests loaded, no datagram flow id):
 *        - more than H2O_HPACK_MAX_HEADERS_HARD_LIMIT (1000) fields -> COMPRESSION (:528-532)
 *        - pseudo-headers (:533-586): only before the first regular field; :authority, :method, :path,
 *          :scheme at most once, :path not empty, :protocol at most once; any other ':' name -> PROTOCOL
 *        - content-length must parse (h2o_strtosize) -> else PROTOCOL (:591-597); expect, host (fills a
 *          missing authority) and datagram-flow-id are taken out of the list; te other than "trailers"
 *          (case-insensitive) and connection / http2-settings / transfer-encoding / upgrade -> PROTOCOL
 *          (:587-619)
 *        - the first H2O_MAX_HEADERS (100) remaining fields go to the request's header list; beyond that
 *          they are dropped and the block ends with H2O_HTTP2_ERROR_INVALID_HEADER_CHAR (:620-637)
 *      Outputs as hhuff_hpack_decode_blocks plus, per block, req[b]; per field, fflags gains
 *      HHUFF_FIELD_HEADER when h2o_add_header took the field.  bstatus[b] is h2o_hpack_parse_request's
 *      return value: 0, -254 (H2O_HTTP2_ERROR_INVALID_HEADER_CHAR: a soft error, the connection lives on),
 *      -1 / -9 (connection errors: later blocks of the connection are HHUFF_BLK_SKIPPED), or the
 *      HHUFF_BLK_* codes.  The field that triggered an error is counted in nfields (it was decoded and,
 *      for incremental indexing, entered the table).  The cache-digest field goes to the header list (h2o
 *      also feeds it to h2o_cache_digests_load_header; that side effect is the caller's). */
#define HHUFF_FIELD_HEADER 0x4u /* fflags: the field is in h2o's h2o_headers_t (h2o_add_header) */
#define HHUFF_HERR_NONE 0u               /* *err_desc == NULL */
#define HHUFF_HERR_SOFT_NAME 1u          /* h2o_hpack_soft_err_found_invalid_char_in_header_name */
#define HHUFF_HERR_SOFT_VALUE 2u         /* h2o_hpack_soft_err_found_invalid_char_in_header_value */
#define HHUFF_HERR_HEADERS_TOO_LONG 3u   /* h2o_hpack_err_headers_too_long */
#define HHUFF_HERR_INVALID_PSEUDO 4u     /* h2o_hpack_err_invalid_pseudo_header */
#define HHUFF_HERR_CONTENT_LENGTH 5u     /* h2o_hpack_err_invalid_content_length_header */
#define HHUFF_HERR_CONNECTION_SPECIFIC 6u /* h2o_hpack_err_unexpected_connection_specific_header */
#define HHUFF_HERR_UPPER_CASE_NAME 7u    /* h2o_hpack_err_found_upper_case_in_header_name */
typedef struct hhuff_request {
    uint64_t content_length; /* h2o's *content_length: SIZE_MAX (all ones) without a content-length field */
    int32_t method, scheme, authority, path, protocol, expect; /* the field (0-based within the block) whose
                                value h2o stored in *method ... *expect, or -1; authority may be a host field */
    uint32_t exists_map;  /* *pseudo_header_exists_map: H2O_HPACK_PARSE_HEADERS_*_EXISTS (hpack.h:81-85) */
    uint32_t nheaders;    /* fields added to the header list */
    uint32_t err;         /* HHUFF_HERR_*: what *err_desc points at when the call returns */
    uint32_t scheme_kind; /* *scheme: 0 unset, 1 H2O_URL_SCHEME_HTTP, 2 _HTTPS, 3 _MASQUE */
} hhuff_request_t;        /* 48 bytes */
int hhuff_hpack_parse_requests(const uint8_t *in, uint64_t in_size, const uint32_t *blk_off, const uint32_t *conn_first,
                               uint32_t nconn, uint32_t table_size, uint8_t *arena, const uint64_t *arena_off,
                               uint32_t *name_off, uint32_t *name_len, uint32_t *value_off, uint32_t *value_len,
                               uint8_t *fflags, uint32_t *nfields, int32_t *bstatus, hhuff_request_t *req,
                               void *scratch, uint64_t scratch_size, unsigned flags, void *stream);

/* (2c'') HTTP/2 response header blocks, client side: the same pass with h2o_hpack_parse_response's rules
 *      (lib/http2/hpack.c:642-750) applied to each field as it is decoded, called as h2o's HTTP/2 client calls
 *      it (lib/common/http2client.c:332 for a response head, :421 for trailers; no datagram flow id):
 *        - a head block must not be empty and must start with :status -> else PROTOCOL, missing mandatory
 *          pseudo header (:652-655, :706-709); :status once, three digits, the first 1-9 (PARSE_DIGIT: the
 *          digits before a bad one stay added); any other pseudo-header, or any in trailers -> PROTOCOL
 *        - more than 1000 fields -> COMPRESSION; content-length, cache-digest and host are listed as they are;
 *          datagram-flow-id is not listed; expect, te, connection, http2-settings, transfer-encoding and
 *          upgrade -> PROTOCOL (unexpected connection-specific header, :712-725)
 *        - the first 100 remaining fields go to the header list, beyond that the block ends with -254
 *      trailers[b] != 0 makes block b a trailers block (status == NULL; NULL: every block is a head; an empty
 *      trailers block fails in decode_header with COMPRESSION, hpack.c:328-329).  Outputs as
 *      hhuff_hpack_parse_requests with res[b] in place of req[b]; bstatus[b] is h2o_hpack_parse_response's
 *      return value (0, -254, -1, -9) or the HHUFF_BLK_* codes. */
#define HHUFF_HERR_MISSING_PSEUDO 9u /* h2o_hpack_err_missing_mandatory_pseudo_header */
typedef struct hhuff_response {
    int32_t status;           /* *status: 0 if none was parsed (trailers: always 0) */
    uint32_t nheaders;        /* fields added to the header list */
    uint32_t err;             /* HHUFF_HERR_*: what *err_desc points at when the call returns */
    int32_t datagram_flow_id; /* HTTP/3: the field whose value h2o stored in *datagram_flow_id, or -1 */
} hhuff_response_t;           /* 16 bytes */
int hhuff_hpack_parse_responses(const uint8_t *in, uint64_t in_size, const uint32_t *blk_off, const uint32_t *conn_first,
                                uint32_t nconn, uint32_t table_size, const uint8_t *trailers, uint8_t *arena,
                                const uint64_t *arena_off, uint32_t *name_off, uint32_t *name_len, uint32_t *value_off,
                                uint32_t *value_len, uint8_t *fflags, uint32_t *nfields, int32_t *bstatus,
                                hhuff_response_t *res, void *scratch, uint64_t scratch_size, unsigned flags, void *stream);

/* (2d) QPACK decoder (QPACK half): h2o's QPACK decoder (lib/http3/qpack.c) for many
 *      connections at once.  One call is one step of every connection c:
 *        encoder stream  in[enc_off[c] .. + enc_len[c]): h2o_qpack_decoder_handle_input (qpack.c:420-485,
 *                        decl. include/h2o/qpack.h) -- the caller's encoder-stream receive buffer, i.e. the
 *                        bytes not consumed by the previous step followed by the new ones
 *        field sections  conn_first[c] .. conn_first[c+1]-1, section k = in[sec_off[k] .. sec_off[k+1])
 *                        (packed back to back): what h2o_qpack_parse_request (qpack.c:830-858) reads --
 *                        parse_decode_context, check_decode_context_blocked, then decode_header field after
 *                        field -- against the table as the connection's encoder stream left it
 *        header_table_size  the decoder's SETTINGS_QPACK_MAX_TABLE_CAPACITY (h2o_qpack_create_decoder,
 *                        qpack.c:240); max_blocked its blocked-streams limit; num_blocked[c] (NULL = 0) the
 *                        caller's count of the connection's blocked streams before this step
 *                        (lib/http3/server.c:1544).  Blocked sections of one step take the free slots in
 *                        section order, as h2o raises num_qpack_blocked for every stream it parks
 *                        (server.c:1553): the first blocked section that finds num_blocked >= max_blocked
 *                        gets HHUFF_QPK_DECOMPRESSION_FAILED.
 *      Table semantics: every section of a step is decoded against the table as the step's WHOLE encoder
 *      stream left it.  h2o decodes a section against the table as it stands when the section arrives;
 *      the two differ only when the same step's encoder stream evicts an entry an earlier-arriving section
 *      still references -- which a compliant encoder never does (RFC 9204 2.1.1: an entry that
 *      unacknowledged sections reference is not evictable).  Against such a peer this call reports
 *      DECOMPRESSION_FAILED where h2o would have decoded the section; a caller that must match h2o
 *      byte for byte there splits the step before the evicting instruction.
 *      Per connection: enc_status[c] = 0, HHUFF_QPK_DECOMPRESSION_FAILED (h2o then closes the connection
 *      with H2O_HTTP3_ERROR_QPACK_ENCODER_STREAM) or HHUFF_QPK_SKIPPED (an earlier step failed);
 *      enc_consumed[c] = bytes of complete instructions consumed (the rest waits for more input);
 *      insert_count[c] as handle_input reports it (the new Insert Count, 0 when nothing was inserted).
 *      Per section k: sstatus[k] = 0, HHUFF_QPK_DECOMPRESSION_FAILED, HHUFF_QPK_BLOCKED (Required Insert
 *      Count not reached and a blocked slot free: h2o parks the stream until more inserts arrive),
 *      HHUFF_QPK_ARENA (a string does not fit arena[arena_off[k] .. min(arena_off[k+1], 2^32)) -- field
 *      offsets are u32 --: a Huffman literal
 *      needs floor(8 len / 5) bytes free, a raw one len, an indexed one its size) or HHUFF_QPK_SKIPPED;
 *      req_insert_count[k] (decoded Required Insert Count, for the Section Acknowledgment); nfields[k]
 *      fields in slots sec_off[k] .. + nfields[k] - 1: name_off/name_len/value_off/value_len (arena
 *      offsets) and fflags = soft bits (HHUFF_SOFT_NAME / _VALUE: decode_header's
 *      H2O_HTTP2_ERROR_INVALID_HEADER_CHAR).  Fields before an error stand.
 *      Device arrays; scratch = hhuff_qpack_scratch_size(nconn, header_table_size) bytes of device memory
 *      (16-byte aligned) that holds the tables: pass HHUFF_QPK_CONTINUE to carry them (and the failed
 *      state) over from the previous call -- connection c of this call is connection c of that one;
 *      without it every connection starts with a fresh decoder; the tables hold scratch offsets, not
 *      addresses, so scratch may be moved between calls.  nsec = conn_first[nconn] (host copy).
 *      in_size <= 2^32 - 3 (offsets are u32).  Encoder streams and sections must not overlap in `in`.
 *      Asynchronous on `stream`: a literal pre-pass (every literal of the step decoded at once), the
 *      encoder streams (one lane per connection, entries booked as references), a table pass, the
 *      sections (one lane per section) and a copy pass.  Stream-ordered pool workspace: 16 bytes per input
 *      byte of field sources, 22 per possible literal (one per input byte) and 1.6 of decoded output --
 *      about 40 bytes per input byte; kept by the pool after the call (hhuff_pool_trim). */
#define HHUFF_QPK_CONTINUE 1u
#define HHUFF_QPK_DECOMPRESSION_FAILED 0x30200 /* H2O_HTTP3_ERROR_QPACK_DECOMPRESSION_FAILED, http3_common.h:73 */
#define HHUFF_QPK_ARENA (-300)
#define HHUFF_QPK_SKIPPED (-301)
#define HHUFF_QPK_BLOCKED (-302)
uint64_t hhuff_qpack_scratch_size(uint32_t nconn, uint32_t header_table_size);
int hhuff_qpack_decode(const uint8_t *in, uint64_t in_size, const uint32_t *enc_off, const uint32_t *enc_len,
                       const uint32_t *sec_off, const uint32_t *conn_first, uint32_t nconn, uint32_t nsec,
                       uint32_t header_table_size, uint64_t max_blocked, const uint32_t *num_blocked, uint8_t *arena,
                       const uint64_t *arena_off, uint32_t *name_off, uint32_t *name_len, uint32_t *value_off,
                       uint32_t *value_len, uint8_t *fflags, uint32_t *nfields, int32_t *sstatus,
                       uint64_t *req_insert_count, int32_t *enc_status, uint32_t *enc_consumed, uint64_t *insert_count,
                       void *scratch, uint64_t scratch_size, unsigned flags, void *stream);

/* (2e') HTTP/3 request sections: the same step with h2o_qpack_parse_request (lib/http3/qpack.c:830-858)
 *      applied to every section as h2o's HTTP/3 server calls it (lib/http3/server.c:1540-1545): the
 *      section's fields go through h2o_hpack_parse_request's rules (qpack.c:848, hpack.c:502-637) with no
 *      cache-digest receiver (a cache-digest field is rejected like the other special fields) and a
 *      datagram-flow-id out-parameter; hard errors other than H2O_HTTP2_ERROR_INVALID_HEADER_CHAR become
 *      HHUFF_QPK_DECOMPRESSION_FAILED (normalize_error_code, :822-828); a section that decoded (0 or
 *      -254) with a Required Insert Count other than 0 gets its Section Acknowledgment (send_header_ack,
 *      :642-649: 0x80 | stream_id[k] as a 7-bit prefix integer) in req[k].ack.
 *      sstatus[k] is h2o_qpack_parse_request's return value: 0, -254 (a soft error, *err_desc in
 *      req[k].req.err), HHUFF_QPK_DECOMPRESSION_FAILED, or HHUFF_QPK_BLOCKED / _ARENA / _SKIPPED as for
 *      hhuff_qpack_decode.  fflags carries HHUFF_FIELD_HEADER for the fields h2o_add_header took.
 *      req[k].req.err is HHUFF_HERR_DECODE when decode_header itself failed (its own description). */
typedef struct hhuff_qpack_request {
    hhuff_request_t req;      /* h2o_hpack_parse_request's out-parameters, as for HTTP/2 */
    int32_t datagram_flow_id; /* the field whose value h2o stored in *datagram_flow_id, or -1 */
    uint32_t ack_len;         /* *outbufsize: bytes of ack (0: no acknowledgment) */
    uint8_t ack[16];          /* the Section Acknowledgment instruction */
} hhuff_qpack_request_t;      /* 72 bytes */
#define HHUFF_HERR_DECODE 8u /* a hard error inside QPACK's decode_header (qpack.c:652-752) */
int hhuff_qpack_parse_requests(const uint8_t *in, uint64_t in_size, const uint32_t *enc_off, const uint32_t *enc_len,
                               const uint32_t *sec_off, const uint32_t *conn_first, uint32_t nconn, uint32_t nsec,
                               uint32_t header_table_size, uint64_t max_blocked, const uint32_t *num_blocked,
                               uint8_t *arena, const uint64_t *arena_off, uint32_t *name_off, uint32_t *name_len,
                               uint32_t *value_off, uint32_t *value_len, uint8_t *fflags, uint32_t *nfields,
                               int32_t *sstatus, uint64_t *req_insert_count, int32_t *enc_status, uint32_t *enc_consumed,
                               uint64_t *insert_count, const uint64_t *stream_id, hhuff_qpack_request_t *req,
                               void *scratch, uint64_t scratch_size, unsigned flags, void *stream);

/* (2e'') HTTP/3 response sections, client side: the step of hhuff_qpack_decode with h2o_qpack_parse_response
 *      (lib/http3/qpack.c:860-882) applied to every section as h2o's HTTP/3 client calls it
 *      (lib/common/http3client.c:542-544: a status and a datagram-flow-id out-parameter; the client has no
 *      blocked-streams budget, so pass max_blocked = 0 to match it): h2o_hpack_parse_response's rules on the
 *      section's fields (as hhuff_hpack_parse_responses, heads only), every hard error -- -254 excepted --
 *      normalised to HHUFF_QPK_DECOMPRESSION_FAILED (:877-878), and the Section Acknowledgment only for a
 *      section that parsed with status 0 and a Required Insert Count other than 0 (:880).  sstatus[k] as for
 *      hhuff_qpack_parse_requests. */
typedef struct hhuff_qpack_response_head {
    hhuff_response_t res;  /* h2o_hpack_parse_response's out-parameters */
    uint32_t ack_len;      /* *outbufsize (0: no acknowledgment) */
    uint32_t reserved;
    uint8_t ack[16];       /* the Section Acknowledgment instruction */
} hhuff_qpack_response_head_t; /* 40 bytes */
int hhuff_qpack_parse_responses(const uint8_t *in, uint64_t in_size, const uint32_t *enc_off, const uint32_t *enc_len,
                                const uint32_t *sec_off, const uint32_t *conn_first, uint32_t nconn, uint32_t nsec,
                                uint32_t header_table_size, uint64_t max_blocked, const uint32_t *num_blocked,
                                uint8_t *arena, const uint64_t *arena_off, uint32_t *name_off, uint32_t *name_len,
                                uint32_t *value_off, uint32_t *value_len, uint8_t *fflags, uint32_t *nfields,
                                int32_t *sstatus, uint64_t *req_insert_count, int32_t *enc_status, uint32_t *enc_consumed,
                                uint64_t *insert_count, const uint64_t *stream_id, hhuff_qpack_response_head_t *res,
                                void *scratch, uint64_t scratch_size, unsigned flags, void *stream);

/* (2f) HTTP/2 response header blocks, encode side (SURVEY f4 encode half): h2o_hpack_flatten_response
 *      (lib/http2/hpack.c:1137-1177) and h2o_hpack_flatten_trailers (:1179-1196) -- and, for h2o's HTTP/2
 *      client (lib/common/http2client.c:1140), h2o_hpack_flatten_request (:1044-1096) -- for many responses of many
 *      connections, with one encoder dynamic table per connection (conn->_output_header_table; do_encode_header
 *      :858-937, at most 32 entries, initial capacity 4096 as lib/http2/connection.c:1847 sets it) kept in
 *      scratch between calls.  A call flattens the responses conn_first[c] .. conn_first[c+1]-1 of every
 *      connection c in order, as lib/http2/stream.c:311-314 / :404-406 and connection.c:1580-1582 call them.
 *        header h    hdr[h]: name in[name_off .. + name_len), value in[value_off .. + value_len), flags:
 *                    HHUFF_HDR_DONT_COMPRESS = h2o_header_t.flags.dont_compress; HHUFF_HDR_TOKEN = the name is
 *                    an h2o token (h2o_iovec_is_token: the header was added with its h2o_token_t) -- set it only
 *                    for names listed in lib/common/token_table.h
 *        response r  res[r] (below): the headers hdr_first .. hdr_first + nhdr - 1 in order (the ranges of two
 *                    responses must not overlap; headers outside every range are ignored); HHUFF_RES_SERVER
 *                    sends server_name (in[server_off .. + server_len), h2o's globalconf->server_name; clear
 *                    it where h2o passes NULL: informational responses); HHUFF_RES_TRAILERS makes r a trailers
 *                    block (flatten_trailers: no :status, server or content-length, END_STREAM);
 *                    HHUFF_RES_REQUEST makes r a request (flatten_request: no :status, server or content-length):
 *                    its first `status` headers are flatten_request's own fields in its order -- :method,
 *                    :scheme, :authority, :path (an old-style CONNECT, method CONNECT without :protocol, has no
 *                    :scheme or :path), :protocol if any, "expect: 100-continue" if send_own_expect -- with
 *                    HHUFF_HDR_TOKEN and no HHUFF_HDR_DONT_COMPRESS; :method GET / POST, :scheme https / http,
 *                    :path / and /index.html among them, and accept-encoding "gzip, deflate" (token) among the
 *                    others, are the one-byte static references h2o writes without its table (:950-985,
 *                    :1083-1086; a scheme named https / http is h2o's H2O_URL_SCHEME_HTTPS / _HTTP)
 *        out         response r's frames (HEADERS, then CONTINUATIONs past max_frame_size, fixup_frame_headers
 *                    :1012-1042) at out + out_off[r]; region [out_off[r], out_off[r+1]) (u64, nres + 1 entries);
 *                    hhuff_hpack_response_bound() is enough for any table state
 *      Per response: out_len[r] = bytes written (frame headers included), headers_size[r] = the payload bytes
 *      (h2o_hpack_flatten_response's return value), rstatus[r] = 0, HHUFF_RES_SPACE (the frames do not fit
 *      the region), HHUFF_RES_EINVAL (status outside 100..999 -- past nhdr for a request --, max_frame_size outside 16384..2^24-1, a string
 *      past in_size) or HHUFF_RES_SKIPPED (an earlier response of the connection failed: its table is no
 *      longer the peer's, h2o would have dropped the connection).  A failed response writes nothing.
 *      Device arrays; scratch = hhuff_hpack_enc_scratch_size(nconn) bytes (16-byte aligned) holding the
 *      tables: HHUFF_ENC_CONTINUE carries them (and the failed state) over from the previous call; without it
 *      every connection starts with an empty table.  nhdr = headers in hdr, nres = conn_first[nconn] (host
 *      copies).  in_size < 2^32.  Asynchronous on `stream`; stream-ordered pool workspace of 36 bytes per
 *      header and 16 per response (hhuff_pool_trim). */
typedef struct hhuff_hpack_header {
    uint32_t name_off, name_len, value_off, value_len;
    uint32_t flags; /* HHUFF_HDR_* */
} hhuff_hpack_header_t; /* 20 bytes */
#define HHUFF_HDR_DONT_COMPRESS 1u
#define HHUFF_HDR_TOKEN 2u
typedef struct hhuff_hpack_response {
    uint64_t content_length;    /* res.content_length: SIZE_MAX (all ones) sends none */
    uint32_t stream_id, status; /* status: res.status (ignored for trailers; own fields of a request) */
    uint32_t hdr_first, nhdr;
    uint32_t header_table_size; /* conn->peer_settings.header_table_size (header_table_adjust_size, :839-856) */
    uint32_t max_frame_size;    /* conn->peer_settings.max_frame_size */
    uint32_t flags;             /* HHUFF_RES_* */
    uint32_t reserved;          /* 0 */
} hhuff_hpack_response_t;       /* 40 bytes */
#define HHUFF_RES_END_STREAM 1u /* is_end_stream */
#define HHUFF_RES_SERVER 2u     /* server_name != NULL */
#define HHUFF_RES_TRAILERS 4u   /* h2o_hpack_flatten_trailers */
#define HHUFF_RES_REQUEST 8u    /* h2o_hpack_flatten_request (status = the number of its own fields) */
#define HHUFF_ENC_CONTINUE 1u
#define HHUFF_RES_SPACE (-300)
#define HHUFF_RES_SKIPPED (-301)
#define HHUFF_RES_EINVAL (-303)
/* A region size that holds response r whatever its connection's table: name_value_bytes = the sum of its
 * headers' name_len + value_len, server_len = 0 without HHUFF_RES_SERVER.  (h2o's own reservation,
 * hpack.c:1141-1152 with calc_capacity :998-1001, plus the CONTINUATION frame headers.) */
static inline uint64_t hhuff_hpack_response_bound(uint64_t name_value_bytes, uint32_t nhdr, uint32_t server_len,
                                                  uint32_t max_frame_size)
{
    uint64_t payload = name_value_bytes + 21ull * nhdr + 5 + 5 + (server_len ? 5ull + server_len + 21 : 0) + 23;
    return 9 + payload + 9 * (payload / (max_frame_size ? max_frame_size : 1) + 1);
}
uint64_t hhuff_hpack_enc_scratch_size(uint32_t nconn);
int hhuff_hpack_flatten_responses(const uint8_t *in, uint64_t in_size, const hhuff_hpack_header_t *hdr, uint32_t nhdr,
                                  const hhuff_hpack_response_t *res, const uint32_t *conn_first, uint32_t nconn,
                                  uint32_t nres, uint32_t server_off, uint32_t server_len, uint8_t *out,
                                  const uint64_t *out_off, uint32_t *out_len, uint32_t *headers_size, int32_t *rstatus,
                                  void *scratch, uint64_t scratch_size, unsigned flags, void *stream);

/* (2g) HTTP/3 response HEADERS frames (QPACK encode half): h2o_qpack_flatten_response
 *      (lib/http3/qpack.c:1352-1399) as h2o's HTTP/3 server calls it (lib/http3/server.c:1680-1683): without an
 *      encoder-stream buffer, so the encoder never inserts into its dynamic table (:1175-1176) and every response
 *      stands alone -- :status, server (HHUFF_RES_SERVER), content-length, the headers (static-table references
 *      through h2o_qpack_lookup_static for token names, literals otherwise; do_flatten_header :1148-1213),
 *      datagram-flow-id (HHUFF_QRES_DATAGRAM: in[dfid_off .. + dfid_len)), behind the section prefix 00 00 and
 *      the HEADERS frame header (type 0x01, QUIC varint length; finalize_flatten :1265-1310).
 *        header h    hdr[h] as for hhuff_hpack_flatten_responses (HHUFF_HDR_TOKEN, HHUFF_HDR_DONT_COMPRESS); the
 *                    ranges hdr_first .. + nhdr of two responses must not overlap
 *        request     HHUFF_QRES_REQUEST: h2o_qpack_flatten_request (:1312-1350) as h2o's HTTP/3 client calls it
 *                    (lib/common/http3client.c:792, no encoder-stream buffer): no :status, server or content-length;
 *                    the headers start with its own fields as for HHUFF_RES_REQUEST (no expect: HTTP/3 has no
 *                    send_own_expect), which flatten exactly as token headers do (its static-indexed http / https
 *                    scheme, :1325-1329, is the static lookup's exact match); datagram-flow-id last as for responses
 *        out         frame r at out + out_off[r]; region [out_off[r], out_off[r+1]) (u64, nres + 1 entries):
 *                    hhuff_qpack_response_bound() always fits
 *      out_len[r] = frame bytes, header_len[r] = *serialized_header_len (the field section, frame header
 *      excluded), rstatus[r] = 0, HHUFF_RES_SPACE or HHUFF_RES_EINVAL (a string past in_size); a failed
 *      response writes nothing.  Device arrays; in_size < 2^32; asynchronous on `stream`; stream-ordered pool
 *      workspace of 24 bytes per header and 32 per response. */
typedef struct hhuff_qpack_response {
    uint64_t content_length; /* res.content_length: SIZE_MAX (all ones) sends none */
    uint32_t status;         /* res.status: a static entry, else the decimal of (uint16_t)status against :status;
                                HHUFF_QRES_REQUEST: the number of own fields (the bytes do not depend on it) */
    uint32_t hdr_first, nhdr;
    uint32_t flags;          /* HHUFF_RES_SERVER, HHUFF_QRES_DATAGRAM */
    uint32_t dfid_off, dfid_len;
} hhuff_qpack_response_t;    /* 32 bytes */
#define HHUFF_QRES_DATAGRAM 8u
#define HHUFF_QRES_REQUEST 16u /* h2o_qpack_flatten_request: status = the number of its own fields */
static inline uint64_t hhuff_qpack_response_bound(uint64_t name_value_bytes, uint32_t nhdr, uint32_t server_len,
                                                  uint32_t dfid_len)
{
    return 9 + 2 + 8 + 23 + 26 + (uint64_t)dfid_len + (server_len ? 12ull + server_len : 0) + 21ull * nhdr +
           name_value_bytes;
}
int hhuff_qpack_flatten_responses(const uint8_t *in, uint64_t in_size, const hhuff_hpack_header_t *hdr, uint32_t nhdr,
                                  const hhuff_qpack_response_t *res, uint32_t nres, uint32_t server_off,
                                  uint32_t server_len, uint8_t *out, const uint64_t *out_off, uint32_t *out_len,
                                  uint32_t *header_len, int32_t *rstatus, void *stream);

/* (3b) Pipelined host path (the socket-buffer -> pinned -> device -> pinned -> pool staging of
 *     SURVEY f3; replaces the caller-side copies around lib/http2/hpack.c:240-241).  Contiguous layout
 *     (in_off[n + 1], implicit output slots) only.  The batch is cut into chunks of about
 *     `chunk_bytes` input bytes (0 = 64 MiB) at multiples of 32 strings; chunks flow through three
 *     streams so that host staging copies, H2D, kernels and D2H of different chunks overlap.  Caller
 *     buffers already pinned (hipHostMalloc / hipHostRegister) are DMA'd directly.  Synchronous; the
 *     results equal hhuff_*_batch_host's.  hhuff_*_batch_host take this path by themselves for
 *     contiguous batches of 128 MiB and more. */
int hhuff_decode_batch_host_pipelined(const uint8_t *in, uint64_t in_size, const uint32_t *in_off, uint32_t n,
                                      const uint32_t *is_name_bits, uint8_t *out, uint64_t out_size,
                                      uint32_t *out_len, uint8_t *status, int device, uint64_t chunk_bytes);
int hhuff_encode_batch_host_pipelined(const uint8_t *in, uint64_t in_size, const uint32_t *in_off, uint32_t n,
                                      uint8_t *out, uint64_t out_size, uint32_t *out_len, uint8_t *status,
                                      int device, uint64_t chunk_bytes);

/* (3c) Packed host path: hhuff_decode_batch_packed / hhuff_encode_batch_packed on host arrays (same layout: every
 *     64-string tile's outputs back to back from the tile's slot position, out_off[n + 1]).  Contiguous layout.
 *     With every array pinned (hipHostMalloc / hipHostRegister), `in` and `out` 16-byte aligned and the u32 arrays
 *     4-byte aligned, the kernels read the input and write the results in host memory themselves and only the
 *     output bytes cross PCIe (the slot layout's unused slot tails do not); otherwise the call stages the batch
 *     through device memory.  out_size >= the slot end (decode floor(8 in_off[n] / 5), encode in_off[n]).
 *     out_off may be NULL: the offsets are then not returned (4 bytes a string fewer across the link) and string i
 *     starts at its tile's position (decode floor(8 in_off[64 t] / 5), encode in_off[64 t], t = i / 64) plus the
 *     out_len of the tile's earlier strings that did not fail.  An encode's status may be NULL (out_len already
 *     says HHUFF_FAIL_LEN); a decode's may not.  Synchronous. */
int hhuff_decode_batch_host_packed(const uint8_t *in, uint64_t in_size, const uint32_t *in_off, uint32_t n,
                                   const uint32_t *is_name_bits, uint8_t *out, uint64_t out_size, uint32_t *out_off,
                                   uint32_t *out_len, uint8_t *status, int device);
int hhuff_encode_batch_host_packed(const uint8_t *in, uint64_t in_size, const uint32_t *in_off, uint32_t n,
                                   uint8_t *out, uint64_t out_size, uint32_t *out_off, uint32_t *out_len,
                                   uint8_t *status, int device);

/* (3d) Multi-device batch (SURVEY 2 new component 5, 8e): one batch over several GPUs of one process, for h2o's
 *     C callers (lib/http2/hpack.c:241, lib/http3/qpack.c:228 -- worker threads, src/main.c:5512) that have no
 *     torch.distributed.  The contiguous layout of hhuff_decode_batch / hhuff_encode_batch (in_off[n + 1], implicit
 *     output slots: decode floor(8 in_off[i] / 5), encode in_off[i]) is cut byte-balanced into ndev shards
 *     (hhuff_shard_bounds with align 64) and shard k runs on devices[k] (NULL: devices 0 .. ndev-1).  Offsets
 *     stay absolute, so every string lands where the one-device call puts it: the shards' outputs are already
 *     concatenated in shard order, and out_len / status are byte for byte the one-device call's.
 *       src_device == HHUFF_HOST_MEMORY: every array is host memory; each device runs its shard through the host
 *         path (zero copy on pinned, aligned arrays, else the chunked pipeline of 3b), all devices at once, each
 *         from its own library thread.  Synchronous; `stream` is ignored.
 *       src_device >= 0: every array is device memory of src_device, ordered on `stream` (a stream of src_device,
 *         NULL the null stream).  The call waits for the work queued before it on `stream` (the cut reads
 *         in_off), then enqueues: the src device's own shard in place on an internal stream of src_device, every
 *         other shard as peer copies (xGMI) of its input bytes, offsets and name bits to scratch on its device,
 *         the kernel there, and peer copies of its output slots, lengths and statuses back; `stream` then waits
 *         for every shard.  Returns once all is enqueued (asynchronous, like hhuff_decode_batch).
 *     ndev == 1 with devices[0] == src_device is the one-device call. */
#define HHUFF_HOST_MEMORY (-1)
int hhuff_decode_batch_multi(int ndev, const int *devices, int src_device, const uint8_t *in, uint64_t in_size,
                             const uint32_t *in_off, uint32_t n, const uint32_t *is_name_bits, uint8_t *out,
                             uint64_t out_size, uint32_t *out_len, uint8_t *status, void *stream);
int hhuff_encode_batch_multi(int ndev, const int *devices, int src_device, const uint8_t *in, uint64_t in_size,
                             const uint32_t *in_off, uint32_t n, uint8_t *out, uint64_t out_size, uint32_t *out_len,
                             uint8_t *status, void *stream);
/* The byte-balanced cut (host arrays, no GPU): bounds[0] = 0, bounds[nshards] = n and, for 0 < k < nshards,
 * bounds[k] = the first string i with in_off[i] >= in_off[0] + floor(k (in_off[n] - in_off[0]) / nshards), rounded
 * down to a multiple of `align` (0 or 1: no rounding).  Non-decreasing.  With align 1 it equals h2o_amd/dist.py
 * byte_balanced_bounds (the torch.distributed path's split). */
int hhuff_shard_bounds(const uint32_t *in_off, uint32_t n, uint32_t nshards, uint32_t align, uint32_t *bounds);

/* ---------------------------------------------------------------------------------------------
 * (4) library info
 * ------------------------------------------------------------------------------------------- */
const char *hhuff_version(void);
/* Text of the last HIP error seen by this thread ("" if none). */
const char *hhuff_last_error_string(void);
/* Number of workgroups the decode / encode launches use on `device` (grid sizing, for profiling). */
/* The prices a mixed-length decode (mean Huffman length 41..128 B) uses to choose between the staged and the
 * stream kernel: out4 = {staged ps per string, staged ps per tile-padded byte, stream ps per string, stream ps
 * per byte}.  A decode never measures them itself: they are fitted MI355X defaults until
 * hhuff_calibrate_decode_prices or hhuff_set_decode_prices runs for the device.  No GPU work.  HHUFF_OK or an
 * error code. */
int hhuff_decode_prices(int device, float *out4);
/* Measure this device's prices now (both kernels timed on two probe batches, about 2 ms; synchronous: it
 * allocates and frees device memory, so call it at start-up, not beside in-flight work) and use them from
 * then on; out4 (may be NULL) receives them.  A failed or implausible fit keeps the prices in effect. */
int hhuff_calibrate_decode_prices(int device, float *out4);
/* Pin the prices of `device` (e.g. a previous calibration's, so every process chooses alike); in4 NULL
 * restores the fitted defaults.  HHUFF_EINVAL for a negative or non-finite value. */
int hhuff_set_decode_prices(int device, const float *in4);
int hhuff_grid_size(int device, int which /* 0 decode, 1 encode */);
/* Which kernel decodes contiguous batches (process-wide; the results are the same, only the speed differs):
 * 0 (default) the staged kernels for short strings and the device-side staged / stream choice for mixed and long
 * ones.  Modes 1 and 2 (the segment kernel -- a tile's bits shared evenly over a wave's lanes -- above a 40-B mean,
 * or for every contiguous batch) exist only in A/B builds of the library (tools/ab.py, -DHHUFF_AB_VARIANTS=1; there
 * HHUFF_DEC_SEG sets the start value): the product library accepts 0 and returns HHUFF_EINVAL for them.
 * Returns the previous mode, or HHUFF_EINVAL. */
int hhuff_set_decode_kernel(int mode);
/* Batches of at least `n` strings leave the 16-B output chunks their tiles share to edge records and a fix-up
 * kernel launched behind the codec kernel; smaller batches store those chunks in the codec kernel (one launch).
 * Default 0xFFFFFFFF: every batch stores them in the kernel.  Process-wide; the results are the same, only the
 * speed differs.  Returns the previous value. */
uint32_t hhuff_set_edge_defer_min(uint32_t n);
/* Return the memory the library's stream-ordered pool on the caller's current device keeps between calls
 * (batch workspaces, edge records) to the driver.  Synchronises the device first.  HHUFF_OK or an error. */
int hhuff_pool_trim(void);

#ifdef __cplusplus
}
#endif
#endif
