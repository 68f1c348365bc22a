// HTTP/2 response header blocks on the GPU, encode side (SURVEY.md 8 f4 encode half):
// h2o_hpack_flatten_response (lib/http2/hpack.c:1137-1177) and h2o_hpack_flatten_trailers (:1179-1196) for
// many connections, each with its encoder dynamic table (do_encode_header :858-937, header_table_add
// :277-317 with at most 32 entries, header_table_adjust_size :839-856).
//
// What a field becomes depends on the table, and the table on every earlier field of the connection, so
// the table work is sequential per connection -- but it needs no output bytes: only lengths and equality.
//   1. prep (hpe_prep_kernel, one lane per header): a 32-bit FNV-1a hash of the name and of the value, the
//      Huffman code bits of each (h2o_hpack_encode_string's length: Huffman when strictly shorter,
//      hpack.c:816-837), and the token facts do_encode_header reads (static name index, dont_compress);
//   2. the walk (hpe_table_kernel, one lane per connection): the table search (hash and length first, bytes
//      only on a hash hit), the representation of each field, its byte length, hence its position in the
//      response; table entries are references to the bytes (this call's input, or the connection's ring);
//   3. emit (hpe_emit_kernel, one lane per field and one per response head): every field writes its own
//      bytes at its place -- prefix integers, raw copies, Huffman codes (encode_core) -- through a register
//      sink, so fields of one response are written in parallel and nothing is written twice;
//   4. frames (hpe_frames_kernel, one workgroup per response longer than max_frame_size): the payload moves
//      apart for the CONTINUATION frame headers, last chunk first (fixup_frame_headers :1012-1042);
//   5. the table pass (hpe_ring_kernel, one wave per connection) copies the live entries' bytes into the
//      connection's other ring, so the next call (HHUFF_ENC_CONTINUE) reads only scratch.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

#include "hhuff.h"
#include "hhuff_device.h"
#include "hhuff_launch.h"
#include "hhuff_tables.h"

namespace hhuff {
namespace {
__device__ const uint32_t e_enc_code[256] = HHUFF_ENC_CODE_INIT;
__device__ const uint8_t e_enc_nbits[256] = HHUFF_ENC_NBITS_INIT;
__device__ const uint8_t e_static_bytes[HHUFF_STATIC_NBYTES] = HHUFF_STATIC_BYTES_INIT;
__device__ const uint16_t e_static_ent[61 * 4] = HHUFF_STATIC_ENT_INIT;
__device__ const uint8_t e_server[8] = {'s', 'e', 'r', 'v', 'e', 'r', 0, 0};

constexpr uint32_t kOverhead = 32;     // HEADER_TABLE_ENTRY_SIZE_OFFSET (hpack.c:30)
constexpr uint32_t kTableOffset = 62;  // HEADER_TABLE_OFFSET (hpack.c:29)
constexpr uint32_t kMaxEntries = 32;   // header_table_add(..., 32) (hpack.c:921)
constexpr uint32_t kInitialCap = 4096; // conn->_output_header_table.hpack_capacity (connection.c:1847)
constexpr uint32_t kRing = 4096;       // live entry bytes never exceed the capacity (<= 4096)
constexpr uint32_t kServerIndex = 54;  // H2O_TOKEN_SERVER's http2_static_table_name_index

// info word of a prepped string pair
constexpr uint32_t kInfoStatic = 0x7Fu;  // static name index (tokens only)
constexpr uint32_t kInfoTokDc = 1u << 8;  // token flag dont_compress (cookie, set-cookie)
constexpr uint32_t kInfoTok = 1u << 9;
constexpr uint32_t kInfoHdrDc = 1u << 10;
constexpr uint32_t kInfoBad = 1u << 11;  // a string past in_size

// op code of a field
constexpr uint32_t kOpIndexed = 0, kOpIdxName = 1, kOpNever = 2, kOpNewName = 3;
constexpr uint32_t kOpAsIs = 1u << 9;  // the value goes as it is (encode_as_is, hpack.c:806-814)
constexpr uint32_t kOpSkip = 1u << 31;

// byte sources of a table entry's name / value
constexpr uint64_t kSrcIn = 0;               // input offset (added in this call)
constexpr uint64_t kSrcScr = 1ull << 62;     // scratch offset (a ring: added by an earlier call)
constexpr uint64_t kSrcConst = 2ull << 62;   // e_server
constexpr uint64_t kSrcOff = (1ull << 62) - 1;

struct EncState {
    uint32_t start, num, ring, failed;
    uint32_t size, cap, pad0, pad1;
};
struct EncEntry {
    uint64_t nsrc, vsrc;
    uint32_t nl, vl, nh, vh;
    uint32_t tok, pad;
};
static_assert(sizeof(EncState) == 32 && sizeof(EncEntry) == 40, "scratch records");
constexpr uint64_t kConnScratch = sizeof(EncState) + kMaxEntries * sizeof(EncEntry) + 2 * kRing;
static_assert(kConnScratch % 16 == 0, "scratch alignment");
}  // namespace

struct HpeArgs {
    const uint8_t* in;
    uint64_t in_size;
    const hhuff_hpack_header_t* hdr;
    uint32_t nhdr;
    const hhuff_hpack_response_t* res;
    const uint32_t* conn_first;
    uint32_t nconn, nres;
    uint32_t server_off, server_len;
    uint8_t* out;
    const uint64_t* out_off;
    uint32_t* out_len;
    uint32_t* headers_size;
    int32_t* rstatus;
    uint8_t* scratch;
    uint32_t flags;
    // workspace
    uint4* rec;      // [nhdr + 1] {name hash, value hash, name code bits, value code bits}; item nhdr: server
    uint32_t* info;  // [nhdr + 1]
    uint4* op;       // [nhdr] {dst lo, dst hi, code, 0}
    uint4* plan;     // [2 nres] {base lo, base hi, payload, total} {size update or ~0, server code, server pos, cl len}
    uint32_t* big;   // [nres + 1]: count, then the responses longer than their max_frame_size
};

namespace {
__device__ __forceinline__ const uint8_t* hpe_src(const HpeArgs& A, uint64_t s) {
    const uint64_t o = s & kSrcOff;
    switch (s >> 62) {
        case 0: return A.in + o;
        case 1: return A.scratch + o;
        default: return e_server + o;
    }
}

__device__ __forceinline__ uint32_t int_len(uint32_t v, uint32_t p) {  // h2o_hpack_encode_int's length (hpack.c:757-772)
    const uint32_t pmax = (1u << p) - 1u;
    if (v < pmax) return 1;
    v -= pmax;
    uint32_t n = 2;
    while (v >= 128) {
        v >>= 7;
        ++n;
    }
    return n;
}

__device__ __forceinline__ bool huff_wins(uint32_t len, uint32_t bits) {  // hpack.c:789-791, :799-800
    return len != 0 && bits <= 8u * len - 8u;
}

__device__ __forceinline__ uint32_t str_len(uint32_t len, uint32_t bits) {  // h2o_hpack_encode_string's length
    if (huff_wins(len, bits)) {
        const uint32_t hb = (bits + 7u) >> 3;
        return int_len(hb, 7) + hb;
    }
    return int_len(len, 7) + len;
}

__device__ __forceinline__ uint32_t digits(uint64_t v) {
    uint32_t n = 1;
    while (v >= 10) {
        v /= 10;
        ++n;
    }
    return n;
}

// FNV-1a over the bytes and their Huffman code bits, one pass
__device__ __forceinline__ void hash_bits(const uint8_t* p, uint32_t len, const uint8_t* nbits, uint32_t& h, uint32_t& bits) {
    h = 2166136261u;
    bits = 0;
    for (uint32_t k = 0; k < len; ++k) {
        const uint32_t b = p[k];
        h = (h ^ b) * 16777619u;
        bits += nbits[b];
    }
}

__device__ __forceinline__ bool lit_eq(const uint8_t* a, const char* lit, uint32_t n) {
    for (uint32_t k = 0; k < n; ++k)
        if (a[k] != (uint8_t)lit[k]) return false;
    return true;
}

__device__ __forceinline__ bool same_bytes(const uint8_t* a, const uint8_t* b, uint32_t n) {
    for (uint32_t k = 0; k < n; ++k)
        if (a[k] != b[k]) return false;
    return true;
}
}  // namespace

// 1. prep: one lane per header (item nhdr: the server name under the server token)
__global__ __launch_bounds__(256) void hpe_prep_kernel(HpeArgs A) {
    __shared__ uint8_t s_nbits[256];
    s_nbits[threadIdx.x] = e_enc_nbits[threadIdx.x];
    __syncthreads();
    for (uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x; i <= A.nhdr; i += (uint64_t)gridDim.x * 256u) {
        uint32_t nh, vh, nb = 0, vb = 0, info;
        if (i == A.nhdr) {
            hash_bits(e_server, 6, s_nbits, nh, nb);
            const bool bad = (uint64_t)A.server_off + A.server_len > A.in_size;
            hash_bits(A.in + A.server_off, bad ? 0u : A.server_len, s_nbits, vh, vb);
            info = kServerIndex | kInfoTok | (bad ? kInfoBad : 0u);
        } else {
            const hhuff_hpack_header_t H = A.hdr[i];
            const bool bad = (uint64_t)H.name_off + H.name_len > A.in_size || (uint64_t)H.value_off + H.value_len > A.in_size;
            const uint32_t nl = bad ? 0u : H.name_len, vl = bad ? 0u : H.value_len;
            const uint8_t* n = A.in + H.name_off;
            hash_bits(n, nl, s_nbits, nh, nb);
            hash_bits(A.in + H.value_off, vl, s_nbits, vh, vb);
            info = (bad ? kInfoBad : 0u) | ((H.flags & HHUFF_HDR_DONT_COMPRESS) ? kInfoHdrDc : 0u);
            if (H.flags & HHUFF_HDR_TOKEN) {
                // lib/common/token_table.h: a token's http2_static_table_name_index is the first static
                // entry with its name; dont_compress is set for cookie and set-cookie
                uint32_t sidx = 0;
                for (uint32_t k = 0; k < 61 && sidx == 0; ++k)
                    if (e_static_ent[4 * k + 1] == nl && same_bytes(e_static_bytes + e_static_ent[4 * k], n, nl)) sidx = k + 1;
                const bool dc = (nl == 6 && lit_eq(n, "cookie", 6)) || (nl == 10 && lit_eq(n, "set-cookie", 10));
                info |= kInfoTok | sidx | (dc ? kInfoTokDc : 0u);
            }
        }
        A.rec[i] = make_uint4(nh, vh, nb, vb);
        A.info[i] = info;
    }
}

namespace {
struct EncTable {  // one connection's encoder table (newest entry = index 62)
    EncEntry* ent;
    uint32_t start, num, size, cap;
    __device__ __forceinline__ uint32_t slot(uint32_t k) const {
        const uint32_t i = start + k;
        return i >= kMaxEntries ? i - kMaxEntries : i;
    }
    __device__ __forceinline__ void evict_one() {  // header_table_evict_one (hpack.c:263-275)
        --num;
        const uint2 l = *reinterpret_cast<const uint2*>(&ent[slot(num)].nl);
        size -= l.x + l.y + kOverhead;
    }
    __device__ void add(const EncEntry& e) {  // header_table_add (hpack.c:277-317), at most 32 entries
        const uint32_t add = e.nl + e.vl + kOverhead;
        while (num != 0 && size + add > cap) evict_one();
        while (num >= kMaxEntries) evict_one();
        if (num == 0 && add > cap) return;
        start = start == 0 ? kMaxEntries - 1 : start - 1;
        ent[start] = e;
        size += add;
        ++num;
    }
};

// do_encode_header (hpack.c:858-937) on item i (a header, or the server name): returns the op code and
// its byte length, and updates the table as h2o does
__device__ uint32_t hpe_field(const HpeArgs& A, EncTable& t, uint32_t i, uint64_t nsrc, uint32_t nl, uint64_t vsrc, uint32_t vl,
                              uint32_t& len) {
    const uint4 rc = A.rec[i];
    const uint32_t info = A.info[i];
    const bool tok = (info & kInfoTok) != 0;
    uint32_t name_index = info & kInfoStatic;  // 0 for non-tokens
    const uint8_t* np = hpe_src(A, nsrc);
    const uint8_t* vp = hpe_src(A, vsrc);
    for (uint32_t k = 0; k < t.num; ++k) {  // newest first (:864-890)
        const EncEntry& e = t.ent[t.slot(k)];
        const uint4 q = *reinterpret_cast<const uint4*>(&e.nl);  // nl, vl, nh, vh
        if (q.x != nl || q.z != rc.x) continue;
        if (tok && !e.tok) continue;  // a token name is compared by pointer (:870-872)
        if (!same_bytes(np, hpe_src(A, e.nsrc), nl)) continue;
        if (!tok && name_index == 0) name_index = k + kTableOffset;  // :875-876
        if (q.y != vl || q.w != rc.y || !same_bytes(vp, hpe_src(A, e.vsrc), vl)) continue;
        len = int_len(k + kTableOffset, 7);  // indexed (:881-884)
        return kOpIndexed | ((k + kTableOffset) << 2);
    }
    bool dc = (info & kInfoHdrDc) != 0;
    if (!dc && tok) dc = (info & kInfoTokDc) != 0;  // :892-893
    if (dc) dc = vl < 20;                           // :894-895
    uint32_t code;
    if (name_index != 0) {
        code = (dc ? kOpNever : kOpIdxName) | (name_index << 2);
        len = int_len(name_index, dc ? 4u : 6u);
    } else {
        code = kOpNewName;
        len = 1u + str_len(nl, rc.z);
    }
    if (dc) {
        len += int_len(vl, 7) + vl;
        code |= kOpAsIs;
    } else {
        len += str_len(vl, rc.w);
        t.add(EncEntry{nsrc, vsrc, nl, vl, rc.x, rc.y, tok ? 1u : 0u, 0u});
    }
    return code;
}
}  // namespace

// 2. the walk: one lane per connection, its responses in order
__global__ __launch_bounds__(256) void hpe_table_kernel(HpeArgs A) {
    for (uint64_t c = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; c < A.nconn; c += (uint64_t)gridDim.x * blockDim.x) {
        uint8_t* scr = A.scratch + c * kConnScratch;
        EncState* ts = reinterpret_cast<EncState*>(scr);
        EncState s0{0u, 0u, 0u, 0u, 0u, kInitialCap, 0u, 0u};
        if (A.flags & HHUFF_ENC_CONTINUE) s0 = *ts;
        EncTable t{reinterpret_cast<EncEntry*>(scr + sizeof(EncState)), s0.start, s0.num, s0.size, s0.cap};
        bool failed = s0.failed != 0;
        for (uint32_t r = A.conn_first[c]; r < A.conn_first[c + 1]; ++r) {
            const hhuff_hpack_response_t R = A.res[r];
            const bool trailers = (R.flags & HHUFF_RES_TRAILERS) != 0;
            const bool server = !trailers && (R.flags & HHUFF_RES_SERVER) && A.server_len != 0;
            int32_t st = 0;
            if (failed) {
                st = HHUFF_RES_SKIPPED;
            } else {
                bool bad = (!trailers && (R.status < 100 || R.status > 999)) || R.max_frame_size < 16384u ||
                           R.max_frame_size > 0xFFFFFFu || (server && (A.info[A.nhdr] & kInfoBad));
                for (uint32_t h = R.hdr_first; h < R.hdr_first + R.nhdr && !bad; ++h) bad = (A.info[h] & kInfoBad) != 0;
                if (bad) st = HHUFF_RES_EINVAL;
            }
            uint32_t pos = 0, su = ~0u, scode = 0, spos = 0, cll = 0;
            const uint64_t base = A.out_off[r];
            if (st == 0) {
                if (R.header_table_size < t.cap) {  // header_table_adjust_size (:839-856)
                    t.cap = R.header_table_size;
                    while (t.num != 0 && t.size > t.cap) t.evict_one();
                    su = t.cap;
                    pos += int_len(su, 5);
                }
                if (!trailers) {
                    const uint32_t s = R.status;  // encode_status (:437-466)
                    pos += (s == 200 || s == 204 || s == 206 || s == 304 || s == 400 || s == 404 || s == 500) ? 1u : 5u;
                }
                if (server) {  // :1159-1163, encode_header_token(H2O_TOKEN_SERVER)
                    uint32_t l;
                    spos = pos;
                    scode = hpe_field(A, t, A.nhdr, kSrcConst, 6, kSrcIn | A.server_off, A.server_len, l);
                    pos += l;
                }
                for (uint32_t h = R.hdr_first; h < R.hdr_first + R.nhdr; ++h) {
                    const hhuff_hpack_header_t H = A.hdr[h];
                    uint32_t l;
                    const uint32_t code = hpe_field(A, t, h, kSrcIn | H.name_off, H.name_len, kSrcIn | H.value_off, H.value_len, l);
                    const uint64_t dst = base + 9u + pos;
                    A.op[h] = make_uint4((uint32_t)dst, (uint32_t)(dst >> 32), code, 0u);
                    pos += l;
                }
                if (!trailers && R.content_length != ~0ull) {  // encode_content_length (:468-485)
                    cll = 3u + digits(R.content_length);
                    pos += cll;
                }
                const uint32_t M = R.max_frame_size;
                const uint64_t total = 9ull + pos + (pos > M ? 9ull * ((pos - 1u) / M) : 0ull);
                if (total > A.out_off[r + 1] - base) {
                    st = HHUFF_RES_SPACE;
                } else {
                    A.out_len[r] = (uint32_t)total;
                    A.headers_size[r] = pos;
                    A.plan[2 * r] = make_uint4((uint32_t)base, (uint32_t)(base >> 32), pos, (uint32_t)total);
                    A.plan[2 * r + 1] = make_uint4(su, server ? scode : kOpSkip, spos, cll);
                    if (pos > M) A.big[1 + atomicAdd(A.big, 1u)] = r;
                }
            }
            if (st != 0) {
                A.out_len[r] = 0;
                A.headers_size[r] = 0;
                A.plan[2 * r + 1] = make_uint4(~0u, kOpSkip, 0u, 0u);
                A.plan[2 * r] = make_uint4(0u, 0u, 0u, 0u);
                for (uint32_t h = R.hdr_first; h < R.hdr_first + R.nhdr; ++h) A.op[h] = make_uint4(0u, 0u, kOpSkip, 0u);
                failed = true;
            }
            A.rstatus[r] = st;
        }
        *ts = EncState{t.start, t.num, s0.ring, failed ? 1u : 0u, t.size, t.cap, 0u, 0u};
    }
}

namespace {
__device__ __forceinline__ void sink_int(RegSink& sink, uint32_t first, uint32_t v, uint32_t p) {  // hpack.c:757-772
    const uint32_t pmax = (1u << p) - 1u;
    if (v < pmax) {
        sink.put1(first | v);
        return;
    }
    sink.put1(first | pmax);
    v -= pmax;
    while (v >= 128) {
        sink.put1(0x80u | (v & 127u));
        v >>= 7;
    }
    sink.put1(v);
}

__device__ __forceinline__ void sink_raw(RegSink& sink, const GlobalSource& src, uint32_t s, uint32_t len) {
    uint32_t a = s & ~3u, rem = len, skip = s & 3u;
    while (rem) {
        const uint32_t w = src.word(a) >> (8 * skip);
        const uint32_t k = min(4u - skip, rem);
        sink.push(w, k);
        rem -= k;
        a += 4;
        skip = 0;
    }
}

// h2o_hpack_encode_string (hpack.c:816-837) of in[s .. s + len) whose code is `bits` long
__device__ __forceinline__ void sink_string(RegSink& sink, const GlobalSource& src, uint32_t s, uint32_t len, uint32_t bits,
                                            const uint2* enc) {
    if (huff_wins(len, bits)) {
        sink_int(sink, 0x80u, (bits + 7u) >> 3, 7);
        encode_core(src, s, len, sink, enc);  // flushes the sink
    } else {
        sink_int(sink, 0u, len, 7);
        sink_raw(sink, src, s, len);
    }
}

__device__ void emit_field(const GlobalSource& src, uint8_t* dst, uint32_t code, uint32_t noff, uint32_t nl, uint32_t voff,
                           uint32_t vl, uint4 rc, const uint2* enc) {
    RegSink sink;
    sink.init(dst);
    const uint32_t kind = code & 3u, idx = (code >> 2) & 0x7Fu;
    switch (kind) {
        case kOpIndexed:
            sink_int(sink, 0x80u, idx, 7);
            sink.finish();
            return;
        case kOpIdxName: sink_int(sink, 0x40u, idx, 6); break;
        case kOpNever: sink_int(sink, 0x10u, idx, 4); break;
        default:
            sink.put1(0x40u);
            sink_string(sink, src, noff, nl, rc.z, enc);
            break;
    }
    if (code & kOpAsIs) {
        sink_int(sink, 0u, vl, 7);
        sink_raw(sink, src, voff, vl);
        sink.finish();
    } else {
        sink_string(sink, src, voff, vl, rc.w, enc);
    }
    sink.finish();
}

__device__ __forceinline__ void put_frame_header(uint8_t* d, uint32_t len, uint32_t type, uint32_t flags, uint32_t sid) {
    d[0] = (uint8_t)(len >> 16);  // h2o_http2_encode_frame_header (lib/http2/frame.c:68-79)
    d[1] = (uint8_t)(len >> 8);
    d[2] = (uint8_t)len;
    d[3] = (uint8_t)type;
    d[4] = (uint8_t)flags;
    d[5] = (uint8_t)(sid >> 24);
    d[6] = (uint8_t)(sid >> 16);
    d[7] = (uint8_t)(sid >> 8);
    d[8] = (uint8_t)sid;
}
}  // namespace

// 3. emit: items 0 .. nhdr-1 are fields, nhdr .. nhdr+nres-1 response heads (frame header, table size
//    update, :status, server, and the content-length at the end)
__global__ __launch_bounds__(256) void hpe_emit_kernel(HpeArgs A) {
    __shared__ uint2 s_enc[256];
    s_enc[threadIdx.x] = make_uint2(e_enc_code[threadIdx.x], e_enc_nbits[threadIdx.x]);
    __syncthreads();
    const GlobalSource src{A.in, A.in_size};
    const uint64_t items = (uint64_t)A.nhdr + A.nres;
    for (uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x; i < items; i += (uint64_t)gridDim.x * 256u) {
        if (i < A.nhdr) {
            const uint4 o = A.op[i];
            if (o.z & kOpSkip) continue;
            const hhuff_hpack_header_t H = A.hdr[i];
            emit_field(src, A.out + ((uint64_t)o.y << 32 | o.x), o.z, H.name_off, H.name_len, H.value_off, H.value_len,
                       A.rec[i], s_enc);
            continue;
        }
        const uint32_t r = (uint32_t)(i - A.nhdr);
        const uint4 p0 = A.plan[2 * r], p1 = A.plan[2 * r + 1];
        if (p0.w == 0) continue;  // failed
        const hhuff_hpack_response_t R = A.res[r];
        uint8_t* base = A.out + ((uint64_t)p0.y << 32 | p0.x);
        const bool trailers = (R.flags & HHUFF_RES_TRAILERS) != 0;
        const uint32_t es = (trailers || (R.flags & HHUFF_RES_END_STREAM)) ? 1u : 0u;
        if (p0.z <= R.max_frame_size) put_frame_header(base, p0.z, 1u, 4u | es, R.stream_id);  // else hpe_frames_kernel
        RegSink sink;
        sink.init(base + 9);
        if (p1.x != ~0u) sink_int(sink, 0x20u, p1.x, 5);  // Dynamic Table Size Update (:852-853)
        if (!trailers) {
            const uint32_t s = R.status;  // encode_status (:437-466)
            const uint32_t c = s == 200 ? 8 : s == 204 ? 9 : s == 206 ? 10 : s == 304 ? 11 : s == 400 ? 12 : s == 404 ? 13 : s == 500 ? 14 : 0;
            if (c) {
                sink.put1(0x80u | c);
            } else {
                sink.put1(8u);
                sink.put1(3u);
                sink.put1('0' + s / 100);
                sink.put1('0' + s / 10 % 10);
                sink.put1('0' + s % 10);
            }
        }
        sink.finish();
        if (!(p1.y & kOpSkip))
            emit_field(src, base + 9 + p1.z, p1.y, 0u, 6u, A.server_off, A.server_len, A.rec[A.nhdr], s_enc);
        if (p1.w) {  // encode_content_length (:468-485): literal without indexing, name index 28, raw digits
            uint8_t* d = base + 9 + p0.z - p1.w;
            d[0] = 0x0f;
            d[1] = 0x0d;
            d[2] = (uint8_t)(p1.w - 3u);
            uint64_t v = R.content_length;
            for (uint32_t k = p1.w - 1; k >= 3; --k) {
                d[k] = (uint8_t)('0' + v % 10);
                v /= 10;
            }
        }
    }
}

// 4. frames: one workgroup per listed response; chunk j (>= 1) of the payload moves up by 9 j bytes,
//    last chunk first and each chunk top-down through LDS, so no byte is overwritten before it is read
__global__ __launch_bounds__(256) void hpe_frames_kernel(HpeArgs A) {
    __shared__ uint8_t s_buf[8192];
    const uint32_t nbig = A.big[0];
    for (uint32_t b = blockIdx.x; b < nbig; b += gridDim.x) {
        const uint32_t r = A.big[1 + b];
        const uint4 p0 = A.plan[2 * r];
        const hhuff_hpack_response_t R = A.res[r];
        uint8_t* base = A.out + ((uint64_t)p0.y << 32 | p0.x);
        const uint32_t P = p0.z, M = R.max_frame_size;
        const uint32_t k = (P + M - 1u) / M;
        for (uint32_t j = k - 1; j >= 1; --j) {
            const uint64_t lo = 9ull + (uint64_t)j * M, hi = 9ull + min((uint64_t)(j + 1) * M, (uint64_t)P);
            const uint64_t shift = 9ull * j;
            for (uint64_t top = hi; top > lo;) {
                const uint64_t bot = top - lo > sizeof(s_buf) ? top - sizeof(s_buf) : lo;
                for (uint64_t q = bot + threadIdx.x; q < top; q += 256) s_buf[q - bot] = base[q];
                __syncthreads();
                for (uint64_t q = bot + threadIdx.x; q < top; q += 256) base[q + shift] = s_buf[q - bot];
                __syncthreads();
                top = bot;
            }
            if (threadIdx.x == 0) {
                const bool last = j == k - 1;
                put_frame_header(base + (uint64_t)j * (M + 9u), last ? (uint32_t)(hi - lo) : M, 9u, last ? 4u : 0u,
                                 R.stream_id);
            }
            __syncthreads();
        }
        if (threadIdx.x == 0) {
            const uint32_t es = ((R.flags & HHUFF_RES_TRAILERS) || (R.flags & HHUFF_RES_END_STREAM)) ? 1u : 0u;
            put_frame_header(base, M, 1u, es, R.stream_id);
        }
        __syncthreads();
    }
}

// 5. the table pass: one wave per connection writes its live entries' bytes, newest first, into the ring
//    they do not use now and points the entries there (as blk_table_kernel does for the decoder)
__global__ __launch_bounds__(256) void hpe_ring_kernel(HpeArgs A) {
    const int lane = threadIdx.x & 63;
    const uint64_t c = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    if (c >= A.nconn) return;
    const uint64_t base = c * kConnScratch;
    EncState* ts = reinterpret_cast<EncState*>(A.scratch + base);
    EncEntry* ent = reinterpret_cast<EncEntry*>(A.scratch + base + sizeof(EncState));
    const EncState s = *ts;
    const uint32_t nring = s.ring ^ 1u;
    const uint64_t rbase = base + sizeof(EncState) + kMaxEntries * sizeof(EncEntry) + (uint64_t)nring * kRing;
    uint32_t carry = 0;
    for (uint32_t k0 = 0; k0 < s.num; k0 += 64) {
        const uint32_t k = k0 + (uint32_t)lane;
        const bool live = k < s.num;
        uint32_t i = s.start + k;
        i = i >= kMaxEntries ? i - kMaxEntries : i;
        EncEntry e{};
        if (live) e = ent[i];
        const uint32_t sz = live ? e.nl + e.vl : 0u;
        const uint32_t dst = carry + wave_excl_scan(sz, lane);
        carry += (uint32_t)__builtin_amdgcn_readlane((int)(dst - carry + sz), 63);
        uint8_t* d = A.scratch + rbase + dst;
        wave_copy64(hpe_src(A, e.nsrc), d, live ? e.nl : 0u, lane);
        wave_copy64(hpe_src(A, e.vsrc), d + e.nl, live ? e.vl : 0u, lane);
        if (live) {
            ent[i].nsrc = kSrcScr | (rbase + dst);
            ent[i].vsrc = kSrcScr | (rbase + dst + e.nl);
        }
    }
    if (lane == 0) ts->ring = nring;
}

uint64_t hpenc_conn_scratch() { return kConnScratch; }

hipError_t launch_hpack_flatten(const uint8_t* in, uint64_t in_size, const hhuff_hpack_header_t* hdr, uint32_t nhdr,
                                const hhuff_hpack_response_t* res, const uint32_t* conn_first, uint32_t nconn, uint32_t nres,
                                uint32_t server_off, uint32_t server_len, uint8_t* out, const uint64_t* out_off,
                                uint32_t* out_len, uint32_t* headers_size, int32_t* rstatus, uint8_t* scratch,
                                uint32_t flags, hipStream_t stream) {
    if (nconn == 0) return hipSuccess;
    const uint64_t ws_bytes = 16ull * (nhdr + 1) + 4ull * (nhdr + 1) + 16ull * nhdr + 32ull * nres + 4ull * (nres + 1) + 64;
    uint8_t* ws = nullptr;
    hipError_t e = work_alloc((void**)&ws, ws_bytes, stream);
    if (e != hipSuccess) return e;
    HpeArgs A{in, in_size, hdr, nhdr, res, conn_first, nconn, nres, server_off, server_len, out, out_off, out_len,
              headers_size, rstatus, scratch, flags, nullptr, nullptr, nullptr, nullptr, nullptr};
    uint8_t* p = ws;
    A.rec = reinterpret_cast<uint4*>(p);
    p += 16ull * (nhdr + 1);
    A.op = reinterpret_cast<uint4*>(p);
    p += 16ull * nhdr;
    A.plan = reinterpret_cast<uint4*>(p);
    p += 32ull * nres;
    A.info = reinterpret_cast<uint32_t*>(p);
    p += 4ull * (nhdr + 1);
    A.big = reinterpret_cast<uint32_t*>(p);
    e = hipMemsetAsync(A.big, 0, 4, stream);
    const uint32_t gp = (uint32_t)std::min<uint64_t>((nhdr + 256ull) / 256u, 8192ull);
    if (e == hipSuccess) {
        hipLaunchKernelGGL(hpe_prep_kernel, dim3(gp), dim3(256), 0, stream, A);
        e = hipGetLastError();
    }
    if (e == hipSuccess) {
        hipLaunchKernelGGL(hpe_table_kernel, dim3((nconn + 255u) / 256u), dim3(256), 0, stream, A);
        e = hipGetLastError();
    }
    if (e == hipSuccess && (uint64_t)nhdr + nres != 0) {
        const uint32_t ge = (uint32_t)std::min<uint64_t>(((uint64_t)nhdr + nres + 255u) / 256u, 16384ull);
        hipLaunchKernelGGL(hpe_emit_kernel, dim3(ge), dim3(256), 0, stream, A);
        e = hipGetLastError();
    }
    if (e == hipSuccess && nres != 0) {
        hipLaunchKernelGGL(hpe_frames_kernel, dim3(min(nres, 512u)), dim3(256), 0, stream, A);
        e = hipGetLastError();
    }
    if (e == hipSuccess) {
        hipLaunchKernelGGL(hpe_ring_kernel, dim3((nconn + 3u) / 4u), dim3(256), 0, stream, A);
        e = hipGetLastError();
    }
    const hipError_t f = hipFreeAsync(ws, stream);
    return e != hipSuccess ? e : f;
}
}  // namespace hhuff
