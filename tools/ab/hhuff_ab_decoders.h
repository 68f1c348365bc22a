// A/B-only decoders, measured and not adopted: the length-sorted decode chunks and
// the segment decoder.  Not part of libhhuff.so: included by hhuff_kernels.hip only when a build defines
// HHUFF_AB_VARIANTS (tools/ab.py build NAME -DHHUFF_AB_VARIANTS ...; the include path adds tools/ab).
#pragma once

// ------------------------------------------------------------------------------------------------
// Length-sorted decode chunks (contiguous layout, slot output, short strings: c2, c4).  A 64-string tile of the
// staged kernel runs as long as its longest string (U[24,72] plain = U[18,54] Huffman bytes: the tile's max is
// ~1.47x its mean).  As encode_sorted_kernel does for encode, a group of 4 waves stages the span of 256
// consecutive strings, counting-sorts them by length and hands wave w the w-th group of 64, so a wave's lanes
// finish nearly together; the slot-layout output of the 256 strings goes out as one region (16-B stores, two
// deferred edges).  The decode tables need one 32-KiB LUT per workgroup, so a workgroup is 16 waves in four
// independent groups (one wave of each group per SIMD), each group on its own chunks with a group barrier of its
// own: an LDS counter and LDS-only fences (s_barrier would make the 16 waves wait for the slowest group, and a
// workgroup-scope fence for their global stores).  While a group's short-string waves wait for its long-string
// wave, the other groups' waves use the SIMD.
// ------------------------------------------------------------------------------------------------
constexpr uint32_t kDsStr = 256;  // strings per chunk (one per thread of a group)
__device__ __forceinline__ void group_sync(uint32_t* ctr, uint32_t& target, uint32_t lane) {
    target += 4u;  // four waves a group, one arrival each
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    if (lane == 0) __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    while (__hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < target) __builtin_amdgcn_s_sleep(1);
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

template <uint32_t CH>
__global__ __launch_bounds__(1024) void decode_sorted_kernel(DecArgs A) {
    constexpr int NV = (CH + 16 * kDsStr - 1) / (16 * kDsStr);  // 16-B span chunks per thread
    constexpr uint32_t OUTS = ((8u * (CH + 16u)) / 5u + 64u + 15u) & ~15u;
    struct __attribute__((aligned(16))) Group {
        uint32_t in[CH / 4 + 16];        // the chunk's span, big-endian dwords (+ read slack)
        uint8_t out[OUTS + 4 * kDsStr];  // slot-layout output of the chunk, then a trash dword per thread
        uint2 str[kDsStr];               // {offset in the span, length | is_name << 31}, then {out_len, status}
        uint16_t perm[kDsStr];
        uint32_t bin[kSortBins];
        uint32_t ctr;
    };
    struct __attribute__((aligned(16))) Smem {
        uint32_t lut[1u << HHUFF_LUT_BITS];
        uint32_t kinfo[32];
        uint32_t ones[(HHUFF_ONES_NENT + 3) & ~3];
        Group g[4];
    };
    __shared__ Smem sm;
    load_dec_tables(sm.lut, sm.kinfo, sm.ones, 1024);
    const uint32_t grp = threadIdx.x >> 8, t = threadIdx.x & 255u, lane = t & 63u;
    Group& G = sm.g[grp];
    if (t < kSortBins) G.bin[t] = 0u;
    if (t == 0) G.ctr = 0u;
    __syncthreads();
    const DecTables T{sm.lut, sm.kinfo, sm.ones};
    uint32_t target = 0;
    const uint64_t nch = ((uint64_t)A.n + kDsStr - 1) / kDsStr;
    const uint64_t cstride = (uint64_t)gridDim.x * 4u;
    uint64_t c = (uint64_t)blockIdx.x * 4u + grp;
    if (c >= nch) return;  // (group-uniform; the other groups never wait for this one)
    struct Chunk {
        uint32_t s, e, lo, hi, nw;
    };
    auto issue = [&](uint64_t cc) {  // clamped: every load issues
        const uint64_t cb = cc * kDsStr;
        const uint64_t i = min(cb + t, (uint64_t)A.n - 1u);
        Chunk q;
        q.s = A.in_off[i];
        q.e = A.in_off[i + 1];
        q.lo = A.in_off[min(cb, (uint64_t)A.n - 1u)];
        q.hi = A.in_off[min(cb + kDsStr, (uint64_t)A.n)];
        q.nw = A.is_name_bits ? A.is_name_bits[i >> 5] : 0u;
        return q;
    };
    auto span_of = [](const Chunk& q) { return q.hi > q.lo ? ((q.hi + 15u) & ~15u) - (q.lo & ~15u) : 0u; };
    uint4 pv[NV];
    auto issue_span = [&](const Chunk& q) {
        const uint32_t a0 = q.lo & ~15u, span = span_of(q);
#pragma unroll
        for (int j = 0; j < NV; ++j) {
            const uint32_t k = (uint32_t)j * (16u * kDsStr) + t * 16u;
            const uint64_t g = (uint64_t)a0 + k;
            if (k < span && span <= CH && g + 16 <= A.in_size) pv[j] = *reinterpret_cast<const uint4*>(A.in + g);
        }
    };
    uint32_t bin = 0, rank = 0;
    // the chunk's span into the input stage (big-endian dwords), its strings' records and their length ranks
    auto prepare = [&](const Chunk& q, uint64_t cc) {
        const uint32_t sp = span_of(q);
        if (sp > CH) return;  // group-uniform: the per-thread path needs none of it
        const uint32_t a0 = q.lo & ~15u;
#pragma unroll
        for (int j = 0; j < NV; ++j) {
            const uint32_t k = (uint32_t)j * (16u * kDsStr) + t * 16u;
            const uint64_t g = (uint64_t)a0 + k;
            if (k < sp) {
                uint4 x = g + 16 <= A.in_size ? pv[j] : load16_tail(A.in, A.in_size, g);
                x = make_uint4(bswap32(x.x), bswap32(x.y), bswap32(x.z), bswap32(x.w));
                *reinterpret_cast<uint4*>(reinterpret_cast<uint8_t*>(G.in) + k) = x;
            }
        }
        const uint64_t i = cc * kDsStr + t;
        const uint32_t ln = i < A.n ? q.e - q.s : 0u;
        const uint32_t nm = i < A.n && A.is_name_bits ? ((q.nw >> (i & 31u)) & 1u) : 0u;
        G.str[t] = make_uint2(q.s - a0, min(ln, kMaxStrLen + 1u) | (nm << 31));
        bin = min(ln, kSortBins - 1u);  // the bulk loop's trip count follows the length
        rank = atomicAdd(&G.bin[bin], 1u);
    };
    Chunk cur = issue(c);
    issue_span(cur);
    prepare(cur, c);
    Chunk nxt = issue(c + cstride < nch ? c + cstride : c);
    __asm__ volatile("" : "+v"(nxt.s), "+v"(nxt.e), "+v"(nxt.lo), "+v"(nxt.hi), "+v"(nxt.nw) : : "memory");
    for (;;) {
        const uint64_t cb = c * kDsStr, i = cb + t;
        const bool valid = i < A.n;
        const uint32_t lo = cur.lo, hi = cur.hi, a0 = lo & ~15u, span = span_of(cur);
        EdgeRec* rec = A.edges + 2 * c;
        const uint64_t cn = c + cstride, cn2 = cn + cstride;
        const bool more = cn < nch;
        group_sync(&G.ctr, target, lane);  // the chunk's stage, records and ranks are in
        if (span > CH) {  // (group-uniform) larger than the stage: one thread per string, global memory
            if (valid) {
                uint32_t ol;
                uint8_t st;
                const bool nm = A.is_name_bits && ((cur.nw >> (i & 31u)) & 1u);
                if (!split_push(A, (uint32_t)i, cur.e - cur.s)) {
                    decode_direct(A, cur.s, cur.e - cur.s, nm, A.out + dec_slot(cur.s), T, ol, st);
                    A.out_len[i] = ol;
                    A.status[i] = st;
                }
            }
            if (t < 2) rec[t].m = make_uint4(0u, 0u, 0u, 0u);  // direct stores: no edges to defer
            if (!more) break;
            issue_span(nxt);
            prepare(nxt, cn);
            Chunk nn = issue(cn2 < nch ? cn2 : cn);
            __asm__ volatile("" : "+v"(nn.s), "+v"(nn.e), "+v"(nn.lo), "+v"(nn.hi), "+v"(nn.nw) : : "memory");
            cur = nxt;
            nxt = nn;
            c = cn;
            continue;
        }
        {  // every wave scans the bin counts (two per lane) and places its threads' strings
            const uint32_t x0 = G.bin[2 * lane], x1 = G.bin[2 * lane + 1];
            const uint32_t ex = wave_excl_scan(x0 + x1, (int)lane);
            const uint32_t eb = (uint32_t)__shfl((int)ex, (int)(bin >> 1)), xb = (uint32_t)__shfl((int)x0, (int)(bin >> 1));
            G.perm[eb + ((bin & 1u) ? xb : 0u) + rank] = (uint16_t)t;
        }
        group_sync(&G.ctr, target, lane);
        if (t < kSortBins) G.bin[t] = 0u;  // read by every wave above: cleared for the next chunk
        if (more) issue_span(nxt);          // the next chunk's span: in flight during the decode
        Chunk nn = issue(cn2 < nch ? cn2 : (more ? cn : c));
        // sorted position t: wave w of the group decodes the w-th length group
        const uint32_t j = G.perm[t];
        const uint2 sj = G.str[j];
        const uint32_t lj = sj.y & 0x7FFFFFFFu;
        const bool vj = cb + j < A.n;
        const uint32_t op0 = (uint32_t)(dec_slot(a0 + sj.x) - (dec_slot(lo) & ~15ull));
        const bool act = vj && lj <= kMaxStrLen;
        const DecResult r = decode_staged_lane_v7(G.in, sj.x, act ? lj : 0u, act, G.out, op0, OUTS + 4u * t, T);
        uint32_t ol = kFailLen, st = kStatusFail;
        if (vj && lj > kMaxStrLen) {
            st = kStatusTooLong;
        } else if (vj && r.ok) {
            ol = r.len;
            st = soft_bits((sj.y >> 31) != 0, r.len, r.flags, r.len ? G.out[op0] : 0u, r.len ? G.out[op0 + r.len - 1] : 0u);
        }
        G.str[j] = make_uint2(ol, st);  // back to the string's own record: stored in string order below
        group_sync(&G.ctr, target, lane);
        const uint2 res = G.str[t];
        if (more) prepare(nxt, cn);  // the input stage and the records are free: the next chunk goes in now
        // the chunk after next's offsets are waited for here, before this chunk's stores (in-order vmcnt)
        __asm__ volatile("" : "+v"(nn.s), "+v"(nn.e), "+v"(nn.lo), "+v"(nn.hi), "+v"(nn.nw) : : "memory");
        if (valid) {
            A.out_len[i] = res.x;
            A.status[i] = (uint8_t)res.y;
        }
        // the slot-layout output region; its first and last 16-B chunks are deferred (edge_fix_kernel)
        {
            const uint64_t olo = dec_slot(lo), ohi = dec_slot(hi), obase = olo & ~15ull;
            const uint32_t ospan = hi > lo ? (uint32_t)(((ohi + 15u) & ~15ull) - obase) : 0u;
            const uint32_t kl = ospan ? (ospan - 1u) & ~15u : 0u;
            for (uint32_t k = t * 16u; k < ospan; k += 16u * kDsStr) {
                const uint64_t g = obase + k;
                const uint4 v = *reinterpret_cast<const uint4*>(G.out + k);
                const bool full = g >= olo && g + 16 <= ohi;
                if (full) st16_out(A.out + g, v);
                if (k == 0 || k == kl) {
                    const uint32_t elo = olo > g ? (uint32_t)(olo - g) : 0u;
                    const uint32_t ehi = ohi - g < 16 ? (uint32_t)(ohi - g) : 16u;
                    EdgeRec* e = rec + (k == 0 ? 0 : 1);
                    e->v = v;
                    e->m = make_uint4((uint32_t)g, (uint32_t)(g >> 32), full ? 0u : elo, full ? 0u : ehi);
                }
            }
            if (t == 0 && (kl == 0 || ospan == 0)) rec[1].m = make_uint4(0u, 0u, 0u, 0u);
            if (t == 0 && ospan == 0) rec[0].m = make_uint4(0u, 0u, 0u, 0u);
        }
        if (!more) break;
        cur = nxt;
        nxt = nn;
        c = cn;
    }
}

// ------------------------------------------------------------------------------------------------
// Segment decode: mixed and long strings, contiguous layout, slot output (SURVEY §7 hard part 2; VERDICT r4
// "next" #1).  One lane per string runs a 64-string tile as long as its longest string (the staged kernel:
// ~4x the mean on Zipf 8..512 B), and one lane per string streaming its own input and output (the stream
// kernel) keeps ~260 B of LDS and two memory streams per lane (1.5 waves a SIMD, 1.44x write traffic).  Here
// the lanes of a wave share the BITS of a tile evenly instead of its strings:
//   tiles     tile t = the strings starting in bytes [t TB, (t+1) TB) of the batch (seg_plan_kernel writes
//             tf[t], the first of them), so a tile's span is below TB + its last string; a last string longer
//             than CAP - TB leaves the span for the split lists (split_decode_kernel) or one lane;
//   stage     the span goes to LDS with 16-B loads, as big-endian dwords (decode_staged_kernel's stage);
//   segments  the span's bits are cut into K <= 64 equal segments [b_k, b_k+1); lane k decodes the symbols
//             that START in its segment, walking from one string into the next;
//   sync      a lane cannot know where a symbol starts at b_k.  It decodes, counting only, from
//             max(b_k - kSegLead, the start of the string holding b_k) to the first symbol boundary f_k >= b_k
//             (Huffman codes resynchronise: on header text ~0.2 % of 256-bit leads are still off the true
//             boundaries), then its segment into a private LDS region, stopping at e_k = the first boundary
//             >= b_k+1.  Lane k is right iff f_k == e_k-1 and lane k - 1 is right (lane 0 starts on a string's
//             first bit); a lane that disagrees decodes its segment again from e_k-1, until no lane changes;
//   ends      string ends inside a segment cost no checked steps: the window's bits past the current string
//             read as ones (13 ones are no code, and a valid string's padding is ones), so a bulk step never
//             takes a symbol of a valid string past its end, and the long-code branch, which sees the ones,
//             closes the string (EOS, padding rule: hpack.c:88-89, 132-133) and moves the lane to the next
//             string's first bit.  A lane records the strings it closes (string, region offset, flags,
//             verdict: <= kSegRecs 16-bit records in four VGPRs);
//   finish    a wave scan places the parts that continue a string from the lane before, per-string counts,
//             flags and first / last bytes meet in LDS (atomics), the parts move (lds_move_or) into a
//             slot-layout stage over the dead input stage, and that goes out with 16-B stores and deferred
//             edges (edge_fix_kernel).
// Same results as decode_core for every string.  A sub-tile in which a lane closes more strings than it can
// record decodes one lane per string from global memory instead (decode_direct).
// ------------------------------------------------------------------------------------------------
#ifndef HHUFF_SEG_LEAD
#define HHUFF_SEG_LEAD 256
#endif
constexpr uint32_t kSegLead = HHUFF_SEG_LEAD;  // bits decoded (counting only) before a segment start inside a string
constexpr uint32_t kSegMinBits = 192;  // shortest segment (small tiles use fewer lanes)
constexpr uint32_t kSegRecs = 8;       // string closes a lane can record
constexpr int32_t kSegIdle = (int32_t)0x80000000;

template <uint32_t CAP>
struct SegGeom {
    static constexpr uint32_t kInStage = CAP + 64u;                         // 16-aligned span (<= CAP + 32) + read slack
    static constexpr uint32_t kFS = ((8u * CAP) / 5u + 48u + 15u) & ~15u;  // slot-layout output stage of a span
    static constexpr uint32_t kStage = kFS > kInStage ? kFS : kInStage;
    static constexpr uint32_t kSegMax = (8u * (CAP + 32u) + 63u) / 64u;  // bits of a segment at most (K = 64)
    static constexpr uint32_t kPW = ((kSegMax + 4u) / 5u + 12u + 3u) & ~3u;  // region bytes per lane
    static constexpr uint32_t kRegOff = 16u + kStage;
    static constexpr uint32_t kAggOff = kRegOff + 64u * kPW;                 // cnt | flags | first | last [64] u32
    static constexpr uint32_t kSbtOff = kAggOff + 4u * 64u * 4u;             // string start bits [68] u32
    static constexpr uint32_t kBuf = kSbtOff + 68u * 4u;
    static_assert(kPW <= 127u, "region offsets are 7-bit record fields");
    static_assert(kSegMinBits <= kSegMax, "segment bound");
};

// tf[t] = the first string starting at or after byte t TB of the batch (relative to in_off[0]), t <= T, where
// T = (in_off[n] - in_off[0]) / TB + 1 is the batch's tile count (tf[T] = n); edge records of tiles T..T_max-1
// (the launch sized them from in_size) are cleared.
__global__ __launch_bounds__(256) void seg_plan_kernel(const uint32_t* __restrict__ in_off, uint32_t n, uint32_t TB,
                                                       uint32_t T_max, uint32_t* __restrict__ tf, EdgeRec* __restrict__ edges) {
    const uint32_t base = in_off[0];
    const uint32_t T = min((in_off[n] - base) / TB + 1u, T_max - 1u);
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i <= n; i += stride) {
        const uint32_t s = in_off[i] - base;
        const uint32_t t_lo = i == 0 ? 0u : (in_off[i - 1] - base) / TB + 1u;
        const uint32_t t_hi = i == n ? T : min(s / TB, T - 1u);
        for (uint32_t t = t_lo; t <= t_hi; ++t) tf[t] = (uint32_t)i;
    }
    for (uint64_t r = 2ull * T + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; r < 2ull * T_max; r += stride)
        edges[r].m = make_uint4(0u, 0u, 0u, 0u);
}

// LDS bytes [0, ospan) to global [gbase, gbase + ospan) keeping [keep_lo, keep_hi): whole chunks with 16-B stores;
// the first / last partial chunk into a deferred-edge record when one is given, else with byte stores (the
// chunk a sub-tile shares with the next one of the same wave).
__device__ __forceinline__ void region_copy_seg(uint8_t* __restrict__ out, uint64_t gbase, const uint8_t* lds, uint32_t ospan,
                                                uint64_t keep_lo, uint64_t keep_hi, int lane, EdgeRec* recL, EdgeRec* recR) {
    const uint32_t kl = ospan ? (ospan - 1u) & ~15u : 0u;
    for (uint32_t k = (uint32_t)lane * 16u; k < ospan; k += 64u * 16u) {
        const uint64_t g = gbase + k;
        const uint4 v = *reinterpret_cast<const uint4*>(lds + k);
        const bool full = g >= keep_lo && g + 16 <= keep_hi;
        const uint32_t lo = keep_lo > g ? (uint32_t)(keep_lo - g) : 0u;
        const uint32_t hi = keep_hi - g < 16 ? (uint32_t)(keep_hi - g) : 16u;
        EdgeRec* r = k == 0 && recL ? recL : (k == kl && recR ? recR : nullptr);
        if (full) {
            *reinterpret_cast<uint4*>(out + g) = v;
        } else if (r == nullptr) {
            for (uint32_t b = lo; b < hi; ++b) out[g + b] = lds[k + b];
        }
        if (r) {
            r->v = v;
            r->m = make_uint4((uint32_t)g, (uint32_t)(g >> 32), full ? 0u : lo, full ? 0u : hi);
        }
        if (k == 0 && kl == 0 && recL && recR) recR->m = make_uint4(0u, 0u, 0u, 0u);
    }
    if (ospan == 0 && lane == 0) {
        if (recL) recL->m = make_uint4(0u, 0u, 0u, 0u);
        if (recR) recR->m = make_uint4(0u, 0u, 0u, 0u);
    }
}

template <int WAVES, uint32_t CAP, uint32_t TB>
__global__ __launch_bounds__(WAVES * 64) void decode_seg_kernel(DecArgs A, const uint32_t* __restrict__ tf, uint32_t tmax) {
    using G = SegGeom<CAP>;
    constexpr uint32_t kLMax = CAP - TB;  // longest string a tile keeps as its last one
    static_assert(TB < CAP, "tile budget");
    struct __attribute__((aligned(16))) Smem {
        uint32_t lut[1u << HHUFF_LUT_BITS];
        uint32_t kinfo[32];
        uint32_t ones[(HHUFF_ONES_NENT + 3) & ~3];
        uint8_t buf[WAVES][G::kBuf];
    };
    __shared__ Smem sm;
    load_dec_tables(sm.lut, sm.kinfo, sm.ones, WAVES * 64);
    __syncthreads();
    const DecTables Tb{sm.lut, sm.kinfo, sm.ones};
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint8_t* const buf = sm.buf[wave];
    uint8_t* const stage8 = buf + 16;  // input stage, then (once the walk is done) the slot-layout output stage
    const lds_u32* st = (const lds_u32*)(uint32_t*)stage8;
    const uint32_t fsa = lds_addr(stage8);
    const uint32_t r0 = lds_addr(buf + G::kRegOff) + (uint32_t)lane * G::kPW;  // this lane's region
    uint32_t* const acnt = reinterpret_cast<uint32_t*>(buf + G::kAggOff);
    uint32_t* const aflg = acnt + 64;  // bits 0-1 invalid-char flags, 3 verdict ok, 4 closed
    uint32_t* const afst = acnt + 128;  // (lane << 8 | first byte of the part), min over parts
    uint32_t* const alst = acnt + 192;  // (lane << 8 | last byte of the part), max over parts
    uint32_t* const sbt = reinterpret_cast<uint32_t*>(buf + G::kSbtOff);
    const uint32_t n = A.n;
    const uint32_t base = A.in_off[0];
    const uint32_t ntiles = min((A.in_off[n] - base) / TB + 1u, tmax - 1u);  // as seg_plan_kernel
    const uint32_t tstride = gridDim.x * WAVES;
    PROF_DECL  // profile builds: setup / lead / bulk / checked / places+moves / copy-out / fallback, slot 0

    using PF = SpanPrefetch<(G::kInStage + 1023u) / 1024u>;
    // Tiles in batches of 64 per wave (lane j: tile tb + j tstride): string range and span (after the last
    // string's exclusion) come in one round of loads per batch; then each tile's offsets and span are loaded
    // into registers while the tile before is decoded, and waited for before that tile's stores (loads and
    // stores complete in order on gfx950: a load waited for behind stores would wait for them too).
    for (uint32_t tb = blockIdx.x * WAVES + wave; tb < ntiles; tb += 64u * tstride) {
        const uint32_t nt = min(64u, (ntiles - tb + tstride - 1u) / tstride);
        const uint32_t tj = tb + min((uint32_t)lane, nt - 1u) * tstride;
        const uint32_t ti0 = tf[tj], ti1 = tf[tj + 1u];
        const uint32_t tlo = A.in_off[ti0], thi = A.in_off[ti1], tpl = A.in_off[ti1 > ti0 ? ti1 - 1u : ti0];
        const bool tex = ti1 > ti0 && thi - tpl > kLMax;  // the tile's last string leaves the span
        const uint32_t thi2 = tex ? tpl : thi;
        const uint64_t texm = __builtin_amdgcn_ballot_w64(tex);
        PF pf;
        uint32_t nx_s = 0, nx_e = 0, nx_nm = 0;
        auto issue = [&](uint32_t j) {  // tile j's first 64 strings' offsets and its span, into registers
            const uint32_t i0 = (uint32_t)__builtin_amdgcn_readlane((int)ti0, (int)j);
            const uint32_t i1 = (uint32_t)__builtin_amdgcn_readlane((int)ti1, (int)j);
            const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)tlo, (int)j);
            const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)thi2, (int)j);
            const uint32_t m = min(64u, i1 - i0);
            const uint32_t i = min(i0 + min((uint32_t)lane, m ? m - 1u : 0u), n - 1u);
            nx_s = A.in_off[i];
            nx_e = A.in_off[i + 1u];
            nx_nm = A.is_name_bits ? A.is_name_bits[i >> 5] : 0u;
            const uint32_t a0 = lo & ~15u;
            pf.issue(A.in, A.in_size, a0, hi > lo ? ((hi + 15u) & ~15u) - a0 : 0u, lane);
        };
        auto consume_next = [&]() {  // wait for the prefetched registers (before a tile's stores)
            __asm__ volatile("" : : "v"(nx_s), "v"(nx_e), "v"(nx_nm));
#pragma unroll
            for (int c = 0; c < (int)((G::kInStage + 1023u) / 1024u); ++c)
                __asm__ volatile("" : : "v"(pf.v[c].x), "v"(pf.v[c].y), "v"(pf.v[c].z), "v"(pf.v[c].w));
        };
        issue(0u);
    for (uint32_t j = 0; j < nt; ++j) {
        const uint32_t t = tb + j * tstride;
        const uint32_t i0 = (uint32_t)__builtin_amdgcn_readlane((int)ti0, (int)j);
        const uint32_t i1 = (uint32_t)__builtin_amdgcn_readlane((int)ti1, (int)j);
        const uint32_t t_lo = (uint32_t)__builtin_amdgcn_readlane((int)tlo, (int)j);
        const uint32_t t_hi = (uint32_t)__builtin_amdgcn_readlane((int)thi2, (int)j);
        const bool t_ex = ((texm >> j) & 1ull) != 0;
        const uint32_t c_s = nx_s, c_e = nx_e, c_nm = nx_nm;  // this tile's prefetched offsets (first 64 strings)
        EdgeRec* const erec = A.edges + 2ull * t;
        if (i0 >= i1) {  // inside a long string of an earlier tile: no bytes of ours
            if (lane == 0) erec[0].m = erec[1].m = make_uint4(0u, 0u, 0u, 0u);
            if (j + 1u < nt) issue(j + 1u);
            continue;
        }
        for (uint32_t g0 = i0; g0 < i1; g0 += 64u) {
            const uint32_t m = min(64u, i1 - g0);
            const bool first_sub = g0 == i0, last_sub = g0 + 64u >= i1;
            const bool mine = (uint32_t)lane < m;
            const uint32_t i = g0 + min((uint32_t)lane, m - 1u);
            uint32_t s = c_s, e = c_e, nmw = c_nm;
            if (!first_sub) {  // later sub-tiles of a tile of more than 64 strings: loaded here
                s = A.in_off[i];
                e = A.in_off[i + 1];
                nmw = A.is_name_bits ? A.is_name_bits[i >> 5] : 0u;
            }
            const uint32_t len = e - s;
            const bool is_name = mine && A.is_name_bits && ((nmw >> (i & 31u)) & 1u);
            // the tile's last string, when longer than the stage allows, leaves the span
            const bool exl = last_sub && t_ex;
            const bool excl = exl && (uint32_t)lane == m - 1u;
            const uint32_t mw = m - (exl ? 1u : 0u);  // strings the lanes walk
            const uint32_t lo = first_sub ? t_lo : (uint32_t)__builtin_amdgcn_readfirstlane((int)s);
            const uint32_t hi = last_sub ? t_hi : (uint32_t)__builtin_amdgcn_readlane((int)e, (int)(m - 1u));
            const uint32_t a0 = lo & ~15u;
            const uint32_t span = hi > lo ? ((hi + 15u) & ~15u) - a0 : 0u;
            const uint32_t Bb = 8u * (lo - a0), Bend = 8u * (hi - a0);
            acnt[lane] = 0u;
            aflg[lane] = 0u;
            afst[lane] = 0xFFFFFFFFu;
            alst[lane] = 0u;
            sbt[lane] = (uint32_t)lane < mw ? 8u * (s - a0) : Bend;
            if (lane < 4) sbt[64 + lane] = Bend;
            if (first_sub) {
                pf.template commit<true>(reinterpret_cast<uint32_t*>(stage8), A.in, A.in_size, a0, span, lane);
                if (j + 1u < nt) issue(j + 1u);  // in flight during this tile's walk
            } else {
                PF pf2;
                pf2.issue(A.in, A.in_size, a0, span, lane);
                pf2.template commit<true>(reinterpret_cast<uint32_t*>(stage8), A.in, A.in_size, a0, span, lane);
            }
            wave_lds_sync();

            PROF_MARK(0);
            // ---- segments ----
            const uint32_t total = Bend - Bb;
            const uint32_t K = total ? min(64u, (total + kSegMinBits - 1u) / kSegMinBits) : 0u;
            const uint32_t SEG = K ? (total + K - 1u) / K : 0u;
            const uint32_t bk = Bb + (uint32_t)lane * SEG;
            const bool act = (uint32_t)lane < K && bk < Bend;
            const int32_t stop = (int32_t)min(bk + SEG, Bend);
            // the string holding bit p: the first of the strings starting at p (empty ones first), else the one p
            // lies inside
            auto locate = [&](uint32_t p) -> uint32_t {
                uint32_t l = 0;  // first l with sbt[l] >= p
#pragma unroll
                for (uint32_t step = 32; step; step >>= 1)
                    if (sbt[l + step - 1u] < p) l += step;
                if (l >= mw || sbt[l] > p) l -= 1u;
                return l;
            };

            // per-lane walk state
            int32_t pm = 0, q = 0, lim = kSegIdle, E = 0;
            uint32_t x0 = 0, x1 = 0, x2 = 0;
            auto reload = [&]() {
                q = pm >> 5;
                x0 = st[q];
                x1 = st[q + 1];
                x2 = st[q + 2];
            };
            auto advance = [&](int32_t cons) {
                pm += cons;
                const int32_t qn = pm >> 5;
                const bool adv = qn != q;
                x0 = adv ? x1 : x0;
                x1 = adv ? x2 : x1;
                q = qn;
                x2 = st[q + 2];
            };
            auto long_entry = [&](uint32_t w) -> uint32_t {  // the leading-ones table entry for window w
                const uint32_t k = min((uint32_t)__builtin_clz(~w | 1u), 30u);
                const uint32_t ki = Tb.kinfo[k];
                return Tb.ones[(ki & 0xFFFFu) + (((w << (k + 1)) >> 1) >> (31 - (ki >> 16)))];
            };

            // ---- lead: count from max(b_k - kSegLead, string start) to the first boundary f >= b_k ----
            uint32_t f = bk;
            {
                const uint32_t j = act ? locate(bk) : 0u;
                const uint32_t Bj = act ? sbt[j] : 0u;
                const uint32_t ls = bk - Bj <= kSegLead ? Bj : bk - kSegLead;
                bool lend = false;
                if (act) {
                    pm = (int32_t)ls - 1;
                    E = (int32_t)sbt[j + 1u];
                    reload();
                    lim = ls < bk ? (int32_t)bk - 26 : kSegIdle;
                }
                auto lstep = [&](bool longchk) {
                    if (pm < lim) {
                        const uint32_t w = __builtin_amdgcn_alignbit(x0, x1, ~(uint32_t)pm);
                        const uint32_t e = Tb.lut[w >> (32 - HHUFF_LUT_BITS)];
                        const uint32_t sl = (uint32_t)((int32_t)e >> 31);
                        uint32_t cons = lut_l12(e);
                        const uint32_t eb = Tb.lut[(w << cons) >> (32 - HHUFF_LUT_BITS)];
                        cons += lut_l12(eb);
                        if (longchk && __builtin_amdgcn_ballot_w64(sl != 0u) != 0) {
                            if (sl) {
                                const int32_t L = (int32_t)((long_entry(w) >> 9) & 31u);
                                const bool fits = L + pm < E;
                                cons = fits ? (uint32_t)L : 0u;
                                if (!fits) lend = true, lim = kSegIdle;
                            }
                        }
                        advance((int32_t)cons);
                    }
                };
                for (;;) {
                    lstep(false);
                    lstep(true);
                    if (!__any(pm < lim)) break;
                }
                for (;;) {  // one symbol a step up to b_k
                    const bool go = act && !lend && pm + 1 < (int32_t)bk;
                    if (!__any(go)) break;
                    if (go) {
                        const uint32_t w = __builtin_amdgcn_alignbit(x0, x1, ~(uint32_t)pm);
                        const uint32_t e = Tb.lut[w >> (32 - HHUFF_LUT_BITS)];
                        const int32_t L = (int32_t)e < 0 ? (int32_t)((long_entry(w) >> 9) & 31u) : (int32_t)lut_l1(e);
                        if (L + pm < E)
                            advance(L);
                        else
                            lend = true;  // no code fits: the string's padding (its verdict is the lane before's)
                    }
                }
                if (act) f = lend ? (uint32_t)E : (uint32_t)(pm + 1);
            }
            PROF_MARK(1);

            // ---- walk [f, first boundary >= stop) into the region; again from e_k-1 where lanes disagree ----
            uint32_t o = r0, pstart = 0, nrec = 0, accb = 0, accl = 0, l = 0, lf = 0, ek = f;
            uint64_t rlo = 0, rhi = 0;
            bool need = act;
            for (uint32_t round = 0;; ++round) {  // <= K + 1 rounds: lane r is final after round r
                bool done = true;
                if (need) {
                    l = lf = locate(f);
                    E = (int32_t)sbt[l + 1u];
                    pm = (int32_t)f - 1;
                    reload();
                    o = r0;
                    pstart = nrec = accb = accl = 0;
                    rlo = rhi = 0;
                    done = (int32_t)f >= stop || l >= mw;
                    lim = done ? kSegIdle : stop - 26;
                } else {
                    lim = kSegIdle;
                }
                // close the current string: verdict, record, next string's first bit
                auto close = [&](bool ok) {
                    const uint32_t fl = ((accb >> 24) | (accb >> 26) | (accl >> 14)) & 3u;
                    const uint32_t off = ok ? o - r0 : pstart;  // a failed string keeps no bytes
                    const uint32_t rec = l | (off << 6) | (fl << 13) | ((ok ? 1u : 0u) << 15);
                    rhi = (rhi << 16) | (rlo >> 48);
                    rlo = (rlo << 16) | rec;
                    nrec += 1u;
                    o = r0 + off;
                    pstart = off;
                    accb = accl = 0;
                    pm = E - 1;
                    q = pm >> 5;
                    x0 = st[q];
                    x1 = st[q + 1];
                    l += 1u;
                    const bool end = l >= mw || E >= stop;
                    E = (int32_t)sbt[l + 1u];  // l + 1 <= 65: sbt[mw..67] = Bend
                    if (end) done = true, lim = kSegIdle;
                };
                auto sstep = [&](bool longchk) {
                    if (pm < lim) {
                        const uint32_t w = __builtin_amdgcn_alignbit(x0, x1, ~(uint32_t)pm);
                        const int32_t d = E - pm - 1;  // string bits left
                        const uint32_t wm = w | (uint32_t)(0xFFFFFFFFull >> (uint32_t)min(max(d, 0), 32));
                        const uint32_t e = Tb.lut[wm >> (32 - HHUFF_LUT_BITS)];
                        const uint32_t sl = (uint32_t)((int32_t)e >> 31);
                        bulk_put2(o, e, 0u);
                        o += (e >> 28) & 3u;
                        accb |= e;
                        uint32_t cons = lut_l12(e);
                        {
                            const uint32_t eb = Tb.lut[(wm << cons) >> (32 - HHUFF_LUT_BITS)];
                            bulk_put2(o, eb, 0u);
                            o += (eb >> 28) & 3u;
                            accb |= eb;
                            cons += lut_l12(eb);
                        }
                        if (longchk && __builtin_amdgcn_ballot_w64(sl != 0u) != 0) {
                            if (sl) {
                                const uint32_t le = long_entry(wm);
                                const int32_t L = (int32_t)((le >> 9) & 31u);
                                const bool eos = (le & 0x1FFu) == kEos;
                                if (L <= d && !eos) {
                                    lds_st8(o, le);
                                    o += 1u;
                                    accl |= le;
                                    cons = (uint32_t)L;
                                } else {  // EOS inside the string (hpack.c:88-89), or no code fits: the string ends
                                    close(!(eos && L <= d) && d >= 0 && d <= 7 && wm == 0xFFFFFFFFu);
                                    cons = 0u;
                                }
                            }
                        }
                        advance((int32_t)cons);
                    }
                };
                for (;;) {
                    sstep(false);
                    sstep(true);
                    if (!__any(pm < lim)) break;
                }
                PROF_MARK(2);
                for (;;) {  // one symbol a step up to the stop
                    const bool go = !done && pm + 1 < stop;
                    if (!__any(go)) break;
                    if (go) {
                        const uint32_t w = __builtin_amdgcn_alignbit(x0, x1, ~(uint32_t)pm);
                        const int32_t d = E - pm - 1;
                        const uint32_t wm = w | (uint32_t)(0xFFFFFFFFull >> (uint32_t)min(max(d, 0), 32));
                        const uint32_t e = Tb.lut[wm >> (32 - HHUFF_LUT_BITS)];
                        uint32_t sym = e, L = lut_l1(e), fl = e & (3u << 24);
                        bool eos = false;
                        if ((int32_t)e < 0) {
                            const uint32_t le = long_entry(wm);
                            sym = le;
                            L = (le >> 9) & 31u;
                            fl = (le >> 14) << 24 & (3u << 24);
                            eos = (le & 0x1FFu) == kEos;
                        }
                        if ((int32_t)L <= d && !eos) {
                            lds_st8(o, sym);
                            o += 1u;
                            accb |= fl;
                            advance((int32_t)L);
                        } else {
                            close(!(eos && (int32_t)L <= d) && d >= 0 && d <= 7 && wm == 0xFFFFFFFFu);
                            advance(0);
                        }
                    }
                }
                // a string whose last symbol ends exactly here is closed by the lane that took that symbol (no
                // padding bits: the next string starts here, past the stop or not)
                if (!done && pm + 1 == E) close(true);
                if (need) ek = (uint32_t)(pm + 1);
                PROF_MARK(3);
                const uint32_t eprev = (uint32_t)__shfl((int)ek, lane > 0 ? lane - 1 : 0);
                const bool mism = act && lane > 0 && f != eprev;
                if (__builtin_amdgcn_ballot_w64(mism) == 0 || round > 65u) break;
                need = mism;
                if (mism) f = eprev;
            }
            const bool ovf = act && nrec > kSegRecs;
            if (__builtin_amdgcn_ballot_w64(ovf) != 0) {
                // more closes than records: one lane per string from global memory (output byte-exact)
                if (mine && (uint32_t)lane < mw) {
                    uint32_t ol;
                    uint8_t stt;
                    decode_direct(A, s, len, is_name, A.out + dec_slot(s), Tb, ol, stt);
                    A.out_len[i] = ol;
                    A.status[i] = stt;
                }
                if (lane == 0) {
                    if (first_sub) erec[0].m = make_uint4(0u, 0u, 0u, 0u);
                    if (last_sub) erec[1].m = make_uint4(0u, 0u, 0u, 0u);
                }
                PROF_MARK(6);
            } else {
                // ---- places: the part continuing the lane before's last string follows it (affine scan) ----
                const uint32_t tlen = act ? (o - r0) - pstart : 0u;  // the trailing part's bytes
                const bool cont = act && f < Bend && f > sbt[lf];
                const bool through = act && nrec == 0u;
                const uint32_t tprev = (uint32_t)__shfl((int)tlen, lane > 0 ? lane - 1 : 0);
                const bool thprev = __shfl((int)through, lane > 0 ? lane - 1 : 0) != 0;
                uint32_t sa = cont && thprev && lane > 0 ? 1u : 0u, sbv = cont && lane > 0 ? tprev : 0u;
#pragma unroll
                for (int d = 1; d < 64; d <<= 1) {
                    const uint32_t ap = (uint32_t)__shfl_up((int)sa, d), bp = (uint32_t)__shfl_up((int)sbv, d);
                    if (lane >= d) {
                        sbv = sa ? bp + sbv : sbv;
                        sa = sa & ap;
                    }
                }
                const uint32_t prefix = sbv;
                // the lane's parts, oldest first: its records, then the trailing part
                auto part = [&](uint32_t k, uint32_t& pl, uint32_t& pend, uint32_t& pfl) {
                    if (k < nrec) {
                        const uint32_t sh = nrec - 1u - k;
                        const uint32_t rec = (uint32_t)((sh < 4u ? rlo >> (16u * sh) : rhi >> (16u * (sh - 4u))) & 0xFFFFu);
                        pl = rec & 63u;
                        pend = (rec >> 6) & 127u;
                        pfl = ((rec >> 13) & 3u) | (1u << 4) | ((rec >> 15) << 3);
                    } else {
                        pl = l;
                        pend = o - r0;
                        pfl = ((accb >> 24) | (accb >> 26) | (accl >> 14)) & 3u;
                    }
                };
                if (act) {
                    uint32_t ps = 0;
                    for (uint32_t k = 0; k <= nrec; ++k) {
                        uint32_t pl, pend, pfl;
                        part(k, pl, pend, pfl);
                        if (pl < mw) {
                            atomicOr(&aflg[pl], pfl);
                            if (pend > ps) {
                                atomicAdd(&acnt[pl], pend - ps);
                                atomicMin(&afst[pl], ((uint32_t)lane << 8) | lds_ld8(r0 + ps));
                                atomicMax(&alst[pl], ((uint32_t)lane << 8) | lds_ld8(r0 + pend - 1u));
                            }
                        }
                        ps = pend;
                    }
                }
                const uint64_t obase = dec_slot(lo) & ~15ull;
                const uint32_t ospan = hi > lo ? (uint32_t)(((dec_slot(hi) + 15u) & ~15ull) - obase) : 0u;
                wave_lds_sync();
#ifndef HHUFF_SEG_NOFIN  // ablation builds: no moves and no copy-out (output wrong by design)
                lds_zero(stage8, 0u, (ospan + 15u) & ~15u, lane);
                wave_lds_sync();
                if (act) {
                    uint32_t ps = 0;
                    for (uint32_t k = 0; k <= nrec; ++k) {
                        uint32_t pl, pend, pfl;
                        part(k, pl, pend, pfl);
                        if (pl < mw && pend > ps && (aflg[pl] & 0x18u) == 0x18u) {
                            const uint32_t dst = (uint32_t)(dec_slot(a0 + sbt[pl] / 8u) - obase) + (k == 0 && cont ? prefix : 0u);
                            lds_move_or(r0 + ps, fsa + dst, pend - ps);
                        }
                        ps = pend;
                    }
                }
                wave_lds_sync();
                consume_next();
                PROF_MARK(4);
                region_copy_seg(A.out, obase, stage8, ospan, dec_slot(lo), dec_slot(hi), lane, first_sub ? erec : nullptr,
                                last_sub ? erec + 1 : nullptr);
#else
                consume_next();
                if (lane == 0) {
                    if (first_sub) erec[0].m = make_uint4(0u, 0u, 0u, 0u);
                    if (last_sub) erec[1].m = make_uint4(0u, 0u, 0u, 0u);
                }
#endif
                if (mine && (uint32_t)lane < mw) {
                    if (len == 0) {
                        A.out_len[i] = 0u;
                        A.status[i] = soft_bits(is_name, 0u, 0u, 0u, 0u);
                    } else {
                        const uint32_t fl = aflg[lane], cnt = acnt[lane];
                        const bool ok = (fl & 0x18u) == 0x18u;
                        A.out_len[i] = ok ? cnt : kFailLen;
                        A.status[i] = ok ? soft_bits(is_name, cnt, fl & 3u, afst[lane] & 0xFFu, alst[lane] & 0xFFu) : kStatusFail;
                    }
                }
            }
            PROF_MARK(5);
            if (excl) {  // the long last string: too long, listed for split decode, or this lane
                if (len > kMaxStrLen) {
                    A.out_len[i] = kFailLen;
                    A.status[i] = kStatusTooLong;
                } else if (!split_push(A, i, len)) {
                    uint32_t ol;
                    uint8_t stt;
                    decode_direct(A, s, len, is_name, A.out + dec_slot(s), Tb, ol, stt);
                    A.out_len[i] = ol;
                    A.status[i] = stt;
                }
            }
            wave_lds_sync();
        }
    }
    }
    PROF_FLUSH(0);
}

