// hhuff_variants.h -- kernel variants kept for A/B builds (included by hhuff_kernels.hip after every helper
// they use).  Each was built to parity and measured against the default kernel (DESIGN.md (e), round 5;
// profiles/r05*): none is instantiated unless its build flag is set (HHUFF_DEC_SW, HHUFF_STREAM2,
// HHUFF_STREAM_RK, HHUFF_ENC_INPLACE, HHUFF_DEC_RUN).
#pragma once

// ------------------------------------------------------------------------------------------------
// Staged decode with store waves (HHUFF_DEC_SW; contiguous layout, slot output, deferred edges).  On gfx950
// loads and stores share one in-order counter, so in decode_staged_kernel the next tile's prefetched span is
// waited for behind the previous tile's output stores: with no stores at all the c4 decode runs 19 % faster
// (profiles/r05t_nt_store_ab.jsonl).  Here 15 waves decode and never store: a wave leaves its tile's output
// stage, lengths, statuses and region in LDS and posts the tile (an LDS flag); the 16th wave reads the stage
// out into registers, hands it back (another flag) and issues the stores.  A decode wave waits for its stage
// only before the next tile's steps write into it.  LDS-only fences, so no wave waits on global memory for a
// hand-over.  Same results as decode_staged_kernel.
// ------------------------------------------------------------------------------------------------
#ifndef HHUFF_DEC_SW_NSW  // store waves of decode_staged_sw_kernel's 16, and the tiles one takes at once
#define HHUFF_DEC_SW_NSW 2
#endif
#ifndef HHUFF_DEC_SW_NB
#define HHUFF_DEC_SW_NB 2
#endif
constexpr uint32_t kSwSkip = 0xFFFFFFFEu;  // a posted length the store wave skips (listed / past n)
struct SwTile {                            // a posted tile: its output region and records
    uint64_t gbase, keep_lo, keep_hi;
    uint32_t ospan, rec, base, pad;
};
__device__ __forceinline__ uint32_t lds_ld_acq(const uint32_t* p) {
    const uint32_t v = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
    return v;
}
__device__ __forceinline__ void lds_st_rel(uint32_t* p, uint32_t v) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
template <int IN_STAGE, int OUT_STAGE, int NSW>
__global__ __launch_bounds__(1024) void decode_staged_sw_kernel(DecArgs A) {
    constexpr int NDW = 16 - NSW;  // decode waves; waves NDW.. store (store wave s serves decode waves s, s + NSW, ...)
    constexpr int NB = HHUFF_DEC_SW_NB;  // tiles a store wave takes at once
    constexpr uint32_t Z = IN_STAGE + OUT_STAGE + 256u;
    constexpr int NCHO = (OUT_STAGE + 1023) / 1024;
    struct __attribute__((aligned(16))) Smem {
        uint32_t lut[1u << HHUFF_LUT_BITS];
        uint32_t kinfo[32];
        uint32_t ones[(HHUFF_ONES_NENT + 3) & ~3];
        uint8_t buf[NDW][Z + 16];
        SwTile tile[NDW];
        uint32_t len[NDW][64];
        uint8_t st[NDW][64];
        uint32_t posted[NDW], drained[NDW], finished;
    };
    __shared__ Smem sm;
    load_dec_tables(sm.lut, sm.kinfo, sm.ones, 1024);
    if (threadIdx.x < NDW) sm.posted[threadIdx.x] = sm.drained[threadIdx.x] = 0u;
    if (threadIdx.x == 0) sm.finished = 0u;
    __syncthreads();
    const DecTables T{sm.lut, sm.kinfo, sm.ones};
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;

    if (wave >= NDW) {  // ---- a store wave ----
        const int sw = wave - NDW;
        const bool mine = lane < NDW && lane % NSW == sw;  // lane w watches decode wave w
        uint32_t drained = 0;  // lane w: tiles of decode wave w stored so far
        for (;;) {
            const uint32_t posted = mine ? lds_ld_acq(&sm.posted[lane]) : 0u;
            const uint64_t ready = __builtin_amdgcn_ballot_w64(mine && posted != drained);
            if (ready == 0) {
                if (lds_ld_acq(&sm.finished) == (uint32_t)NDW) {  // every wave is done: one last look
                    const uint32_t p2 = mine ? lds_ld_acq(&sm.posted[lane]) : 0u;
                    if (__builtin_amdgcn_ballot_w64(mine && p2 != drained) == 0) break;
                    continue;
                }
                __builtin_amdgcn_s_sleep(1);
                continue;
            }
            // up to NB ready tiles at once: their stages read out, handed back with one fence, then stored
            int ws[NB];
            SwTile d[NB];
            uint4 v[NB][NCHO];
            uint32_t ol[NB];
            uint8_t stt[NB];
            uint64_t left = ready;
#pragma unroll
            for (int b = 0; b < NB; ++b) {
                ws[b] = left ? __builtin_ctzll(left) : -1;
                left &= left - 1u;
                if (ws[b] >= 0) {  // (wave-uniform)
                    const int w = ws[b];
                    const SwTile x = sm.tile[w];  // (wave-uniform: into SGPRs)
                    auto u64 = [](uint64_t q) {
                        return (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)q) |
                               (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(q >> 32)) << 32;
                    };
                    d[b].gbase = u64(x.gbase);
                    d[b].keep_lo = u64(x.keep_lo);
                    d[b].keep_hi = u64(x.keep_hi);
                    d[b].ospan = (uint32_t)__builtin_amdgcn_readfirstlane((int)x.ospan);
                    d[b].rec = (uint32_t)__builtin_amdgcn_readfirstlane((int)x.rec);
                    d[b].base = (uint32_t)__builtin_amdgcn_readfirstlane((int)x.base);
                    const uint8_t* obuf = sm.buf[w] + IN_STAGE;
#pragma unroll
                    for (int c = 0; c < NCHO; ++c) {
                        const uint32_t kk = (uint32_t)c * 1024u + (uint32_t)lane * 16u;
                        if (kk < d[b].ospan) v[b][c] = *reinterpret_cast<const uint4*>(obuf + kk);
                    }
                    ol[b] = sm.len[w][lane];
                    stt[b] = sm.st[w][lane];
                }
            }
            // the stages and records are in registers: hand the stages back (the fence waits for these reads)
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
#pragma unroll
            for (int b = 0; b < NB; ++b) {
                if (ws[b] >= 0) {
                    const uint32_t pw = (uint32_t)__builtin_amdgcn_readlane((int)posted, ws[b]);
                    if (lane == ws[b]) drained = pw;
                    if (lane == 0) __hip_atomic_store(&sm.drained[ws[b]], pw, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                }
            }
#pragma unroll
            for (int b = 0; b < NB; ++b) {
                if (ws[b] < 0) continue;
                EdgeRec* rec = A.edges + 2 * (uint64_t)d[b].rec;
                const uint32_t kl = d[b].ospan ? (d[b].ospan - 1u) & ~15u : 0u;
#pragma unroll
                for (int c = 0; c < NCHO; ++c) {
                    const uint32_t kk = (uint32_t)c * 1024u + (uint32_t)lane * 16u;
                    if (kk < d[b].ospan) {
                        const uint64_t g = d[b].gbase + kk;
                        const bool full = g >= d[b].keep_lo && g + 16 <= d[b].keep_hi;
                        if (full) st16_out(A.out + g, v[b][c]);
                        if (kk == 0 || kk == kl) {
                            const uint32_t lo = d[b].keep_lo > g ? (uint32_t)(d[b].keep_lo - g) : 0u;
                            const uint32_t hi = d[b].keep_hi - g < 16 ? (uint32_t)(d[b].keep_hi - g) : 16u;
                            EdgeRec* r = rec + (kk == 0 ? 0 : 1);
                            r->v = v[b][c];
                            r->m = make_uint4((uint32_t)g, (uint32_t)(g >> 32), full ? 0u : lo, full ? 0u : hi);
                            if (kl == 0) rec[1].m = make_uint4(0u, 0u, 0u, 0u);
                        }
                    }
                }
                if (d[b].ospan == 0 && lane == 0) {
                    rec[0].m = make_uint4(0u, 0u, 0u, 0u);
                    rec[1].m = make_uint4(0u, 0u, 0u, 0u);
                }
                if (ol[b] != kSwSkip) {
                    A.out_len[d[b].base + (uint32_t)lane] = ol[b];
                    A.status[d[b].base + (uint32_t)lane] = stt[b];
                }
            }
        }
        return;
    }

    // ---- the decode waves: decode_staged_kernel's pipeline (slot layout), stores handed to the store wave ----
    uint8_t* const buf = sm.buf[wave];
    const uint64_t stride = (uint64_t)gridDim.x * NDW * 64;
    uint64_t base = ((uint64_t)blockIdx.x * NDW + wave) * 64;
    uint32_t seq = 0;  // tiles this wave has posted
    if (base >= A.n) {
        if (lane == 0) __hip_atomic_fetch_add(&sm.finished, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
        return;
    }
    struct Plan {
        uint32_t s, len, op0;
        uint32_t lo, hi, ospan;
        bool valid, fits;
        __device__ __forceinline__ uint32_t a0() const { return lo & ~15u; }
        __device__ __forceinline__ uint32_t span() const { return hi > lo ? ((hi + 15u) & ~15u) - a0() : 0u; }
        __device__ __forceinline__ uint64_t olo() const { return dec_slot(lo); }
        __device__ __forceinline__ uint64_t ohi() const { return dec_slot(hi); }
        __device__ __forceinline__ uint64_t obase() const { return olo() & ~15ull; }
    };
    auto plan = [&](uint64_t b, const TileIn& ti) {
        Plan P;
        const Tile t = finish_tile(b, lane, A.n, ti, false);
        P.s = t.s;
        P.len = t.len;
        P.valid = t.valid;
        P.lo = __builtin_amdgcn_readfirstlane(t.lo);
        P.hi = __builtin_amdgcn_readfirstlane(t.hi);
        P.ospan = P.hi > P.lo ? (uint32_t)(P.ohi() - P.obase()) : 0u;
        P.op0 = t.len ? (uint32_t)(dec_slot(t.s) - P.obase()) : 0u;
        P.fits = P.span() <= IN_STAGE && P.ospan <= OUT_STAGE;
        return P;
    };
    SpanPrefetch<(IN_STAGE + 1023) / 1024> pf;
    TileIn ti = issue_tile(base, lane, A.n, A.in_off, nullptr, A.is_name_bits, nullptr);
    Plan cur = plan(base, ti);
    uint32_t cur_name = ti.name_word;
    if (cur.fits) pf.issue(A.in, A.in_size, cur.a0(), cur.span(), lane);
    bool have_next = base + stride < A.n;
    ti = issue_tile(base + stride, lane, A.n, A.in_off, nullptr, A.is_name_bits, nullptr);
    if (cur.fits) pf.template commit<true>(reinterpret_cast<uint32_t*>(buf), A.in, A.in_size, cur.a0(), cur.span(), lane);
    Plan nxt;
    uint32_t nxt_name = 0;
    if (have_next) {
        nxt = plan(base + stride, ti);
        nxt_name = ti.name_word;
        if (nxt.fits) pf.issue(A.in, A.in_size, nxt.a0(), nxt.span(), lane);
        ti = issue_tile(base + 2 * stride, lane, A.n, A.in_off, nullptr, A.is_name_bits, nullptr);
    }
    uint32_t* stage = reinterpret_cast<uint32_t*>(buf);
    uint8_t* obuf = buf + IN_STAGE;
    for (;;) {
        const uint64_t nbase = base + stride;
        const Plan& t = cur;
        const uint32_t ti_i = (uint32_t)base + (uint32_t)lane;
        const bool is_name = t.valid && A.is_name_bits ? ((cur_name >> (ti_i & 31)) & 1u) : false;
        uint32_t ol = 0;
        uint8_t st = 0;
        bool listed = false;
        if (cur.fits) {
            // the store wave has read the last posted tile's stage out before this tile's steps overwrite it
            while (lds_ld_acq(&sm.drained[wave]) != seq) __builtin_amdgcn_s_sleep(1);
            wave_lds_sync();
            const bool act = t.valid && t.len <= kMaxStrLen;
            const uint32_t rel = t.len ? t.s - cur.a0() : 0u;
            const DecResult r = decode_staged_lane_v7(stage, rel, t.len, act, obuf, cur.op0, OUT_STAGE + 4u * (uint32_t)lane, T);
            if (t.valid && t.len > kMaxStrLen) {
                ol = kFailLen;
                st = kStatusTooLong;
            } else if (r.ok) {
                ol = r.len;
                const uint32_t first = r.len ? obuf[cur.op0] : 0u, lastc = r.len ? obuf[cur.op0 + r.len - 1] : 0u;
                st = soft_bits(is_name, r.len, r.flags, first, lastc);
            } else {
                ol = kFailLen;
                st = kStatusFail;
            }
            // post the tile: lengths, statuses and region into LDS, then the flag
            sm.len[wave][lane] = t.valid ? ol : kSwSkip;
            sm.st[wave][lane] = st;
            if (lane == 0) {
                SwTile d;
                d.gbase = cur.obase();
                d.keep_lo = cur.olo();
                d.keep_hi = cur.ohi();
                d.ospan = cur.ospan;
                d.rec = (uint32_t)(base >> 6);
                d.base = (uint32_t)base;
                d.pad = 0;
                sm.tile[wave] = d;
            }
            ++seq;
            if (lane == 0) lds_st_rel(&sm.posted[wave], seq);
        } else if (t.valid) {  // a tile larger than the stages: this wave stores it itself (no edges to defer)
            if (split_push(A, ti_i, t.len)) {
                listed = true;
            } else {
                decode_direct(A, t.s, t.len, is_name, A.out + dec_slot(t.s), T, ol, st);
            }
        }
        if (!cur.fits) {
            if (lane == 0) {
                A.edges[2 * (base >> 6)].m = make_uint4(0u, 0u, 0u, 0u);
                A.edges[2 * (base >> 6) + 1].m = make_uint4(0u, 0u, 0u, 0u);
            }
            if (t.valid && !listed) {
                A.out_len[ti_i] = ol;
                A.status[ti_i] = st;
            }
        }
        // ---- the next tile: commit its span (the input stage is free), plan + prefetch the one after ----
        if (have_next && nxt.fits)
            pf.template commit<true>(stage, A.in, A.in_size, nxt.a0(), nxt.span(), lane);
        const bool have_nn = have_next && nbase + stride < A.n;
        Plan nn = plan(nbase + stride, ti);
        const uint32_t nn_name = ti.name_word;
        if (have_nn && nn.fits) pf.issue(A.in, A.in_size, nn.a0(), nn.span(), lane);
        ti = issue_tile(nbase + 2 * stride, lane, A.n, A.in_off, nullptr, A.is_name_bits, nullptr);
        if (!have_next) break;
        cur = nxt;
        cur_name = nxt_name;
        nxt = nn;
        nxt_name = nn_name;
        have_next = have_nn;
        base = nbase;
    }
    if (lane == 0) __hip_atomic_fetch_add(&sm.finished, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}


// ------------------------------------------------------------------------------------------------
// Streaming decode v2 (mixed and long lengths; same results as decode_stream_kernel / decode_core).  The
// rounds of decode_stream_kernel, with no global-memory round trip on a lane's way from one string to the
// next -- there every string start cost a dependent chain (the work counter, the string's offsets, its first
// window) that stalled the whole wave once per round in which any lane took a string:
//   * a wave claims batches of 64 strings from the counter one batch ahead and keeps each batch's fields in
//     registers (lane l holds string b + l: offset, length, is-name bit, destination); a lane takes its next
//     string by ds_bpermute from them;
//   * a lane whose string ends inside this round's window reserves its next string at the start of the
//     round and prefetches that string's first window (in place of its own continuation) for the next round;
//   * one per-lane LDS buffer of BW dwords (odd: lanes at the same position hit distinct banks) holds the
//     output from its start and the window at its end; a round's output grows at most 1.6x as fast as the
//     window is consumed and starts 0.6 of a window below it, so it never overtakes unread window bytes.
// ------------------------------------------------------------------------------------------------
// 16 bytes of LDS at a 4-aligned address (the odd-stride buffers are not 16-aligned)
__device__ __forceinline__ uint4 lds_ld16(const uint8_t* p) {
    const uint32_t* q = reinterpret_cast<const uint32_t*>(p);
    return make_uint4(q[0], q[1], q[2], q[3]);
}
__device__ __forceinline__ void lds_st16(uint8_t* p, uint4 v) {
    uint32_t* q = reinterpret_cast<uint32_t*>(p);
    q[0] = v.x, q[1] = v.y, q[2] = v.z, q[3] = v.w;
}
// store_range16 with the chunk in registers
__device__ __forceinline__ void store_range16v(uint8_t* __restrict__ g, uint4 v, uint32_t lo, uint32_t hi) {
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (uint32_t k = 0; k < 4; ++k)
        if (lo <= 4u * k && 4u * k + 4u <= hi) *reinterpret_cast<uint32_t*>(g + 4u * k) = w[k];
    const uint64_t q0 = (uint64_t)v.y << 32 | v.x, q1 = (uint64_t)v.w << 32 | v.z;
    auto byte_at = [&](uint32_t a) { return (uint32_t)((a < 8u ? q0 : q1) >> (8u * (a & 7u))); };
    const uint32_t e0 = min(hi, (lo + 3u) & ~3u);
    const uint32_t s1 = max(max(lo, hi & ~3u), e0);
#pragma unroll
    for (uint32_t j = 0; j < 3; ++j) {
        if (lo + j < e0) g[lo + j] = (uint8_t)byte_at(lo + j);
        if (s1 + j < hi) g[s1 + j] = (uint8_t)byte_at(s1 + j);
    }
}

// ------------------------------------------------------------------------------------------------
// Stream decode with the output in registers (round 5; VERDICT r4 "next" #1 route b).  decode_stream_kernel keeps
// a 160-B LDS output buffer per lane beside its 100-B window: 6 waves a CU, 1.5 a SIMD, 56 % of wave cycles
// parked.  Here a lane's output goes into one 16-B chunk held in four VGPRs, aligned to the output's 16-B grid:
// a full chunk leaves with one 16-B store (the first chunk of a string, shared with the string before, with
// byte-exact stores), the partial chunk simply stays in its registers from round to round, and the string's
// last chunk leaves byte-exact at its end.  No output buffer and no flush phase: 16 waves a CU fit the LDS (the
// 32-KiB LUT + 100 B of window per lane).  (Round 2 measured a register output with a 4-B store per dword: c3
// 0.316 -> 0.360 ms; here one 16-B store per 16 bytes, no more stores than the LDS version's flush.)
// ------------------------------------------------------------------------------------------------
struct RegChunk {  // 16 output bytes at global [g, g + 16): L = bytes 0..7, H = 8..15; p bytes filled; lo = first ours
    uint64_t L, H;
    uint64_t g;
    uint32_t p, lo;
    __device__ __forceinline__ void start(uint64_t dst) {
        g = dst & ~15ull;
        p = lo = (uint32_t)(dst & 15u);
        L = H = 0;
    }
    __device__ __forceinline__ void flush_full(uint8_t* __restrict__ out) {
        const uint4 v = make_uint4((uint32_t)L, (uint32_t)(L >> 32), (uint32_t)H, (uint32_t)(H >> 32));
        if (lo == 0)
            *reinterpret_cast<uint4*>(out + g) = v;
        else
            store_range16v(out + g, v, lo, 16u);
    }
    __device__ __forceinline__ void flush_part(uint8_t* __restrict__ out) {  // the string's last bytes
        if (p > lo) store_range16v(out + g, make_uint4((uint32_t)L, (uint32_t)(L >> 32), (uint32_t)H, (uint32_t)(H >> 32)),
                                   lo, p);
    }
    // n (0..2) bytes of v at position p; a chunk that fills up leaves at once (the second byte of a pair at p = 15
    // starts the next chunk)
    __device__ __forceinline__ void put(uint8_t* __restrict__ out, uint32_t v, uint32_t n) {
        const uint64_t x = (uint64_t)(v & (n >= 2u ? 0xFFFFu : (n ? 0xFFu : 0u)));
        const uint32_t sh = 8u * p;
        L |= sh < 64u ? x << sh : 0ull;
        H |= sh >= 64u ? x << (sh - 64u) : (sh > 48u ? x >> (64u - sh) : 0ull);
        p += n;
        if (p >= 16u) {
            flush_full(out);
            g += 16u;
            lo = 0;
            p -= 16u;
            L = p ? x >> 8 : 0ull;  // (p is 0 or 1)
            H = 0;
        }
    }
};

template <int WAVES, int NW>
__global__ __launch_bounds__(WAVES * 64) void decode_stream_rk_kernel(DecArgs A, unsigned long long* __restrict__ counter) {
    static_assert(NW >= 8 && NW % 4 == 0, "window shape");
    constexpr uint32_t kWS = NW + 1;  // odd dword stride: lanes at the same q hit distinct banks
    struct __attribute__((aligned(16))) Smem {
        uint32_t lut[1u << HHUFF_LUT_BITS];
        uint32_t kinfo[32];
        uint32_t ones[(HHUFF_ONES_NENT + 3) & ~3];
        uint32_t win[WAVES * 64][kWS];  // [0]: the dword before the window (read, never used)
    };
    if (A.gate && *A.gate != kGateStream) return;  // block-uniform: decode_select_kernel chose the staged kernel
    __shared__ Smem sm;
    load_dec_tables(sm.lut, sm.kinfo, sm.ones, WAVES * 64);
    __syncthreads();
    const DecTables T{sm.lut, sm.kinfo, sm.ones};
    const int lane = threadIdx.x & 63;
    uint32_t* win = &sm.win[threadIdx.x][1];
    const lds_u32* st = (const lds_u32*)win;
    constexpr int32_t kLimW = 32 * (NW - 2) - 30;  // bulk steps start below this window bit
    constexpr int32_t kFinal = 32 * (NW - 2);      // a string ending at or before this bit ends in the window

    uint4 pfv[NW / 4];
    uint64_t pfa = ~0ull;
    bool busy = false, is_name = false;
    uint32_t i = 0, s = 0, len = 0, P = 0, ocnt = 0, flags = 0, first = 0, lastb = 0, fail = 0;
    RegChunk ch;
    ch.start(0);
    uint64_t bnext = 0, bend = 0;
    bool qdone = false;
    const uint64_t nwork = A.n_dev ? (uint64_t)*A.n_dev : (uint64_t)A.n;

    for (;;) {
        // ---- 1. idle lanes take strings ----
        for (int it = 0; it < 2; ++it) {
            const uint64_t need = __builtin_amdgcn_ballot_w64(!busy);
            if (need == 0) break;
            if (bnext >= bend) {
                if (qdone) break;
                uint64_t b = 0;
                if (lane == 0) b = atomicAdd(counter, 64ull);
                b = ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(b >> 32)) << 32) |
                    (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)b);
                if (b >= nwork) {
                    qdone = true;
                    break;
                }
                bnext = b;
                bend = min(b + 64u, nwork);
            }
            const uint32_t rank = (uint32_t)__builtin_amdgcn_mbcnt_hi((uint32_t)(need >> 32),
                                                                      __builtin_amdgcn_mbcnt_lo((uint32_t)need, 0u));
            if (!busy && bnext + rank < bend) {
                i = (uint32_t)(bnext + rank);
                s = A.in_off[i];
                len = A.in_len ? A.in_len[i] : A.in_off[i + 1] - s;
                is_name = A.is_name_bits ? ((A.is_name_bits[i >> 5] >> (i & 31)) & 1u) : false;
                const uint64_t dst = A.out_off ? (uint64_t)A.out_off[i] : dec_slot(s);
                if (len > kMaxStrLen) {
                    A.out_len[i] = kFailLen;
                    A.status[i] = kStatusTooLong;
                } else if (!split_push(A, i, len)) {
                    busy = true;
                    ch.start(dst);
                    P = ocnt = flags = first = lastb = fail = 0;
                }
            }
            bnext = min(bend, bnext + (uint64_t)__builtin_popcountll(need));
        }
        if (!__any(busy)) {
            if (qdone) break;
            continue;
        }

        // ---- 2. the lane's window (as decode_stream_kernel) ----
        const uint64_t cur = (uint64_t)s + (P >> 3);
        const uint64_t wb = cur & ~3ull;
        const uint64_t rem = (uint64_t)len * 8u - P;
        if (busy) {
            if (wb != pfa) {
#pragma unroll
                for (int j = 0; j < NW / 4; ++j) pfv[j] = load16_bounded(A.in, A.in_size, wb + 16u * j);
            }
#pragma unroll
            for (int j = 0; j < NW / 4; ++j) {
                win[4 * j + 0] = bswap32(pfv[j].x);
                win[4 * j + 1] = bswap32(pfv[j].y);
                win[4 * j + 2] = bswap32(pfv[j].z);
                win[4 * j + 3] = bswap32(pfv[j].w);
            }
            pfa = rem + 8u * (uint32_t)(cur - wb) + (P & 7u) > 32u * (NW - 2) ? wb + 4u * (NW - 3) : ~0ull;
            if (pfa != ~0ull) {
#pragma unroll
                for (int j = 0; j < NW / 4; ++j) pfv[j] = load16_bounded(A.in, A.in_size, pfa + 16u * j);
            }
        }
        int32_t pm = busy ? (int32_t)(8u * (uint32_t)(cur - wb) + (P & 7u)) - 1 : -1;
        const int32_t pm0 = pm;
        const int32_t end = busy ? (int32_t)min((uint64_t)(pm + 1) + rem, (uint64_t)0x40000000u) : 0;
        const bool fin = busy && end <= kFinal;
        int32_t q = pm >> 5;
        uint32_t x0 = st[q], x1 = st[q + 1], x2 = st[q + 2];
        uint32_t accb = 0, acc1 = 0, accl = 0, parked = busy ? 0u : 1u;
        uint32_t made = 0;
        int32_t lim = busy ? min(end - 26, kLimW) : (int32_t)0x80000000;
        auto advance = [&](int32_t cons) {
            pm += cons;
            const int32_t qn = pm >> 5;
            const bool adv = qn != q;
            x0 = adv ? x1 : x0;
            x1 = adv ? x2 : x1;
            q = qn;
            x2 = st[q + 2];
        };
        // n symbol bytes (the low n of v) to the output, first / last byte remembered
        auto emit = [&](uint32_t v, uint32_t n) {
            first = (ocnt + made) == 0u && n ? (v & 0xFFu) : first;
            lastb = n == 2u ? ((v >> 8) & 0xFFu) : (n ? (v & 0xFFu) : lastb);
            made += n;
            ch.put(A.out, v, n);
        };

        // ---- 3a. bulk ----
        auto bstep = [&](bool longchk) {
            if (pm < lim) {
                const uint32_t w = __builtin_amdgcn_alignbit(x0, x1, ~(uint32_t)pm);
                const uint32_t e = T.lut[w >> (32 - HHUFF_LUT_BITS)];
                const uint32_t sl = (uint32_t)((int32_t)e >> 31);
                emit(lut_pair(e), (e >> 28) & 3u);
                accb |= e;
                uint32_t cons = lut_l12(e);
                {
                    const uint32_t eb = T.lut[(w << cons) >> (32 - HHUFF_LUT_BITS)];
                    emit(lut_pair(eb), (eb >> 28) & 3u);
                    accb |= eb;
                    cons += lut_l12(eb);
                }
                if (longchk && __builtin_amdgcn_ballot_w64(sl != 0u) != 0) {
                    if (sl) {
                        const uint32_t k = min((uint32_t)__builtin_clz(~w | 1u), 30u);
                        const uint32_t ki = T.kinfo[k];
                        const uint32_t le = T.ones[(ki & 0xFFFFu) + (((w << (k + 1)) >> 1) >> (31 - (ki >> 16)))];
                        const int32_t L = (le >> 9) & 31u;
                        const bool fits = L + pm < end;
                        const bool eos = (le & 0x1FFu) == kEos;
                        fail |= fits && eos ? 1u : 0u;  // EOS inside the string (hpack.c:88-89)
                        if (fits && !eos) {
                            emit(le, 1u);
                            accl |= le;
                            cons = (uint32_t)L;
                        } else {
                            parked = 1u;
                            lim = (int32_t)0x80000000;
                        }
                    }
                }
                advance((int32_t)cons);
            }
        };
        for (;;) {
            bstep(false);
            bstep(true);
            if (!__any(pm < lim)) break;
        }

        // ---- 3b. tail: lanes whose string ends in this window, one symbol a step checked against the end ----
        bool tdone = !(fin && !parked);
        for (;;) {
            const bool go = !tdone;
            if (!__any(go)) break;
            if (go) {
                const uint32_t w = __builtin_amdgcn_alignbit(x0, x1, ~(uint32_t)pm);
                const uint32_t e = T.lut[w >> (32 - HHUFF_LUT_BITS)];
                uint32_t sym = e, L = lut_l1(e), fl = e & (3u << 24);
                bool eos = false;
                if ((int32_t)e < 0) {
                    const uint32_t k = min((uint32_t)__builtin_clz(~w | 1u), 30u);
                    const uint32_t ki = T.kinfo[k];
                    const uint32_t le = T.ones[(ki & 0xFFFFu) + (((w << (k + 1)) >> 1) >> (31 - (ki >> 16)))];
                    sym = le;
                    L = (le >> 9) & 31u;
                    fl = ((le >> 14) & 3u) << 24;
                    eos = (le & 0x1FFu) == kEos;
                }
                const int32_t R = end - 1 - pm;  // string bits left
                if ((int32_t)L <= R && !eos) {
                    emit(sym, 1u);
                    acc1 |= fl;
                    advance((int32_t)L);
                } else {
                    fail |= eos && (int32_t)L <= R ? 1u : 0u;  // EOS inside the string (hpack.c:88-89)
                    tdone = true;  // no code fits: the padding
                }
            }
        }

        // ---- 4. finish strings ----
        if (busy) {
            flags |= ((accb >> 24) | (accb >> 26) | (acc1 >> 24) | (accl >> 14)) & 3u;
            const bool done = parked || fin;
            bool ok = false;
            if (fin && !parked && !fail) {  // padding: at most 7 bits, all ones (hpack.c:132-133)
                const int32_t R = end - 1 - pm;
                const uint32_t w = __builtin_amdgcn_alignbit(x0, x1, ~(uint32_t)pm);
                ok = R >= 0 && R <= 7 && (w | (0xFFFFFFFFu >> R)) == 0xFFFFFFFFu;
            }
            ocnt += made;
            P += (uint32_t)(pm - pm0);
            if (done) {
                if (ok) ch.flush_part(A.out);
                A.out_len[i] = ok ? ocnt : kFailLen;
                A.status[i] = ok ? soft_bits(is_name, ocnt, flags, first, lastb) : kStatusFail;
                busy = false;
            }
        }
    }
}

struct StreamBatch {  // lane l: string b + l of a claimed batch of 64 (cnt of them exist)
    uint64_t b;
    uint32_t cnt;
    uint32_t s, lw;  // offset; length (clamped to kMaxStrLen + 1) | is-name << 31
    uint32_t dst;    // explicit destination (out_off) or 0
};

template <int WAVES, int NW, int BW>
__global__ __launch_bounds__(WAVES * 64) void decode_stream2_kernel(DecArgs A, unsigned long long* __restrict__ counter) {
    static_assert(NW >= 8 && NW % 4 == 0 && (BW & 1) == 1, "window shape; odd buffer stride");
    // in place: output [0, ...) below the window at WOFF (dwords [WOFF/4 - 1, WOFF/4 + NW) with the dword read
    // before it), then a trash dword.  Output after c window bytes <= 15 + 1.6 c + 3 bytes, unread window >=
    // WOFF + c: WOFF >= 15 + 0.6 (4 NW) + 3
    constexpr uint32_t WOFF = ((15u + (12u * NW + 4u) / 5u + 3u + 4u) + 3u) & ~3u;
    static_assert(WOFF + 4u * NW + 4u <= 4u * BW, "buffer too small for the window");
    static_assert(15 + (32 * (NW - 2)) / 5 + 2 < WOFF + 4 * NW, "output past the window's end");
    struct __attribute__((aligned(16))) Smem {
        uint32_t lut[1u << HHUFF_LUT_BITS];
        uint32_t kinfo[32];
        uint32_t ones[(HHUFF_ONES_NENT + 3) & ~3];
        uint32_t buf[WAVES * 64][BW];
    };
    if (A.gate && *A.gate != kGateStream) return;  // block-uniform: decode_select_kernel chose the staged kernel
    __shared__ Smem sm;
    load_dec_tables(sm.lut, sm.kinfo, sm.ones, WAVES * 64);
    __syncthreads();
    const DecTables T{sm.lut, sm.kinfo, sm.ones};
    const int lane = threadIdx.x & 63;
    uint8_t* obuf = reinterpret_cast<uint8_t*>(sm.buf[threadIdx.x]);
    uint32_t* win = reinterpret_cast<uint32_t*>(obuf + WOFF);
    const lds_u32* st = (const lds_u32*)win;
    const uint32_t ob = lds_addr(obuf), trash = ob + WOFF + 4u * NW + 3u;
    constexpr int32_t kLimW = 32 * (NW - 2) - 30;  // bulk steps start below this window bit
    constexpr int32_t kFinal = 32 * (NW - 2);      // a string ending at or before this bit ends in the window

    const uint64_t nwork = A.n_dev ? (uint64_t)*A.n_dev : (uint64_t)A.n;
    if (nwork == 0) return;
    auto claim = [&](StreamBatch& X) {
        uint64_t b = 0;
        if (lane == 0) b = atomicAdd(counter, 64ull);
        b = ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(b >> 32)) << 32) |
            (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)b);
        X.b = b;
        X.cnt = b < nwork ? (uint32_t)min(nwork - b, (uint64_t)64) : 0u;
        const uint64_t i = min(b + (uint64_t)lane, nwork - 1u);  // clamped: every load issues
        X.s = A.in_off[i];
        const uint32_t len = A.in_len ? A.in_len[i] : A.in_off[i + 1] - X.s;
        const uint32_t nm = A.is_name_bits ? (A.is_name_bits[i >> 5] >> (i & 31)) & 1u : 0u;
        X.lw = min(len, kMaxStrLen + 1u) | nm << 31;
        X.dst = A.out_off ? A.out_off[i] : 0u;
    };
    StreamBatch QA, QB;
    claim(QA);
    claim(QB);
    uint32_t qpos = 0;  // wave-uniform: strings of QA taken so far
    // hand the queue's next strings to the lanes in `need` (in lane order); false where the queue is dry
    auto take = [&](uint64_t need, uint32_t& i, uint32_t& s, uint32_t& lw, uint64_t& dst) {
        const uint32_t rank = (uint32_t)__builtin_amdgcn_mbcnt_hi((uint32_t)(need >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)need, 0u));
        const uint32_t k = qpos + rank;
        const bool inA = k < 64u;
        const uint32_t src = (k & 63u) << 2;
        const uint32_t sa = (uint32_t)__builtin_amdgcn_ds_bpermute((int)src, (int)QA.s);
        const uint32_t la = (uint32_t)__builtin_amdgcn_ds_bpermute((int)src, (int)QA.lw);
        const uint32_t da = A.out_off ? (uint32_t)__builtin_amdgcn_ds_bpermute((int)src, (int)QA.dst) : 0u;
        // QB only when the takers run past QA (wave-uniform): its loads, issued at its claim, are waited
        // for only here
        uint32_t sb = 0, lb = 0, db = 0;
        if (qpos + (uint32_t)__builtin_popcountll(need) > 64u) {
            sb = (uint32_t)__builtin_amdgcn_ds_bpermute((int)src, (int)QB.s);
            lb = (uint32_t)__builtin_amdgcn_ds_bpermute((int)src, (int)QB.lw);
            if (A.out_off) db = (uint32_t)__builtin_amdgcn_ds_bpermute((int)src, (int)QB.dst);
        }
        const bool ok = ((need >> lane) & 1u) && (inA ? k < QA.cnt : (QA.cnt == 64u && k - 64u < QB.cnt));
        i = (uint32_t)((inA ? QA.b : QB.b) + (k & 63u));
        s = inA ? sa : sb;
        lw = inA ? la : lb;
        dst = A.out_off ? (uint64_t)(inA ? da : db) : dec_slot(s);
        qpos += (uint32_t)__builtin_popcountll(need);
        if (qpos >= 64u) {  // QA is used up: QB moves up, the next batch is claimed behind it
            QA = QB;
            qpos -= 64u;
            claim(QB);
        }
        return ok;
    };
    auto dry = [&]() { return qpos >= QA.cnt && (QA.cnt < 64u || QB.cnt == 0u); };  // wave-uniform

    // per-lane string state; the reserved next string; the prefetched window (its input address: pfa)
    bool busy = false, head = false, is_name = false, rv = false;
    uint32_t i = 0, s = 0, len = 0, P = 0, ocnt = 0, flags = 0, first = 0, lastb = 0, fail = 0;
    uint64_t dst = 0;
    uint32_t ri = 0, rs = 0, rlw = 0;
    uint64_t rdst = 0;
    uint4 pfv[NW / 4];
    uint64_t pfa = ~0ull;
    PROF_DECL

    for (;;) {
        // ---- 1. lanes without a string start their reserved one (or take one now: the first round, or after
        //      a string that failed early) ----
        {
            const uint64_t need = __builtin_amdgcn_ballot_w64(!busy && !rv);
            if (need != 0 && !dry()) rv = take(need, ri, rs, rlw, rdst) || rv;
        }
        if (!busy && rv) {
            rv = false;
            i = ri, s = rs, len = rlw & 0x7FFFFFFFu, is_name = (rlw >> 31) != 0, dst = rdst;
            if (len > kMaxStrLen) {
                A.out_len[i] = kFailLen;
                A.status[i] = kStatusTooLong;
            } else {
                busy = true;
                head = (dst & 15u) != 0;
                P = ocnt = flags = first = lastb = fail = 0;
            }
        }
        if (!__any(busy)) {
            if (dry() && !__any(rv)) {
                PROF_FLUSH(0);
                break;
            }
            continue;
        }
        PROF_MARK(0);

        // ---- 2. the lane's window: NW dwords from its current byte (dword-aligned), prefetched last round
        //      unless the string started unannounced ----
        const uint64_t cur = (uint64_t)s + (P >> 3);
        const uint64_t wb = cur & ~3ull;
        const uint64_t rem = (uint64_t)len * 8u - P;  // string bits left
        if (busy) {
            if (wb != pfa) {
#pragma unroll
                for (int j = 0; j < NW / 4; ++j) pfv[j] = load16_bounded(A.in, A.in_size, wb + 16u * j);
            }
#pragma unroll
            for (int j = 0; j < NW / 4; ++j) {
                win[4 * j + 0] = bswap32(pfv[j].x);
                win[4 * j + 1] = bswap32(pfv[j].y);
                win[4 * j + 2] = bswap32(pfv[j].z);
                win[4 * j + 3] = bswap32(pfv[j].w);
            }
        }
        int32_t pm = busy ? (int32_t)(8u * (uint32_t)(cur - wb) + (P & 7u)) - 1 : -1;
        const int32_t pm0 = pm;
        const int32_t end = busy ? (int32_t)min((uint64_t)(pm + 1) + rem, (uint64_t)0x40000000u) : 0;
        const bool fin = busy && end <= kFinal;
        // ---- 3. a lane whose string ends in this window reserves its next one and prefetches that string's
        //      first window; the others prefetch their continuation ----
        {
            const uint64_t need = __builtin_amdgcn_ballot_w64(fin && !rv);
            if (need != 0 && !dry()) rv = take(need, ri, rs, rlw, rdst) || rv;
        }
        {
            const bool cont = busy && !fin;  // the string goes on past this window
            pfa = cont ? wb + 4u * (NW - 3) : (fin && rv && (rlw & 0x7FFFFFFFu) <= kMaxStrLen) ? (uint64_t)(rs & ~3u) : ~0ull;
            if (pfa != ~0ull) {
#pragma unroll
                for (int j = 0; j < NW / 4; ++j) pfv[j] = load16_bounded(A.in, A.in_size, pfa + 16u * j);
            }
        }
        PROF_MARK(1);
        const uint32_t h0 = (uint32_t)((dst + ocnt) & 15u);  // buffer offset of this round's first byte
        uint32_t o = ob + h0;
        int32_t q = pm >> 5;
        uint32_t x0 = st[q], x1 = st[q + 1], x2 = st[q + 2];
        uint32_t accb = 0, acc1 = 0, acc2 = 0, accl = 0, parked = busy ? 0u : 1u;
        int32_t lim = busy ? min(end - 26, kLimW) : (int32_t)0x80000000;
        auto advance = [&](int32_t cons) {
            pm += cons;
            const int32_t qn = pm >> 5;
            const bool adv = qn != q;
            x0 = adv ? x1 : x0;
            x1 = adv ? x2 : x1;
            q = qn;
            x2 = st[q + 2];
        };

        // ---- 4a. bulk (decode_staged_lane_v7's step) ----
        auto bstep = [&](bool longchk) {
            if (pm < lim) {
                const uint32_t w = __builtin_amdgcn_alignbit(x0, x1, ~(uint32_t)pm);
                const uint32_t e = T.lut[w >> (32 - HHUFF_LUT_BITS)];
                const uint32_t sl = (uint32_t)((int32_t)e >> 31);
                bulk_put2(o, e, trash);
                o += (e >> 28) & 3u;
                accb |= e;
                uint32_t cons = lut_l12(e);  // LONG entries carry L12 = 0
                {
                    const uint32_t wb2 = w << cons;
                    const uint32_t eb = T.lut[wb2 >> (32 - HHUFF_LUT_BITS)];
                    bulk_put2(o, eb, trash);
                    o += (eb >> 28) & 3u;
                    accb |= eb;
                    cons += lut_l12(eb);
                }
                if (longchk && __builtin_amdgcn_ballot_w64(sl != 0u) != 0) {
                    if (sl) {
                        const uint32_t k = min((uint32_t)__builtin_clz(~w | 1u), 30u);
                        const uint32_t ki = T.kinfo[k];
                        const uint32_t le = T.ones[(ki & 0xFFFFu) + (((w << (k + 1)) >> 1) >> (31 - (ki >> 16)))];
                        const int32_t L = (le >> 9) & 31u;
                        const uint32_t fits = (uint32_t)((L + pm - end) >> 31);
                        const uint32_t eos = (le & 0x1FFu) == kEos ? 0xFFFFFFFFu : 0u;
                        const uint32_t okm = fits & ~eos;
                        fail |= fits & eos & 1u;  // EOS inside the string (hpack.c:88-89)
                        lds_st8(sel_bits(okm, o, trash), le);
                        o -= okm;
                        accl |= le & okm;
                        cons = okm & (uint32_t)L;
                        parked |= ~okm & 1u;
                        lim = (int32_t)sel_bits(okm, (uint32_t)lim, 0x80000000u);
                    }
                }
                advance((int32_t)cons);
            }
        };
        for (;;) {
            bstep(false);
            bstep(true);
            if (!__any(pm < lim)) break;
        }
        PROF_MARK(2);

        // ---- 4b. tail: lanes whose string ends in this window ----
        int32_t c = (fin && !parked) ? pm - end : 0x40000000;
        if (__any(fin)) {
            int32_t prog = 0;
            auto step = [&](bool longchk) {
                const uint32_t w = __builtin_amdgcn_alignbit(x0, x1, ~(uint32_t)pm);
                const uint32_t e = T.lut[w >> (32 - HHUFF_LUT_BITS)];
                const int32_t L1 = lut_l1(e), L12 = lut_l12(e);
                const int32_t s1 = L1 + c, s2 = L12 + c;
                const uint32_t m1 = (uint32_t)((s1 & ~(int32_t)e) >> 31);
                const uint32_t m2 = (uint32_t)((s2 & (int32_t)(e << 1)) >> 31);
                int32_t cons = (int32_t)sel_bits(m2, (uint32_t)L12, m1 & (uint32_t)L1);
                lds_st8(sel_bits(m1, o - m2, trash), lut_sym2(e));
                lds_st8(sel_bits(m1, o, trash), e);
                o = o - m1 - m2;
                acc1 |= e & m1;
                acc2 |= e & m2;
                {
                    const uint32_t wb2 = w << cons;
                    const uint32_t eb = T.lut[wb2 >> (32 - HHUFF_LUT_BITS)];
                    const int32_t cb = c + cons;
                    const int32_t L1b = lut_l1(eb), L12b = lut_l12(eb);
                    const uint32_t m1b = (uint32_t)(((L1b + cb) & ~(int32_t)eb) >> 31);
                    const uint32_t m2b = (uint32_t)(((L12b + cb) & (int32_t)(eb << 1)) >> 31);
                    lds_st8(sel_bits(m1b, o - m2b, trash), lut_sym2(eb));
                    lds_st8(sel_bits(m1b, o, trash), eb);
                    o = o - m1b - m2b;
                    acc1 |= eb & m1b;
                    acc2 |= eb & m2b;
                    cons += (int32_t)sel_bits(m2b, (uint32_t)L12b, m1b & (uint32_t)L1b);
                }
                const bool lact = (s1 & (int32_t)e) < 0;
                uint32_t consl = 0;
                if (longchk && __builtin_amdgcn_ballot_w64(lact) != 0) {
                    if (lact) {
                        const uint32_t k = min((uint32_t)__builtin_clz(~w | 1u), 30u);
                        const uint32_t ki = T.kinfo[k];
                        const uint32_t le = T.ones[(ki & 0xFFFFu) + (((w << (k + 1)) >> 1) >> (31 - (ki >> 16)))];
                        const int32_t L = (le >> 9) & 31u;
                        const uint32_t fits = (uint32_t)((L + c) >> 31);
                        const uint32_t eos = (le & 0x1FFu) == kEos ? 0xFFFFFFFFu : 0u;
                        const uint32_t okm = fits & ~eos;
                        fail |= fits & eos & 1u;
                        lds_st8(sel_bits(okm, o, trash), le);
                        o -= okm;
                        accl |= le & okm;
                        consl = okm & (uint32_t)L;
                        c = (int32_t)sel_bits(okm, (uint32_t)c, 0x40000000u);
                    }
                }
                cons |= (int32_t)consl;
                c += cons;
                advance(cons);
                prog = cons;
            };
            step(true);
            for (;;) {
                step(false);
                step(true);
                if (!__any(prog != 0)) break;
            }
        }
        PROF_MARK(3);

        // ---- 5. flush whole chunks, carry the partial one; finish strings ----
        if (busy) {
            flags |= ((accb >> 24) | (accb >> 26) | (acc1 >> 24) | (acc2 >> 26) | (accl >> 14)) & 3u;
            const uint32_t nb = o - ob;  // buffer bytes: h0 carried (or, at a string's start, foreign) + produced
            const uint32_t made = nb - h0;
            if (made) {
                if (ocnt == 0) first = obuf[h0];
                lastb = obuf[nb - 1u];
            }
            const bool done = parked || fin;
            const bool ok = fin && !parked && !fail && [&] {
                const uint32_t R = ~(uint32_t)c;
                const uint32_t w = __builtin_amdgcn_alignbit(x0, x1, ~(uint32_t)pm);
                return R <= 7 && (w | (0xFFFFFFFFu >> (R & 31u))) == 0xFFFFFFFFu;
            }();
            uint8_t* gchunk = A.out + ((dst + ocnt) & ~15ull);
            const uint32_t hs = (uint32_t)(dst & 15u);  // head chunk: the string's bytes start here
#ifdef HHUFF_X_NOSTORE  // ablation builds (output wrong by design): no global stores at all
            if (false) {
#else
            if (!done || ok) {  // a failed string's output is unspecified: skip its last stores
#endif
                const uint32_t nfull = nb >> 4;
                for (uint32_t k = 0; k < nfull; ++k) {
                    const uint4 v = lds_ld16(obuf + 16u * k);
                    if (head && k == 0)
                        store_range16v(gchunk, v, hs, 16u);
                    else
                        *reinterpret_cast<uint4*>(gchunk + 16u * k) = v;
                }
                head = head && nfull == 0;
                const uint32_t part = nb & 15u;
                if (done) {
                    if (part > (head ? hs : 0u))
                        store_range16v(gchunk + 16u * nfull, lds_ld16(obuf + 16u * nfull), head ? hs : 0u, part);
                } else if (nfull) {
                    lds_st16(obuf, lds_ld16(obuf + 16u * nfull));
                }
            }
            ocnt += made;
            P += (uint32_t)(pm - pm0);
            if (done) {
#ifndef HHUFF_X_NOSTORE
                A.out_len[i] = ok ? ocnt : kFailLen;
                A.status[i] = ok ? soft_bits(is_name, ocnt, flags, first, lastb) : kStatusFail;
#endif
                busy = false;
            }
        }
        PROF_MARK(4);
    }
}


// ------------------------------------------------------------------------------------------------
// In-place sorted encode (HHUFF_ENC_INPLACE; review r4 next 3).  encode_sorted_kernel's chunks with one stage
// instead of two, so a workgroup of 4 waves holds 512 strings and each thread encodes a sorted pair (ranks t and
// NS - 1 - t): the lanes' work is even across the workgroup (no wave waits at a barrier for a longest length
// group) at the same 16 waves a CU.  A string's output slot is its own input range, so its codes overwrite its
// own bytes:
//   * a lane clears exactly its own bytes of each input word as it reads it (one ds_and_rtn: the word's value
//     comes back, the neighbours' bytes stay), one word ahead of the word it encodes, so its OR-placed codes
//     land on zeros and the slot's tail is zero at the end;
//   * codes that would end past the words it has read (a prefix of long codes outrunning the input) are not
//     placed: the lane counts on, and a string that stays shorter than its input is encoded again from global
//     memory after the chunk's encode barrier (`redo`; strings of random bytes fail on their own);
//   * each thread puts the next chunk's span into the stage piece by piece as it copies its pieces out.
// Same results as encode_core (hpack.c:774-804).
// ------------------------------------------------------------------------------------------------
struct EncIP {
    const uint2* enc;
    uint32_t obase;  // LDS byte address of the stage (input and MSB-first output)
    uint32_t tb;     // next stage bit
    uint32_t tlim;   // stage bit at which the string fails
    bool live, fail, haz;
    // one masked dword (a string's first or last word): rlim = the stage bit below which every word is read
    __device__ __forceinline__ void put4(uint2 e0, uint2 e1, uint2 e2, uint2 e3, bool on, uint32_t rlim) {
        const uint32_t n01 = e0.y + e1.y, n23 = e2.y + e3.y, n = n01 + n23;
        const bool lng = max(max(e0.y, e1.y), max(e2.y, e3.y)) > 16u;
        const bool over = on && live && tb + n >= tlim;
        fail = fail || over;
        live = live && !over;
        haz = haz || (on && live && tb + n > rlim);
        const bool put = on && live && !haz;
        if (__any(put && lng)) {
            if (put && lng) {
                place_bits(obase, tb, (uint64_t)e0.x << e1.y | e1.x, n01);
                place_bits(obase, tb + n01, (uint64_t)e2.x << e3.y | e3.x, n23);
            }
        }
        const bool f = put && !lng;
        const uint32_t p01 = e0.x << e1.y | e1.x, p23 = e2.x << e3.y | e3.x;
        const uint64_t cc = f ? ((uint64_t)p01 << n23 | p23) : 0ull;
        place_bits(obase, tb, cc, f ? n : 0u);
        tb += (on && live) ? n : 0u;  // a lane past its read words counts on (its verdict decides the redo)
    }
    // one whole dword (bulk), predicates as VGPR masks (EncV2::put4m); hzm: sticky "stopped placing" mask
    __device__ __forceinline__ void put4m(uint2 e0, uint2 e1, uint2 e2, uint2 e3, uint32_t onm, uint32_t rlim,
                                          uint32_t& hzm) {
        const uint32_t n01 = e0.y + e1.y, n23 = e2.y + e3.y, n = n01 + n23;
        const uint32_t mx = max(max(e0.y, e1.y), max(e2.y, e3.y));
        const uint32_t lngm = (uint32_t)((int32_t)(16u - mx) >> 31);
        const uint32_t nm = n & onm;
        const uint32_t okm = (uint32_t)((int32_t)(tb + nm - tlim) >> 31);        // still below the fail bit
        const uint32_t rdm = ~(uint32_t)((int32_t)(rlim - (tb + nm)) >> 31);     // ends inside the read words
        hzm |= onm & okm & ~rdm;
        const uint32_t putm = onm & okm & ~hzm;
        if (__builtin_amdgcn_ballot_w64((putm & lngm) != 0u) != 0) {
            if (putm & lngm) {
                place_bits(obase, tb, (uint64_t)e0.x << e1.y | e1.x, n01);
                place_bits(obase, tb + n01, (uint64_t)e2.x << e3.y | e3.x, n23);
            }
        }
        const uint32_t fm = putm & ~lngm;
        const uint32_t p01 = e0.x << e1.y | e1.x, p23 = e2.x << e3.y | e3.x;
        const uint64_t cc = ((uint64_t)p01 << n23 | p23) & ((uint64_t)fm << 32 | fm);
        const uint32_t nf = n & fm;
        const uint64_t t = cc << ((64u - nf) & 63u);
        const uint32_t sh = tb & 31u;
        const uint64_t u = t >> sh;
        const uint32_t a = obase + ((tb >> 3) & ~3u);
        lds_or32(a, (uint32_t)(u >> 32));
        lds_or32(a + 4u, (uint32_t)u);
        if (__builtin_amdgcn_ballot_w64(sh + nf > 64u) != 0) {
            if (sh + nf > 64u) lds_or32(a + 8u, (uint32_t)t << (32u - sh));
        }
        tb += nm;
    }
};

// Encode stage bytes [start, start + len) in place (stage at LDS byte address sbase; `last`: the stage's last
// word offset, where reads are clamped).  Returns the code bits or kFailLen; redo = the codes were counted
// but not all placed (the string is still to be encoded: encode_redo).
__device__ __forceinline__ uint32_t encode_inplace_lane(uint32_t sbase, uint32_t last, uint32_t start, uint32_t len,
                                                        bool active, const uint2* __restrict__ enc, uint32_t limit,
                                                        bool& redo) {
    const uint32_t end = start + len;
    const uint32_t a0 = start & ~3u, a0w = a0 >> 2, lastw = last >> 2;
    const uint32_t ndw = active ? (end - a0 + 3u) >> 2 : 0u;  // the string's words [a0w, a0w + ndw)
    const uint32_t jl = active ? (end - a0) >> 2 : 0u;        // whole words [1, jl) after word 0; tail word jl
    // the stage holds big-endian words (committed byte-swapped): string byte k of a word at bits 31 - 8k, the
    // same place the MSB-first output puts stream byte k -- so a lane's codes fall on its own bytes
    const uint32_t mfirst = 0xFFFFFFFFu >> (8u * (start & 3u));
    const uint32_t mlast = (uint32_t)(0xFFFFFFFFull << ((32u - 8u * (end & 3u)) & 31u));
    auto mo = [&](uint32_t q) -> uint32_t {  // this string's bytes of its word q
        const uint32_t m = (q == 0 ? mfirst : 0xFFFFFFFFu) & (q + 1u == ndw ? mlast : 0xFFFFFFFFu);
        return q < ndw ? m : 0u;
    };
    auto rc = [&](uint32_t q) -> uint32_t {  // read word q and clear this string's bytes of it
        const uint32_t idx = min(a0w + q, lastw);
        return __hip_atomic_fetch_and((lds_u32*)(size_t)(sbase + 4u * idx), ~mo(q), __ATOMIC_RELAXED,
                                      __HIP_MEMORY_SCOPE_WORKGROUP);
    };
    const uint32_t startbit = 8u * start, base = 32u * a0w;
    EncIP E{enc, sbase, startbit, limit >= 0x40000000u ? 0x7FFFFFFFu : startbit + limit, active, false, false};
    auto masked = [&](uint32_t w, uint32_t vm, bool on, uint32_t rlim) {
        vm = on ? vm : 0u;
        const uint32_t iw = ~vm & 0x01010101u;
        E.put4(enc[__builtin_amdgcn_perm(iw, w, 0x0C0C0703u)], enc[__builtin_amdgcn_perm(iw, w, 0x0C0C0602u)],
               enc[__builtin_amdgcn_perm(iw, w, 0x0C0C0501u)], enc[__builtin_amdgcn_perm(iw, w, 0x0C0C0400u)], on, rlim);
    };
    const uint32_t w0 = rc(0);
    uint32_t wn = rc(1);  // one word ahead: read (and cleared) before word 0's codes are placed
    uint32_t wt = wn;     // the tail word's value (word jl), kept as the bulk loop reads past it
    masked(w0, mo(0), active && ndw != 0, base + 32u * min(2u, ndw));
    {
        const uint32_t jlv = E.live ? jl : 0u;  // a lane that failed in word 0 places nothing more
        const uint32_t jend = wave_max_u32(jlv);
        uint32_t hzm = E.haz ? 0xFFFFFFFFu : 0u;
        for (uint32_t j = 1; j < jend; ++j) {  // bulk: whole words
            const uint32_t w = wn;
            wn = rc(j + 1u);
            wt = j + 1u == jl ? wn : wt;
            const uint32_t onm = j < jlv ? 0xFFFFFFFFu : 0u;
            E.put4m(enc[w >> 24], enc[(w >> 16) & 0xFFu], enc[(w >> 8) & 0xFFu], enc[w & 0xFFu], onm,
                    base + 32u * min(j + 2u, ndw), hzm);
        }
        E.haz = E.haz || hzm != 0u;
    }
    E.fail = E.fail || (E.live && E.tb >= E.tlim);
    E.live = E.live && !E.fail;
    masked(wt, mlast, active && (end & 3u) != 0 && jl >= 1u, base + 32u * ndw);  // tail
    if (E.fail || !active) return kFailLen;
    if (E.haz) {
        redo = true;
        return E.tb - startbit;
    }
    const uint32_t p = (0u - E.tb) & 7u;  // EOS-prefix padding (hpack.c:795-798)
    place_bits(sbase, E.tb, (1ull << p) - 1ull, p);
    return E.tb - startbit;
}

// A string encode_inplace_lane stopped placing: its bytes cleared and its codes placed again, reading the
// input from global memory (after the chunk's encode barrier: every lane's reads are done).
__device__ __forceinline__ void encode_redo(uint32_t sbase, const uint8_t* __restrict__ in, uint64_t in_size, uint64_t g0,
                                         uint32_t start, uint32_t len, const uint2* __restrict__ enc) {
    const uint32_t end = start + len, a0w = start >> 2, ndw = (end - (start & ~3u) + 3u) >> 2;
    const uint32_t mfirst = 0xFFFFFFFFu >> (8u * (start & 3u));  // (big-endian stage words)
    const uint32_t mlast = (uint32_t)(0xFFFFFFFFull << ((32u - 8u * (end & 3u)) & 31u));
    for (uint32_t q = 0; q < ndw; ++q) {
        const uint32_t m = (q == 0 ? mfirst : 0xFFFFFFFFu) & (q + 1u == ndw ? mlast : 0xFFFFFFFFu);
        __hip_atomic_fetch_and((lds_u32*)(size_t)(sbase + 4u * (a0w + q)), ~m, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    const GlobalSource src{in, in_size};
    uint32_t tb = 8u * start;
    const uint64_t g1 = g0 + len;
    for (uint64_t a = g0 & ~3ull; a < g1; a += 4) {
        const uint32_t w = src.word(a);
        for (uint32_t k = 0; k < 4; ++k) {
            if (a + k < g0 || a + k >= g1) continue;
            const uint2 e = enc[(w >> (8 * k)) & 0xFFu];
            place_bits(sbase, tb, e.x, e.y);
            tb += e.y;
        }
    }
    const uint32_t p = (0u - tb) & 7u;
    place_bits(sbase, tb, (1ull << p) - 1ull, p);
}

// a chunk's two strings per thread (offsets) and its span bounds (made wave-uniform once landed)
struct PairChunk {
    uint32_t s0, e0, s1, e1, lo, hi;
};
#ifndef HHUFF_ENCI_EARLY_SPAN
#define HHUFF_ENCI_EARLY_SPAN 0
#endif
#ifndef HHUFF_ENCI_WPE  // waves per SIMD the register allocation is held to (4: 128 VGPRs)
#define HHUFF_ENCI_WPE 4
#endif
template <int NS, int CH, int SPT>
__global__ __launch_bounds__(NS / SPT) __attribute__((amdgpu_waves_per_eu(HHUFF_ENCI_WPE, HHUFF_ENCI_WPE))) void encode_inplace_kernel(EncArgs A) {
    static_assert(SPT == 1 || SPT == 2, "one string a thread, or a sorted pair");
    constexpr uint32_t NT = NS / SPT;
    constexpr int NV = (CH + 16 * NT - 1) / (16 * NT);  // 16-B span pieces per thread
    __shared__ __attribute__((aligned(16))) uint2 s_enc[512];  // 256..511: bytes outside a string
    __shared__ __attribute__((aligned(16))) uint32_t s_st[CH / 4 + 8];
    __shared__ uint2 s_str[NS];  // {offset in the span, length} of chunk string t (.x: then its encoded length)
    __shared__ uint16_t s_perm[NS];
    __shared__ uint32_t s_bin[kSortBins];
    __shared__ uint32_t s_redo;
    const uint32_t t = threadIdx.x, lane = t & 63u;
    const uint32_t sbase = lds_addr(s_st);
    for (uint32_t k = t; k < 512; k += NT) s_enc[k] = k < 256 ? make_uint2(g_enc_code[k], g_enc_nbits[k]) : make_uint2(0u, 0u);
    const uint32_t nch = (uint32_t)(((uint64_t)A.n + NS - 1) / NS);  // (32-bit chunk and string indices)
    uint32_t c = blockIdx.x;
    if (c >= nch) return;
    auto issue_chunk = [&](uint32_t qb) {  // (clamped: every load issues)
        PairChunk q;
        const uint32_t i0 = min(qb + t, A.n - 1u), i1 = min(qb + t + NT, A.n - 1u);
        q.s0 = A.in_off[i0];
        q.e0 = A.in_off[i0 + 1];
        q.s1 = SPT == 2 ? A.in_off[i1] : 0u;
        q.e1 = SPT == 2 ? A.in_off[i1 + 1] : 0u;
        q.lo = A.in_off[min(qb, A.n - 1u)];
        q.hi = A.in_off[min(qb + NS, A.n)];
        return q;
    };
    auto land = [](PairChunk& q) {  // its loads are waited for here; the bounds then live in SGPRs
        __asm__ volatile("" : "+v"(q.s0), "+v"(q.e0), "+v"(q.s1), "+v"(q.e1), "+v"(q.lo), "+v"(q.hi) : : "memory");
        q.lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)q.lo);
        q.hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)q.hi);
    };
    auto span_of = [](const PairChunk& q) { return q.hi > q.lo ? ((q.hi + 15u) & ~15u) - (q.lo & ~15u) : 0u; };
    auto issue_span = [&](uint4 (&v)[NV], const PairChunk& q) {
        const uint32_t a0 = q.lo & ~15u, span = span_of(q);
#pragma unroll
        for (int j = 0; j < NV; ++j) {
            const uint32_t k = (uint32_t)j * (16u * NT) + t * 16u;
            const uint64_t g = (uint64_t)a0 + k;
            if (k < span && span <= (uint32_t)CH && g + 16 <= A.in_size) v[j] = *reinterpret_cast<const uint4*>(A.in + g);
        }
    };
    // piece j of q's span (the input's end: bounded), its words byte-swapped: the stage holds big-endian words
    auto piece = [&](const uint4 (&v)[NV], int j, const PairChunk& q) {
        const uint64_t g = (uint64_t)(q.lo & ~15u) + (uint32_t)j * (16u * NT) + t * 16u;
        const uint4 x = g + 16 <= A.in_size ? v[j] : load16_tail(A.in, A.in_size, g);
        return make_uint4(bswap32(x.x), bswap32(x.y), bswap32(x.z), bswap32(x.w));
    };
    uint32_t bin[2], rank[2];
    auto meta = [&](const PairChunk& q, uint32_t qb) {  // the chunk's string records and length ranks
        const uint32_t ss[2] = {q.s0, q.s1}, ee[2] = {q.e0, q.e1};
#pragma unroll
        for (int u = 0; u < SPT; ++u) {
            const uint32_t tt = t + (uint32_t)u * NT;
            const uint32_t ln = qb + tt < A.n ? ee[u] - ss[u] : 0u;
            s_str[tt] = make_uint2(ss[u] - (q.lo & ~15u), ln);
            bin[u] = ln ? min((ss[u] + ln - (ss[u] & ~3u)) >> 2, kSortBins - 1u) : 0u;
            rank[u] = atomicAdd(&s_bin[bin[u]], 1u);
        }
    };
    for (uint32_t k = t; k < kSortBins; k += NT) s_bin[k] = 0u;
    if (t == 0) s_redo = 0u;
    __syncthreads();
    uint4 pv[NV];
    PairChunk cur = issue_chunk(c * NS);
    land(cur);
    issue_span(pv, cur);
    if (span_of(cur) <= (uint32_t)CH) {
#pragma unroll
        for (int j = 0; j < NV; ++j) {
            const uint32_t k = (uint32_t)j * (16u * NT) + t * 16u;
            if (k < span_of(cur)) *reinterpret_cast<uint4*>(reinterpret_cast<uint8_t*>(s_st) + k) = piece(pv, j, cur);
        }
        meta(cur, c * NS);
    }
    PairChunk nxt = issue_chunk((c + gridDim.x < nch ? c + gridDim.x : c) * NS);
    land(nxt);  // (once)
    for (;;) {
        const uint32_t cb = c * NS;
        const uint32_t lo = cur.lo, hi = cur.hi, a0 = lo & ~15u, span = span_of(cur);
        EdgeRec* rec = A.edges + 2 * c;
        const uint32_t cn = c + gridDim.x, cn2 = cn + gridDim.x;
        const bool more = cn < nch;
        __syncthreads();  // barrier 1: the chunk's stage, records and ranks are in
        if (span > (uint32_t)CH) {  // (workgroup-uniform) a chunk larger than the stage: one thread per string
            const uint32_t ss[2] = {cur.s0, cur.s1}, ee[2] = {cur.e0, cur.e1};
#pragma unroll
            for (int u = 0; u < SPT; ++u) {
                const uint32_t i = cb + t + (uint32_t)u * NT;
                const uint32_t len = i < A.n ? ee[u] - ss[u] : 0u;
                uint32_t ol = kFailLen;
                if (i < A.n && len <= kMaxStrLen) {
                    RegSink sink;
                    sink.init(A.out + ss[u]);
                    ol = encode_core(GlobalSource{A.in, A.in_size}, ss[u], len, sink, s_enc);
                }
                if (i < A.n) finish_encode(A, i, len, ol);
            }
            if (t < 2) rec[t].m = make_uint4(0u, 0u, 0u, 0u);  // direct stores: no edges to defer
            if (!more) break;
            issue_span(pv, nxt);
            if (span_of(nxt) <= (uint32_t)CH) {
#pragma unroll
                for (int j = 0; j < NV; ++j) {
                    const uint32_t k = (uint32_t)j * (16u * NT) + t * 16u;
                    if (k < span_of(nxt)) *reinterpret_cast<uint4*>(reinterpret_cast<uint8_t*>(s_st) + k) = piece(pv, j, nxt);
                }
                meta(nxt, cn * NS);
            }
            PairChunk nn = issue_chunk((cn2 < nch ? cn2 : cn) * NS);
            land(nn);
            cur = nxt;
            nxt = nn;
            c = cn;
            continue;
        }
        {  // every wave scans the bin counts (two per lane)
            const uint32_t x0 = s_bin[2 * lane], x1 = s_bin[2 * lane + 1];
            const uint32_t ex = wave_excl_scan(x0 + x1, (int)lane);
#pragma unroll
            for (int u = 0; u < SPT; ++u) {
                const uint32_t eb = (uint32_t)__shfl((int)ex, (int)(bin[u] >> 1)), xb = (uint32_t)__shfl((int)x0, (int)(bin[u] >> 1));
                s_perm[eb + ((bin[u] & 1u) ? xb : 0u) + rank[u]] = (uint16_t)(t + (uint32_t)u * NT);
            }
        }
        __syncthreads();  // barrier 2: the sorted order is in
        for (uint32_t k = t; k < kSortBins; k += NT) s_bin[k] = 0u;
#if HHUFF_ENCI_EARLY_SPAN  // the next chunk's span in flight during the encode (its 28 VGPRs spill the encode)
        if (more) issue_span(pv, nxt);
#endif
#if HHUFF_ENCI_EARLY_SPAN
        PairChunk nn = issue_chunk((cn2 < nch ? cn2 : (more ? cn : c)) * NS);
#endif
        uint32_t rdo[2] = {0u, 0u};  // a string to encode again: its span offset | its length << 16
#pragma unroll
        for (int u = 0; u < SPT; ++u) {  // sorted positions t and NS - 1 - t: a short and a long string
            const uint32_t j = s_perm[u == 0 ? t : NS - 1u - t];
            const uint2 sj = s_str[j];
            const bool act = cb + j < A.n && sj.y != 0 && sj.y <= kMaxStrLen;
            bool rd = false;
            const uint32_t tb = encode_inplace_lane(sbase, span - 4u, sj.x, sj.y, act, s_enc,
                                                    act ? 8 * sj.y - 7 : 0xFFFFFFFFu, rd);
            s_str[j].x = act && tb != kFailLen ? (tb + 7) >> 3 : kFailLen;
            if (rd) {
                s_redo = 1u;
                rdo[u] = sj.x | sj.y << 16;  // (offsets and lengths < CH < 2^16)
            }
        }
        __syncthreads();  // barrier 3: every string encoded (or counted)
        if (s_redo != 0u) {  // (workgroup-uniform) strings whose codes outran their reads: encoded again
#pragma unroll
            for (int u = 0; u < SPT; ++u)
                if (rdo[u] >> 16)
                    encode_redo(sbase, A.in, A.in_size, (uint64_t)a0 + (rdo[u] & 0xFFFFu), rdo[u] & 0xFFFFu, rdo[u] >> 16, s_enc);
            __syncthreads();
            if (t == 0) s_redo = 0u;
        }
#if !HHUFF_ENCI_EARLY_SPAN
        // the next chunk's span and the chunk after next's offsets: in flight while the records are read and
        // ranked (issued during the encode, their registers would spill the encode's)
        if (more) issue_span(pv, nxt);
        PairChunk nn = issue_chunk((cn2 < nch ? cn2 : (more ? cn : c)) * NS);
#endif
        const uint2 r0 = s_str[t], r1 = SPT == 2 ? s_str[t + NT] : make_uint2(0u, 0u);  // {encoded length, length}
        // the chunk after next's offsets and the next span land here, before this chunk's stores (no load is
        // waited for behind a data-dependent number of stores)
        land(nn);
#pragma unroll
        for (int j = 0; j < NV; ++j) __asm__ volatile("" : "+v"(pv[j].x), "+v"(pv[j].y), "+v"(pv[j].z), "+v"(pv[j].w) : : "memory");
        const uint32_t nspan = more ? span_of(nxt) : 0u;
        const bool ncommit = nspan <= (uint32_t)CH;
        if (more && ncommit) meta(nxt, cn * NS);  // (s_str is read above)
        if (cb + t < A.n) finish_encode(A, cb + t, r0.y, r0.x);
        if (SPT == 2 && cb + t + NT < A.n) finish_encode(A, cb + t + NT, r1.y, r1.x);
        // copy out the stage's MSB-first words (byte-swapped) and put the next span in, piece by piece: each
        // thread writes only the pieces it has just read.  The chunk's first and last pieces are deferred.
        const uint32_t kl = (span - 1u) & ~15u;
#pragma unroll
        for (int j = 0; j < NV; ++j) {
            const uint32_t k = (uint32_t)j * (16u * NT) + t * 16u;
            uint4* sp = reinterpret_cast<uint4*>(reinterpret_cast<uint8_t*>(s_st) + k);
            uint4 v = make_uint4(0u, 0u, 0u, 0u);
            if (k < span) v = *sp;
            if (ncommit && k < nspan) *sp = piece(pv, j, nxt);
            if (k < span) {
                const uint64_t g = (uint64_t)a0 + k;
                v = make_uint4(bswap32(v.x), bswap32(v.y), bswap32(v.z), bswap32(v.w));
                const bool full = g >= lo && g + 16 <= hi;
                if (full) st16_out(A.out + g, v);
                if (k == 0 || k == kl) {
                    const uint32_t elo = lo > g ? (uint32_t)(lo - g) : 0u;
                    const uint32_t ehi = hi - g < 16 ? (uint32_t)(hi - g) : 16u;
                    EdgeRec* ed = rec + (k == 0 ? 0 : 1);
                    ed->v = v;
                    ed->m = make_uint4((uint32_t)g, (uint32_t)(g >> 32), full ? 0u : elo, full ? 0u : ehi);
                }
            }
        }
        if (t == 0 && (kl == 0 || span == 0)) rec[1].m = make_uint4(0u, 0u, 0u, 0u);  // one piece, or none
        if (t == 0 && span == 0) rec[0].m = make_uint4(0u, 0u, 0u, 0u);
        if (!more) break;
        cur = nxt;
        nxt = nn;
        c = cn;
    }
}

// ------------------------------------------------------------------------------------------------
// Run decode (HHUFF_DEC_RUN; contiguous layout, slot output; mixed and long lengths).  decode_stream_kernel's
// lanes take one string at a time, and a lane whose string ends inside its window idles for the rest of the
// round: on c3's long half that spread costs 24 % against the same bytes at one length (profiles/
// r05ac_c3_decomposition_ab.jsonl), and every string starts behind a dependent take (counter, offsets, window).
// Here a lane takes a run of RL consecutive strings (their RL + 1 offsets and is-name word in registers), and a
// string that ends inside the window is followed at once by the run's next string, whose bytes are already in
// the window (consecutive strings are adjacent): the round goes on in sub-rounds until every lane has used its
// window.  Measured slower (c3 0.395 / 0.565 ms with runs of 2 / 4 strings against 0.296; c5 0.631 / 0.822
// against 0.431, profiles/r05af_run_decode_ab.jsonl): c3 and c5 give a lane only 5-11 strings, so runs leave
// too few units to balance the lanes, and the sub-rounds cost more than the idle window they recover.
// A string's output is flushed when it ends (its head and tail chunks byte-exact, as the stream kernel
// does at a string's end); the next string's output starts a fresh buffer at its own slot.  The continuation
// window of a run is always the next NW dwords, so it is prefetched a round ahead.
// ------------------------------------------------------------------------------------------------
template <int WAVES, int NW, int OUT, int RL>
__global__ __launch_bounds__(WAVES * 64) void decode_run_kernel(DecArgs A, unsigned long long* __restrict__ counter) {
    static_assert(NW >= 8 && NW % 4 == 0 && OUT % 16 == 0 && 32 % RL == 0, "window shape; runs inside a name word");
    static_assert(15 + (32 * (NW - 2)) / 5 + 2 < OUT, "output buffer too small for a window");
    constexpr uint32_t kWS = NW + 1;
    struct __attribute__((aligned(16))) Smem {
        uint32_t lut[1u << HHUFF_LUT_BITS];
        uint32_t kinfo[32];
        uint32_t ones[(HHUFF_ONES_NENT + 3) & ~3];
        uint8_t out[WAVES * 64][OUT];
        uint32_t win[WAVES * 64][kWS];
    };
    __shared__ Smem sm;
    load_dec_tables(sm.lut, sm.kinfo, sm.ones, WAVES * 64);
    __syncthreads();
    const DecTables T{sm.lut, sm.kinfo, sm.ones};
    const int lane = threadIdx.x & 63;
    uint32_t* win = &sm.win[threadIdx.x][1];
    const lds_u32* st = (const lds_u32*)win;
    uint8_t* obuf = sm.out[threadIdx.x];
    const uint32_t ob = lds_addr(obuf), trash = ob + OUT - 1u;
    constexpr int32_t kLimW = 32 * (NW - 2) - 30;
    constexpr int32_t kFinal = 32 * (NW - 2);

    // per-lane run state: strings [rs + k, rs + kcnt); ro[0], ro[1] bound the current string (popped as strings end)
    uint32_t ro[RL + 1];
    uint32_t rs = 0, k = 0, kcnt = 0, nmw = 0, rend = 0;
    // per-lane string state
    uint4 pfv[NW / 4];
    uint64_t pfa = ~0ull;
    bool busy = false, head = false, is_name = false;
    uint32_t i = 0, s = 0, len = 0, P = 0, ocnt = 0, flags = 0, first = 0, lastb = 0, fail = 0;
    uint64_t dst = 0;
    uint64_t bnext = 0, bend = 0;
    bool qdone = false;
    const uint64_t nwork = (uint64_t)A.n;
    const uint64_t nruns = (nwork + RL - 1) / RL;
    // the current string of the run (ro[0], ro[1]); too long / listed strings are settled and skipped here
    auto start_string = [&]() {
        busy = false;
        while (k < kcnt) {
            i = rs + k;
            s = ro[0];
            len = ro[1] - ro[0];
            is_name = ((nmw >> (i & 31u)) & 1u) != 0;
            dst = dec_slot(s);
            bool skip = false;
            if (len > kMaxStrLen) {
                A.out_len[i] = kFailLen;
                A.status[i] = kStatusTooLong;
                skip = true;
            } else if (split_push(A, i, len)) {
                skip = true;
            }
            if (!skip) {
                busy = true;
                head = (dst & 15u) != 0;
                P = ocnt = flags = first = lastb = fail = 0;
                return;
            }
#pragma unroll
            for (int j = 0; j < RL; ++j) ro[j] = ro[j + 1];
            ++k;
        }
    };
    PROF_DECL

    for (;;) {
        // ---- 1. lanes without a run take one (a wave claims 64 runs at a time) ----
        for (int it = 0; it < 2; ++it) {
            const uint64_t need = __builtin_amdgcn_ballot_w64(!busy && k >= kcnt);
            if (need == 0) break;
            if (bnext >= bend) {
                if (qdone) break;
                uint64_t b = 0;
                if (lane == 0) b = atomicAdd(counter, 64ull);
                b = ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(b >> 32)) << 32) |
                    (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)b);
                if (b >= nruns) {
                    qdone = true;
                    break;
                }
                bnext = b;
                bend = min(b + 64u, nruns);
            }
            const uint32_t rank = (uint32_t)__builtin_amdgcn_mbcnt_hi((uint32_t)(need >> 32),
                                                                      __builtin_amdgcn_mbcnt_lo((uint32_t)need, 0u));
            if (!busy && k >= kcnt && bnext + rank < bend) {
                rs = (uint32_t)((bnext + rank) * RL);
                kcnt = (uint32_t)min((uint64_t)RL, nwork - rs);
                k = 0;
#pragma unroll
                for (int j = 0; j <= RL; ++j) ro[j] = A.in_off[min((uint64_t)rs + j, nwork)];
                nmw = A.is_name_bits ? A.is_name_bits[rs >> 5] : 0u;
                rend = A.in_off[rs + kcnt];  // the run's end byte
                start_string();
            }
            bnext = min(bend, bnext + (uint64_t)__builtin_popcountll(need));
        }
        if (!__any(busy)) {
            if (qdone) {
                PROF_FLUSH(0);
                break;
            }
            continue;
        }
        PROF_MARK(0);

        // ---- 2. the lane's window: NW dwords from its current byte; the run's continuation prefetched ----
        const uint64_t cur = (uint64_t)s + (P >> 3);
        // the prefetched window when the lane's byte lies in its first 16 bytes (a run's next round, or a string
        // that starts past the last round's window), else the dword holding the byte
        const uint64_t wb = pfa != ~0ull && cur >= pfa && cur < pfa + 16u ? pfa : cur & ~3ull;
        if (busy) {
            if (wb != pfa) {
#pragma unroll
                for (int j = 0; j < NW / 4; ++j) pfv[j] = load16_bounded(A.in, A.in_size, wb + 16u * j);
            }
#pragma unroll
            for (int j = 0; j < NW / 4; ++j) {
                win[4 * j + 0] = bswap32(pfv[j].x);
                win[4 * j + 1] = bswap32(pfv[j].y);
                win[4 * j + 2] = bswap32(pfv[j].z);
                win[4 * j + 3] = bswap32(pfv[j].w);
            }
            // a round stops at or past window bit kLimW: the run's next round starts in the dword at 4 (NW - 3)
            pfa = (uint64_t)rend > wb + 4u * (NW - 3) ? wb + 4u * (NW - 3) : ~0ull;
            if (pfa != ~0ull) {
#pragma unroll
                for (int j = 0; j < NW / 4; ++j) pfv[j] = load16_bounded(A.in, A.in_size, pfa + 16u * j);
            }
        }
        // the current string inside this window
        int32_t pm = busy ? (int32_t)(8u * (uint32_t)(cur - wb) + (P & 7u)) - 1 : -1;
        int32_t pm0 = pm;
        int32_t end = busy ? (int32_t)min((uint64_t)(pm + 1) + ((uint64_t)len * 8u - P), (uint64_t)0x40000000u) : 0;
        bool fin = busy && end <= kFinal;
        uint32_t h0 = (uint32_t)((dst + ocnt) & 15u);
        uint32_t o = ob + h0;
        int32_t q = pm >> 5;
        uint32_t x0 = st[q], x1 = st[q + 1], x2 = st[q + 2];
        uint32_t accb = 0, acc1 = 0, acc2 = 0, accl = 0, parked = busy ? 0u : 1u;
        int32_t lim = busy ? min(end - 26, kLimW) : (int32_t)0x80000000;
        auto advance = [&](int32_t cons) {
            pm += cons;
            const int32_t qn = pm >> 5;
            const bool adv = qn != q;
            x0 = adv ? x1 : x0;
            x1 = adv ? x2 : x1;
            q = qn;
            x2 = st[q + 2];
        };
        int32_t c = 0;
        bool waiting = false;  // the lane's string starts past this window: it begins next round
        for (;;) {  // ---- 3. sub-rounds: bulk, tail, and the run's next strings inside this window ----
            auto bstep = [&](bool longchk) {
                if (pm < lim) {
                    const uint32_t w = __builtin_amdgcn_alignbit(x0, x1, ~(uint32_t)pm);
                    const uint32_t e = T.lut[w >> (32 - HHUFF_LUT_BITS)];
                    const uint32_t sl = (uint32_t)((int32_t)e >> 31);
                    bulk_put2(o, e, trash);
                    o += (e >> 28) & 3u;
                    accb |= e;
                    uint32_t cons = lut_l12(e);
                    {
                        const uint32_t wb2 = w << cons;
                        const uint32_t eb = T.lut[wb2 >> (32 - HHUFF_LUT_BITS)];
                        bulk_put2(o, eb, trash);
                        o += (eb >> 28) & 3u;
                        accb |= eb;
                        cons += lut_l12(eb);
                    }
                    if (longchk && __builtin_amdgcn_ballot_w64(sl != 0u) != 0) {
                        if (sl) {
                            const uint32_t kk = min((uint32_t)__builtin_clz(~w | 1u), 30u);
                            const uint32_t ki = T.kinfo[kk];
                            const uint32_t le = T.ones[(ki & 0xFFFFu) + (((w << (kk + 1)) >> 1) >> (31 - (ki >> 16)))];
                            const int32_t L = (le >> 9) & 31u;
                            const uint32_t fits = (uint32_t)((L + pm - end) >> 31);
                            const uint32_t eos = (le & 0x1FFu) == kEos ? 0xFFFFFFFFu : 0u;
                            const uint32_t okm = fits & ~eos;
                            fail |= fits & eos & 1u;
                            lds_st8(sel_bits(okm, o, trash), le);
                            o -= okm;
                            accl |= le & okm;
                            cons = okm & (uint32_t)L;
                            parked |= ~okm & 1u;
                            lim = (int32_t)sel_bits(okm, (uint32_t)lim, 0x80000000u);
                        }
                    }
                    advance((int32_t)cons);
                }
            };
            for (;;) {
                bstep(false);
                bstep(true);
                if (!__any(pm < lim)) break;
            }
            c = (fin && !parked) ? pm - end : 0x40000000;
            if (__any(fin)) {
                int32_t prog = 0;
                auto step = [&](bool longchk) {
                    const uint32_t w = __builtin_amdgcn_alignbit(x0, x1, ~(uint32_t)pm);
                    const uint32_t e = T.lut[w >> (32 - HHUFF_LUT_BITS)];
                    const int32_t L1 = lut_l1(e), L12 = lut_l12(e);
                    const int32_t s1 = L1 + c, s2 = L12 + c;
                    const uint32_t m1 = (uint32_t)((s1 & ~(int32_t)e) >> 31);
                    const uint32_t m2 = (uint32_t)((s2 & (int32_t)(e << 1)) >> 31);
                    int32_t cons = (int32_t)sel_bits(m2, (uint32_t)L12, m1 & (uint32_t)L1);
                    lds_st8(sel_bits(m1, o - m2, trash), lut_sym2(e));
                    lds_st8(sel_bits(m1, o, trash), e);
                    o = o - m1 - m2;
                    acc1 |= e & m1;
                    acc2 |= e & m2;
                    {
                        const uint32_t wb2 = w << cons;
                        const uint32_t eb = T.lut[wb2 >> (32 - HHUFF_LUT_BITS)];
                        const int32_t cb = c + cons;
                        const int32_t L1b = lut_l1(eb), L12b = lut_l12(eb);
                        const uint32_t m1b = (uint32_t)(((L1b + cb) & ~(int32_t)eb) >> 31);
                        const uint32_t m2b = (uint32_t)(((L12b + cb) & (int32_t)(eb << 1)) >> 31);
                        lds_st8(sel_bits(m1b, o - m2b, trash), lut_sym2(eb));
                        lds_st8(sel_bits(m1b, o, trash), eb);
                        o = o - m1b - m2b;
                        acc1 |= eb & m1b;
                        acc2 |= eb & m2b;
                        cons += (int32_t)sel_bits(m2b, (uint32_t)L12b, m1b & (uint32_t)L1b);
                    }
                    const bool lact = (s1 & (int32_t)e) < 0;
                    uint32_t consl = 0;
                    if (longchk && __builtin_amdgcn_ballot_w64(lact) != 0) {
                        if (lact) {
                            const uint32_t kk = min((uint32_t)__builtin_clz(~w | 1u), 30u);
                            const uint32_t ki = T.kinfo[kk];
                            const uint32_t le = T.ones[(ki & 0xFFFFu) + (((w << (kk + 1)) >> 1) >> (31 - (ki >> 16)))];
                            const int32_t L = (le >> 9) & 31u;
                            const uint32_t fits = (uint32_t)((L + c) >> 31);
                            const uint32_t eos = (le & 0x1FFu) == kEos ? 0xFFFFFFFFu : 0u;
                            const uint32_t okm = fits & ~eos;
                            fail |= fits & eos & 1u;
                            lds_st8(sel_bits(okm, o, trash), le);
                            o -= okm;
                            accl |= le & okm;
                            consl = okm & (uint32_t)L;
                            c = (int32_t)sel_bits(okm, (uint32_t)c, 0x40000000u);
                        }
                    }
                    cons |= (int32_t)consl;
                    c += cons;
                    advance(cons);
                    prog = cons;
                };
                step(true);
                for (;;) {
                    step(false);
                    step(true);
                    if (!__any(prog != 0)) break;
                }
            }
            // strings that ended in this window: settle and flush them, then the run's next string
            const bool ended = busy && (parked || fin);
            if (!__any(ended)) break;
            bool again = false;
            if (ended) {
                flags |= ((accb >> 24) | (accb >> 26) | (acc1 >> 24) | (acc2 >> 26) | (accl >> 14)) & 3u;
                const uint32_t nb = o - ob;
                const uint32_t made = nb - h0;
                if (made) {
                    if (ocnt == 0) first = obuf[h0];
                    lastb = obuf[nb - 1u];
                }
                const bool ok = fin && !parked && !fail && [&] {
                    const uint32_t R = ~(uint32_t)c;
                    const uint32_t w = __builtin_amdgcn_alignbit(x0, x1, ~(uint32_t)pm);
                    return R <= 7 && (w | (0xFFFFFFFFu >> (R & 31u))) == 0xFFFFFFFFu;
                }();
                if (ok) {  // a failed string's output is unspecified
                    uint8_t* gchunk = A.out + ((dst + ocnt) & ~15ull);
                    const uint32_t hs = head ? (uint32_t)(dst & 15u) : 0u;
                    const uint32_t nfull = nb >> 4;
                    for (uint32_t kc = 0; kc < nfull; ++kc) {
                        const uint32_t c0 = 16u * kc;
                        if (c0 + 16u <= hs) continue;
                        if (c0 < hs)
                            store_range16(gchunk + c0, obuf + c0, hs - c0, 16u);
                        else
                            *reinterpret_cast<uint4*>(gchunk + c0) = *reinterpret_cast<const uint4*>(obuf + c0);
                    }
                    const uint32_t c0 = 16u * nfull;
                    const uint32_t lo = hs > c0 ? hs - c0 : 0u;
                    if (nb - c0 > lo) store_range16(gchunk + c0, obuf + c0, lo, nb - c0);
                }
                ocnt += made;
                A.out_len[i] = ok ? ocnt : kFailLen;
                A.status[i] = ok ? soft_bits(is_name, ocnt, flags, first, lastb) : kStatusFail;
                // the run's next string: its bytes follow at once, in this window if it starts before its end
#pragma unroll
                for (int j = 0; j < RL; ++j) ro[j] = ro[j + 1];
                ++k;
                start_string();
                if (busy) {
                    const int64_t rel = (int64_t)s - (int64_t)wb;  // >= 0: runs are contiguous
                    pm = (int32_t)(8 * rel) - 1;
                    pm0 = pm;
                    end = (int32_t)min((uint64_t)(pm + 1) + (uint64_t)len * 8u, (uint64_t)0x40000000u);
                    fin = end <= kFinal;
                    h0 = (uint32_t)(dst & 15u);
                    o = ob + h0;
                    accb = acc1 = acc2 = accl = 0;
                    parked = 0;
                    // bulk only from a start inside the window's bulk range; a start past it waits for the next round
                    const bool inside = pm + 1 < kFinal;
                    lim = inside ? min(end - 26, kLimW) : (int32_t)0x80000000;
                    fin = fin && inside;
                    if (inside) {
                        q = pm >> 5;
                        x0 = st[q];
                        x1 = st[q + 1];
                        x2 = st[q + 2];
                        again = true;
                    } else {
                        waiting = true;
                    }
                } else {
                    fin = false;
                    lim = (int32_t)0x80000000;
                    parked = 1;
                }
            }
            if (!__any(again)) break;
        }
        PROF_MARK(2);

        // ---- 4. strings that go on past this window: whole chunks out, the partial one carried ----
        if (busy && !waiting) {
            flags |= ((accb >> 24) | (accb >> 26) | (acc1 >> 24) | (acc2 >> 26) | (accl >> 14)) & 3u;
            const uint32_t nb = o - ob;
            const uint32_t made = nb - h0;
            if (made) {
                if (ocnt == 0) first = obuf[h0];
                lastb = obuf[nb - 1u];
            }
            uint8_t* gchunk = A.out + ((dst + ocnt) & ~15ull);
            const uint32_t hs = head ? (uint32_t)(dst & 15u) : 0u;
            const uint32_t nfull = nb >> 4;
            for (uint32_t kc = 0; kc < nfull; ++kc) {
                const uint32_t c0 = 16u * kc;
                if (c0 + 16u <= hs) continue;
                if (c0 < hs)
                    store_range16(gchunk + c0, obuf + c0, hs - c0, 16u);
                else
                    *reinterpret_cast<uint4*>(gchunk + c0) = *reinterpret_cast<const uint4*>(obuf + c0);
            }
            if (nfull) {
                head = false;
                const uint32_t c0 = 16u * nfull;
                for (uint32_t r = 0; c0 + 16u * r < nb; ++r)
                    *reinterpret_cast<uint4*>(obuf + 16u * r) = *reinterpret_cast<const uint4*>(obuf + c0 + 16u * r);
            }
            ocnt += made;
            P += (uint32_t)(pm - pm0);
        }
        PROF_MARK(4);
    }
}

