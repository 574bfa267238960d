/* Device-side helpers for gfx950 (wave64): tile keys, wave aggregation,
 * block scans.  Wave width is hard-coded to 64 (CDNA). */
#pragma once
#include "hm_common.h"

#define HM_WAVE 64

/* ---- tile keys ----
 * Keys are row-major: a level's key holds the (row, col) offsets of a point's
 * tile inside its bucket as (row << s) | col, s bits each; a digit is the
 * top w bits of both, (row >> s' << w) | (col >> s').  Buckets carry their
 * tile as coord = (row << 32) | col. */

/* output cell key (include/heatmap_amd.h HM_KEY) */
__device__ __forceinline__ uint64_t hm_key(int z, uint64_t row, uint64_t col)
{
    return ((uint64_t)z << 58) | (row << 29) | col;
}

/* cell i of the row-major (2^lg)^2 block of zoom z whose corner tile at zoom
 * z - lg is `coord` */
__device__ __forceinline__ uint64_t hm_cell_key(int z, uint64_t coord, int lg, uint32_t i)
{
    const uint64_t row = ((coord >> 32) << lg) | (i >> lg);
    const uint64_t col = ((coord & 0xFFFFFFFFull) << lg) | (i & ((1u << lg) - 1u));
    return hm_key(z, row, col);
}

/* sum of the 4 children of cell i of the next (coarser) level: the child
 * block is row-major with side 2^(lgn+1) at v */
template <typename T>
__device__ __forceinline__ T hm_sum4(const T* v, uint32_t i, int lgn)
{
    const uint32_t r = i >> lgn, c = i & ((1u << lgn) - 1u);
    const uint32_t side = 2u << lgn;
    const uint32_t j = (r << (lgn + 2)) | (c << 1);
    return (T)(v[j] + v[j + 1] + v[j + side] + v[j + side + 1]);
}

/* linear block id of a 2-D grid (hm_grid2) */
__device__ __forceinline__ uint32_t hm_block_id() { return blockIdx.y * gridDim.x + blockIdx.x; }

/* ---- wave helpers ---- */
__device__ __forceinline__ int hm_lane() { return (int)__lane_id(); }

__device__ __forceinline__ uint32_t hm_mbcnt(uint64_t mask)
{
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0u));
}

/* inclusive wave prefix sum: DPP row shifts 1, 2, 4, 8 scan each row of 16
 * lanes (out-of-row sources read 0), then row_bcast:15 / row_bcast:31 carry
 * rows 0 -> 1, 2 -> 3 and rows 0-1 -> 2-3 (6 VALU, no LDS permutes).  Every
 * lane must be active. */
#define HM_DPP_ADD(v, ctrl, rows) \
    (v) += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(v), (ctrl), (rows), 0xF, false)
__device__ __forceinline__ uint32_t hm_wave_incl_scan(uint32_t v)
{
    HM_DPP_ADD(v, 0x111, 0xF);   /* row_shr:1 */
    HM_DPP_ADD(v, 0x112, 0xF);   /* row_shr:2 */
    HM_DPP_ADD(v, 0x114, 0xF);   /* row_shr:4 */
    HM_DPP_ADD(v, 0x118, 0xF);   /* row_shr:8 */
    HM_DPP_ADD(v, 0x142, 0xA);   /* row_bcast:15 into rows 1, 3 */
    HM_DPP_ADD(v, 0x143, 0xC);   /* row_bcast:31 into rows 2, 3 */
    return v;
}

__device__ __forceinline__ uint64_t hm_wave_incl_scan64(uint64_t v)
{
    const int lane = hm_lane();
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        uint64_t t = __shfl_up(v, o, 64);
        if (lane >= o) v += t;
    }
    return v;
}

__device__ __forceinline__ uint32_t hm_wave_sum(uint32_t v)
{
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

/* Workgroup barrier that orders LDS only: __syncthreads() also releases
 * global memory, i.e. waits (vmcnt(0)) for every global load and store the
 * wave has in flight -- prefetched points included.  For kernels whose waves
 * share data through LDS alone. */
__device__ __forceinline__ void hm_lds_barrier()
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

/* Block-wide exclusive scan of one value per thread; returns the block total
 * in *total.  `scratch` needs (blockDim/64 + 1) u32 of LDS.  LDS_ONLY: the
 * barriers are hm_lds_barrier(). */
template <int THREADS, bool LDS_ONLY = false>
__device__ __forceinline__ uint32_t hm_block_excl_scan(uint32_t v, uint32_t* scratch, uint32_t* total)
{
    constexpr int NW = THREADS / 64;
    const int lane = hm_lane();
    const int w = threadIdx.x >> 6;
    uint32_t inc = hm_wave_incl_scan(v);
    if (lane == 63) scratch[w] = inc;
    if (LDS_ONLY) hm_lds_barrier(); else __syncthreads();
    if (w == 0) {
        uint32_t s = lane < NW ? scratch[lane] : 0u;
        uint32_t si = hm_wave_incl_scan(s);
        if (lane < NW) scratch[lane] = si - s;
        if (lane == NW - 1) scratch[NW] = si;
    }
    if (LDS_ONLY) hm_lds_barrier(); else __syncthreads();
    uint32_t r = scratch[w] + inc - v;
    *total = scratch[NW];
    if (LDS_ONLY) hm_lds_barrier(); else __syncthreads();
    return r;
}

template <int THREADS>
__device__ __forceinline__ uint64_t hm_block_excl_scan64(uint64_t v, unsigned long long* scratch, uint64_t* total)
{
    constexpr int NW = THREADS / 64;
    const int lane = hm_lane();
    const int w = threadIdx.x >> 6;
    const uint64_t inc = hm_wave_incl_scan64(v);
    if (lane == 63) scratch[w] = inc;
    __syncthreads();
    if (w == 0) {
        const uint64_t s = lane < NW ? scratch[lane] : 0ull;
        const uint64_t si = hm_wave_incl_scan64(s);
        if (lane < NW) scratch[lane] = si - s;
        if (lane == NW - 1) scratch[NW] = si;
    }
    __syncthreads();
    const uint64_t r = scratch[w] + inc - v;
    *total = scratch[NW];
    __syncthreads();
    return r;
}

/* Digit slots d = q * THREADS + t of thread t (q < PER): a wave's lanes own
 * consecutive digits, so per-digit global counters they update coalesce.
 * Exclusive offsets in digit order (q major, then thread) from ONE 64-bit
 * block scan of the PER counts packed in 64/PER-bit fields (each count, and
 * the block's total per q, must stay below 2^(64/PER)). */
template <int THREADS, int PER>
__device__ __forceinline__ void hm_digit_offsets(const uint32_t (&cnt)[PER], uint32_t (&off)[PER],
                                                 unsigned long long* scratch)
{
    constexpr int FB = 64 / PER;
    constexpr uint64_t FM = (FB == 64) ? ~0ull : ((1ull << FB) - 1);
    uint64_t packed = 0;
#pragma unroll
    for (int q = 0; q < PER; q++) packed |= (uint64_t)cnt[q] << (FB * q);
    uint64_t tot;
    const uint64_t o = hm_block_excl_scan64<THREADS>(packed, scratch, &tot);
    uint32_t base = 0;
#pragma unroll
    for (int q = 0; q < PER; q++) {
        off[q] = base + (uint32_t)((o >> (FB * q)) & FM);
        base += (uint32_t)((tot >> (FB * q)) & FM);
    }
}

/* LDS histogram increment / slot reservation, branch-free.  The lanes whose
 * key equals the first active lane's are added by one atomic of their first
 * lane (the skew case, SURVEY.md section 7 hard part 3: a wave of one key
 * costs one atomic, not 64 serialised ones); every other valid lane adds 1 to
 * its own key; lanes with nothing to add hit a private dummy slot, so no
 * branch, leader election loop or exec-mask juggling is needed -- those made
 * the partition kernels scalar-issue bound.  `dummy` is the index of 64
 * spare words at the end of the same array (an index select, not a pointer
 * select, and non-short-circuit logic: either of those makes the compiler
 * emit exec-mask branches). */
__device__ __forceinline__ void hm_lds_count(uint32_t* hist, uint32_t dummy, uint32_t key, bool valid)
{
    const uint32_t k0 = __builtin_amdgcn_readfirstlane(key);
    const bool same = valid & (key == k0);
    const uint64_t m = __ballot(same);
    const uint32_t r = hm_mbcnt(m);
    const bool lead = same & (r == 0);
    const bool own = valid & !same;
    const uint32_t i = lead ? k0 : (own ? key : dummy + (uint32_t)hm_lane());
    const uint32_t inc = lead ? (uint32_t)__popcll(m) : (uint32_t)own;
    atomicAdd(&hist[i], inc);
}

__device__ __forceinline__ uint32_t hm_lds_claim(uint32_t* cur, uint32_t dummy, uint32_t key, bool valid)
{
    const uint32_t k0 = __builtin_amdgcn_readfirstlane(key);
    const bool same = valid & (key == k0);
    const uint64_t m = __ballot(same);
    const uint32_t r = hm_mbcnt(m);
    const bool lead = same & (r == 0);
    const bool own = valid & !same;
    const uint32_t i = lead ? k0 : (own ? key : dummy + (uint32_t)hm_lane());
    const uint32_t inc = lead ? (uint32_t)__popcll(m) : (uint32_t)own;
    const uint32_t old = atomicAdd(&cur[i], inc);
    const uint32_t base = __builtin_amdgcn_readlane(old, m ? __ffsll((unsigned long long)m) - 1 : 0);
    return same ? base + r : old;
}

/* LDS histogram increment that merges only when it pays: when more than
 * HM_MERGE_MIN valid lanes hold lane 0's key (wave-uniform test) those are one
 * atomic of their first lane; otherwise every valid lane adds 1 on its own
 * (the LDS serialises the few same-address lanes of a spread-out wave for
 * less than the merge's VALU work costs).  `dummy_lane`: this lane's private
 * dummy word. */
#ifndef HM_MERGE_MIN
#define HM_MERGE_MIN 8
#endif
__device__ __forceinline__ void hm_lds_count_fast(uint32_t* hist, uint32_t dummy_lane, uint32_t key, bool valid)
{
    const uint32_t k0 = __builtin_amdgcn_readfirstlane(key);
    /* (the raw ballot: __ballot materialises the predicate in a VGPR first;
     * a 32-bit popcount compare stays on the scalar unit) */
    const uint64_t m = __builtin_amdgcn_ballot_w64(key == k0) & __builtin_amdgcn_ballot_w64(valid);
    if ((uint32_t)__builtin_popcount((uint32_t)m) + (uint32_t)__builtin_popcount((uint32_t)(m >> 32)) >
        HM_MERGE_MIN) {
        const int l = __ffsll((unsigned long long)m) - 1;
        const bool same = (m >> hm_lane()) & 1ull;
        const bool lead = hm_lane() == l;
        atomicAdd(&hist[(valid & (!same | lead)) ? key : dummy_lane], lead ? (uint32_t)__popcll(m) : 1u);
    } else {
        atomicAdd(&hist[valid ? key : dummy_lane], 1u);
    }
}

/* hm_lds_claim split in two, so several claims can be in flight: prep, the
 * atomic (atomicAdd(&cur[g.idx], g.inc)), then pos.  The lanes whose key
 * equals lane 0's (straight-line code: every lane active) are one atomic of
 * lane 0; if lane 0 holds no valid key none merge.  `dummy_lane` = the
 * caller's private dummy word of this lane. */
struct HmClaim {
    bool same;
    uint32_t r, idx, inc;
};

__device__ __forceinline__ HmClaim hm_claim_prep(uint32_t key, bool valid, uint32_t dummy_lane)
{
    HmClaim g;
    const uint32_t k0 = __builtin_amdgcn_readfirstlane(key);
    g.same = valid & (key == k0);
    const uint64_t m = __ballot(g.same);
    g.r = hm_mbcnt(m);
    const bool lead = g.same & (g.r == 0);
    const bool own = valid & !g.same;
    g.idx = (lead | own) ? key : dummy_lane;
    g.inc = lead ? (uint32_t)__popcll(m) : (uint32_t)own;
    return g;
}

__device__ __forceinline__ uint32_t hm_claim_pos(const HmClaim& g, uint32_t old)
{
    /* a non-empty group holds lane 0, which added for it */
    return g.same ? __builtin_amdgcn_readfirstlane(old) + g.r : old;
}

/* Multi-round wave aggregation for LDS histograms and slot claims.  Round r
 * takes the first lane not yet grouped, and every lane holding its key joins
 * that group; after HM_MERGE_ROUNDS rounds the remaining lanes go alone.  The
 * grouping needs only the keys (ballots, readlane), so a claim still costs ONE
 * atomic instruction per key for the whole wave: a group's first lane adds the
 * group size, a lone lane adds 1, every other lane hits its private dummy word.
 * Skewed keys (a few hot digits per wave: hotspot clouds) then cost no
 * same-address serialisation, which single-round merging (lanes equal to the
 * first lane only) left to the 2nd, 3rd ... hottest digit. */
#ifndef HM_MERGE_ROUNDS
#define HM_MERGE_ROUNDS 1
#endif
struct HmMerge {
    uint64_t m[HM_MERGE_ROUNDS];
    int l[HM_MERGE_ROUNDS];
    uint32_t idx, inc;
};

__device__ __forceinline__ HmMerge hm_merge_prep(uint32_t key, bool valid, uint32_t dummy)
{
    HmMerge g;
    uint64_t un = __ballot(valid);
    const int lane = hm_lane();
    uint32_t inc = 0;
    bool lead = false;
#pragma unroll
    for (int r = 0; r < HM_MERGE_ROUNDS; r++) {
        const int l = un ? __ffsll((unsigned long long)un) - 1 : 0;
        const uint32_t kr = __builtin_amdgcn_readlane(key, l);
        const uint64_t m = un & __ballot(key == kr);
        g.m[r] = m;
        g.l[r] = l;
        const bool me = (lane == l) & (m != 0);
        lead |= me;
        inc = me ? (uint32_t)__popcll(m) : inc;
        un &= ~m;
    }
    const bool own = valid & (((un >> lane) & 1ull) != 0);
    g.idx = (lead | own) ? key : dummy + (uint32_t)lane;
    g.inc = own ? 1u : inc;
    return g;
}

/* position claimed by this lane, from the atomic's old value */
__device__ __forceinline__ uint32_t hm_merge_pos(const HmMerge& g, uint32_t old)
{
    const int lane = hm_lane();
    uint32_t pos = old;
#pragma unroll
    for (int r = 0; r < HM_MERGE_ROUNDS; r++) {
        const uint32_t b = __builtin_amdgcn_readlane(old, g.l[r]);
        pos = ((g.m[r] >> lane) & 1ull) ? b + hm_mbcnt(g.m[r]) : pos;
    }
    return pos;
}

__device__ __forceinline__ void hm_lds_count_m(uint32_t* hist, uint32_t dummy, uint32_t key, bool valid)
{
    const HmMerge g = hm_merge_prep(key, valid, dummy);
    atomicAdd(&hist[g.idx], g.inc);
}

__device__ __forceinline__ uint32_t hm_lds_claim_m(uint32_t* cur, uint32_t dummy, uint32_t key, bool valid)
{
    const HmMerge g = hm_merge_prep(key, valid, dummy);
    return hm_merge_pos(g, atomicAdd(&cur[g.idx], g.inc));
}

/* LDS slot of cell (r, c) = (r << w) | c of a row-major 2^w x 2^w histogram:
 * the column is rotated by 8 r, so a 2-D cluster of cells spreads over more
 * LDS banks than the few of its columns */
__device__ __forceinline__ uint32_t hm_skew(uint32_t d, int w)
{
    const uint32_t m = (1u << w) - 1u;
    return (d & ~m) | ((d + ((d >> w) << 3)) & m);
}

/* LDS slot of digit d in the partition kernels' digit counters (cur[]): the
 * hm_skew rotation, so that a hotspot's 2-D cluster of digits (same columns,
 * consecutive rows) does not pile onto the few banks of its columns */
#ifndef HM_SKEW_CUR
#define HM_SKEW_CUR 1
#endif
__device__ __forceinline__ uint32_t hm_cur_slot(uint32_t d, int w) { return HM_SKEW_CUR ? hm_skew(d, w) : d; }

/* level-1 digit slot: cold digits (< HM_MAX_F1, a 2-D grid) skewed as
 * hm_cur_slot, hot-tile digits as they are (no 2-D structure) */
__device__ __forceinline__ uint32_t hm_dslot(uint32_t d, int w) { return d < 1024u ? hm_cur_slot(d, w) : d; }
