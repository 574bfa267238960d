/* gfx950 kernels of the general count path.
 *
 * The fast pipeline (hm_kernels.hip) counts the points of one group whose
 * zoom-Z tile lies in [0, 2^Z)^2.  Everything else is counted here:
 *   - kept points whose tile lies outside that square: |lat| > 85.0511...,
 *     lon outside [-180, 180).  The reference bins them with negative rows and
 *     columns >= 2^z (tile.py:17,21 has no clamp; heatmap.py:27-36 keeps them);
 *   - grouped counts (hm_count_grouped): one count per (group, zoom, row, col)
 *     in one pass, the per-user keys of heatmap.py:64-75.
 *
 * Input: exact zoom-Z tiles (int64 row, col) and an optional u32 group.  A
 * point's key is 128 bits (hm_genkey.h),
 *     sr + 16 (5) | sc + 2^47 (48) | group (32) | morton(ro, co) (2Z)
 * where sr = row >> Z and sc = col >> Z (arithmetic shifts) name the point's
 * zoom-0 tile ("super tile", any integers) and ro, co its tile's offsets inside
 * it.  The zoom-(Z-k) cell of the point is the key with its low 2k bits
 * cleared: the shift of a tile (exact for negative rows and
 * huge columns too) only drops Morton bits.  So one LSD radix sort of the keys
 * orders every zoom at once, and the zoom cascade is a run-length reduction of
 * the previous zoom's sorted unique cells.
 *
 * Radix sort: keys only, 8-bit digits, LSD, stable, one sweep per digit
 * (k_rx_onesweep); digits that are the same in every key (an OR/AND
 * reduction taken while the keys are built) are skipped.
 */
#include <hip/hip_runtime.h>
#include <utility>
#include "hm_device.h"
#include "hm_pipeline.h"
#include "../../include/heatmap_amd.h"

#include "hm_genkey.h"

/* ------------------------------------------------------------------------ */
/* keys                                                                      */
/* ------------------------------------------------------------------------ */
/* Keys live as two u64 arrays (low and high halves).  When the high halves
 * are all equal (one super tile and groups < 2^(64 - 2Z): the usual case)
 * the sort and the cascade move only the low halves ("narrow", KT =
 * uint64_t) and the high half is a constant of the call; otherwise both
 * (KT = hm_u128). */

template <typename KT> __device__ __forceinline__ KT hm_kld(const uint64_t* lo, const uint64_t* hi, uint64_t i);
template <> __device__ __forceinline__ uint64_t hm_kld<uint64_t>(const uint64_t* lo, const uint64_t*, uint64_t i)
{
    return lo[i];
}
template <> __device__ __forceinline__ hm_u128 hm_kld<hm_u128>(const uint64_t* lo, const uint64_t* hi, uint64_t i)
{
    return ((hm_u128)hi[i] << 64) | (hm_u128)lo[i];
}
__device__ __forceinline__ void hm_kst(uint64_t* lo, uint64_t*, uint64_t i, uint64_t k) { lo[i] = k; }
__device__ __forceinline__ void hm_kst(uint64_t* lo, uint64_t* hi, uint64_t i, hm_u128 k)
{
    lo[i] = (uint64_t)k;
    hi[i] = (uint64_t)(k >> 64);
}
__device__ __forceinline__ hm_u128 hm_k128(uint64_t k, uint64_t hic) { return ((hm_u128)hic << 64) | (hm_u128)k; }
__device__ __forceinline__ hm_u128 hm_k128(hm_u128 k, uint64_t) { return k; }
__device__ __forceinline__ uint64_t hm_kshfl_up(uint64_t k) { return __shfl_up((unsigned long long)k, 1, 64); }
__device__ __forceinline__ hm_u128 hm_kshfl_up(hm_u128 k)
{
    return ((hm_u128)__shfl_up((unsigned long long)(k >> 64), 1, 64) << 64) |
           (hm_u128)__shfl_up((unsigned long long)k, 1, 64);
}
__device__ __forceinline__ uint64_t hm_kshfl_down(uint64_t k) { return __shfl_down((unsigned long long)k, 1, 64); }
__device__ __forceinline__ hm_u128 hm_kshfl_down(hm_u128 k)
{
    return ((hm_u128)__shfl_down((unsigned long long)(k >> 64), 1, 64) << 64) |
           (hm_u128)__shfl_down((unsigned long long)k, 1, 64);
}

/* OR / AND of the keys into orand[0..3] (lo, hi | lo, hi) */
__device__ __forceinline__ void hm_orand_flush(unsigned long long* orand, unsigned long long o_lo,
                                               unsigned long long o_hi, unsigned long long n_lo,
                                               unsigned long long n_hi)
{
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        o_lo |= __shfl_xor(o_lo, o, 64);
        o_hi |= __shfl_xor(o_hi, o, 64);
        n_lo &= __shfl_xor(n_lo, o, 64);
        n_hi &= __shfl_xor(n_hi, o, 64);
    }
    if (hm_lane() == 0) {
        atomicOr(&orand[0], o_lo);
        atomicOr(&orand[1], o_hi);
        atomicAnd(&orand[2], n_lo);
        atomicAnd(&orand[3], n_hi);
    }
}

/* the same, one set of atomics per 256-thread block (every thread calls):
 * same-address atomics serialise (~88 per us a word) */
__device__ __forceinline__ void hm_orand_flush_block(unsigned long long* orand, unsigned long long o_lo,
                                                     unsigned long long o_hi, unsigned long long n_lo,
                                                     unsigned long long n_hi)
{
    __shared__ unsigned long long red[4][4];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        o_lo |= __shfl_xor(o_lo, o, 64);
        o_hi |= __shfl_xor(o_hi, o, 64);
        n_lo &= __shfl_xor(n_lo, o, 64);
        n_hi &= __shfl_xor(n_hi, o, 64);
    }
    const int w = threadIdx.x >> 6;
    if (hm_lane() == 0) {
        red[0][w] = o_lo;
        red[1][w] = o_hi;
        red[2][w] = n_lo;
        red[3][w] = n_hi;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int q = 1; q < 4; q++) {
            o_lo |= red[0][q];
            o_hi |= red[1][q];
            n_lo &= red[2][q];
            n_hi &= red[3][q];
        }
        atomicOr(&orand[0], o_lo);
        atomicOr(&orand[1], o_hi);
        atomicAnd(&orand[2], n_lo);
        atomicAnd(&orand[3], n_hi);
    }
}

__global__ __launch_bounds__(256) void k_gen_keys(HmGenArgs a)
{
    const uint64_t n = a.n;
    const uint64_t stride = (uint64_t)gridDim.x * 256;
    unsigned long long o_lo = 0, o_hi = 0, n_lo = ~0ull, n_hi = ~0ull;
    const int Z = a.Z;
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += stride) {
        const int64_t r = a.row[i], c = a.col[i];
        bool ok;
        const hm_u128 k = hm_gen_key(r, c, a.group ? a.group[i] : 0u, Z, &ok);
        if (!ok) {
            /* representable by the reference, beyond this path's key */
            const uint64_t src = a.index ? (uint64_t)a.index[i] : i;
            atomicMin(a.err_word, ((unsigned long long)src << 8) | (unsigned long long)HM_E_RANGE);
        }
        hm_kst(a.klo, a.khi, i, k);
        o_lo |= (unsigned long long)k;
        o_hi |= (unsigned long long)(k >> 64);
        n_lo &= (unsigned long long)k;
        n_hi &= (unsigned long long)(k >> 64);
    }
    hm_orand_flush_block(a.orand, o_lo, o_hi, n_lo, n_hi);
}

/* ------------------------------------------------------------------------ */
/* zoom cascade: run-length reduction of sorted cells                        */
/* ------------------------------------------------------------------------ */

/* One zoom step per launch.  The input is a sorted list of level-(z+1) cells
 * (or, at the first step, the sorted raw keys, every one a point), each with
 * its END: the inclusive prefix of the counts, so a cell's count is END[i] -
 * END[i-1].  A zoom-z cell is the key with two more low bits cleared; its END is the END of the last fine
 * cell of its run -- prefixes survive coarsening, so no count is ever summed.
 * The step writes the unique zoom-z keys and their ENDs, compacted: a head's
 * slot is the number of heads before it, from a block scan of head ballots
 * and a decoupled look-back over the tiles (tiles taken in order from a
 * ticket, so every predecessor is held by a running block).  In the same
 * pass it writes the records of its input level (level z+1, at the running
 * record offset + i).  Sizes stay on the device: the step reads its item
 * count from the previous step's m_out, so the zoom cascade runs without a
 * host round trip.  Traffic per step (narrow keys): 12 B read per input
 * cell, 12 B written per output cell, one record per input cell. */
#define HM_CS_THREADS 256
#ifndef HM_CS_IT
#define HM_CS_IT 16
#endif
#define HM_CS_TILE (HM_CS_THREADS * HM_CS_IT)
#define HM_CS_FLAG_AGG 1ull
#define HM_CS_FLAG_INC 2ull
#define HM_CS_VBITS 38

/* one (group,) z, row, col, count record at slot q; width 2 (packed grouped
 * records, hm_count_grouped_packed, in-square cells only): keys[q] =
 * HM_KEY(z, row, col), counts[q] = group << 32 | count */
__device__ __forceinline__ void hm_put_record(const HmGenEmit& e, uint64_t q, uint32_t g, int z, int64_t row,
                                              int64_t col, uint64_t cnt)
{
    if (q >= e.capacity) return;
    if (e.width == 2) {
        e.keys[q] = ((uint64_t)z << 58) | ((uint64_t)row << 29) | (uint64_t)col;
        e.counts[q] = ((uint64_t)g << 32) | cnt;
        return;
    }
    int64_t* r = e.cells + q * e.width;
    int f = 0;
    if (e.width == 5) r[f++] = (int64_t)g;
    r[f++] = z;
    r[f++] = row;
    r[f++] = col;
    r[f] = (int64_t)cnt;
}

/* split mode (hm_count fallback): cells inside [0, 2^z)^2 go out as
 * (HM_KEY, count), the others as records */
__device__ __forceinline__ bool hm_in_square(int64_t row, int64_t col, int z)
{
    return (uint64_t)row < (1ull << z) && (uint64_t)col < (1ull << z);
}

__device__ __forceinline__ void hm_put_key(const HmGenEmit& e, uint64_t p, int z, int64_t row, int64_t col,
                                           uint64_t cnt)
{
    if (p >= e.kcapacity) return;
    e.keys[p] = ((uint64_t)z << 58) | ((uint64_t)row << 29) | (uint64_t)col;
    e.counts[p] = cnt;
}

__device__ __forceinline__ uint64_t hm_cs_word(uint64_t epoch, uint64_t flag, uint64_t v)
{
    return (epoch << 40) | (flag << HM_CS_VBITS) | v;
}

/* exclusive prefix of the tiles before `tile` (wave-parallel look-back over
 * 64 predecessors at a time; a tile < 0 reads as an inclusive 0) */
__device__ uint64_t hm_cs_lookback(uint64_t* st, int64_t tile, uint64_t epoch)
{
    const int lane = hm_lane();
    uint64_t excl = 0;
    int64_t p = tile - 1;
    while (p >= 0) {
        const int64_t q = p - lane;
        const uint64_t wv = q >= 0 ? __hip_atomic_load(st + q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                   : hm_cs_word(epoch, HM_CS_FLAG_INC, 0);
        const uint64_t fl = (wv >> 40) == epoch ? (wv >> HM_CS_VBITS) & 3ull : 0ull;
        const uint64_t mi = __builtin_amdgcn_ballot_w64(fl == HM_CS_FLAG_INC);
        const uint64_t mr = __builtin_amdgcn_ballot_w64(fl != 0);
        const uint64_t upto = mi ? ((mi & (0ull - mi)) << 1) - 1 : ~0ull;   /* lanes up to the first inclusive */
        if ((mr & upto) != upto) {
            __builtin_amdgcn_s_sleep(1);
            continue;
        }
        uint64_t v = ((upto >> lane) & 1ull) ? (wv & ((1ull << HM_CS_VBITS) - 1)) : 0ull;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
        excl += v;
        if (mi) break;
        p -= 64;
    }
    return excl;
}

template <typename KT>
__global__ __launch_bounds__(HM_CS_THREADS) void k_cascade(HmCascArgs a)
{
    constexpr int NW = HM_CS_THREADS / 64, NF = HM_CS_IT * NW;   /* (round, wave) fragments of a tile */
    __shared__ uint32_t wtot[NF];
    __shared__ KT kfirst[NF + 1], klast[NF + 1];   /* klast[f + 1]: last key of fragment f; [0]: item t0 - 1 */
    __shared__ uint32_t elast[NF + 1];
    __shared__ int64_t stage[NW][64 * 5];               /* a wave's records, written out contiguously */
    __shared__ uint32_t wsq[NF], wrc[NF];   /* split mode: per-fragment key / record counts, then offsets */
    __shared__ uint32_t tile_s;
    __shared__ uint64_t excl_s;
    __shared__ unsigned long long bsq_s, brc_s;
    const uint64_t m = a.m_in ? (uint64_t)*a.m_in : a.m_host;
    const uint64_t ntiles = (m + HM_CS_TILE - 1) / HM_CS_TILE;
    const int lane = hm_lane(), w = threadIdx.x >> 6;
    const KT keep_bits = ~((((KT)1) << a.clr) - 1);
    const unsigned long long rb = a.rbase_in ? *a.rbase_in : 0ull;
    const int W = a.e.width;
    /* packed records (width 2) go straight from the lanes: consecutive lanes
     * write consecutive 8-B words of the two arrays */
    const bool packed = a.emit && W == 2;
    const bool staged = a.emit && !a.e.split && !packed, split = a.emit && a.e.split;
    if (blockIdx.x == 0 && threadIdx.x == 0 && a.rbase_out) *a.rbase_out = rb + m;
    if (m == 0 && blockIdx.x == 0 && threadIdx.x == 0) *a.m_out = 0u;
    for (;;) {
        if (threadIdx.x == 0) tile_s = atomicAdd(a.ticket, 1u);
        __syncthreads();
        const uint64_t tile = tile_s;
        if (tile >= ntiles) break;
        const uint64_t t0 = tile * HM_CS_TILE;
        /* every load of the tile first: items, and the items either side */
        KT k[HM_CS_IT];
        uint32_t e[HM_CS_IT];
#pragma unroll
        for (int r = 0; r < HM_CS_IT; r++) {
            const uint64_t i = t0 + (uint64_t)r * HM_CS_THREADS + threadIdx.x;
            const bool v = i < m;
            k[r] = v ? hm_kld<KT>(a.kin_lo, a.kin_hi, i) : (KT)0;
            e[r] = a.ein ? (v ? a.ein[i] : 0u) : (uint32_t)(i + 1);
        }
        if (threadIdx.x == 0) {
            klast[0] = t0 ? hm_kld<KT>(a.kin_lo, a.kin_hi, t0 - 1) : (KT)0;
            elast[0] = t0 ? (a.ein ? a.ein[t0 - 1] : (uint32_t)t0) : 0u;
        }
        if (threadIdx.x == HM_CS_THREADS - 1)
            kfirst[NF] = t0 + HM_CS_TILE < m ? hm_kld<KT>(a.kin_lo, a.kin_hi, t0 + HM_CS_TILE) : (KT)0;
#pragma unroll
        for (int r = 0; r < HM_CS_IT; r++) {
            const int f = r * NW + w;
            if (lane == 0) kfirst[f] = k[r];
            if (lane == 63) {
                klast[f + 1] = k[r];
                elast[f + 1] = e[r];
            }
        }
        __syncthreads();
        uint32_t fl[HM_CS_IT];
#pragma unroll
        for (int r = 0; r < HM_CS_IT; r++) {
            const int f = r * NW + w;
            const uint64_t i = t0 + (uint64_t)r * HM_CS_THREADS + threadIdx.x;
            const bool v = i < m;
            KT kp = hm_kshfl_up(k[r]), kn = hm_kshfl_down(k[r]);
            uint32_t ep = __shfl_up(e[r], 1, 64);
            if (lane == 0) {
                kp = klast[f];
                ep = elast[f];
            }
            if (lane == 63) kn = kfirst[f + 1];
            const KT kz = k[r] & keep_bits;
            const bool head = v && (i == 0 || (kp & keep_bits) != kz);
            const bool tail = v && (i + 1 == m || (kn & keep_bits) != kz);
            uint32_t xs = 0;
            if (a.emit) {
                const uint64_t cnt = (uint64_t)(e[r] - ep);
                if (packed) {
                    uint32_t g = 0;
                    int64_t row = 0, col = 0;
                    if (v) {
                        hm_gen_decode(hm_k128(k[r], a.hic), a.Z, a.zin, &g, &row, &col);
                        hm_put_record(a.e, rb + i, g, a.zin, row, col, cnt);
                    }
                } else if (staged) {
                    /* the wave's 64 records are consecutive: stage them, then
                     * store whole 8-B words across the lanes */
                    const uint64_t i0 = t0 + (uint64_t)r * HM_CS_THREADS + (uint64_t)w * 64;
                    uint32_t g = 0;
                    int64_t row = 0, col = 0;
                    if (v) hm_gen_decode(hm_k128(k[r], a.hic), a.Z, a.zin, &g, &row, &col);
                    int64_t* sp = &stage[w][lane * W];
                    int q = 0;
                    if (W == 5) sp[q++] = (int64_t)g;
                    sp[q++] = a.zin;
                    sp[q++] = row;
                    sp[q++] = col;
                    sp[q] = (int64_t)cnt;
                    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
                    __builtin_amdgcn_wave_barrier();
                    const uint64_t nv = i0 < m ? min<uint64_t>(64, m - i0) : 0;
                    const uint64_t q0 = rb + i0;
                    uint64_t nw = q0 < a.e.capacity ? min<uint64_t>(nv, a.e.capacity - q0) * W : 0;
                    int64_t* dst = a.e.cells + q0 * W;
                    for (uint32_t x = lane; x < nw; x += 64) dst[x] = stage[w][x];
                    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
                    __builtin_amdgcn_wave_barrier();
                } else {
                    /* split: classify now, reserve per tile, write after the
                     * look-back (one cursor atomic per tile and kind) */
                    bool sq = false;
                    if (v) {
                        uint32_t g;
                        int64_t row, col;
                        hm_gen_decode(hm_k128(k[r], a.hic), a.Z, a.zin, &g, &row, &col);
                        sq = hm_in_square(row, col, a.zin);
                    }
                    const uint64_t ms = __builtin_amdgcn_ballot_w64(sq), mx = __builtin_amdgcn_ballot_w64(v && !sq);
                    if (lane == 0) {
                        wsq[f] = (uint32_t)__popcll(ms);
                        wrc[f] = (uint32_t)__popcll(mx);
                    }
                    xs = (uint32_t)sq << 30 | (uint32_t)(v && !sq) << 31;
                }
            }
            const uint64_t hb = __builtin_amdgcn_ballot_w64(head);
            if (lane == 0) wtot[f] = (uint32_t)__popcll(hb);
            k[r] = kz;
            fl[r] = (uint32_t)head | ((uint32_t)tail << 1) | (hm_mbcnt(hb) << 2) | xs;
        }
        __syncthreads();
        if (w == 0) {
            const uint32_t x = lane < NF ? wtot[lane] : 0u;
            uint32_t inc = x;
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                const uint32_t y = __shfl_up(inc, o, 64);
                if (lane >= o) inc += y;
            }
            const uint64_t agg = __shfl(inc, 63, 64);
            if (lane < NF) wtot[lane] = inc - x;
            if (lane == 0)
                __hip_atomic_store(a.tstat + tile, hm_cs_word(a.epoch, tile ? HM_CS_FLAG_AGG : HM_CS_FLAG_INC, agg),
                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const uint64_t excl = tile ? hm_cs_lookback(a.tstat, (int64_t)tile, a.epoch) : 0ull;
            if (lane == 0) {
                if (tile)
                    __hip_atomic_store(a.tstat + tile, hm_cs_word(a.epoch, HM_CS_FLAG_INC, excl + agg),
                                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (tile + 1 == ntiles) *a.m_out = (uint32_t)(excl + agg);
                excl_s = excl;
            }
            if (split) {
                const uint32_t xq = lane < NF ? wsq[lane] : 0u, xr = lane < NF ? wrc[lane] : 0u;
                uint32_t iq = xq, ir = xr;
#pragma unroll
                for (int o = 1; o < 64; o <<= 1) {
                    const uint32_t yq = __shfl_up(iq, o, 64), yr = __shfl_up(ir, o, 64);
                    if (lane >= o) {
                        iq += yq;
                        ir += yr;
                    }
                }
                const uint32_t tq = __shfl(iq, 63, 64), tr = __shfl(ir, 63, 64);
                if (lane < NF) {
                    wsq[lane] = iq - xq;
                    wrc[lane] = ir - xr;
                }
                if (lane == 0) {
                    bsq_s = tq ? atomicAdd(a.e.kcursor, (unsigned long long)tq) : 0ull;
                    brc_s = tr ? atomicAdd(a.e.xcursor, (unsigned long long)tr) : 0ull;
                }
            }
        }
        __syncthreads();
        const uint64_t excl = excl_s;
#pragma unroll
        for (int r = 0; r < HM_CS_IT; r++) {
            const uint64_t j = excl + wtot[r * NW + w] + ((fl[r] >> 2) & 0x7fu);
            if (fl[r] & 1u) hm_kst(a.kout_lo, a.kout_hi, j, k[r]);
            if (fl[r] & 2u) a.eout[j + (fl[r] & 1u) - 1] = e[r];
        }
        if (split) {
            /* the input cells again (L2-warm), to their reserved slots */
#pragma unroll 1
            for (int r = 0; r < HM_CS_IT; r++) {
                const int f = r * NW + w;
                const bool sq = (fl[r] >> 30) & 1u, rc = fl[r] >> 31;
                const uint64_t ms = __builtin_amdgcn_ballot_w64(sq), mx = __builtin_amdgcn_ballot_w64(rc);
                if (sq || rc) {
                    const uint64_t i = t0 + (uint64_t)r * HM_CS_THREADS + threadIdx.x;
                    const KT kk = hm_kld<KT>(a.kin_lo, a.kin_hi, i);
                    const uint32_t ep = i ? (a.ein ? a.ein[i - 1] : (uint32_t)i) : 0u;
                    uint32_t g;
                    int64_t row, col;
                    hm_gen_decode(hm_k128(kk, a.hic), a.Z, a.zin, &g, &row, &col);
                    const uint64_t cnt = (uint64_t)(e[r] - ep);
                    if (sq) hm_put_key(a.e, bsq_s + wsq[f] + hm_mbcnt(ms), a.zin, row, col, cnt);
                    else hm_put_record(a.e, brc_s + wrc[f] + hm_mbcnt(mx), g, a.zin, row, col, cnt);
                }
            }
        }
        __syncthreads();
    }
}

/* Two zoom steps per launch (packed records, width 2): the sorted level-zin
 * cells in, the records of levels zin AND zin - 1 out, and the level-(zin - 2)
 * cells for the next launch -- the level-(zin - 1) cells are never written
 * and read back (24 of every 80 bytes a pair of single steps moves).
 * A level-(zin - 1) cell holds at most 4 input cells (one zoom, one group),
 * so the last input cell of its run finds the END before the run at most 4
 * items back (lane shuffles; lanes 0..3 read the previous fragment's last 4
 * items from LDS) and writes the record; its slot is the number of
 * level-(zin - 1) heads up to it, from a second look-back (tstat2, wave 1)
 * beside the output level's (tstat, wave 0).  a.clr: low key bits cleared
 * for the OUTPUT level (zin - 2). */
#ifndef HM_CS2_IT
#define HM_CS2_IT 16                /* k_cascade2: items per thread of a tile */
#endif
#define HM_CS2_TILE (HM_CS_THREADS * HM_CS2_IT)
template <typename KT>
__device__ __forceinline__ KT hm_kshfl_up_d(KT k, int d);
template <>
__device__ __forceinline__ uint64_t hm_kshfl_up_d<uint64_t>(uint64_t k, int d)
{
    return __shfl_up((unsigned long long)k, d, 64);
}
template <>
__device__ __forceinline__ hm_u128 hm_kshfl_up_d<hm_u128>(hm_u128 k, int d)
{
    return ((hm_u128)__shfl_up((unsigned long long)(k >> 64), d, 64) << 64) |
           (hm_u128)__shfl_up((unsigned long long)k, d, 64);
}

template <typename KT>
__global__ __launch_bounds__(HM_CS_THREADS) void k_cascade2(HmCascArgs a)
{
    constexpr int NW = HM_CS_THREADS / 64, NF = HM_CS2_IT * NW;   /* (round, wave) fragments of a tile */
    __shared__ uint32_t wtot[NF], wtot1[NF];
    __shared__ KT kfirst[NF + 1];
    __shared__ KT klast4[NF + 1][4];      /* [f + 1][j]: lane 60 + j of fragment f; [0]: items t0 - 4 .. t0 - 1 */
    __shared__ uint32_t elast4[NF + 1][4];
    __shared__ uint32_t tile_s;
    __shared__ uint64_t excl_s, excl1_s;
    const uint64_t m = a.m_in ? (uint64_t)*a.m_in : a.m_host;
    const uint64_t ntiles = (m + HM_CS2_TILE - 1) / HM_CS2_TILE;
    const int lane = hm_lane(), w = threadIdx.x >> 6;
    const KT keep1 = ~((((KT)1) << (a.clr - 2)) - 1);   /* level zin - 1 */
    const KT keep2 = ~((((KT)1) << a.clr) - 1);         /* level zin - 2 (the output) */
    const unsigned long long rb = *a.rbase_in, rb1 = rb + m;
    if (m == 0 && blockIdx.x == 0 && threadIdx.x == 0) {
        *a.m_out = 0u;
        *a.rbase_out = rb1;
    }
    for (;;) {
        if (threadIdx.x == 0) tile_s = atomicAdd(a.ticket, 1u);
        __syncthreads();
        const uint64_t tile = tile_s;
        if (tile >= ntiles) break;
        const uint64_t t0 = tile * HM_CS2_TILE;
        KT k[HM_CS2_IT];
        uint32_t e[HM_CS2_IT];
#pragma unroll
        for (int r = 0; r < HM_CS2_IT; r++) {
            const uint64_t i = t0 + (uint64_t)r * HM_CS_THREADS + threadIdx.x;
            const bool v = i < m;
            k[r] = v ? hm_kld<KT>(a.kin_lo, a.kin_hi, i) : (KT)0;
            e[r] = v ? a.ein[i] : 0u;
        }
        if (threadIdx.x < 4) {
            const int64_t j = (int64_t)t0 - 4 + (int64_t)threadIdx.x;
            klast4[0][threadIdx.x] = j >= 0 ? hm_kld<KT>(a.kin_lo, a.kin_hi, (uint64_t)j) : (KT)0;
            elast4[0][threadIdx.x] = j >= 0 ? a.ein[j] : 0u;
        }
        if (threadIdx.x == HM_CS_THREADS - 1)
            kfirst[NF] = t0 + HM_CS2_TILE < m ? hm_kld<KT>(a.kin_lo, a.kin_hi, t0 + HM_CS2_TILE) : (KT)0;
#pragma unroll
        for (int r = 0; r < HM_CS2_IT; r++) {
            const int f = r * NW + w;
            if (lane == 0) kfirst[f] = k[r];
            if (lane >= 60) {
                klast4[f + 1][lane - 60] = k[r];
                elast4[f + 1][lane - 60] = e[r];
            }
        }
        __syncthreads();
        uint32_t fl[HM_CS2_IT];
#pragma unroll
        for (int r = 0; r < HM_CS2_IT; r++) {
            const int f = r * NW + w;
            const uint64_t i = t0 + (uint64_t)r * HM_CS_THREADS + threadIdx.x;
            const bool v = i < m;
            KT kp = hm_kshfl_up(k[r]), kn = hm_kshfl_down(k[r]);
            uint32_t ep = __shfl_up(e[r], 1, 64);
            if (lane == 0) {
                kp = klast4[f][3];
                ep = elast4[f][3];
            }
            if (lane == 63) kn = kfirst[f + 1];
            const KT k1 = k[r] & keep1, k2 = k[r] & keep2;
            const bool head1 = v && (i == 0 || (kp & keep1) != k1);
            const bool tail1 = v && (i + 1 == m || (kn & keep1) != k1);
            const bool head2 = v && (i == 0 || (kp & keep2) != k2);
            const bool tail2 = v && (i + 1 == m || (kn & keep2) != k2);
            /* the input level's record (its cells are compact: slot rb + i) */
            if (v) {
                uint32_t g;
                int64_t row, col;
                hm_gen_decode(hm_k128(k[r], a.hic), a.Z, a.zin, &g, &row, &col);
                hm_put_record(a.e, rb + i, g, a.zin, row, col, (uint64_t)(e[r] - (i ? ep : 0u)));
            }
            const uint64_t hb1 = __builtin_amdgcn_ballot_w64(head1), hb2 = __builtin_amdgcn_ballot_w64(head2);
            /* the lane of this cell's level-(zin - 1) run head, 64: before the fragment */
            const uint64_t below = hb1 & (((2ull << lane) - 1ull) | (lane == 63 ? ~0ull : 0ull));
            const uint32_t hl = below ? 63u - (uint32_t)__builtin_clzll(below) : 64u;
            if (lane == 0) {
                wtot[f] = (uint32_t)__popcll(hb2);
                wtot1[f] = (uint32_t)__popcll(hb1);
            }
            fl[r] = (uint32_t)head2 | ((uint32_t)tail2 << 1) | (hm_mbcnt(hb2) << 2) | ((uint32_t)tail1 << 9) |
                    ((hm_mbcnt(hb1) + (uint32_t)head1) << 10) | (hl << 17);
        }
        __syncthreads();
        if (w < 2) {
            /* wave 0: the output level's heads; wave 1: level zin - 1's */
            uint32_t* wt = w ? wtot1 : wtot;
            uint64_t* st = w ? a.tstat2 : a.tstat;
            const uint32_t x = lane < NF ? wt[lane] : 0u;
            uint32_t inc = x;
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                const uint32_t y = __shfl_up(inc, o, 64);
                if (lane >= o) inc += y;
            }
            const uint64_t agg = __shfl(inc, 63, 64);
            if (lane < NF) wt[lane] = inc - x;
            if (lane == 0)
                __hip_atomic_store(st + tile, hm_cs_word(a.epoch, tile ? HM_CS_FLAG_AGG : HM_CS_FLAG_INC, agg),
                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const uint64_t excl = tile ? hm_cs_lookback(st, (int64_t)tile, a.epoch) : 0ull;
            if (lane == 0) {
                if (tile)
                    __hip_atomic_store(st + tile, hm_cs_word(a.epoch, HM_CS_FLAG_INC, excl + agg), __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
                if (w == 0) {
                    if (tile + 1 == ntiles) *a.m_out = (uint32_t)(excl + agg);
                    excl_s = excl;
                } else {
                    if (tile + 1 == ntiles) *a.rbase_out = rb1 + excl + agg;
                    excl1_s = excl;
                }
            }
        }
        __syncthreads();
        const uint64_t excl = excl_s, excl1 = excl1_s;
#pragma unroll
        for (int r = 0; r < HM_CS2_IT; r++) {
            const int f = r * NW + w;
            const uint64_t j = excl + wtot[r * NW + w] + ((fl[r] >> 2) & 0x7fu);
            if (fl[r] & 1u) hm_kst(a.kout_lo, a.kout_hi, j, k[r] & keep2);
            if (fl[r] & 2u) a.eout[j + (fl[r] & 1u) - 1] = e[r];
            /* the END before this cell's level-(zin - 1) run: its head's
             * predecessor (one lane shuffle, every lane active), the previous
             * fragment's last item for a head at lane 0, and for a run that
             * began before the fragment (lanes 0..2: runs hold <= 4 cells)
             * the first of that fragment's last items with another key */
            const uint32_t hl = fl[r] >> 17;
            uint32_t eb = __shfl(e[r], hl >= 1u && hl < 64u ? (int)hl - 1 : 0, 64);
            if ((fl[r] >> 9) & 1u) {
                const KT k1 = k[r] & keep1;
                if (hl == 0u) {
                    eb = elast4[f][3];
                } else if (hl == 64u) {
                    const int64_t i0 = (int64_t)t0 + (int64_t)f * 64;   /* item of lane 0 */
                    eb = 0u;
                    for (int jj = 3; jj >= 0; jj--) {
                        if (i0 - 4 + jj < 0) break;
                        if ((klast4[f][jj] & keep1) != k1) {
                            eb = elast4[f][jj];
                            break;
                        }
                    }
                }
                /* the level-(zin - 1) record, by the last cell of its run */
                const uint64_t q = excl1 + wtot1[f] + ((fl[r] >> 10) & 0x7fu) - 1;
                uint32_t g;
                int64_t row, col;
                hm_gen_decode(hm_k128(k1, a.hic), a.Z, a.zin - 1, &g, &row, &col);
                hm_put_record(a.e, rb1 + q, g, a.zin - 1, row, col, (uint64_t)(e[r] - eb));
            }
        }
        __syncthreads();
    }
}

/* the records of the last level (nothing below it to fold into); split mode
 * reserves its slots once per block and kind */
template <typename KT>
__global__ __launch_bounds__(256) void k_cascade_emit(HmCascArgs a)
{
    __shared__ uint32_t wq[4], wr[4];
    __shared__ unsigned long long bq_s, br_s;
    const uint64_t m = a.m_in ? (uint64_t)*a.m_in : a.m_host;
    const unsigned long long rb = *a.rbase_in;
    if (blockIdx.x == 0 && threadIdx.x == 0) *a.rbase_out = rb + m;
    const uint64_t stride = (uint64_t)gridDim.x * 256;
    const uint64_t m_up = (m + 255) & ~255ull;   /* whole blocks: split mode reserves per block */
    const int lane = hm_lane(), w = threadIdx.x >> 6;
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < m_up; i += stride) {
        const bool v = i < m;
        const KT k = v ? hm_kld<KT>(a.kin_lo, a.kin_hi, i) : (KT)0;
        const uint32_t e = v ? a.ein[i] : 0u, ep = (v && i) ? a.ein[i - 1] : 0u;
        const uint64_t cnt = (uint64_t)(e - ep);
        uint32_t g = 0;
        int64_t row = 0, col = 0;
        if (v) hm_gen_decode(hm_k128(k, a.hic), a.Z, a.zin, &g, &row, &col);
        if (!a.e.split) {
            if (v) hm_put_record(a.e, rb + i, g, a.zin, row, col, cnt);
            continue;
        }
        const bool sq = v && hm_in_square(row, col, a.zin), rc = v && !sq;
        const uint64_t ms = __builtin_amdgcn_ballot_w64(sq), mx = __builtin_amdgcn_ballot_w64(rc);
        if (lane == 0) {
            wq[w] = (uint32_t)__popcll(ms);
            wr[w] = (uint32_t)__popcll(mx);
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            uint32_t tq = 0, tr = 0;
            for (int x = 0; x < 4; x++) {
                const uint32_t q = wq[x], r = wr[x];
                wq[x] = tq;
                wr[x] = tr;
                tq += q;
                tr += r;
            }
            bq_s = tq ? atomicAdd(a.e.kcursor, (unsigned long long)tq) : 0ull;
            br_s = tr ? atomicAdd(a.e.xcursor, (unsigned long long)tr) : 0ull;
        }
        __syncthreads();
        if (sq) hm_put_key(a.e, bq_s + wq[w] + hm_mbcnt(ms), a.zin, row, col, cnt);
        if (rc) hm_put_record(a.e, br_s + wr[w] + hm_mbcnt(mx), g, a.zin, row, col, cnt);
        __syncthreads();
    }
}

/* ------------------------------------------------------------------------ */
/* one-sweep LSD radix sort (keys only, stable)                              */
/* ------------------------------------------------------------------------ */
/* The digit histograms of every pass come from ONE read of the keys
 * (k_rx_hist_all); a pass is then one kernel: a block takes the next tile of
 * HM_OS_TILE keys from a ticket, ranks them (per wave: 8-ballot digit match
 * in key order; waves in order), publishes its per-digit counts and resolves
 * its per-digit global offsets with a decoupled look-back over the earlier
 * tiles (one thread per digit), then writes the tile through LDS in digit
 * order, so a digit's keys leave as one contiguous run.  Per pass: 8 B read
 * and 8 B written per narrow key (16 + 16 wide), plus 2 KB of look-back
 * words per tile. */
#define HM_OS_THREADS 256
#ifndef HM_OS_LB
#define HM_OS_LB 4                  /* one-sweep look-back: predecessors per round trip */
#endif
/* keys per thread: 32 narrow keys (211 VGPRs, 72 KB of LDS: 2 blocks per
 * CU; 16 measured 1.1 ms slower per grouped call), 16 wide ones */
template <typename KT> struct HmOs {
    static constexpr int IT = sizeof(KT) == 8 ? 32 : 16;
    static constexpr int TILE = HM_OS_THREADS * IT;
};
#define HM_OS_TILE_MIN (HM_OS_THREADS * 16)   /* look-back words are sized for the smaller tiles */
#define HM_OS_MAXP 16

struct HmRxAll {
    const uint64_t* lo;
    const uint64_t* hi;
    uint64_t n;
    int np;
    int sh[HM_OS_MAXP];
    unsigned long long* hist;   /* [np][256] */
};

template <typename KT>
__global__ __launch_bounds__(256) void k_rx_hist_all(HmRxAll a)
{
    __shared__ uint32_t h[HM_OS_MAXP * 256];
    for (int i = threadIdx.x; i < a.np * 256; i += 256) h[i] = 0;
    __syncthreads();
    const uint64_t stride = (uint64_t)gridDim.x * 256;
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < a.n; i += stride) {
        const KT k = hm_kld<KT>(a.lo, a.hi, i);
        for (int p = 0; p < a.np; p++) atomicAdd(&h[p * 256 + ((uint32_t)(k >> a.sh[p]) & 0xFFu)], 1u);
    }
    __syncthreads();
    for (int i = threadIdx.x; i < a.np * 256; i += 256)
        if (h[i]) atomicAdd(&a.hist[i], (unsigned long long)h[i]);
}

/* exclusive digit offsets of every pass, in place (one wave per pass) */
__global__ __launch_bounds__(64) void k_rx_digit_offsets(unsigned long long* hist)
{
    unsigned long long* hp = hist + blockIdx.x * 256;
    const int lane = hm_lane();
    unsigned long long v[4], t = 0;
#pragma unroll
    for (int q = 0; q < 4; q++) {
        v[q] = hp[lane * 4 + q];
        t += v[q];
    }
    unsigned long long inc = t;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const unsigned long long y = __shfl_up(inc, o, 64);
        if (lane >= o) inc += y;
    }
    unsigned long long b = inc - t;
#pragma unroll
    for (int q = 0; q < 4; q++) {
        hp[lane * 4 + q] = b;
        b += v[q];
    }
}

struct HmRxPass {
    const uint64_t* ilo;
    const uint64_t* ihi;
    uint64_t* olo;
    uint64_t* ohi;
    uint64_t n;
    int sh;
    const unsigned long long* goff;   /* 256 exclusive digit offsets of this pass */
    uint64_t* tstat;                  /* [tiles][256] look-back words */
    uint64_t epoch;
    unsigned* ticket;
};

template <typename KT>
__global__ __launch_bounds__(HM_OS_THREADS) void k_rx_onesweep(HmRxPass a)
{
    constexpr int HM_OS_IT = HmOs<KT>::IT, HM_OS_TILE = HmOs<KT>::TILE;
    __shared__ KT stage[HM_OS_TILE];
    __shared__ uint32_t wcnt[4][256];
    __shared__ uint32_t dbase[256];      /* tile-local start of each digit */
    __shared__ uint64_t gbase[256];      /* global start of each digit's run of this tile */
    __shared__ uint32_t wtot[4];
    __shared__ uint32_t tile_s;
    const int w = threadIdx.x >> 6, lane = hm_lane();
    const int sh = a.sh;
    const uint64_t ntiles = (a.n + HM_OS_TILE - 1) / HM_OS_TILE;
    for (;;) {
        if (threadIdx.x == 0) tile_s = atomicAdd(a.ticket, 1u);
        wcnt[0][threadIdx.x] = 0;
        wcnt[1][threadIdx.x] = 0;
        wcnt[2][threadIdx.x] = 0;
        wcnt[3][threadIdx.x] = 0;
        __syncthreads();
        const uint64_t tile = tile_s;
        if (tile >= ntiles) break;
        const uint64_t t0 = tile * HM_OS_TILE + (uint64_t)w * (HM_OS_TILE / 4);
        KT k[HM_OS_IT];
        uint32_t rk[HM_OS_IT / 2];
#pragma unroll
        for (int r = 0; r < HM_OS_IT; r++) {
            const uint64_t i = t0 + (uint64_t)r * 64 + lane;
            const bool v = i < a.n;
            k[r] = v ? hm_kld<KT>(a.ilo, a.ihi, i) : ~(KT)0;
        }
#pragma unroll
        for (int r = 0; r < HM_OS_IT; r++) {
            const uint64_t i = t0 + (uint64_t)r * 64 + lane;
            const bool v = i < a.n;
            const uint32_t d = (uint32_t)(k[r] >> sh) & 0xFFu;
            uint64_t m = __builtin_amdgcn_ballot_w64(v);
#pragma unroll
            for (int b = 0; b < 8; b++) {
                const uint64_t bb = __builtin_amdgcn_ballot_w64((d >> b) & 1u);
                m &= ((d >> b) & 1u) ? bb : ~bb;
            }
            const uint32_t below = hm_mbcnt(m);
            const uint32_t prev = wcnt[w][d];
            __builtin_amdgcn_wave_barrier();
            if (v && below == 0) wcnt[w][d] = prev + (uint32_t)__popcll(m);
            __builtin_amdgcn_wave_barrier();
            const uint32_t rank = v ? prev + below : 0xFFFFu;
            if (r & 1) rk[r >> 1] |= rank << 16;
            else rk[r >> 1] = rank;
        }
        __syncthreads();
        /* thread t owns digit t: wave prefixes, tile count, look-back */
        const uint32_t d = threadIdx.x;
        const uint32_t c0 = wcnt[0][d], c1 = wcnt[1][d], c2 = wcnt[2][d], c3 = wcnt[3][d];
        const uint32_t cnt = c0 + c1 + c2 + c3;
        uint64_t* st = a.tstat + tile * 256 + d;
        __hip_atomic_store(st, hm_cs_word(a.epoch, tile ? HM_CS_FLAG_AGG : HM_CS_FLAG_INC, cnt), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
        /* look back HM_OS_LB predecessors per round trip (a tile mostly finds
         * a run of aggregate-only predecessors before an inclusive one; one
         * load per step made the walk 35% of a pass) */
        uint64_t excl = 0;
        for (int64_t p = (int64_t)tile - 1; p >= 0;) {
            uint64_t wv[HM_OS_LB];
#pragma unroll
            for (int q = 0; q < HM_OS_LB; q++)
                wv[q] = p - q >= 0 ? __hip_atomic_load(a.tstat + (uint64_t)(p - q) * 256 + d, __ATOMIC_RELAXED,
                                                       __HIP_MEMORY_SCOPE_AGENT)
                                   : hm_cs_word(a.epoch, HM_CS_FLAG_INC, 0);
            int adv = 0;
            bool done = false;
#pragma unroll
            for (int q = 0; q < HM_OS_LB; q++) {
                if (done || adv < q) break;
                const uint64_t f = (wv[q] >> 40) == a.epoch ? (wv[q] >> HM_CS_VBITS) & 3ull : 0ull;
                if (!f) break;
                excl += wv[q] & ((1ull << HM_CS_VBITS) - 1);
                adv++;
                done = f == HM_CS_FLAG_INC;
            }
            if (done) break;
            if (!adv) __builtin_amdgcn_s_sleep(1);
            p -= adv;
        }
        if (tile)
            __hip_atomic_store(st, hm_cs_word(a.epoch, HM_CS_FLAG_INC, excl + cnt), __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
        /* tile-local digit starts: exclusive scan of cnt over the 256 digits */
        uint32_t inc = cnt;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = __shfl_up(inc, o, 64);
            if (lane >= o) inc += y;
        }
        if (lane == 63) wtot[w] = inc;
        __syncthreads();
        uint32_t wo = 0;
        for (int q = 0; q < w; q++) wo += wtot[q];
        const uint32_t db = wo + inc - cnt;
        dbase[d] = db;
        gbase[d] = a.goff[d] + excl;
        __syncthreads();
        /* wave prefixes per digit into wcnt (read back per key) */
        wcnt[0][d] = db;
        wcnt[1][d] = db + c0;
        wcnt[2][d] = db + c0 + c1;
        wcnt[3][d] = db + c0 + c1 + c2;
        __syncthreads();
#pragma unroll
        for (int r = 0; r < HM_OS_IT; r++) {
            const uint32_t rank = (rk[r >> 1] >> ((r & 1) * 16)) & 0xFFFFu;
            if (rank != 0xFFFFu) {
                const uint32_t dd = (uint32_t)(k[r] >> sh) & 0xFFu;
                stage[wcnt[w][dd] + rank] = k[r];
            }
        }
        __syncthreads();
        const uint32_t valid = (uint32_t)min<uint64_t>(HM_OS_TILE, a.n - tile * HM_OS_TILE);
        for (uint32_t j = threadIdx.x; j < valid; j += HM_OS_THREADS) {
            const KT kk = stage[j];
            const uint32_t dg = (uint32_t)(kk >> sh) & 0xFFu;
            hm_kst(a.olo, a.ohi, gbase[dg] + (j - dbase[dg]), kk);
        }
        __syncthreads();
    }
}

/* grouped counts from tiles (hm_count_grouped_tiles): list the kept ones,
 * one output reservation per block step of 256 * HM_TL_PPT points (as
 * k_project_list: a per-wave reservation on one counter saturates it) */
#define HM_TL_PPT 16
__global__ __launch_bounds__(256) void k_tiles_list(const int64_t* __restrict__ rows, const int64_t* __restrict__ cols,
                                                    const uint8_t* __restrict__ keep, const uint32_t* __restrict__ group,
                                                    int64_t n, int64_t* row, int64_t* col, uint32_t* grp, int64_t* idx,
                                                    unsigned long long* count)
{
    __shared__ uint32_t scr[256 / 64 + 1];
    __shared__ unsigned long long base_s;
    constexpr int64_t TILE = 256 * HM_TL_PPT;
    for (int64_t t0 = (int64_t)blockIdx.x * TILE; t0 < n; t0 += (int64_t)gridDim.x * TILE) {
        uint32_t pm = 0;
#pragma unroll
        for (int k = 0; k < HM_TL_PPT; k++) {
            const int64_t i = t0 + (int64_t)k * 256 + threadIdx.x;
            pm |= (uint32_t)(i < n && (!keep || keep[i])) << k;
        }
        uint32_t tot;
        uint32_t pos = hm_block_excl_scan<256>((uint32_t)__popc(pm), scr, &tot);
        if (threadIdx.x == 0) base_s = tot ? atomicAdd(count, (unsigned long long)tot) : 0ull;
        __syncthreads();
        const unsigned long long b = base_s;
        __syncthreads();
#pragma unroll
        for (int k = 0; k < HM_TL_PPT; k++) {
            if ((pm >> k) & 1u) {
                const int64_t i = t0 + (int64_t)k * 256 + threadIdx.x;
                const uint64_t q = b + pos++;
                row[q] = rows[i];
                col[q] = cols[i];
                grp[q] = group ? group[i] : 0u;
                idx[q] = i;
            }
        }
    }
}

/* ------------------------------------------------------------------------ */
/* launchers                                                                 */
/* ------------------------------------------------------------------------ */

static unsigned hm_ggrid(uint64_t n, unsigned per, unsigned cap)
{
    uint64_t b = (n + per - 1) / per;
    if (b > cap) b = cap;
    return (unsigned)(b ? b : 1);
}

void hm_launch_gen_keys(hipStream_t s, const HmGenArgs& a)
{
    hipLaunchKernelGGL(k_gen_keys, dim3(hm_ggrid(a.n, 256, 4096)), dim3(256), 0, s, a);
}

uint64_t hm_rx_os_tiles(uint64_t n) { return (n + HM_OS_TILE_MIN - 1) / HM_OS_TILE_MIN; }

/* LSD sort of n keys (lo[0], hi[0]) over the digits at shifts sh[0..np)
 * (ascending); (lo[1], hi[1]) is the other buffer.  state = 256 B tickets +
 * 16 x 2 KB histograms + tiles x 2 KB look-back words, zeroed here.  Returns
 * the index of the buffer that holds the sorted keys. */
int hm_launch_rx_sort(hipStream_t s, bool wide, uint64_t* const* lo, uint64_t* const* hi, uint64_t n, const int* sh,
                      int np, uint8_t* state)
{
    if (np == 0) return 0;
    const uint64_t nt = wide ? (n + HmOs<hm_u128>::TILE - 1) / HmOs<hm_u128>::TILE
                             : (n + HmOs<uint64_t>::TILE - 1) / HmOs<uint64_t>::TILE;
    (void)hipMemsetAsync(state, 0, 256 + HM_OS_MAXP * 2048 + nt * 2048, s);
    HmRxAll h;
    h.lo = lo[0];
    h.hi = hi[0];
    h.n = n;
    h.np = np;
    for (int p = 0; p < np; p++) h.sh[p] = sh[p];
    h.hist = (unsigned long long*)(state + 256);
    if (wide)
        hipLaunchKernelGGL(k_rx_hist_all<hm_u128>, dim3(hm_ggrid(n, 256 * 16, 2048)), dim3(256), 0, s, h);
    else
        hipLaunchKernelGGL(k_rx_hist_all<uint64_t>, dim3(hm_ggrid(n, 256 * 16, 2048)), dim3(256), 0, s, h);
    hipLaunchKernelGGL(k_rx_digit_offsets, dim3(np), dim3(64), 0, s, h.hist);
    int cur = 0;
    for (int p = 0; p < np; p++) {
        HmRxPass x;
        x.ilo = lo[cur];
        x.ihi = hi[cur];
        x.olo = lo[1 - cur];
        x.ohi = hi[1 - cur];
        x.n = n;
        x.sh = sh[p];
        x.goff = h.hist + p * 256;
        x.tstat = (uint64_t*)(state + 256 + HM_OS_MAXP * 2048);
        x.epoch = (uint64_t)p + 1;
        x.ticket = (unsigned*)state + p;
        if (wide)
            hipLaunchKernelGGL(k_rx_onesweep<hm_u128>, dim3(hm_ggrid(nt, 1, 512)), dim3(HM_OS_THREADS), 0, s, x);
        else
            hipLaunchKernelGGL(k_rx_onesweep<uint64_t>, dim3(hm_ggrid(nt, 1, 1024)), dim3(HM_OS_THREADS), 0, s, x);
        cur = 1 - cur;
    }
    return cur;
}

void hm_launch_cascade(hipStream_t s, const HmCascArgs& a, uint64_t bound, int emit_only, bool wide)
{
    if (emit_only == 2) {   /* two zoom steps (k_cascade2) */
        if (wide)
            hipLaunchKernelGGL(k_cascade2<hm_u128>, dim3(hm_ggrid(bound, HM_CS2_TILE, 2048)), dim3(HM_CS_THREADS), 0,
                               s, a);
        else
            hipLaunchKernelGGL(k_cascade2<uint64_t>, dim3(hm_ggrid(bound, HM_CS2_TILE, 2048)), dim3(HM_CS_THREADS), 0,
                               s, a);
        return;
    }
    if (emit_only) {
        if (wide)
            hipLaunchKernelGGL(k_cascade_emit<hm_u128>, dim3(hm_ggrid(bound, 256, 4096)), dim3(256), 0, s, a);
        else
            hipLaunchKernelGGL(k_cascade_emit<uint64_t>, dim3(hm_ggrid(bound, 256, 4096)), dim3(256), 0, s, a);
    } else {
        if (wide)
            hipLaunchKernelGGL(k_cascade<hm_u128>, dim3(hm_ggrid(bound, HM_CS_TILE, 2048)), dim3(HM_CS_THREADS), 0, s,
                               a);
        else
            hipLaunchKernelGGL(k_cascade<uint64_t>, dim3(hm_ggrid(bound, HM_CS_TILE, 2048)), dim3(HM_CS_THREADS), 0,
                               s, a);
    }
}

/* look-back words per level: sized for the smaller of the two kernels' tiles */
uint64_t hm_cascade_tiles(uint64_t n)
{
    constexpr uint64_t t = HM_CS_TILE < HM_CS2_TILE ? HM_CS_TILE : HM_CS2_TILE;
    return (n + t - 1) / t;
}

void hm_launch_tiles_list(hipStream_t s, const int64_t* rows, const int64_t* cols, const uint8_t* keep,
                          const uint32_t* group, int64_t n, int64_t* row, int64_t* col, uint32_t* grp, int64_t* idx,
                          unsigned long long* count)
{
    hipLaunchKernelGGL(k_tiles_list, dim3(hm_ggrid((uint64_t)n, 256 * HM_TL_PPT, 4096)), dim3(256), 0, s, rows, cols, keep, group,
                       n, row, col, grp, idx, count);
}

/* ------------------------------------------------------------------------ */
/* row JSON text: one thread per bin writes  ["{"] "z_r_c": V.0 ("}" | ", ")  */
/* ------------------------------------------------------------------------ */

__device__ __forceinline__ uint8_t* hm_put_u64(uint8_t* p, uint64_t x)
{
    char d[20];
    int k = 0;
    do {
        d[k++] = (char)('0' + x % 10);
        x /= 10;
    } while (x);
    while (k) *p++ = (uint8_t)d[--k];
    return p;
}

__global__ __launch_bounds__(256) void k_format_bins(HmFormatArgs a)
{
    const uint64_t stride = (uint64_t)gridDim.x * 256;
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < (uint64_t)a.n; i += stride) {
        uint8_t* p = a.text + a.offset[i];
        if (a.head[i]) *p++ = '{';
        *p++ = '"';
        p = hm_put_u64(p, (uint64_t)a.zoom[i]);
        *p++ = '_';
        p = hm_put_u64(p, (uint64_t)a.row[i]);
        *p++ = '_';
        p = hm_put_u64(p, (uint64_t)a.col[i]);
        *p++ = '"';
        *p++ = ':';
        *p++ = ' ';
        p = hm_put_u64(p, (uint64_t)a.value[i]);
        *p++ = '.';
        *p++ = '0';
        if (a.last[i]) {
            *p++ = '}';
        } else {
            *p++ = ',';
            *p++ = ' ';
        }
    }
}

void hm_launch_format_bins(hipStream_t s, const HmFormatArgs& a)
{
    if (a.n <= 0) return;
    const uint64_t blocks = std::min<uint64_t>(8192, ((uint64_t)a.n + 255) / 256);
    hipLaunchKernelGGL(k_format_bins, dim3((unsigned)blocks), dim3(256), 0, s, a);
}

/* row ids: one thread per row writes  name|span|tz_tr_tc  */
__global__ __launch_bounds__(256) void k_format_ids(HmIdArgs a)
{
    const uint64_t stride = (uint64_t)gridDim.x * 256;
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < (uint64_t)a.n; i += stride) {
        uint8_t* p = a.text + a.offset[i];
        const int64_t l = a.label[i], t = a.span[i];
        for (int64_t q = a.name_off[l]; q < a.name_off[l + 1]; q++) *p++ = a.names[q];
        *p++ = '|';
        for (int64_t q = a.span_off[t]; q < a.span_off[t + 1]; q++) *p++ = a.spans[q];
        *p++ = '|';
        p = hm_put_u64(p, (uint64_t)a.tz[i]);
        *p++ = '_';
        p = hm_put_u64(p, (uint64_t)a.tr[i]);
        *p++ = '_';
        p = hm_put_u64(p, (uint64_t)a.tc[i]);
    }
}

void hm_launch_format_ids(hipStream_t s, const HmIdArgs& a)
{
    if (a.n <= 0) return;
    const uint64_t blocks = std::min<uint64_t>(8192, ((uint64_t)a.n + 255) / 256);
    hipLaunchKernelGGL(k_format_ids, dim3((unsigned)blocks), dim3(256), 0, s, a);
}
