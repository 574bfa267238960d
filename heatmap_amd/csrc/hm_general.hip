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
 * point's key is 128 bits,
 *     group (32) | sr + 16 (5) | sc + 2^47 (48) | morton(ro, co) (2Z)
 * where sr = row >> Z and sc = col >> Z (arithmetic shifts) name the point's
 * zoom-0 tile ("super tile", any integers) and ro, co its tile's offsets inside
 * it.  The zoom-(Z-k) cell of the point is key >> 2k: the shift of a tile
 * (exact for negative rows and huge columns too) only drops
 * Morton bits.  So one LSD radix sort of the keys orders every zoom at once,
 * and the zoom cascade is a run-length reduction of the previous zoom's sorted
 * unique cells: zoom Z-k+1's cells shifted by 2 are non-decreasing.
 *
 * Radix sort: keys only, 8-bit digits, LSD, stable; digits that are the same
 * in every key (an OR/AND reduction taken while the keys are built) are
 * skipped.  A wave owns a tile of 1024 consecutive keys; its per-digit ranks
 * come from an 8-ballot match in tile order, so the scatter is stable.
 */
#include <hip/hip_runtime.h>
#include "hm_device.h"
#include "hm_pipeline.h"
#include "../../include/heatmap_amd.h"

typedef unsigned __int128 hm_u128;

__device__ __forceinline__ hm_u128 hm_ld128(const ulonglong2* p, uint64_t i)
{
    const ulonglong2 v = p[i];
    return ((hm_u128)v.y << 64) | (hm_u128)v.x;
}

__device__ __forceinline__ void hm_st128(ulonglong2* p, uint64_t i, hm_u128 k)
{
    p[i] = make_ulonglong2((unsigned long long)k, (unsigned long long)(k >> 64));
}

/* 21 -> 42 bit spread / compact (Morton halves) */
__device__ __forceinline__ uint64_t hm_spread21(uint64_t x)
{
    x &= 0x1FFFFFull;
    x = (x | (x << 16)) & 0x0000FFFF0000FFFFull;
    x = (x | (x << 8)) & 0x00FF00FF00FF00FFull;
    x = (x | (x << 4)) & 0x0F0F0F0F0F0F0F0Full;
    x = (x | (x << 2)) & 0x3333333333333333ull;
    return (x | (x << 1)) & 0x5555555555555555ull;
}

__device__ __forceinline__ uint64_t hm_compact21(uint64_t x)
{
    x &= 0x5555555555555555ull;
    x = (x | (x >> 1)) & 0x3333333333333333ull;
    x = (x | (x >> 2)) & 0x0F0F0F0F0F0F0F0Full;
    x = (x | (x >> 4)) & 0x00FF00FF00FF00FFull;
    x = (x | (x >> 8)) & 0x0000FFFF0000FFFFull;
    return (x | (x >> 16)) & 0x00000000FFFFFFFFull;
}

#define HM_GEN_SR_BIAS 16
#define HM_GEN_SC_BITS 48
#define HM_GEN_SC_BIAS (1ll << 47)

/* ------------------------------------------------------------------------ */
/* keys                                                                      */
/* ------------------------------------------------------------------------ */

__global__ __launch_bounds__(256) void k_gen_keys(HmGenArgs a)
{
    const uint64_t n = a.n;
    const uint64_t stride = (uint64_t)gridDim.x * 256;
    unsigned long long o_lo = 0, o_hi = 0, n_lo = ~0ull, n_hi = ~0ull;
    const int Z = a.Z;
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += stride) {
        const int64_t r = a.row[i], c = a.col[i];
        const int64_t sr = r >> Z, sc = c >> Z;
        const uint64_t m = (hm_spread21((uint64_t)r & ((1ull << Z) - 1)) << 1) |
                           hm_spread21((uint64_t)c & ((1ull << Z) - 1));
        hm_u128 k = 0;
        if (sr >= -HM_GEN_SR_BIAS && sr < HM_GEN_SR_BIAS && sc >= -HM_GEN_SC_BIAS && sc < HM_GEN_SC_BIAS) {
            const uint64_t g = a.group ? (uint64_t)a.group[i] : 0ull;
            const hm_u128 root = ((hm_u128)g << 53) | ((hm_u128)(uint64_t)(sr + HM_GEN_SR_BIAS) << 48) |
                                 (hm_u128)(uint64_t)(sc + HM_GEN_SC_BIAS);
            k = (root << (2 * Z)) | (hm_u128)m;
        } else {
            /* representable by the reference, beyond this path's key */
            const uint64_t src = a.index ? (uint64_t)a.index[i] : i;
            atomicMin(a.err_word, ((unsigned long long)src << 8) | (unsigned long long)HM_E_RANGE);
        }
        hm_st128(a.keys, i, k);
        o_lo |= (unsigned long long)k;
        o_hi |= (unsigned long long)(k >> 64);
        n_lo &= (unsigned long long)k;
        n_hi &= (unsigned long long)(k >> 64);
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        o_lo |= __shfl_xor(o_lo, o, 64);
        o_hi |= __shfl_xor(o_hi, o, 64);
        n_lo &= __shfl_xor(n_lo, o, 64);
        n_hi &= __shfl_xor(n_hi, o, 64);
    }
    if (hm_lane() == 0) {
        atomicOr(&a.orand[0], o_lo);
        atomicOr(&a.orand[1], o_hi);
        atomicAnd(&a.orand[2], n_lo);
        atomicAnd(&a.orand[3], n_hi);
    }
}

/* ------------------------------------------------------------------------ */
/* LSD radix sort pass (keys only, stable)                                   */
/* ------------------------------------------------------------------------ */

#define HM_RX_WT 1024                 /* keys per wave tile */
#define HM_RX_J (HM_RX_WT / 64)

__device__ __forceinline__ uint32_t hm_rx_digit(hm_u128 k, int sh) { return (uint32_t)(k >> sh) & 0xFFu; }

/* per wave tile: digit histogram, digit-major into hist[d * ntiles + t] */
__global__ __launch_bounds__(256) void k_rx_hist(const ulonglong2* __restrict__ keys, uint64_t n, int sh,
                                                 uint64_t ntiles, uint64_t* __restrict__ hist)
{
    __shared__ uint32_t h[4][256];
    const int w = threadIdx.x >> 6, lane = hm_lane();
    const uint64_t t = (uint64_t)blockIdx.x * 4 + w;
#pragma unroll
    for (int q = 0; q < 4; q++) h[w][lane * 4 + q] = 0;
    __syncthreads();
    if (t < ntiles) {
        for (int j = 0; j < HM_RX_J; j++) {
            const uint64_t i = t * HM_RX_WT + (uint64_t)j * 64 + lane;
            if (i < n) atomicAdd(&h[w][hm_rx_digit(hm_ld128(keys, i), sh)], 1u);
        }
    }
    __syncthreads();
    if (t < ntiles) {
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const uint32_t d = lane * 4 + q;
            hist[(uint64_t)d * ntiles + t] = h[w][d];
        }
    }
}

/* stable scatter: keys of a wave tile in index order; the lanes of one
 * 64-key step holding digit d are matched with 8 ballots, ranked by lane */
__global__ __launch_bounds__(256) void k_rx_scatter(const ulonglong2* __restrict__ in, ulonglong2* __restrict__ out,
                                                    uint64_t n, int sh, uint64_t ntiles, const uint64_t* __restrict__ off)
{
    __shared__ uint32_t base[4][256];
    const int w = threadIdx.x >> 6, lane = hm_lane();
    const uint64_t t = (uint64_t)blockIdx.x * 4 + w;
    if (t < ntiles) {
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const uint32_t d = lane * 4 + q;
            base[w][d] = (uint32_t)off[(uint64_t)d * ntiles + t];
        }
    }
    __syncthreads();
    if (t >= ntiles) return;   /* wave-uniform */
    for (int j = 0; j < HM_RX_J; j++) {
        const uint64_t i = t * HM_RX_WT + (uint64_t)j * 64 + lane;
        const bool v = i < n;
        const hm_u128 k = v ? hm_ld128(in, i) : (hm_u128)0;
        const uint32_t d = hm_rx_digit(k, sh);
        uint64_t m = __ballot(v);
#pragma unroll
        for (int b = 0; b < 8; b++) {
            const uint64_t bb = __ballot((d >> b) & 1u);
            m &= ((d >> b) & 1u) ? bb : ~bb;
        }
        const uint32_t rank = hm_mbcnt(m);
        const uint32_t p = base[w][d] + rank;
        __builtin_amdgcn_wave_barrier();
        if (v && rank == 0) base[w][d] = p + (uint32_t)__popcll(m);
        __builtin_amdgcn_wave_barrier();
        if (v) hm_st128(out, p, k);
    }
}

/* ------------------------------------------------------------------------ */
/* zoom cascade: run-length reduction of sorted cells                        */
/* ------------------------------------------------------------------------ */

/* head flags and counts of (key >> s) over a sorted list */
__global__ __launch_bounds__(256) void k_rle_prep(const ulonglong2* __restrict__ keys, const uint64_t* __restrict__ cnt,
                                                  uint64_t n, int s, uint64_t* __restrict__ flag, uint64_t* __restrict__ c)
{
    const uint64_t stride = (uint64_t)gridDim.x * 256;
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += stride) {
        const hm_u128 k = hm_ld128(keys, i) >> s;
        const bool head = i == 0 || (hm_ld128(keys, i - 1) >> s) != k;
        flag[i] = head;
        c[i] = cnt ? cnt[i] : 1ull;
    }
}

/* unique keys at their index; segment end (inclusive count prefix) per cell */
__global__ __launch_bounds__(256) void k_rle_scatter(const ulonglong2* __restrict__ keys, uint64_t n, int s,
                                                     const uint64_t* __restrict__ flag, const uint64_t* __restrict__ idx,
                                                     const uint64_t* __restrict__ S, const uint64_t* __restrict__ c,
                                                     ulonglong2* __restrict__ okey, uint64_t* __restrict__ oend)
{
    const uint64_t stride = (uint64_t)gridDim.x * 256;
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += stride) {
        const uint64_t j = idx[i] + flag[i] - 1;   /* segment of i (idx: exclusive head count) */
        if (flag[i]) hm_st128(okey, j, hm_ld128(keys, i) >> s);
        if (i + 1 == n || flag[i + 1]) oend[j] = S[i] + c[i];
    }
}

/* counts of zoom z's cells (next level's input) and their records */
__global__ __launch_bounds__(256) void k_rle_emit(HmGenEmit e, const ulonglong2* __restrict__ okey,
                                                  const uint64_t* __restrict__ oend, uint64_t u, int z,
                                                  uint64_t* __restrict__ ocnt, uint64_t base, int emit)
{
    const uint64_t stride = (uint64_t)gridDim.x * 256;
    const hm_u128 mm = ((hm_u128)1 << (2 * z)) - 1;
    const uint64_t u_up = (u + 63) & ~63ull;   /* split mode appends per wave */
    for (uint64_t j = (uint64_t)blockIdx.x * 256 + threadIdx.x; j < u_up; j += stride) {
        const bool in = j < u;
        uint64_t cnt = 0;
        int64_t row = 0, col = 0;
        hm_u128 root = 0;
        if (in) {
            cnt = oend[j] - (j ? oend[j - 1] : 0ull);
            ocnt[j] = cnt;
            const hm_u128 k = hm_ld128(okey, j);
            root = k >> (2 * z);
            const uint64_t m = (uint64_t)(k & mm);
            const int64_t sr = (int64_t)(uint64_t)((root >> 48) & 31) - HM_GEN_SR_BIAS;
            const int64_t sc = (int64_t)(uint64_t)(root & ((((hm_u128)1) << HM_GEN_SC_BITS) - 1)) - HM_GEN_SC_BIAS;
            /* sr * 2^z, sc * 2^z as unsigned shifts (two's complement) */
            row = (int64_t)(((uint64_t)sr << z) + hm_compact21(m >> 1));
            col = (int64_t)(((uint64_t)sc << z) + hm_compact21(m));
        }
        if (!emit) continue;
        uint64_t q = base + j;
        bool rec = in;
        if (e.split) {
            /* hm_count fallback: cells inside [0, 2^z)^2 as (HM_KEY, count),
             * the others as records; one append per wave and kind */
            const bool sq = in && (uint64_t)row < (1ull << z) && (uint64_t)col < (1ull << z);
            rec = in && !sq;
            const uint64_t ms = __ballot(sq), mx = __ballot(rec);
            const int ls = ms ? __ffsll((unsigned long long)ms) - 1 : 0;
            const int lx = mx ? __ffsll((unsigned long long)mx) - 1 : 0;
            unsigned long long bs = 0, bx = 0;
            if (ms && hm_lane() == ls) bs = atomicAdd(e.kcursor, (unsigned long long)__popcll(ms));
            if (mx && hm_lane() == lx) bx = atomicAdd(e.xcursor, (unsigned long long)__popcll(mx));
            bs = __shfl(bs, ls, 64);
            bx = __shfl(bx, lx, 64);
            if (sq) {
                const uint64_t p = bs + hm_mbcnt(ms);
                if (p < e.kcapacity) {
                    e.keys[p] = ((uint64_t)z << 58) | ((uint64_t)row << 29) | (uint64_t)col;
                    e.counts[p] = cnt;
                }
            }
            q = bx + hm_mbcnt(mx);
        }
        if (!rec || q >= e.capacity) continue;
        int64_t* r = e.cells + q * e.width;
        int f = 0;
        if (e.width == 5) r[f++] = (int64_t)(uint64_t)(root >> 53);
        r[f++] = z;
        r[f++] = row;
        r[f++] = col;
        r[f] = (int64_t)cnt;
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
    hipLaunchKernelGGL(k_gen_keys, dim3(hm_ggrid(a.n, 256, 8192)), dim3(256), 0, s, a);
}

uint64_t hm_rx_tiles(uint64_t n) { return (n + HM_RX_WT - 1) / HM_RX_WT; }

void hm_launch_rx_pass(hipStream_t s, const ulonglong2* in, ulonglong2* out, uint64_t n, int sh, uint64_t* hist,
                       uint64_t* off, uint64_t* partial, uint64_t* total)
{
    const uint64_t nt = hm_rx_tiles(n);
    const unsigned blocks = (unsigned)((nt + 3) / 4);
    hipLaunchKernelGGL(k_rx_hist, dim3(blocks), dim3(256), 0, s, in, n, sh, nt, hist);
    hm_launch_scan(s, hist, nt * 256, partial, off, total);
    hipLaunchKernelGGL(k_rx_scatter, dim3(blocks), dim3(256), 0, s, in, out, n, sh, nt, off);
}

void hm_launch_rle_prep(hipStream_t s, const ulonglong2* keys, const uint64_t* cnt, uint64_t n, int sh, uint64_t* flag,
                        uint64_t* c)
{
    hipLaunchKernelGGL(k_rle_prep, dim3(hm_ggrid(n, 256, 16384)), dim3(256), 0, s, keys, cnt, n, sh, flag, c);
}

void hm_launch_rle_scatter(hipStream_t s, const ulonglong2* keys, uint64_t n, int sh, const uint64_t* flag,
                           const uint64_t* idx, const uint64_t* S, const uint64_t* c, ulonglong2* okey, uint64_t* oend)
{
    hipLaunchKernelGGL(k_rle_scatter, dim3(hm_ggrid(n, 256, 16384)), dim3(256), 0, s, keys, n, sh, flag, idx, S, c,
                       okey, oend);
}

void hm_launch_rle_emit(hipStream_t s, const HmGenEmit& e, const ulonglong2* okey, const uint64_t* oend, uint64_t u,
                        int z, uint64_t* ocnt, uint64_t base, int emit)
{
    hipLaunchKernelGGL(k_rle_emit, dim3(hm_ggrid(u, 256, 16384)), dim3(256), 0, s, e, okey, oend, u, z, ocnt, base,
                       emit);
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
