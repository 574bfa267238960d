/* gfx950 kernels of the multi-GPU cell exchange (heatmap_amd/multigpu.py).
 *
 * The reference's only data exchange is Spark's two shuffles per level:
 * reduceByKey (heatmap.py:111) sums the counts of a cell key, groupByKey
 * (heatmap.py:112) collects a heatmap row's bins on one executor.  Across GPUs
 * every rank counts its shard with hm_count, then:
 *   k_cells_route     per cell: zooms <= dense_zmax are added into a dense
 *                     Morton-ordered u64 grid (zoom z at offset (4^z - 1)/3;
 *                     summed across ranks by one RCCL reduce); sparser zooms
 *                     are routed to the rank that owns their heatmap row
 *                     (zoom, row >> delta, col >> delta): the groupByKey key,
 *                     so a row's bins meet on one rank.  Block-local owner
 *                     histograms reserve each block's output with one atomic
 *                     per owner; the cells then land grouped by owner, ready
 *                     for one RCCL all-to-all.
 *   k_cells_merge     received cells -> device hash table (hm_table.h):
 *                     equal keys from several ranks sum their counts;
 *   k_table_extract   the table's occupied slots -> (key, count) lists;
 *   k_dense_extract   the reduced dense grid -> non-empty cells (root rank).
 */
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <type_traits>

#include "hm_device.h"
#include "hm_pipeline.h"
#include "hm_table.h"

#define HM_ROUTE_THREADS 256
#define HM_MAX_RANKS 64

/* owner rank of a cell: multiplicative hash of its heatmap-row key (and, for
 * grouped cells, the group: the row id is user|alltime|tile, heatmap.py:55) */
__device__ __forceinline__ uint32_t hm_owner(uint64_t key, int delta, int nranks, uint64_t gmix = 0)
{
    const int64_t z = (int64_t)(key >> 58);
    const int64_t r = (int64_t)((key >> 29) & 0x1FFFFFFFull), c = (int64_t)(key & 0x1FFFFFFFull);
    const int64_t rk = ((z << 48) ^ ((r >> delta) << 24) ^ (c >> delta)) + (int64_t)(gmix * 0xD6E8FEB86659FD93ull);
    const int64_t h = (int64_t)((uint64_t)rk * 0x9E3779B97F4A7C15ull) >> 33;   /* wrapping multiply */
    const int64_t m = h % nranks;
    return (uint32_t)(m < 0 ? m + nranks : m);
}

__device__ __forceinline__ uint64_t hm_spread29(uint64_t v)
{
    v &= 0xFFFFFFFFull;
    v = (v | (v << 16)) & 0x0000FFFF0000FFFFull;
    v = (v | (v << 8)) & 0x00FF00FF00FF00FFull;
    v = (v | (v << 4)) & 0x0F0F0F0F0F0F0F0Full;
    v = (v | (v << 2)) & 0x3333333333333333ull;
    return (v | (v << 1)) & 0x5555555555555555ull;
}

__device__ __forceinline__ uint64_t hm_compact29(uint64_t v)
{
    v &= 0x5555555555555555ull;
    v = (v | (v >> 1)) & 0x3333333333333333ull;
    v = (v | (v >> 2)) & 0x0F0F0F0F0F0F0F0Full;
    v = (v | (v >> 4)) & 0x00FF00FF00FF00FFull;
    v = (v | (v >> 8)) & 0x0000FFFF0000FFFFull;
    return (v | (v >> 16)) & 0x00000000FFFFFFFFull;
}

/* 10-byte exchange record of a sparse cell: its key in 48 bits (zoom << 42 |
 * row << 21 | col: zooms <= 21, so row and col fit 21 bits) and a u32 count,
 * as five u16 words (2-byte aligned, one all-to-all for keys and counts) */
__device__ __forceinline__ void hm_rec_put(uint16_t* r, uint64_t k, uint32_t c)
{
    const uint64_t p = ((k >> 58) << 42) | (((k >> 29) & 0x1FFFFFull) << 21) | (k & 0x1FFFFFull);
    r[0] = (uint16_t)p;
    r[1] = (uint16_t)(p >> 16);
    r[2] = (uint16_t)(p >> 32);
    r[3] = (uint16_t)c;
    r[4] = (uint16_t)(c >> 16);
}
__device__ __forceinline__ uint64_t hm_rec_key(const uint16_t* r)
{
    const uint64_t p = (uint64_t)r[0] | ((uint64_t)r[1] << 16) | ((uint64_t)r[2] << 32);
    return ((p >> 42) << 58) | (((p >> 21) & 0x1FFFFFull) << 29) | (p & 0x1FFFFFull);
}
__device__ __forceinline__ uint32_t hm_rec_count(const uint16_t* r) { return (uint32_t)r[3] | ((uint32_t)r[4] << 16); }

/* a record through the two aligned 8-byte words around it (2 loads, not 5
 * strided u16 ones; reads up to 6 bytes either side, inside the record's
 * 8-byte words -- the caller takes the u16 form for a run's last record) */
__device__ __forceinline__ void hm_rec_load(const uint16_t* r, uint64_t& key, uint32_t& cnt)
{
    const uintptr_t A = (uintptr_t)r;
    const uint64_t* q = (const uint64_t*)(A & ~(uintptr_t)7);
    const uint32_t sh = (uint32_t)(A & 7) * 8;
    const uint64_t q0 = q[0], q1 = q[1];
    const uint64_t lo = sh ? (q0 >> sh) | (q1 << (64 - sh)) : q0;
    const uint32_t hi = (uint32_t)(q1 >> sh) & 0xFFFFu;
    const uint64_t p = lo & 0xFFFFFFFFFFFFull;
    key = ((p >> 42) << 58) | (((p >> 21) & 0x1FFFFFull) << 29) | (p & 0x1FFFFFull);
    cnt = (uint32_t)(lo >> 48) | (hi << 16);
}

/* pass 1 (count) / pass 2 (scatter) over the same block-contiguous cells:
 * both passes see identical per-block owner counts, so pass 1's block totals,
 * scanned owner-major, are pass 2's reservations (slots inside a block's
 * reservation are claimed with LDS atomics, any order) */
template <bool SCATTER>
__global__ __launch_bounds__(HM_ROUTE_THREADS) void k_cells_route(HmRouteArgs a)
{
    __shared__ uint32_t hist[HM_MAX_RANKS + 64];   /* + 64 dummy words (hm_lds_claim) */
    __shared__ uint64_t base[HM_MAX_RANKS];
    const int tid = threadIdx.x;
    if (tid < a.nranks) hist[tid] = 0;
    if (SCATTER && tid < a.nranks) base[tid] = a.block_off[(uint64_t)tid * gridDim.x + blockIdx.x];
    __syncthreads();
    const uint64_t per = (a.n + gridDim.x - 1) / gridDim.x;
    const uint64_t b0 = (uint64_t)blockIdx.x * per, b1 = min(b0 + per, (uint64_t)a.n);
    for (uint64_t i0 = b0; i0 < b1; i0 += HM_ROUTE_THREADS) {
        const uint64_t i = i0 + tid;
        const bool in = i < b1;
        const uint64_t k = in ? a.keys[i] : 0ull;
        const int z = (int)(k >> 58);
        const bool dense = in && z <= a.dense_zmax;
        if (!SCATTER && dense) {
            const uint64_t r = (k >> 29) & 0x1FFFFFFFull, c = k & 0x1FFFFFFFull;
            const uint64_t off = ((1ull << (2 * z)) - 1) / 3;
            atomicAdd((unsigned long long*)&a.grid[off + ((hm_spread29(r) << 1) | hm_spread29(c))],
                      (unsigned long long)a.counts[i]);
        }
        const bool sp = in && !dense;
        const uint32_t g = a.grouped && in ? (uint32_t)(a.counts[i] >> 32) : 0u;
        const uint32_t o = sp ? hm_owner(k, a.delta, a.nranks, a.grouped ? (uint64_t)g + 1 : 0ull) : 0u;
        if (SCATTER) {
            const uint32_t pos = hm_lds_claim(hist, HM_MAX_RANKS, o, sp);
            if (sp) {
                const uint64_t q = base[o] + pos;
                if (a.rec_out) {
                    hm_rec_put(a.rec_out + 5 * q, k, (uint32_t)a.counts[i]);
                } else if (a.grouped) {
                    a.keys_out[q] = hm_gkey(k, g);
                    a.counts_out32[q] = (uint32_t)a.counts[i];
                } else {
                    a.keys_out[q] = k;
                    if (a.counts_out32) a.counts_out32[q] = (uint32_t)a.counts[i];
                    else a.counts_out[q] = a.counts[i];
                }
            }
        } else {
            hm_lds_count(hist, HM_MAX_RANKS, o, sp);
            /* wide: a count needs 64 bits, or (10-byte records) a key does not
             * fit 48 bits (zoom > 21, row or column >= 2^21) */
            const bool kw = (a.rec_out || a.grouped) && (z > 21 || ((k >> 29) & 0x1FFFFFFFull) >= (1ull << 21) ||
                                                         (k & 0x1FFFFFFFull) >= (1ull << 21));
            /* grouped: the count field is 32 bits already; the group must fit the merge key */
            const bool cw = a.grouped ? g >= (1u << HM_GKEY_GROUP_BITS) : (a.counts[i] >> 32) != 0ull;
            if (a.wide && __any(sp && (cw || kw)) && (tid & 63) == 0)
                atomicOr(a.wide, 1ull);
        }
    }
    __syncthreads();
    if (!SCATTER && tid < a.nranks) a.block_cnt[(uint64_t)tid * gridDim.x + blockIdx.x] = hist[tid];
}

template <typename CT>
__global__ __launch_bounds__(256) void k_cells_merge(const uint64_t* __restrict__ keys, const CT* __restrict__ counts,
                                                     uint64_t n, HmsTable t)
{
    uint32_t overflow = 0;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
        hms_insert(t, keys[i], counts[i], &overflow);
    const uint64_t of = hms_wave_sum(overflow);
    if ((threadIdx.x & 63) == 0 && of) atomicAdd(&t.state[HMS_ST_OVERFLOW], (unsigned long long)of);
}

/* one run of distinct keys (one rank's cells): only the key claim is atomic,
 * the count a plain store or read-modify-write (hms_insert_unique) */
__global__ __launch_bounds__(256) void k_cells_merge_unique(const uint64_t* __restrict__ keys,
                                                            const uint64_t* __restrict__ counts, uint64_t n,
                                                            HmsTable t)
{
    uint32_t overflow = 0;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
        hms_insert_unique(t, keys[i], counts[i], &overflow);
    const uint64_t of = hms_wave_sum(overflow);
    if ((threadIdx.x & 63) == 0 && of) atomicAdd(&t.state[HMS_ST_OVERFLOW], (unsigned long long)of);
}

/* occupied slots -> (key, count).  Block b owns the contiguous slot range
 * [b C, b C + C): a first sweep counts its occupied slots and ONE atomic per
 * block reserves their output range; a second sweep writes them in slot order
 * (per 1024-slot step: wave ballots + a block scan).  One reservation per
 * 64-slot wave put a million same-address atomics on the cursor for a 64M-slot
 * table (~88 per us: 12.6 ms); now it is a few thousand. */
#define HM_TX_THREADS 256
#define HM_TX_SPT 4
__global__ __launch_bounds__(HM_TX_THREADS) void k_table_extract(HmsTable t, uint64_t* __restrict__ keys_out,
                                                               uint64_t* __restrict__ counts_out, uint64_t cap,
                                                               unsigned long long* cursor, uint64_t chunk)
{
    __shared__ uint32_t wsum[HM_TX_THREADS / 64 + 1];
    __shared__ unsigned long long sbase;
    const uint64_t n = t.mask + 1;
    const uint64_t b0 = (uint64_t)blockIdx.x * chunk, b1 = min(b0 + chunk, n);
    if (b0 >= n) return;
    const ulonglong2* slots = (const ulonglong2*)t.slots;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    constexpr uint32_t STEP = HM_TX_THREADS * HM_TX_SPT;
    uint32_t c = 0;
    for (uint64_t i = b0 + tid; i < b1; i += HM_TX_THREADS) c += slots[i].x != HMS_EMPTY;
    c = hm_wave_sum(c);
    if (lane == 0) wsum[w] = c;
    __syncthreads();
    if (tid == 0) {
        uint32_t tot = 0;
        for (int k = 0; k < HM_TX_THREADS / 64; k++) tot += wsum[k];
        sbase = tot ? atomicAdd(cursor, (unsigned long long)tot) : 0ull;
    }
    __syncthreads();
    uint64_t base = sbase;
    for (uint64_t s0 = b0; s0 < b1; s0 += STEP) {
        ulonglong2 sl[HM_TX_SPT];
        uint64_t bal[HM_TX_SPT];
        uint32_t mine = 0;
#pragma unroll
        for (int k = 0; k < HM_TX_SPT; k++) {
            const uint64_t i = s0 + (uint64_t)(w * HM_TX_SPT + k) * 64 + lane;   /* a wave's 4 x 64 slots */
            sl[k] = i < b1 ? slots[i] : make_ulonglong2(HMS_EMPTY, 0ull);
            bal[k] = __ballot(sl[k].x != HMS_EMPTY);
            mine += (uint32_t)__popcll(bal[k]);
        }
        __syncthreads();
        if (lane == 0) wsum[w] = mine;
        __syncthreads();
        uint32_t before = 0, tot = 0;
        for (int k = 0; k < HM_TX_THREADS / 64; k++) {
            before += k < w ? wsum[k] : 0u;
            tot += wsum[k];
        }
        uint64_t pos = base + before;
#pragma unroll
        for (int k = 0; k < HM_TX_SPT; k++) {
            if (sl[k].x != HMS_EMPTY) {
                const uint64_t q = pos + hm_mbcnt(bal[k]);
                if (q < cap) {
                    keys_out[q] = sl[k].x;
                    counts_out[q] = sl[k].y;
                }
            }
            pos += (uint32_t)__popcll(bal[k]);
        }
        base += tot;
    }
}

/* non-empty cells of the dense grid (zooms 0..dense_zmax) */
__global__ __launch_bounds__(256) void k_dense_extract(const uint64_t* __restrict__ grid, uint64_t total,
                                                       int dense_zmax, uint64_t* __restrict__ keys_out,
                                                       uint64_t* __restrict__ counts_out, uint64_t cap,
                                                       unsigned long long* cursor)
{
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i0 = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) & ~63ull; i0 < total; i0 += stride) {
        const uint64_t i = i0 + lane;
        const uint64_t v = i < total ? grid[i] : 0ull;
        const uint64_t bal = __ballot(v != 0);
        if (!bal) continue;
        unsigned long long first = 0;
        if (lane == 0) first = atomicAdd(cursor, (unsigned long long)__popcll(bal));
        first = __shfl(first, 0, 64);
        if (v) {
            int z = 0;
            while (z < dense_zmax && i >= (((1ull << (2 * (z + 1))) - 1) / 3)) z++;
            const uint64_t m = i - ((1ull << (2 * z)) - 1) / 3;
            const uint64_t pos = first + hm_mbcnt(bal);
            if (pos < cap) {
                keys_out[pos] = ((uint64_t)z << 58) | (hm_compact29(m >> 1) << 29) | hm_compact29(m);
                counts_out[pos] = v;
            }
        }
    }
}

/* ---- bucketed merge (hm_cells_merge / hm_cells_merge_runs) ----
 * The owner of a multi-GPU exchange receives every rank's cells of its rows,
 * one run per sender (~28M cells at 1.25e9 points per rank).  Inserting them
 * one by one into a 1 GB global hash table is a random read-modify-write per
 * cell; here the cells are first hash-partitioned into buckets of ~2048
 * (two streaming passes), then one block per bucket sums equal keys in LDS
 * and writes the distinct cells with one output reservation. */
__device__ __forceinline__ uint32_t hm_mb_bucket(uint64_t k, int lb)
{
    return lb ? (uint32_t)(hms_hash(k) >> (64 - lb)) : 0u;
}

/* Hash partition of (key, count) cells, one pass (HmMbPass).  The count
 * pass histograms each chunk's digits; the scatter pass takes a chunk 4096
 * cells at a time, orders them by digit in LDS and writes every digit's
 * cells as one contiguous run at its running offset (a wave's stores are
 * consecutive words: a direct 4096-way scatter wrote one partial line per
 * cell and took 1.2 ms for 28M cells). */
#define HM_MB_PPT 16
#define HM_MB_TILE (256 * HM_MB_PPT)
#define HM_MB_MAXD 128
template <bool SCATTER>
__global__ __launch_bounds__(256) void k_mb_pass(HmMbPass a)
{
    __shared__ uint32_t hist[HM_MB_MAXD];
    __shared__ uint32_t toff[HM_MB_MAXD];
    __shared__ unsigned long long gb[HM_MB_MAXD];
    __shared__ uint32_t scr[256 / 64 + 1];
    __shared__ unsigned long long sk[SCATTER ? HM_MB_TILE : 1], sc[SCATTER ? HM_MB_TILE : 1];
    __shared__ uint8_t sd[SCATTER ? HM_MB_TILE : 1];
    const int tid = threadIdx.x;
    const uint32_t s = blockIdx.x / a.C, c = blockIdx.x % a.C;
    const uint32_t nd = 1u << a.bits, dm = nd - 1u;
    const uint64_t s0 = a.segoff ? a.segoff[(uint64_t)s * a.segstride] : 0ull;
    const uint64_t s1 = a.segoff ? a.segoff[(uint64_t)(s + 1) * a.segstride] : a.n;
    const uint64_t len = s1 - s0;
    const uint64_t c0 = s0 + len * c / a.C, c1 = s0 + len * (c + 1) / a.C;
    const uint64_t cbase = ((uint64_t)s << a.bits) * a.C + c;   /* + d * C */
    for (uint32_t d = tid; d < nd; d += 256) {
        hist[d] = 0;
        if (SCATTER) gb[d] = a.off[cbase + (uint64_t)d * a.C];
    }
    __syncthreads();
    if (!SCATTER) {
        for (uint64_t i = c0 + tid; i < c1; i += 256) {
            const uint64_t k = a.rin ? hm_rec_key(a.rin + 5 * i) : a.kin[i];
            atomicAdd(&hist[(uint32_t)(hms_hash(k) >> a.shift) & dm], 1u);
        }
        __syncthreads();
        for (uint32_t d = tid; d < nd; d += 256) a.cnt[cbase + (uint64_t)d * a.C] = hist[d];
        return;
    }
    for (uint64_t t0 = c0; t0 < c1; t0 += HM_MB_TILE) {
        const uint32_t tn = (uint32_t)min((uint64_t)HM_MB_TILE, c1 - t0);
        uint64_t k[HM_MB_PPT], cc[HM_MB_PPT];
        uint32_t d[HM_MB_PPT], r[HM_MB_PPT];
#pragma unroll
        for (int j = 0; j < HM_MB_PPT; j++) {
            const uint32_t i = j * 256 + tid;
            const bool v = i < tn;
            if (a.rin) {
                k[j] = v ? hm_rec_key(a.rin + 5 * (t0 + i)) : 0ull;
                cc[j] = v ? (uint64_t)hm_rec_count(a.rin + 5 * (t0 + i)) : 0ull;
            } else {
                k[j] = v ? a.kin[t0 + i] : 0ull;
                cc[j] = v ? (a.cin32 ? (uint64_t)a.cin32[t0 + i] : a.cin[t0 + i]) : 0ull;
            }
        }
#pragma unroll
        for (int j = 0; j < HM_MB_PPT; j++) {
            const bool v = (uint32_t)(j * 256 + tid) < tn;
            d[j] = (uint32_t)(hms_hash(k[j]) >> a.shift) & dm;
            r[j] = v ? atomicAdd(&hist[d[j]], 1u) : 0u;
        }
        __syncthreads();
        uint32_t tot;
        const uint32_t o = hm_block_excl_scan<256>(tid < (int)nd ? hist[tid] : 0u, scr, &tot);
        if (tid < (int)nd) toff[tid] = o;
        __syncthreads();
#pragma unroll
        for (int j = 0; j < HM_MB_PPT; j++) {
            if ((uint32_t)(j * 256 + tid) < tn) {
                const uint32_t pos = toff[d[j]] + r[j];
                sk[pos] = k[j];
                sc[pos] = cc[j];
                sd[pos] = (uint8_t)d[j];
            }
        }
        __syncthreads();
        for (uint32_t i = tid; i < tn; i += 256) {
            const uint32_t dd = sd[i];
            const uint64_t dst = gb[dd] + (i - toff[dd]);
            a.kout[dst] = sk[i];
            a.cout[dst] = sc[i];
        }
        __syncthreads();
        if (tid < (int)nd) {
            gb[tid] += hist[tid];
            hist[tid] = 0;
        }
        __syncthreads();
    }
}

void hm_launch_mb_pass(hipStream_t s, const HmMbPass& a, bool scatter)
{
    const unsigned g = a.nseg * a.C;
    if (scatter)
        hipLaunchKernelGGL(k_mb_pass<true>, dim3(g), dim3(256), 0, s, a);
    else
        hipLaunchKernelGGL(k_mb_pass<false>, dim3(g), dim3(256), 0, s, a);
}

/* one bucket per block: its cells into an LDS table (P sub-passes by hash
 * bits when the bucket is large, so a table never holds more than ~half its
 * slots), distinct cells out */
__global__ __launch_bounds__(HM_MB_THREADS) void k_mb_merge(HmMergeArgs a)
{
    __shared__ unsigned long long tk[HM_MB_TS];
    __shared__ unsigned long long tc[HM_MB_TS];
    __shared__ uint32_t scr[HM_MB_THREADS / 64 + 1];
    __shared__ unsigned long long sbase;
    __shared__ uint32_t full;
    const uint32_t b = blockIdx.x;
    const uint64_t e0 = a.boff[(uint64_t)b * a.nblocks], e1 = a.boff[(uint64_t)(b + 1) * a.nblocks];
    if (e1 == e0) return;
    const uint64_t size = e1 - e0;
    const uint32_t P = (uint32_t)((size + HM_MB_TS / 2 - 1) / (HM_MB_TS / 2));
    constexpr int SPT = HM_MB_TS / HM_MB_THREADS;
    for (uint32_t pass = 0; pass < P; pass++) {
        for (int j = 0; j < SPT; j++) {
            tk[j * HM_MB_THREADS + threadIdx.x] = HMS_EMPTY;
            tc[j * HM_MB_THREADS + threadIdx.x] = 0;
        }
        if (threadIdx.x == 0) full = 0;
        __syncthreads();
        for (uint64_t i = e0 + threadIdx.x; i < e1; i += HM_MB_THREADS) {
            const uint64_t k = a.pkeys[i];
            const uint64_t h = hms_hash(k);
            if ((uint32_t)((h >> 32) % P) != pass) continue;
            uint32_t sl = (uint32_t)h & (HM_MB_TS - 1);
            int probes = 0;
            for (;;) {
                const unsigned long long o = atomicCAS(&tk[sl], (unsigned long long)HMS_EMPTY, (unsigned long long)k);
                if (o == HMS_EMPTY || o == k) {
                    atomicAdd(&tc[sl], (unsigned long long)a.pcounts[i]);
                    break;
                }
                sl = (sl + 1) & (HM_MB_TS - 1);
                if (++probes == HM_MB_TS) {
                    full = 1;
                    break;
                }
            }
        }
        __syncthreads();
        if (full) {
            if (threadIdx.x == 0) atomicOr(a.overflow, 1ull);
            return;
        }
        uint32_t c = 0;
        for (int j = 0; j < SPT; j++) c += tk[threadIdx.x * SPT + j] != HMS_EMPTY;
        uint32_t tot;
        uint32_t off = hm_block_excl_scan<HM_MB_THREADS>(c, scr, &tot);
        if (threadIdx.x == 0) sbase = atomicAdd(a.cursor, (unsigned long long)tot);
        __syncthreads();
        const uint64_t base = sbase;
        for (int j = 0; j < SPT; j++) {
            const uint32_t sl = threadIdx.x * SPT + j;
            if (tk[sl] != HMS_EMPTY) {
                const uint64_t q = base + off++;
                if (q < a.cap) {
                    a.keys_out[q] = tk[sl];
                    a.counts_out[q] = tc[sl];
                }
            }
        }
        __syncthreads();
    }
}

void hm_launch_mb_merge(hipStream_t s, const HmMergeArgs& a)
{
    hipLaunchKernelGGL(k_mb_merge, dim3(1u << a.lb), dim3(HM_MB_THREADS), 0, s, a);
}

/* ---- the pieces exchange (hm_cells_route_pieces / hm_cells_merge_pieces) ----
 * The sender's route already partitions its cells by owner; it now orders each
 * owner's group by the first merge digit as well (the top `bits` bits of the
 * merge key's hash), so the owner skips the first partition pass: it gathers
 * digit s's piece of every sender (one chunked segment per digit), partitions
 * it by the next bits, and merges buckets of <= ~1000 cells in LDS. */
#ifndef HM_XR_PPT
#define HM_XR_PPT 16
#endif
#define HM_XR_TILE (256 * HM_XR_PPT)
#ifndef HM_XRC_PPT
#define HM_XRC_PPT 16                /* the count pass's cells in flight a thread */
#endif

struct HmXCell {
    uint32_t d;     /* digit, or ~0u: not routed (dense zoom / past the input) */
    uint64_t mk;    /* merge key */
};

__device__ __forceinline__ HmXCell hm_xr_cell(const HmRouteArgs& a, uint64_t k, uint64_t cn, bool in)
{
    HmXCell x;
    const int z = (int)(k >> 58);
    const bool sp = in && z > a.dense_zmax;
    const uint32_t g = a.grouped ? (uint32_t)(cn >> 32) : 0u;
    x.mk = a.grouped ? hm_gkey(k, g) : k;
    const uint32_t o = sp ? hm_owner(k, a.delta, a.nranks, a.grouped ? (uint64_t)g + 1 : 0ull) : 0u;
    const uint32_t h = a.bits ? (uint32_t)(hms_hash(x.mk) >> (64 - a.bits)) : 0u;
    /* group position of owner o: rank order, or (self >= 0) that owner last */
    const uint32_t po = a.self < 0 ? o : (o == (uint32_t)a.self ? (uint32_t)a.nranks - 1u : o - (o > (uint32_t)a.self));
    x.d = sp ? (po << a.bits) | h : ~0u;
    return x;
}

/* count pass: per-block digit histogram (+ the dense grid's atomics and the
 * wide flag, as k_cells_route<false>) */
__global__ __launch_bounds__(256) void k_xroute_count(HmRouteArgs a)
{
    __shared__ uint32_t hist[HM_XR_MAXD];
    const int tid = threadIdx.x;
    const uint32_t D = (uint32_t)a.nranks << a.bits;
    for (uint32_t d = tid; d < D; d += 256) hist[d] = 0;
    __syncthreads();
    const uint64_t c0 = a.n * blockIdx.x / gridDim.x, c1 = a.n * (blockIdx.x + 1) / gridDim.x;
    for (uint64_t t0 = c0; t0 < c1; t0 += 256 * HM_XRC_PPT) {
        uint64_t k[HM_XRC_PPT];
#pragma unroll
        for (int j = 0; j < HM_XRC_PPT; j++) {
            const uint64_t i = t0 + j * 256 + tid;
            k[j] = i < c1 ? a.keys[i] : 0ull;
        }
#pragma unroll
        for (int j = 0; j < HM_XRC_PPT; j++) {
            const uint64_t i = t0 + j * 256 + tid;
            const bool in = i < c1;
            const int z = (int)(k[j] >> 58);
            const bool dense = in && z <= a.dense_zmax;
            /* counts: the dense cells' (grid sums) and grouped cells' (the group
             * picks the owner); the wide checks are the scatter pass's */
            const uint64_t cn = (dense || (in && a.grouped)) ? a.counts[i] : 0ull;
            if (dense) {
                const uint64_t r = (k[j] >> 29) & 0x1FFFFFFFull, c = k[j] & 0x1FFFFFFFull;
                const uint64_t off = ((1ull << (2 * z)) - 1) / 3;
                atomicAdd((unsigned long long*)&a.grid[off + ((hm_spread29(r) << 1) | hm_spread29(c))],
                          (unsigned long long)cn);
            }
            const HmXCell x = hm_xr_cell(a, k[j], cn, in);
            if (x.d != ~0u) atomicAdd(&hist[x.d], 1u);
        }
    }
    __syncthreads();
    for (uint32_t d = tid; d < D; d += 256) a.block_cnt[(uint64_t)d * a.C + blockIdx.x] = hist[d];
}

/* scatter pass: each 2048-cell tile is ordered by digit in LDS, then every
 * digit's cells are written as one run at the block's running offset (the
 * runs of consecutive tiles of a block continue each other).  OUT: 0 records
 * (REC10), 1 u64 keys + u64 counts, 2 u64 keys + u32 counts (U32, G12) */
template <int OUT>
__global__ __launch_bounds__(256) void k_xroute_scatter(HmRouteArgs a)
{
    typedef typename std::conditional<OUT == 1, unsigned long long, uint32_t>::type CT;
    __shared__ uint32_t hist[HM_XR_MAXD];
    __shared__ uint32_t toff[HM_XR_MAXD];
    __shared__ unsigned long long gb[HM_XR_MAXD];
    __shared__ uint32_t scr[256 / 64 + 1];
    __shared__ unsigned long long sk[HM_XR_TILE];
    __shared__ CT sc[HM_XR_TILE];
    __shared__ uint16_t sd[HM_XR_TILE];
    const int tid = threadIdx.x;
    const uint32_t D = (uint32_t)a.nranks << a.bits;
    const uint32_t per = (D + 255) / 256;   /* digits per thread in the tile scan */
    for (uint32_t d = tid; d < D; d += 256) {
        hist[d] = 0;
        gb[d] = a.block_off[(uint64_t)d * a.C + blockIdx.x];
    }
    __syncthreads();
    const uint64_t c0 = a.n * blockIdx.x / gridDim.x, c1 = a.n * (blockIdx.x + 1) / gridDim.x;
    for (uint64_t t0 = c0; t0 < c1; t0 += HM_XR_TILE) {
        uint64_t k[HM_XR_PPT], cn[HM_XR_PPT];
        uint32_t d[HM_XR_PPT], r[HM_XR_PPT];
#pragma unroll
        for (int j = 0; j < HM_XR_PPT; j++) {
            const uint64_t i = t0 + j * 256 + tid;
            k[j] = i < c1 ? a.keys[i] : 0ull;
            cn[j] = i < c1 ? a.counts[i] : 0ull;
        }
        bool wide = false;
#pragma unroll
        for (int j = 0; j < HM_XR_PPT; j++) {
            const HmXCell x = hm_xr_cell(a, k[j], cn[j], t0 + j * 256 + tid < c1);
            d[j] = x.d;
            if (x.d != ~0u && OUT != 1) {
                /* wide: a count needs 64 bits, a grouped cell's group passes the
                 * merge key's field, or (records and grouped keys) the key
                 * passes 48 bits (zoom > 21, row or column >= 2^21) */
                const uint64_t kk = k[j];
                const bool kw = (OUT == 0 || a.grouped) &&
                                ((kk >> 58) > 21 || ((kk >> 29) & 0x1FFFFFFFull) >= (1ull << 21) ||
                                 (kk & 0x1FFFFFFFull) >= (1ull << 21));
                const bool cw = a.grouped ? (cn[j] >> 32) >= (1ull << HM_GKEY_GROUP_BITS) : (cn[j] >> 32) != 0ull;
                wide |= kw || cw;
            }
            if (OUT == 2 && a.grouped) k[j] = x.mk;
            r[j] = x.d != ~0u ? atomicAdd(&hist[x.d], 1u) : 0u;
        }
        if (OUT != 1 && a.wide && __any(wide) && (tid & 63) == 0) atomicOr(a.wide, 1ull);
        __syncthreads();
        uint32_t loc = 0;
        for (uint32_t q = 0; q < per; q++) {
            const uint32_t dd = tid * per + q;
            loc += dd < D ? hist[dd] : 0u;
        }
        uint32_t tot;
        uint32_t o = hm_block_excl_scan<256>(loc, scr, &tot);
        for (uint32_t q = 0; q < per; q++) {
            const uint32_t dd = tid * per + q;
            if (dd < D) {
                toff[dd] = o;
                o += hist[dd];
            }
        }
        __syncthreads();
#pragma unroll
        for (int j = 0; j < HM_XR_PPT; j++) {
            if (d[j] != ~0u) {
                const uint32_t pos = toff[d[j]] + r[j];
                sk[pos] = k[j];
                sc[pos] = (CT)cn[j];
                sd[pos] = (uint16_t)d[j];
            }
        }
        __syncthreads();
        for (uint32_t i = tid; i < tot; i += 256) {
            const uint32_t dd = sd[i];
            const uint64_t q = gb[dd] + (i - toff[dd]);
            if (OUT == 0) {
                hm_rec_put(a.rec_out + 5 * q, sk[i], (uint32_t)sc[i]);
            } else {
                a.keys_out[q] = sk[i];
                if (OUT == 1) a.counts_out[q] = sc[i];
                else a.counts_out32[q] = (uint32_t)sc[i];
            }
        }
        __syncthreads();
        for (uint32_t dd = tid; dd < D; dd += 256) {
            gb[dd] += hist[dd];
            hist[dd] = 0;
        }
        __syncthreads();
    }
}

/* per-owner rows of the device sizes array: sent, wide, pieces */
__global__ __launch_bounds__(256) void k_xroute_sizes(HmRouteArgs a)
{
    const uint32_t S = 1u << a.bits, D = (uint32_t)a.nranks << a.bits;
    const unsigned long long wide = a.wide ? *a.wide : 0ull;
    for (uint32_t d = threadIdx.x; d < D; d += 256) {
        const uint32_t p = d >> a.bits, s = d & (S - 1);   /* group position p -> owner o */
        const uint32_t o = a.self < 0 ? p : (p == (uint32_t)a.nranks - 1u ? (uint32_t)a.self : p + (p >= (uint32_t)a.self));
        long long* row = a.sizes + (uint64_t)o * a.stride;
        row[2 + s] = (long long)(a.block_off[(uint64_t)(d + 1) * a.C] - a.block_off[(uint64_t)d * a.C]);
        if (s == 0) {
            row[0] = (long long)(a.block_off[(uint64_t)(d + S) * a.C] - a.block_off[(uint64_t)d * a.C]);
            row[1] = wide ? 1ll : 0ll;
        }
    }
}

void hm_launch_xroute(hipStream_t s, const HmRouteArgs& a, bool scatter, int layout)
{
    if (!scatter)
        hipLaunchKernelGGL(k_xroute_count, dim3(a.C), dim3(256), 0, s, a);
    else if (layout == 10)
        hipLaunchKernelGGL(k_xroute_scatter<0>, dim3(a.C), dim3(256), 0, s, a);
    else if (layout == 8)
        hipLaunchKernelGGL(k_xroute_scatter<1>, dim3(a.C), dim3(256), 0, s, a);
    else
        hipLaunchKernelGGL(k_xroute_scatter<2>, dim3(a.C), dim3(256), 0, s, a);
}

void hm_launch_xroute_sizes(hipStream_t s, const HmRouteArgs& a)
{
    hipLaunchKernelGGL(k_xroute_sizes, dim3(1), dim3(256), 0, s, a);
}

/* owner: partition digit s's pieces by the next bits.  IN: 0 records, 1 u32
 * counts, 2 u64 counts (kept u64 in the output) */
#ifndef HM_MG_PPT
#define HM_MG_PPT 8
#endif
#define HM_MG_TILE (256 * HM_MG_PPT)
#define HM_MG_MAXD 256
#define HM_MG_MAXR 64
template <bool SCATTER, int IN>
__global__ __launch_bounds__(256) void k_mb_gather(HmMbGather a)
{
    typedef typename std::conditional<IN == 2, unsigned long long, uint32_t>::type CT;
    __shared__ uint32_t hist[HM_MG_MAXD];
    __shared__ uint32_t toff[HM_MG_MAXD];
    __shared__ unsigned long long gb[HM_MG_MAXD];
    __shared__ unsigned long long vp[HM_MG_MAXR + 1], kp[HM_MG_MAXR], cp[HM_MG_MAXR];
    __shared__ uint32_t scr[256 / 64 + 1];
    __shared__ unsigned long long sk[SCATTER ? HM_MG_TILE : 1];
    __shared__ CT sc[SCATTER ? HM_MG_TILE : 1];
    __shared__ uint8_t sd[SCATTER ? HM_MG_TILE : 1];
    const int tid = threadIdx.x;
    const uint32_t s = blockIdx.x / a.C, c = blockIdx.x % a.C;
    const uint32_t R = a.R, nd = 1u << a.bits, dm = nd - 1u;
    if (tid <= (int)R) vp[tid] = a.vpre[(uint64_t)s * (R + 1) + tid];
    if (tid < (int)R) {
        kp[tid] = a.kp[(uint64_t)s * R + tid];
        cp[tid] = a.cp ? a.cp[(uint64_t)s * R + tid] : 0ull;
    }
    const uint64_t cbase = ((uint64_t)s << a.bits) * a.C + c;   /* + d * C */
    for (uint32_t d = tid; d < nd; d += 256) {
        hist[d] = 0;
        if (SCATTER && !a.fill) gb[d] = a.off[cbase + (uint64_t)d * a.C];
    }
    __syncthreads();
    const uint64_t len = vp[R];
    const uint64_t c0 = len * c / a.C, c1 = len * (c + 1) / a.C;
    for (uint64_t t0 = c0; t0 < c1; t0 += HM_MG_TILE) {
        const uint32_t tn = (uint32_t)min((uint64_t)HM_MG_TILE, c1 - t0);
        uint64_t k[HM_MG_PPT];
        CT cc[HM_MG_PPT];
#pragma unroll
        for (int j = 0; j < HM_MG_PPT; j++) {
            const uint32_t i = j * 256 + tid;
            k[j] = 0ull;
            cc[j] = 0;
            if (i < tn) {
                const uint64_t v = t0 + i;
                uint32_t lo = 0, hi = R;   /* the last piece starting at or before v */
                while (hi - lo > 1) {
                    const uint32_t mid = (lo + hi) >> 1;
                    if (vp[mid] <= v) lo = mid;
                    else hi = mid;
                }
                const uint64_t e = v - vp[lo];
                if (IN == 0) {
                    const uint16_t* rp = (const uint16_t*)kp[lo] + 5 * e;
                    if (v + 1 < vp[lo + 1]) {
                        uint32_t c32;
                        hm_rec_load(rp, k[j], c32);
                        cc[j] = c32;
                    } else {   /* a piece's last record: nothing read past it */
                        k[j] = hm_rec_key(rp);
                        cc[j] = hm_rec_count(rp);
                    }
                } else {
                    k[j] = ((const uint64_t*)kp[lo])[e];
                    cc[j] = IN == 1 ? (CT)((const uint32_t*)cp[lo])[e] : (CT)((const uint64_t*)cp[lo])[e];
                }
            }
        }
        if (!SCATTER) {
#pragma unroll
            for (int j = 0; j < HM_MG_PPT; j++)
                if ((uint32_t)(j * 256 + tid) < tn) atomicAdd(&hist[(uint32_t)(hms_hash(k[j]) >> a.shift) & dm], 1u);
            continue;
        }
        uint32_t d[HM_MG_PPT], r[HM_MG_PPT];
#pragma unroll
        for (int j = 0; j < HM_MG_PPT; j++) {
            const bool v = (uint32_t)(j * 256 + tid) < tn;
            d[j] = (uint32_t)(hms_hash(k[j]) >> a.shift) & dm;
            r[j] = v ? atomicAdd(&hist[d[j]], 1u) : 0u;
        }
        __syncthreads();
        uint32_t tot;
        const uint32_t o = hm_block_excl_scan<256>(tid < (int)nd ? hist[tid] : 0u, scr, &tot);
        if (tid < (int)nd) {
            toff[tid] = o;
            if (a.fill) {
                /* fill mode: this tile's run of digit tid, claimed in its bucket */
                const uint32_t h = hist[tid];
                const uint64_t bk = ((uint64_t)s << a.bits) + tid;
                const uint64_t at = h ? atomicAdd(a.fill + bk, (unsigned long long)h) : 0ull;
                if (at + h > a.bcap) {
                    atomicOr(a.over, 1ull);
                    gb[tid] = ~0ull;
                } else {
                    gb[tid] = bk * a.bcap + at;
                }
            }
        }
        __syncthreads();
#pragma unroll
        for (int j = 0; j < HM_MG_PPT; j++) {
            if ((uint32_t)(j * 256 + tid) < tn) {
                const uint32_t pos = toff[d[j]] + r[j];
                sk[pos] = k[j];
                sc[pos] = cc[j];
                sd[pos] = (uint8_t)d[j];
            }
        }
        __syncthreads();
        for (uint32_t i = tid; i < tn; i += 256) {
            const uint32_t dd = sd[i];
            if (a.fill && gb[dd] == ~0ull) continue;
            const uint64_t dst = gb[dd] + (i - toff[dd]);
            a.kout[dst] = sk[i];
            ((CT*)a.cout)[dst] = sc[i];
        }
        __syncthreads();
        if (tid < (int)nd) {
            if (!a.fill) gb[tid] += hist[tid];
            hist[tid] = 0;
        }
        __syncthreads();
    }
    if (!SCATTER) {
        __syncthreads();
        for (uint32_t d = tid; d < nd; d += 256) a.cnt[cbase + (uint64_t)d * a.C] = hist[d];
    }
}

void hm_launch_mb_gather(hipStream_t s, const HmMbGather& a, bool scatter)
{
    const unsigned g = a.S * a.C;
#define HM_MG_L(SC, IN) hipLaunchKernelGGL((k_mb_gather<SC, IN>), dim3(g), dim3(256), 0, s, a)
    if (a.in_layout == 10) {
        if (scatter) HM_MG_L(true, 0);
        else HM_MG_L(false, 0);
    } else if (a.in_layout == 8) {
        if (scatter) HM_MG_L(true, 2);
        else HM_MG_L(false, 2);
    } else {
        if (scatter) HM_MG_L(true, 1);
        else HM_MG_L(false, 1);
    }
#undef HM_MG_L
}

/* buckets of <= ~1000 cells, 256-thread blocks each looping over buckets
 * b = blockIdx, + gridDim, ... (a few blocks per CU): a 2048-slot LDS table,
 * distinct cells out in slot order (a wave's stores consecutive), one output
 * reservation per bucket.  The next bucket's cells (<= 4 a thread) are loaded
 * into registers while this one is merged, and its bounds one bucket earlier
 * still, so a block's loads overlap its LDS work.  C32: u32 input counts
 * and (TC32) u32 table counts -- 24 KB, 6 blocks a CU; a sum that carries out
 * of 32 bits sets the overflow flag (the caller's global table takes over). */
#ifndef HM_MB2_TC32
#define HM_MB2_TC32 1
#endif
#define HM_MB2_PF ((HM_MB2_TS / 2 + HM_MB2_T - 1) / HM_MB2_T)
template <bool C32>
__global__ __launch_bounds__(HM_MB2_T) void k_mb_merge2(HmMergeArgs a)
{
    constexpr bool TC32 = C32 && HM_MB2_TC32;
    typedef typename std::conditional<TC32, uint32_t, unsigned long long>::type TC;
    __shared__ unsigned long long tk[HM_MB2_TS];
    __shared__ TC tc[HM_MB2_TS];
    constexpr int SPT = HM_MB2_TS / HM_MB2_T, NW = HM_MB2_T / 64, PF = HM_MB2_PF;
    constexpr int NF = SPT * NW, FPL = (NF + 63) / 64;   /* fragments, per lane of the scan */
    __shared__ uint32_t wc[NF + 1];
    __shared__ unsigned long long sbase;
    __shared__ uint32_t full;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const uint32_t nb = 1u << a.lb, G = gridDim.x;
    auto bounds = [&](uint32_t bb, uint64_t& f0, uint64_t& f1) {
        if (a.bfill) {
            f0 = (uint64_t)bb * a.bcap;
            f1 = bb < nb ? f0 + min((uint64_t)a.bfill[bb], a.bcap) : f0;
        } else {
            f0 = bb < nb ? a.boff[(uint64_t)bb * a.nblocks] : 0ull;
            f1 = bb < nb ? a.boff[(uint64_t)(bb + 1) * a.nblocks] : 0ull;
        }
    };
    auto fetch = [&](uint64_t f0, uint64_t f1, uint64_t (&k)[PF], uint32_t (&c)[PF], uint64_t (&c64)[PF]) {
#pragma unroll
        for (int j = 0; j < PF; j++) {
            const uint64_t i = f0 + j * HM_MB2_T + tid;
            const bool v = i < f1;
            k[j] = v ? a.pkeys[i] : HMS_EMPTY;
            if (C32) c[j] = v ? a.pcounts32[i] : 0u;
            else c64[j] = v ? a.pcounts[i] : 0ull;
        }
    };
#pragma unroll
    for (int j = 0; j < SPT; j++) {
        tk[j * HM_MB2_T + tid] = HMS_EMPTY;
        tc[j * HM_MB2_T + tid] = 0;
    }
    if (tid == 0) full = 0;
    uint64_t e0, e1, n0, n1;
    bounds(blockIdx.x, e0, e1);
    bounds(blockIdx.x + G, n0, n1);
    uint64_t ck[PF], cc64[PF];
    uint32_t cc[PF];
    fetch(e0, e1, ck, cc, cc64);
    __syncthreads();
    for (uint32_t b = blockIdx.x; b < nb; b += G) {
        const uint64_t size = e1 - e0;
        const bool fast = size <= (uint64_t)PF * HM_MB2_T;
        const uint32_t P = fast ? 1u : (uint32_t)((size + HM_MB2_TS / 2 - 1) / (HM_MB2_TS / 2));
        auto insert = [&](uint64_t k, uint64_t c, uint32_t pass) {
            if (k == HMS_EMPTY) return;
            const uint64_t h = hms_hash(k);
            if (P > 1 && (uint32_t)((h >> 32) % P) != pass) return;
            uint32_t sl = (uint32_t)h & (HM_MB2_TS - 1);
            for (int probes = 0;; probes++) {
                const unsigned long long o = atomicCAS(&tk[sl], (unsigned long long)HMS_EMPTY, (unsigned long long)k);
                if (o == HMS_EMPTY || o == k) {
                    if (TC32) {
                        if (atomicAdd((uint32_t*)&tc[sl], (uint32_t)c) + (uint32_t)c < (uint32_t)c) full = 1;
                    } else {
                        atomicAdd((unsigned long long*)&tc[sl], (unsigned long long)c);
                    }
                    return;
                }
                sl = (sl + 1) & (HM_MB2_TS - 1);
                if (probes == HM_MB2_TS) {
                    full = 1;
                    return;
                }
            }
        };
        for (uint32_t pass = 0; pass < P; pass++) {
            if (fast) {
#pragma unroll
                for (int j = 0; j < PF; j++) insert(ck[j], C32 ? (uint64_t)cc[j] : cc64[j], 0);
            } else {
                for (uint64_t i0 = e0; i0 < e1; i0 += PF * HM_MB2_T) {
                    uint64_t k[PF], c64[PF];
                    uint32_t c[PF];
                    fetch(i0, min(e1, i0 + (uint64_t)PF * HM_MB2_T), k, c, c64);
#pragma unroll
                    for (int j = 0; j < PF; j++) insert(k[j], C32 ? (uint64_t)c[j] : c64[j], pass);
                }
            }
            __syncthreads();
            if (full) {
                if (tid == 0) atomicOr(a.overflow, 1ull);
                return;
            }
            uint64_t bal[SPT];
#pragma unroll
            for (int j = 0; j < SPT; j++) {
                bal[j] = __ballot(tk[j * HM_MB2_T + tid] != HMS_EMPTY);
                if (lane == 0) wc[j * NW + w] = (uint32_t)__popcll(bal[j]);
            }
            __syncthreads();
            if (w == 0) {
                /* exclusive scan of the NF fragment counts, FPL consecutive ones a lane */
                uint32_t f[FPL], v = 0;
#pragma unroll
                for (int q = 0; q < FPL; q++) {
                    f[q] = lane * FPL + q < NF ? wc[lane * FPL + q] : 0u;
                    v += f[q];
                }
                const uint32_t inc = hm_wave_incl_scan(v);
                uint32_t o = inc - v;
#pragma unroll
                for (int q = 0; q < FPL; q++) {
                    if (lane * FPL + q < NF) wc[lane * FPL + q] = o;
                    o += f[q];
                }
                if (lane == 63) sbase = inc ? atomicAdd(a.cursor, (unsigned long long)inc) : 0ull;
            }
            if (pass + 1 == P) {
                /* the next bucket: its cells now, the one after's bounds */
                e0 = n0;
                e1 = n1;
                bounds(b + 2 * G, n0, n1);
                if (e1 - e0 <= (uint64_t)PF * HM_MB2_T) fetch(e0, e1, ck, cc, cc64);
            }
            __syncthreads();
            const uint64_t base = sbase;
#pragma unroll
            for (int j = 0; j < SPT; j++) {
                const uint32_t sl = j * HM_MB2_T + tid;
                if ((bal[j] >> lane) & 1ull) {
                    const uint64_t q = base + wc[j * NW + w] + hm_mbcnt(bal[j]);
                    if (q < a.cap) {
                        a.keys_out[q] = tk[sl];
                        a.counts_out[q] = (uint64_t)tc[sl];
                    }
                    tk[sl] = HMS_EMPTY;
                    tc[sl] = 0;
                }
            }
            __syncthreads();
        }
    }
}

void hm_launch_mb_merge2(hipStream_t s, const HmMergeArgs& a)
{
    /* as many blocks as fit the CUs at once (each loops over buckets) */
    static int cus = 0, per32 = 0, per64 = 0;
    if (!cus) {
        int dev = 0;
        (void)hipGetDevice(&dev);
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) cus = 256;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per32, k_mb_merge2<true>, HM_MB2_T, 0) != hipSuccess ||
            per32 < 1)
            per32 = 1;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per64, k_mb_merge2<false>, HM_MB2_T, 0) != hipSuccess ||
            per64 < 1)
            per64 = 1;
    }
    const unsigned per = (unsigned)(a.pcounts32 ? per32 : per64);
    const dim3 g(std::min(1u << a.lb, per * (unsigned)cus)), t(HM_MB2_T);
    if (a.pcounts32) hipLaunchKernelGGL(k_mb_merge2<true>, g, t, 0, s, a);
    else hipLaunchKernelGGL(k_mb_merge2<false>, g, t, 0, s, a);
}

static unsigned hm_mgrid(uint64_t n, unsigned cap)
{
    uint64_t b = (n + 255) / 256;
    if (b > cap) b = cap;
    return (unsigned)(b ? b : 1);
}

unsigned hm_route_blocks(uint64_t n) { return hm_mgrid(n, 1024); }

void hm_launch_cells_route(hipStream_t s, const HmRouteArgs& a, bool scatter)
{
    const unsigned g = hm_route_blocks(a.n);
    if (scatter)
        hipLaunchKernelGGL(k_cells_route<true>, dim3(g), dim3(HM_ROUTE_THREADS), 0, s, a);
    else
        hipLaunchKernelGGL(k_cells_route<false>, dim3(g), dim3(HM_ROUTE_THREADS), 0, s, a);
}

void hm_launch_cells_merge_unique(hipStream_t s, const uint64_t* keys, const uint64_t* counts, uint64_t n,
                                  const HmsTable& t)
{
    if (n) hipLaunchKernelGGL(k_cells_merge_unique, dim3(hm_mgrid(n, 8192)), dim3(256), 0, s, keys, counts, n, t);
}

void hm_launch_cells_merge(hipStream_t s, const uint64_t* keys, const uint64_t* counts, uint64_t n, const HmsTable& t)
{
    if (n) hipLaunchKernelGGL(k_cells_merge<uint64_t>, dim3(hm_mgrid(n, 8192)), dim3(256), 0, s, keys, counts, n, t);
}

void hm_launch_cells_merge32(hipStream_t s, const uint64_t* keys, const uint32_t* counts, uint64_t n,
                             const HmsTable& t)
{
    if (n) hipLaunchKernelGGL(k_cells_merge<uint32_t>, dim3(hm_mgrid(n, 8192)), dim3(256), 0, s, keys, counts, n, t);
}

void hm_launch_table_extract(hipStream_t s, const HmsTable& t, uint64_t* keys_out, uint64_t* counts_out, uint64_t cap,
                             unsigned long long* cursor)
{
    const uint64_t n = t.mask + 1;
    uint64_t chunk = 16384;
    while ((n + chunk - 1) / chunk > 16384) chunk <<= 1;
    hipLaunchKernelGGL(k_table_extract, dim3((unsigned)((n + chunk - 1) / chunk)), dim3(HM_TX_THREADS), 0, s, t,
                       keys_out, counts_out, cap, cursor, chunk);
}

void hm_launch_dense_extract(hipStream_t s, const uint64_t* grid, uint64_t total, int dense_zmax, uint64_t* keys_out,
                             uint64_t* counts_out, uint64_t cap, unsigned long long* cursor)
{
    hipLaunchKernelGGL(k_dense_extract, dim3(hm_mgrid(total, 4096)), dim3(256), 0, s, grid, total, dense_zmax,
                       keys_out, counts_out, cap, cursor);
}
