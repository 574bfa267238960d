/* gfx950 kernels of the heatmap hot path.
 *
 * Path (SURVEY.md section 8a, a-1 .. a-11), one hm_count() call:
 *
 *   k_project_partition   fp64 lat/lon SoA -> tile row/col at zoom Z (exact,
 *                         hm_project.h) -> row-major key -> LDS counting sort of an
 *                         8192-point tile by the key's top digit (zoom z1
 *                         tile); writes the tile's keys (u32/u16, top digit
 *                         dropped) contiguously and one run record per
 *                         non-empty digit.  Reads 16 B/point, writes 4 B/point.
 *   k_partition           the same counting sort one level down, gathering a
 *                         parent bucket's runs (wave per run).  Levels stop at
 *                         zoom zb = Z - 7, whose buckets hold 128x128 zoom-Z
 *                         bins.
 *   k_aggregate           per zoom-zb bucket: LDS-privatised dense 128x128 u32
 *                         histogram of the u16 in-bucket keys (wave-aggregated
 *                         atomics), then an in-LDS 4:1 pyramid emitting every
 *                         non-empty cell of zooms Z .. zb+1.  Buckets larger
 *                         than one work item merge through global atomics and
 *                         k_aggregate_merged emits them.
 *   k_pool                per parent bucket: dense LDS array of its children's
 *                         totals -> 4:1 pyramid -> zooms z_l .. z_{l-1}+1; the
 *                         root emits zooms z1 .. 0.
 *   k_runscan / scans / k_compact: turn per-digit run counters into compact,
 *                         parent-major bucket lists and work-item prefixes.
 *
 * Every coarser tile is a right shift of the zoom-Z row and column, which is
 * the reference's tile-centre re-projection on the shift window (SURVEY.md
 * a-4) and the direct projection at every zoom (a-1).  Counts are integers (u32
 * per call, u64 out): the reference's float sums of 1.0 are exact below 2^53.
 */
#include <hip/hip_runtime.h>
#include "hm_genkey.h"
#include "hm_device.h"
#include "hm_project.h"
#include "hm_pipeline.h"

#ifdef HM_STAMPS
/* phase timing (profiling builds only, tools/stamps.py): thread 0 of the first
 * HM_STAMP_BLOCKS blocks of one kernel records s_memtime at up to 12 points.
 * HM_STAMPS = 1: k_partition, 2: k_project_partition, 3: k_partition_fr, 4: k_l1_fast,
 * 5: k_aggregate */
#define HM_STAMP_BLOCKS 65536
__device__ unsigned long long g_stamps[HM_STAMP_BLOCKS * 12];
#define HM_STAMP_M(m, k)                                                                       \
    do {                                                                                       \
        if (HM_STAMPS == (m) && threadIdx.x == 0 && hm_block_id() < HM_STAMP_BLOCKS)           \
            g_stamps[hm_block_id() * 12 + (k)] = __builtin_amdgcn_s_memtime();                 \
    } while (0)
#define HM_STAMP_V(m, k, v)                                                                    \
    do {                                                                                       \
        if (HM_STAMPS == (m) && threadIdx.x == 0 && hm_block_id() < HM_STAMP_BLOCKS)           \
            g_stamps[hm_block_id() * 12 + (k)] = (v);                                          \
    } while (0)
extern "C" int hm_debug_stamps(void* host, size_t bytes)
{
    return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(g_stamps), bytes, 0, hipMemcpyDeviceToHost);
}
#else
#define HM_STAMP_M(m, k) do { } while (0)
#define HM_STAMP_V(m, k, v) do { } while (0)
#endif
#define HM_STAMP(k) HM_STAMP_M(1, k)

#define HM_YTAB_N (HM_YTAB_ROWS * HM_YTAB_STRIDE)
__constant__ double c_ytab[HM_YTAB_N] = HM_YTAB_INIT;

__device__ __forceinline__ void hm_load_ytab(double* tab)
{
    for (int i = threadIdx.x; i < HM_YTAB_N; i += blockDim.x) tab[i] = c_ytab[i];
}

/* ------------------------------------------------------------------------ */
/* projection API kernel (hm_project)                                        */
/* ------------------------------------------------------------------------ */

__global__ __launch_bounds__(256) void k_project(const double* __restrict__ lat, const double* __restrict__ lon,
                                                 int64_t n, int zoom, int64_t* __restrict__ row,
                                                 int64_t* __restrict__ col, uint8_t* __restrict__ status,
                                                 unsigned long long* err_word, unsigned long long* slow_count)
{
    __shared__ double tab[HM_YTAB_N];
    hm_load_ytab(tab);
    __syncthreads();
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        int64_t r = 0, c = 0;
        int slow = 0;
        int st = hm_project_point(lat[i], lon[i], zoom, &r, &c, &slow, tab);
        if (HM_UNLIKELY(st == HM_E_RANGE)) {
            /* the row projected (its errors come first), the column is beyond
             * int64: return it exactly, as an integer-valued double */
            if (hm_row(lat[i], zoom, &r, &slow, tab) == HM_OK) {
                c = __double_as_longlong(floor((lon[i] + 180.0) / 360.0 * hm_exp2i(zoom)));
                st = HM_BIGCOL;
            }
        }
        const bool good = st == HM_OK || st == HM_BIGCOL;
        row[i] = good ? r : 0;
        col[i] = good ? c : 0;
        status[i] = (uint8_t)st;
        if (HM_UNLIKELY(!good)) atomicMin(err_word, ((unsigned long long)i << 8) | (unsigned long long)st);
        const uint64_t sm = __ballot(slow);
        if (sm && hm_lane() == __ffsll((unsigned long long)sm) - 1) atomicAdd(slow_count, (unsigned long long)__popcll(sm));
    }
}

/* wave-aggregated append to the exotic list (every lane of the wave calls) */
__device__ __forceinline__ void hm_exotic_append(const HmExotic& x, bool p, int64_t r, int64_t c, int64_t i)
{
    const uint64_t m = __ballot(p);
    if (!m) return;
    const int lead = __ffsll((unsigned long long)m) - 1;
    unsigned long long b = 0;
    if (hm_lane() == lead) b = atomicAdd(x.count, (unsigned long long)__popcll(m));
    b = __shfl(b, lead, 64);
    const uint64_t q = b + hm_mbcnt(m);
    if (p && q < x.cap) {
        x.row[q] = r;
        x.col[q] = c;
        x.idx[q] = i;
    }
}


/* a value the compiler must recompute where it is used (keeps per-lane
 * 64-bit addresses from being hoisted out of a loop and spilled) */
__device__ __forceinline__ uint32_t hm_opaque(uint32_t x)
{
    asm volatile("" : "+v"(x));
    return x;
}

/* the point stream: 16 GB per 1e9 points read once, with the non-temporal
 * hint (HM_L1_NT) so it does not push level 1's partly written key lines out
 * of L2 (each region line fills over many tiles; evicted early, it is written
 * back several times) */
#ifndef HM_L1_NT
#define HM_L1_NT 1
#endif
typedef double hm_d2v __attribute__((ext_vector_type(2)));
__device__ __forceinline__ double2 hm_stream_load2(const double2* p)
{
    if (HM_L1_NT) {
        const hm_d2v v = __builtin_nontemporal_load((const hm_d2v*)p);
        return make_double2(v.x, v.y);
    }
    return *p;
}

/* hot-tile lookup of zoom-zb tile (rs, cs) in the LDS table image: h when the
 * tile is hot, >= 2^16 otherwise (hm_pipeline.h) */
__device__ __forceinline__ uint32_t hm_hot_find(const uint2* tab, uint32_t rs, uint32_t cs)
{
    const uint2 e = tab[hm_hot_bucket(rs, cs)];
    const uint32_t tk = rs << HM_HOT_TAG;
    return min(e.x ^ tk, e.y ^ tk);
}

/* ------------------------------------------------------------------------ */
/* level 1: projection fused with the first partition                        */
/* ------------------------------------------------------------------------ */

template <typename OutT, int MODE, bool FULL>
__global__ __launch_bounds__(HM_P1_THREADS, HM_P1_WAVES) void k_project_partition(HmPart1Args a)
{
    __shared__ uint32_t cur[HM_D1 + 64];   /* + 64 dummy words (hm_lds_count) */
    /* the staged keys; until the projection is done it holds the hot-tile hash */
    __shared__ __attribute__((aligned(16))) OutT stage[HM_T1 + 64];
    /* digit of each staged key; until the count is done it holds each
     * digit's region (base, capacity << 1 | sharded) for this tile */
    __shared__ __attribute__((aligned(8))) uint16_t sdig[HM_T1 + 64];
    __shared__ unsigned long long scr[HM_P1_THREADS / 64 + 1];
    /* the projection's polynomial table; after the projection it holds, per
     * digit, (region position - stage offset) */
    __shared__ double tab[HM_YTAB_N];
    /* the hot-tile table lives in the stage and the region info in sdig when
     * they fit (8192-point tiles), else in arrays of their own */
    constexpr bool HSEP = sizeof(OutT) * HM_T1 < HM_HOT_SLOTS * 4;
    constexpr bool RSEP = sizeof(uint16_t) * HM_T1 < HM_D1 * sizeof(uint2);
    __shared__ __attribute__((aligned(16))) uint32_t hsep[HSEP ? HM_HOT_SLOTS : 4];
    __shared__ __attribute__((aligned(8))) uint2 rsep[RSEP ? HM_D1 : 1];
    static_assert(sizeof(double) * HM_YTAB_N >= HM_D1 * 4, "dbase lives in the polynomial table");
    uint4* const hsh4 = HSEP ? (uint4*)hsep : (uint4*)stage;
    uint32_t* const dbase = (uint32_t*)tab;
    uint2* const rinfo = RSEP ? rsep : (uint2*)sdig;
    constexpr bool FROM_TILES = MODE == 1;
    const int tid = threadIdx.x;
    const int F = 1 << a.dbits;
    /* hot tiles of this call (block-uniform; the count is an L2-hot word) */
    const uint32_t H = a.hot_z >= 0 ? *a.hot_n : 0u;
    const int64_t base = (a.tile0 + (int64_t)blockIdx.x) * HM_T1;   /* first input point */
    /* the resolved-redo launch is sized for the list's capacity; its length
     * is read here (no host round trip) */
    const int64_t n = (FROM_TILES && a.n_dev) ? min((int64_t)*a.n_dev, a.n) : a.n;
    if (base >= n) return;
    if (MODE == 0) HM_STAMP_M(2, 0);
    const uint32_t lim = 1u << a.Z;
    const double scale = hm_exp2i(a.Z);
    const double kz = HM_INV360 * scale;
    uint32_t dig[HM_P1_PPT];
    uint32_t rest[HM_P1_PPT];
    int nslow = 0;
    /* the polynomial table's loads go out FIRST: the barrier before the
     * projection waits for them (vmcnt retires in issue order), and must not
     * wait for the tile's 128 KB of points -- the projection then starts as
     * soon as the first points land */
    constexpr bool FULLT = FULL && !FROM_TILES;   /* a whole tile of lat/lon input */
    double2 la[HM_P1_PPT / 2], lo[HM_P1_PPT / 2];
    uint32_t kp[HM_P1_PPT / 2];   /* keep bytes of 2 points (u32: no packing, no early wait) */
    if (FULLT) {
        /* keep bytes first of all: consumed before the points */
        if (a.keep) {
            const uint16_t* kp2 = (const uint16_t*)(a.keep + base);
#pragma unroll
            for (int k = 0; k < HM_P1_PPT / 2; k++) kp[k] = kp2[k * HM_P1_THREADS + tid];
        } else {
#pragma unroll
            for (int k = 0; k < HM_P1_PPT / 2; k++) kp[k] = 0x0101;
        }
    }
    __builtin_amdgcn_sched_barrier(0);
    constexpr int TPT = (HM_YTAB_N + HM_P1_THREADS - 1) / HM_P1_THREADS;
    double tv[TPT];
    if (!FROM_TILES) {
#pragma unroll
        for (int q = 0; q < TPT; q++) {
            const int i = q * HM_P1_THREADS + tid;
            tv[q] = i < HM_YTAB_N ? c_ytab[i] : 0.0;
        }
    }
    /* this thread's digits' region slots, capacities and bases (small, L2-hot
     * tables), also before the points, and without a dependent load: a hot
     * digit's slot is d*8 + (block & 7), a cold one's d*8 (smask 7 or 0), so
     * both candidates are fetched and the mask picks one later.  (Waiting for
     * the mask before the dependent loads would wait for every point load
     * issued before it.) */
    constexpr int PERD = HM_D1 / HM_P1_THREADS;
    static_assert(HM_D1 % HM_P1_THREADS == 0, "digit slots per thread");
    /* digit slot d is live: a cold digit (d < F) or one of the H hot tiles */
    auto live = [&](int d) { return d < F || (d >= HM_MAX_F1 && (uint32_t)(d - HM_MAX_F1) < H); };
    uint32_t smk[PERD], rcap2[PERD][2], rbase2[PERD][2];
#pragma unroll
    for (int q = 0; q < PERD; q++) {
        const int d = q * HM_P1_THREADS + tid;
        const uint32_t s0 = hm_l1i(d, 0), s1 = hm_l1i(d, blockIdx.x & (HM_L1_SHARDS - 1));
        const bool lv = live(d);
        smk[q] = lv ? a.smask[d] : 0u;
        rcap2[q][0] = lv ? a.rcap[s0] : 0u;
        rcap2[q][1] = lv ? a.rcap[s1] : 0u;
        rbase2[q][0] = lv ? a.rbase[s0] : 0u;
        rbase2[q][1] = lv ? a.rbase[s1] : 0u;
    }
    /* the hot-tile table, also ahead of the points (stored to LDS below) */
    constexpr int HV = HM_HOT_SLOTS / 4 / HM_P1_THREADS;
    static_assert(HM_HOT_SLOTS == 4 * HV * HM_P1_THREADS, "the table is HV uint4 per thread");
    uint4 hv[HV];
#pragma unroll
    for (int j = 0; j < HV; j++) hv[j] = H ? ((const uint4*)a.hot_hash)[j * HM_P1_THREADS + tid] : make_uint4(0u, 0u, 0u, 0u);
    __builtin_amdgcn_sched_barrier(0);
    /* issue every load of the tile before any arithmetic: 16 points x 16 B per
     * lane in flight (double2 = two consecutive points of one array).  Full
     * tiles are a launch of their own (FULL): straight-line loads, so the
     * table's wait below counts exactly the loads issued after it; the tail
     * tile's per-lane code would make the compiler drain everything there. */
    if (FULLT) {
        const double2* lat2 = (const double2*)(a.lat + base);
        const double2* lon2 = (const double2*)(a.lon + base);
#pragma unroll
        for (int k = 0; k < HM_P1_PPT / 2; k++) {
            la[k] = lat2[k * HM_P1_THREADS + tid];
            lo[k] = lon2[k * HM_P1_THREADS + tid];
        }
    } else
#pragma unroll
    for (int k = 0; k < HM_P1_PPT / 2; k++) {
        const int64_t i0 = base + 2 * ((int64_t)k * HM_P1_THREADS + tid);
        kp[k] = 0x0101;
        if (i0 + 1 < n) {
            if (FROM_TILES) {
                la[k].x = __longlong_as_double(a.rows_in[i0]);
                la[k].y = __longlong_as_double(a.rows_in[i0 + 1]);
                lo[k].x = __longlong_as_double(a.cols_in[i0]);
                lo[k].y = __longlong_as_double(a.cols_in[i0 + 1]);
            } else {
                la[k] = *(const double2*)(a.lat + i0);
                lo[k] = *(const double2*)(a.lon + i0);
            }
            if (a.keep) kp[k] = (uint16_t)a.keep[i0] | ((uint16_t)a.keep[i0 + 1] << 8);
        } else if (i0 < n) {
            if (FROM_TILES) {
                la[k].x = __longlong_as_double(a.rows_in[i0]);
                lo[k].x = __longlong_as_double(a.cols_in[i0]);
            } else {
                la[k].x = a.lat[i0];
                lo[k].x = a.lon[i0];
            }
            la[k].y = 0.0;
            lo[k].y = 0.0;
            if (a.keep) kp[k] = (uint16_t)a.keep[i0];
        } else {
            la[k] = make_double2(0.0, 0.0);
            lo[k] = make_double2(0.0, 0.0);
        }
    }
    /* LDS set-up after the loads are issued */
    for (int i = tid; i < HM_D1; i += HM_P1_THREADS) cur[i] = 0;
    /* this tile's region of each digit: the registers are free again for
     * the projection, the count reads it back */
#pragma unroll
    for (int q = 0; q < PERD; q++) {
        const int d = q * HM_P1_THREADS + tid;
        const uint32_t sh = smk[q] != 0;
        rinfo[d] = make_uint2(sh ? rbase2[q][1] : rbase2[q][0], ((sh ? rcap2[q][1] : rcap2[q][0]) << 1) | sh);
    }
    if (H) {
#pragma unroll
        for (int j = 0; j < HV; j++) hsh4[j * HM_P1_THREADS + tid] = hv[j];
    }
    if (!FROM_TILES) {
#pragma unroll
        for (int q = 0; q < TPT; q++) {
            const int i = q * HM_P1_THREADS + tid;
            if (i < HM_YTAB_N) tab[i] = tv[q];
        }
    }
    __syncthreads();
    if (MODE == 0) HM_STAMP_M(2, 1);
    /* fast path for every point, branch-free; points the fast path cannot
     * settle (guard band, polar/out-of-range/non-finite input) are marked in
     * `redo` and resolved afterwards in one ballot-guarded pass */
    const int hb = a.restbits >> 1;      /* offset bits per coordinate in rest */
    const int wd = a.dbits >> 1;         /* digit bits per coordinate */
    const uint32_t lowm = (1u << hb) - 1u;
    const int hs = a.Z - a.hot_z;        /* hot keys: offset bits per coordinate */
    const uint32_t hm = (1u << hs) - 1u;
    /* a tile's digit slot (the skewed LDS slot of its digit, hm_cur_slot: one
     * bijection used for every digit table of the block) and key.  A point in
     * a hot tile (one 16-B read of its table bucket: the entry's tile bits
     * cancel in the XOR, so the minimum is h exactly when the tile is there)
     * takes digit HM_MAX_F1 + h and its zoom-Z offset inside the tile. */
    const uint32_t wm = (1u << wd) - 1u;
    auto key_of = [&](uint32_t r, uint32_t c, bool v, uint32_t& dslot, uint32_t& key) {
        const uint32_t rd = r >> hb, cd = c >> hb;
        /* = hm_dslot(rd << wd | cd): the column digit rotated by 8 rows */
        uint32_t dg = (rd << wd) | (HM_SKEW_CUR ? ((cd + (rd << 3)) & wm) : cd);
        key = ((r & lowm) << hb) | (c & lowm);
        if (H) {   /* block-uniform */
            const uint32_t x = hm_hot_find((const uint2*)hsh4, r >> hs, c >> hs);
            const bool hot = x < (uint32_t)HM_HOT_LIMIT;   /* a miss leaves x >= 2^16 */
            dg = hot ? HM_MAX_F1 + x : dg;
            key = hot ? (((r & hm) << hs) | (c & hm)) : key;
        }
        dslot = v ? dg : 0xFFFFFFFFu;
    };
    uint32_t redo = 0;
#pragma unroll
    for (int k = 0; k < HM_P1_PPT; k++) {
        const int64_t i = base + 2 * ((int64_t)(k >> 1) * HM_P1_THREADS + tid) + (k & 1);
        const double pa = (k & 1) ? la[k >> 1].y : la[k >> 1].x;
        const double po = (k & 1) ? lo[k >> 1].y : lo[k >> 1].x;
        int64_t r, c;
        int ok;
        bool dom;
        if (FROM_TILES) {
            r = __double_as_longlong(pa);
            c = __double_as_longlong(po);
            ok = 1;
            dom = ((uint64_t)r < lim) & ((uint64_t)c < lim);
        } else {
            int32_t r32, c32;
            ok = hm_project_fast(pa, po, scale, kz, &r32, &c32, tab);
            r = r32;
            c = c32;
            dom = true;   /* ok implies 0 <= r32, c32 < 2^Z (hm_project_fast) */
        }
        const bool inb = FULLT || i < n;   /* a whole tile is in range */
        const bool kept = ((kp[k >> 1] >> (8 * (k & 1))) & 0xFF) != 0;
        redo |= (uint32_t)(inb & !(ok & dom)) << k;
        const bool v = inb & ok & dom & kept;
        key_of((uint32_t)r, (uint32_t)c, v, dig[k], rest[k]);
        /* pin the key: without it the compiler keeps every point's
         * projection temporaries alive past this point (158 VGPRs, 1 block/CU) */
        asm volatile("" : "+v"(dig[k]), "+v"(rest[k]));
        /* one point at a time: interleaving all eight projections would need
         * ~200 VGPRs and halve occupancy */
        if ((k % HM_P1_ILP) == HM_P1_ILP - 1) __builtin_amdgcn_sched_barrier(0);
    }
    if (MODE == 0) HM_STAMP_M(2, 2);
    if (MODE == 0) {
        /* defer: k_redo resolves these with the exact chain and feeds them
         * back as extra tiles (keeps the exact path out of this kernel's
         * register allocation) */
        if (__ballot(redo != 0))
#pragma unroll
        for (int k = 0; k < HM_P1_PPT; k++) {
            const bool rd = (redo >> k) & 1u;
            const uint64_t m = __ballot(rd);
            if (m) {
                uint64_t b = 0;
                if (hm_lane() == __ffsll((unsigned long long)m) - 1) b = atomicAdd(a.redo_count, (unsigned long long)__popcll(m));
                b = __shfl(b, __ffsll((unsigned long long)m) - 1, 64);
                const uint64_t q = b + hm_mbcnt(m);
                if (rd && q < a.redo_cap)
                    a.redo_idx[q] = (uint32_t)(base + 2 * ((int64_t)(k >> 1) * HM_P1_THREADS + tid) + (k & 1));
            }
        }
        nslow = __popc(redo);
    } else if (__ballot(redo != 0)) {
        /* every lane runs each step (the exotic append is a wave operation) */
#pragma unroll
        for (int k = 0; k < HM_P1_PPT; k++) {
            const bool rd = (redo >> k) & 1u;
            const int64_t i = base + 2 * ((int64_t)(k >> 1) * HM_P1_THREADS + tid) + (k & 1);
            int64_t r = 0, c = 0;
            int st = HM_OK;
            if (rd) {
                const double pa = (k & 1) ? la[k >> 1].y : la[k >> 1].x;
                const double po = (k & 1) ? lo[k >> 1].y : lo[k >> 1].x;
                if (FROM_TILES) {
                    r = __double_as_longlong(pa);
                    c = __double_as_longlong(po);
                } else {
                    /* the literal reference chain (tile.py:17,21), row before column */
                    st = hm_row_exact(pa, a.Z, &r);
                    if (st == HM_OK) st = hm_col_exact(po, a.Z, &c);
                    nslow++;
                }
            }
            const bool kept = ((kp[k >> 1] >> (8 * (k & 1))) & 0xFF) != 0;
            if (rd && st != HM_OK) atomicMin(a.err_word, ((unsigned long long)i << 8) | (unsigned long long)st);
            const bool good = rd & (st == HM_OK) & kept;
            const bool outside = good & (((uint64_t)r >= lim) | ((uint64_t)c >= lim));
            hm_exotic_append(a.x, outside, r, c, i);
            if (good & !outside) key_of((uint32_t)r, (uint32_t)c, true, dig[k], rest[k]);
        }
    }
    if (!FROM_TILES) {
        const uint32_t ws = hm_wave_sum((uint32_t)nslow);
        if (hm_lane() == 0 && ws) atomicAdd(a.slow_count, (unsigned long long)ws);
    }
    /* one returning atomic per point: the digit histogram and the point's
     * rank within its digit (its slot is the digit's offset + rank) */
    const uint32_t dummy = HM_D1 + (uint32_t)hm_lane();
    uint32_t rank[HM_P1_PPT];
#pragma unroll
    for (int k0 = 0; k0 < HM_P1_PPT; k0 += HM_P1_GROUP) {
        HmClaim gm[HM_P1_GROUP];
        uint32_t old[HM_P1_GROUP];
#pragma unroll
        for (int u = 0; u < HM_P1_GROUP; u++) {
            gm[u] = hm_claim_prep(dig[k0 + u], dig[k0 + u] != 0xFFFFFFFFu, dummy);
            old[u] = atomicAdd(&cur[gm[u].idx], gm[u].inc);
        }
#pragma unroll
        for (int u = 0; u < HM_P1_GROUP; u++) rank[k0 + u] = hm_claim_pos(gm[u], old[u]);
    }
    __syncthreads();
    if (MODE == 0) HM_STAMP_M(2, 3);
    /* reserve each digit's keys in its region (one returning atomic per
     * non-empty digit), issued as soon as the histogram is known; the results
     * are consumed only after the scan and the claim below, so the atomic
     * latency hides behind LDS work */
    constexpr int PER = PERD;
    uint32_t cnt[PER];
    uint32_t gpos[PER];
    uint32_t rcap[PER], rbase[PER], dsl[PER];
    /* thread t holds digits q * T + t: a wave's lanes reserve for
     * consecutive digits (coalesced atomics on the shard-major fill words) */
    uint32_t tsum = 0;
#pragma unroll
    for (int q = 0; q < PER; q++) {
        const int d = q * HM_P1_THREADS + tid;
        const uint2 ri = rinfo[d];
        rbase[q] = ri.x;
        rcap[q] = ri.y >> 1;
        dsl[q] = hm_dslot(d, wd);
        const uint32_t slot = hm_l1i(d, (ri.y & 1u) ? (blockIdx.x & (HM_L1_SHARDS - 1)) : 0u);
        cnt[q] = live(d) ? cur[dsl[q]] : 0u;
        gpos[q] = 0;
        if (cnt[q]) gpos[q] = atomicAdd(&a.fill[slot], cnt[q]);
        tsum += cnt[q];
    }
    /* stage ranges in thread order (a thread's digits q = 0.. adjacent): one
     * 32-bit block scan.  Any disjoint ranges do: the copy-out finds each
     * staged key's region through its digit slot */
    uint32_t total;
    uint32_t offq[PER];
    offq[0] = hm_block_excl_scan<HM_P1_THREADS>(tsum, (uint32_t*)scr, &total);
#pragma unroll
    for (int q = 1; q < PER; q++) offq[q] = offq[q - 1] + cnt[q - 1];
#pragma unroll
    for (int q = 0; q < PER; q++) {
        const int d = q * HM_P1_THREADS + tid;
        if (live(d)) cur[dsl[q]] = offq[q];
    }
    __syncthreads();
    if (MODE == 0) HM_STAMP_M(2, 4);
#pragma unroll
    for (int k = 0; k < HM_P1_PPT; k++) {
        const bool v = dig[k] != 0xFFFFFFFFu;
        const uint32_t pos = v ? cur[v ? dig[k] : 0u] + rank[k] : HM_T1 + hm_lane();
        stage[pos] = (OutT)rest[k];
        sdig[pos] = (uint16_t)dig[k];
    }
    /* lane-parallel copy-out: staged key i of digit slot s goes to region
     * position dbase[s] + i (= rbase + gpos + i - offset of its digit), so a
     * wave stores 64 consecutive staged keys (one or a few digits' runs).  A
     * reservation past the region's capacity is dropped and flagged (the host
     * re-runs the level with exact sizes). */
    bool over = false;
#pragma unroll
    for (int q = 0; q < PER; q++) {
        const int d = q * HM_P1_THREADS + tid;
        if (live(d)) {
            const bool fits = cnt[q] && (uint64_t)gpos[q] + cnt[q] <= (uint64_t)rcap[q];
            over |= cnt[q] && !fits;
            dbase[dsl[q]] = fits ? rbase[q] + gpos[q] - offq[q] : 0xFFFFFFFFu;
        }
    }
    if (MODE == 0) HM_STAMP_M(2, 5);
    if (over) atomicOr(a.overflow, 1ull);
    __syncthreads();
    if (MODE == 0) HM_STAMP_M(2, 6);
    {
        /* every LDS read first (a thread copies <= HM_P1_PPT staged keys),
         * then the stores: no load-use round trip per key */
        OutT* out = (OutT*)a.keys_out;
        uint16_t* hout = (uint16_t*)a.keys_hot;
        uint32_t* hout32 = (uint32_t*)a.keys_hot;   /* mid-level hot tiles (a.hot_bytes 4) */
        uint32_t sv[HM_P1_PPT], sl[HM_P1_PPT], sb[HM_P1_PPT];
#pragma unroll
        for (int j = 0; j < HM_P1_PPT; j++) {
            const uint32_t i = j * HM_P1_THREADS + tid;
            const uint32_t ic = i < total ? i : 0u;
            sl[j] = sdig[ic];
            sv[j] = (uint32_t)stage[ic];
        }
#pragma unroll
        for (int j = 0; j < HM_P1_PPT; j++) sb[j] = dbase[sl[j]];
#pragma unroll
        for (int j = 0; j < HM_P1_PPT; j++) {
            const uint32_t i = j * HM_P1_THREADS + tid;
            if (i < total && sb[j] != 0xFFFFFFFFu) {
                if (sl[j] < HM_MAX_F1)
                    out[sb[j] + i] = (OutT)sv[j];
                else if (a.hot_bytes == 4)
                    hout32[sb[j] + i] = sv[j];
                else
                    hout[sb[j] + i] = (uint16_t)sv[j];
            }
        }
    }
    if (MODE == 0) HM_STAMP_M(2, 7);
}

/* ------------------------------------------------------------------------ */
/* level 1, whole lat/lon tiles (the hot launch of every hm_count call)      */
/* ------------------------------------------------------------------------ */
/* k_l1_fast: the same level-1 pass as k_project_partition<OutT, 0, true> --
 * the same regions, reservations, keys and deferred points -- with the
 * per-point instruction budget cut (round 4):
 *
 *  projection  v_fract_f64 gives each coordinate's fraction in one op and the
 *              floor is a truncating convert (both coordinates are positive on
 *              the accepted range); the column is one fma (lon * kz + 180 kz,
 *              inside the same 2^-49 guard); the column range test is
 *              |lon| < 180 on the input (an accepted y lies in [0, 2^z));
 *  hot lookup  row-tagged 2-way buckets (hm_hot_find): the tile's row and
 *              column are shifts of the point's, no tile id is built, and the
 *              digit is ONE min3 over (way 0, way 1, cold slot) because hot
 *              tiles take the LOW slots [0, HM_MAX_HOT) of this kernel's
 *              numbering and cold digits the slots above;
 *  count+rank  one plain returning LDS atomic per point; lanes are grouped on
 *              lane 0's slot only when a wave-uniform test finds >=
 *              HM_L1_MERGE_MIN of them (skewed clouds), so a hotspot wave pays
 *              two VALU ops per point for the test;
 *  staging     each staged entry is (key, destination position): the copy-out
 *              reads one 8-B LDS word per key and needs no per-digit lookup;
 *              the stage holds the cold keys first and the hot keys after them
 *              (one packed 16|16-bit block scan), so the copy-out's two store
 *              kinds are wave-uniform; hot keys are staged in the cold layout
 *              and narrowed to their zb-relative u16 form in the copy-out.
 *
 * Internal slot s: hot tile h -> s = h; cold z1 digit d -> s = HM_MAX_HOT +
 * hm_dslot(d) (the bank-skewed slot).  Thread t owns slots q * T + t. */
#ifndef HM_L1_MERGE_MIN
#define HM_L1_MERGE_MIN 6
#endif
#define HM_L1_SLOTS (HM_MAX_HOT + HM_MAX_F1)
#define HM_L1_CW 1600                       /* slot words (>= HM_L1_SLOTS + 64 dummies), a multiple of 64 */
static_assert(HM_L1_CW >= HM_L1_SLOTS + 64 && HM_L1_CW % 64 == 0, "count and delta words pair as read2st64");
static_assert(HM_L1_SLOTS % HM_P1_THREADS == 0, "slots per thread");

#ifndef HM_L1_FAST
#define HM_L1_FAST 1                        /* 0: k_project_partition, 1: k_l1_fast */
#endif
#ifndef HM_L1_LATE_DEST
#define HM_L1_LATE_DEST 1                   /* destinations resolved after the staging (see the staging) */
#endif
#ifndef HM_L1_WAVES
#define HM_L1_WAVES 4                       /* k_l1_fast: waves per SIMD its registers allow (4: 2 blocks of 8 waves per CU) */
#endif
template <typename OutT, bool KEEP>
__global__ __launch_bounds__(HM_P1_THREADS) __attribute__((amdgpu_waves_per_eu(HM_L1_WAVES, HM_L1_WAVES))) void
k_l1_fast(HmPart1Args a)
{
    /* staged (key, destination), + one pad entry per lane for points that
     * stage nothing; during the projection its first 32 KB hold the
     * polynomial table and the hot-tile table */
    __shared__ __attribute__((aligned(16))) uint2 ent[HM_T1 + 64];
    /* per slot: count (atomics) then stage offset in [0, CW); destination minus
     * stage position in [CW, 2 CW) -- one ds_read2st64_b32 reads both */
    __shared__ uint32_t cw[2 * HM_L1_CW];
    __shared__ uint32_t scr[HM_P1_THREADS / 64 + 1];
    __shared__ uint32_t s_over;
    /* the polynomial table plus one poison row (HM_YTAB_ROWS, NaN
     * coefficients) that the clamped index of |lat| > 90, NaN and inf lands
     * on.  Points with 85.05 < |lat| <= 90 are rejected by the latitude test
     * (an accepted point has Y in (0, 1), 0 < R < 2^Z).  (Poisoning the table
     * down to |lat| > 85 instead saves that test but sends 0.06% of a uniform
     * cloud to the exact path: 46x the deferred points, on one counter.) */
    constexpr int YROWS = HM_YTAB_ROWS + 1;
    constexpr int YN = YROWS * HM_YTAB_STRIDE;
    static_assert(sizeof(double) * YN <= 16384 && HM_HOT_SLOTS * 4 <= 16384, "tables fit the stage");
    double* const tab = (double*)ent;
    uint2* const hot2 = (uint2*)((char*)ent + 16384);
    const int tid = threadIdx.x;
    const int F = 1 << a.dbits;
    const uint32_t H = a.hot_z >= 0 ? *a.hot_n : 0u;
    const int64_t base = (a.tile0 + (int64_t)blockIdx.x) * HM_T1;
    HM_STAMP_M(4, 0);
    const double scale = hm_exp2i(a.Z);
    const double nscale = -scale, hscale = 0.5 * scale;
    const double kz = HM_INV360 * scale;
    const double c180 = 180.0 * kz;
    const double ghalf = 0.5 - HM_Y_EPS * scale;       /* row: |frac - 1/2| < ghalf */
    const double ghalf2 = 0.5 - scale * 0x1p-49;       /* column */
    constexpr int PERD = HM_L1_SLOTS / HM_P1_THREADS;
    const int wd = a.dbits >> 1;
    /* slot -> digit (hot slot h: digit HM_MAX_F1 + h; cold slot: unskewed) */
    auto digit_of = [&](uint32_t sl) -> uint32_t {
        if (sl < HM_MAX_HOT) return HM_MAX_F1 + sl;
        const uint32_t u = sl - HM_MAX_HOT, m = (1u << wd) - 1u;
        return HM_SKEW_CUR ? ((u & ~m) | ((u - ((u >> wd) << 3)) & m)) : u;
    };
    auto live = [&](uint32_t sl) {
        return sl < HM_MAX_HOT ? sl < H : (sl - HM_MAX_HOT) < (uint32_t)F;
    };
    /* keep bytes, then the tables, then the points (vmcnt retires in order) */
    uint32_t kp[HM_P1_PPT / 2];   /* KEEP: the keep bytes (a keep-less call compiles the test away) */
    if (KEEP) {
        const uint16_t* kp2 = (const uint16_t*)(a.keep + base);
#pragma unroll
        for (int k = 0; k < HM_P1_PPT / 2; k++) kp[k] = kp2[k * HM_P1_THREADS + tid];
    } else {
#pragma unroll
        for (int k = 0; k < HM_P1_PPT / 2; k++) kp[k] = 0x0101;
    }
    __builtin_amdgcn_sched_barrier(0);
    constexpr int TPT = (YN + HM_P1_THREADS - 1) / HM_P1_THREADS;
    double tv[TPT];
#pragma unroll
    for (int q = 0; q < TPT; q++) {
        const int i = q * HM_P1_THREADS + tid;
        tv[q] = i >= HM_YTAB_N ? __builtin_nan("") : c_ytab[i];
    }
    uint32_t smk[PERD], rcap2[PERD][2], rbase2[PERD][2];
#pragma unroll
    for (int q = 0; q < PERD; q++) {
        const uint32_t sl = q * HM_P1_THREADS + tid;
        const uint32_t d = digit_of(sl);
        const uint32_t s0 = hm_l1i(d, 0), s1 = hm_l1i(d, blockIdx.x & (HM_L1_SHARDS - 1));
        const bool lv = live(sl);
        smk[q] = lv ? a.smask[d] : 0u;
        rcap2[q][0] = lv ? a.rcap[s0] : 0u;
        rcap2[q][1] = lv ? a.rcap[s1] : 0u;
        rbase2[q][0] = lv ? a.rbase[s0] : 0u;
        rbase2[q][1] = lv ? a.rbase[s1] : 0u;
    }
    constexpr int HV = HM_HOT_SLOTS / 4 / HM_P1_THREADS;
    uint4 hv[HV];
#pragma unroll
    for (int j = 0; j < HV; j++) hv[j] = H ? ((const uint4*)a.hot_hash)[j * HM_P1_THREADS + tid] : make_uint4(0u, 0u, 0u, 0u);
    __builtin_amdgcn_sched_barrier(0);
    double2 la[HM_P1_PPT / 2], lo[HM_P1_PPT / 2];
    {
        const double2* lat2 = (const double2*)(a.lat + base);
        const double2* lon2 = (const double2*)(a.lon + base);
#pragma unroll
        for (int k = 0; k < HM_P1_PPT / 2; k++) {
            la[k] = hm_stream_load2(lat2 + k * HM_P1_THREADS + tid);
            lo[k] = hm_stream_load2(lon2 + k * HM_P1_THREADS + tid);
        }
    }
    for (int i = tid; i < HM_L1_CW; i += HM_P1_THREADS) cw[i] = 0;
    if (tid == 0) s_over = 0;
    if (H) {
#pragma unroll
        for (int j = 0; j < HV; j++) ((uint4*)hot2)[j * HM_P1_THREADS + tid] = hv[j];
    }
#pragma unroll
    for (int q = 0; q < TPT; q++) {
        const int i = q * HM_P1_THREADS + tid;
        if (i < YN) tab[i] = tv[q];
    }
    hm_lds_barrier();
    HM_STAMP_M(4, 1);
    const int hb = a.restbits >> 1;
    const uint32_t lowm = (1u << hb) - 1u;
    const uint32_t keym = (uint32_t)((1ull << (2 * hb)) - 1ull);
    const uint32_t wm = (1u << wd) - 1u;
    const int hs = a.hot_z >= 0 ? a.Z - a.hot_z : 0;
    const uint32_t dummy = HM_L1_SLOTS + (uint32_t)hm_lane();
    uint32_t slot[HM_P1_PPT], key[HM_P1_PPT];
    uint32_t redo = 0;
#pragma unroll
    for (int k = 0; k < HM_P1_PPT; k++) {
        const double pa = (k & 1) ? la[k >> 1].y : la[k >> 1].x;
        const double po = (k & 1) ? lo[k >> 1].y : lo[k >> 1].x;
        /* row: Y = 1/2 - sign(lat) g(90 - |lat|) (hm_fast_g), R = Y 2^Z */
        const double dd = 90.0 - fabs(pa);
        const uint32_t dh = (uint32_t)(hm_d2u(dd) >> 32);
        constexpr uint32_t I0 = (1023u + HM_YTAB_E0) << HM_YTAB_K;
        const uint32_t ii = min((dh >> (20 - HM_YTAB_K)) - I0, (uint32_t)HM_YTAB_ROWS);   /* wraps below d = 4 */
        const double dlo = hm_u2d((uint64_t)(dh & ~((1u << (20 - HM_YTAB_K)) - 1u)) << 32);
        const double t = dd - dlo;
        const double* cf = tab + ii * HM_YTAB_STRIDE;
        double p = cf[5];
        p = fma(p, t, cf[4]);
        p = fma(p, t, cf[3]);
        p = fma(p, t, cf[2]);
        p = fma(p, t, cf[1]);
        p = fma(p, t, cf[0]);
        const double R = fma(copysign(p, pa), nscale, hscale);
        const double fr = __builtin_amdgcn_fract(R);
        /* column: y = (lon + 180) / 360 * 2^z within 2^(z-51.3); guard 2^(z-49) */
        const double y = fma(po, kz, c180);
        const double fc = __builtin_amdgcn_fract(y);
        /* |lat| <= HM_LAT_SQ as dd >= 90 - HM_LAT_SQ: both differences are
         * exact for |lat| in [45, 180] (Sterbenz), dd >= 45 below, NaN fails */
        const bool ok = (int)(dd >= 90.0 - HM_LAT_SQ) & (int)(fabs(fr - 0.5) < ghalf) & (int)(fabs(po) < 180.0) &
                        (int)(fabs(fc - 0.5) < ghalf2);
        const uint32_t r = (uint32_t)(int32_t)R;   /* truncation = floor: R, y > 0 when ok */
        const uint32_t c = (uint32_t)(int32_t)y;
        const bool kept = ((kp[k >> 1] >> (8 * (k & 1))) & 0xFFu) != 0;
        redo |= (uint32_t)!ok << k;
        /* cold slot: bank-skewed z1 digit above the hot slots */
        const uint32_t rd = r >> hb, cd = c >> hb;
        const uint32_t rdw = (rd << wd) + HM_MAX_HOT;
        uint32_t sl = HM_SKEW_CUR ? (((cd + (rd << 3)) & wm) | rdw) : (cd | rdw);
        if (H) sl = min(hm_hot_find(hot2, r >> hs, c >> hs), sl);   /* block-uniform */
        key[k] = ((r << hb) | (c & lowm)) & keym;
        slot[k] = (ok & kept) ? sl : dummy;
        asm volatile("" : "+v"(slot[k]), "+v"(key[k]));
        __builtin_amdgcn_sched_barrier(0);
    }
    HM_STAMP_M(4, 2);
    /* deferred points: k_redo resolves them exactly */
    if (__builtin_amdgcn_ballot_w64(redo != 0)) {
#pragma unroll
        for (int k = 0; k < HM_P1_PPT; k++) {
            const bool rd = (redo >> k) & 1u;
            const uint64_t m = __builtin_amdgcn_ballot_w64(rd);
            if (m) {
                uint64_t b = 0;
                if (hm_lane() == __ffsll((unsigned long long)m) - 1) b = atomicAdd(a.redo_count, (unsigned long long)__popcll(m));
                b = __shfl(b, __ffsll((unsigned long long)m) - 1, 64);
                const uint64_t q = b + hm_mbcnt(m);
                if (rd && q < a.redo_cap)
                    a.redo_idx[q] = (uint32_t)(base + 2 * ((int64_t)(k >> 1) * HM_P1_THREADS + tid) + (k & 1));
            }
        }
        const uint32_t ws = hm_wave_sum((uint32_t)__popc(redo));
        if (hm_lane() == 0 && ws) atomicAdd(a.slow_count, (unsigned long long)ws);
    }
    /* count + rank: one returning atomic per point; a wave whose lanes mostly
     * share lane 0's slot adds for them once (lane 0 adds the group size, the
     * rest of the group hits private dummy words) */
    uint32_t rank[HM_P1_PPT];
    uint32_t merged = 0;   /* wave-uniform: points whose atomic was grouped */
#pragma unroll
    for (int k = 0; k < HM_P1_PPT; k++) {
        const uint32_t k0 = __builtin_amdgcn_readfirstlane(slot[k]);
        const uint64_t m = __builtin_amdgcn_ballot_w64(slot[k] == k0);
        const uint32_t pm = (uint32_t)__builtin_popcount((uint32_t)m) + (uint32_t)__builtin_popcount((uint32_t)(m >> 32));
        uint32_t idx = slot[k], inc = 1u;
        if (pm >= HM_L1_MERGE_MIN) {
            merged |= 1u << k;
            const bool in = (m >> hm_lane()) & 1ull;
            idx = (in && hm_lane() != 0) ? dummy : idx;
            inc = hm_lane() == 0 ? pm : inc;
        }
        rank[k] = atomicAdd(&cw[idx], inc);
    }
    if (merged) {
#pragma unroll
        for (int k = 0; k < HM_P1_PPT; k++)
            if ((merged >> k) & 1u) {
                const uint32_t k0 = __builtin_amdgcn_readfirstlane(slot[k]);
                const uint64_t m = __builtin_amdgcn_ballot_w64(slot[k] == k0);
                const uint32_t r0 = __builtin_amdgcn_readfirstlane(rank[k]);
                if ((m >> hm_lane()) & 1ull) rank[k] = r0 + hm_mbcnt(m);
            }
    }
    hm_lds_barrier();
    HM_STAMP_M(4, 3);
    /* reservations: one returning global atomic per non-empty (digit, shard) */
    uint32_t cnt[PERD], gpos[PERD];
#pragma unroll
    for (int q = 0; q < PERD; q++) {
        const uint32_t sl = q * HM_P1_THREADS + tid;
        const uint32_t d = digit_of(sl);
        const uint32_t sh = smk[q] != 0 ? (blockIdx.x & (HM_L1_SHARDS - 1)) : 0u;
        cnt[q] = live(sl) ? cw[sl] : 0u;
        gpos[q] = 0;
        if (cnt[q]) gpos[q] = atomicAdd(&a.fill[hm_l1i(d, sh)], cnt[q]);
    }
    /* stage offsets: cold slots (q >= QH) first, hot slots (q < QH) after
     * them, from one scan of (cold count | hot count << 16) */
    constexpr int QH = HM_MAX_HOT / HM_P1_THREADS;
    static_assert(HM_MAX_HOT % HM_P1_THREADS == 0 && QH >= 1 && QH < PERD, "slots q < QH are the hot tiles");
    uint32_t csum = 0, hsum = 0;
#pragma unroll
    for (int q = 0; q < PERD; q++) (q < QH ? hsum : csum) += cnt[q];
    uint32_t tot2;
    const uint32_t pre = hm_block_excl_scan<HM_P1_THREADS, true>(csum | (hsum << 16), scr, &tot2);
    const uint32_t C = tot2 & 0xFFFFu, total = C + (tot2 >> 16);
    uint32_t offq[PERD];
    {
        uint32_t oc = pre & 0xFFFFu, oh = C + (pre >> 16);
#pragma unroll
        for (int q = 0; q < PERD; q++) {
            offq[q] = q < QH ? oh : oc;
            (q < QH ? oh : oc) += cnt[q];
        }
    }
    bool over = false;
    /* a slot's destination delta: its region base + reservation - stage
     * offset; a region that overflowed: destinations >= 0xFFF00000 (no key
     * position reaches it), dropped by the copy-out */
    auto deltas = [&]() {
#pragma unroll
        for (int q = 0; q < PERD; q++) {
            const uint32_t sl = q * HM_P1_THREADS + tid;
            if (live(sl)) {
                const uint32_t rc = smk[q] != 0 ? rcap2[q][1] : rcap2[q][0];
                const uint32_t rb = smk[q] != 0 ? rbase2[q][1] : rbase2[q][0];
                const bool fits = (uint64_t)gpos[q] + cnt[q] <= (uint64_t)rc;
                over |= cnt[q] && !fits;
                cw[HM_L1_CW + sl] = (fits ? rb + gpos[q] : 0xFFF00000u) - offq[q];
            }
        }
        if (over) {
            atomicOr(a.overflow, 1ull);
            s_over = 1;
        }
    };
#pragma unroll
    for (int q = 0; q < PERD; q++) {
        const uint32_t sl = q * HM_P1_THREADS + tid;
        if (live(sl)) cw[sl] = offq[q];
    }
    if (!HM_L1_LATE_DEST) deltas();
    hm_lds_barrier();
    HM_STAMP_M(4, 4);
    /* staging, branch-free: a point that stages nothing writes its lane's pad
     * entry.  HM_L1_LATE_DEST: the entry holds its slot, and the destination
     * deltas are written after the staging, so the reservation atomics'
     * round trip overlaps it (the copy-out looks the delta up per key) */
#pragma unroll
    for (int k = 0; k < HM_P1_PPT; k++) {
        const uint32_t o = cw[slot[k]];   /* (dummies: in range, unused) */
        const uint32_t pos = slot[k] < HM_L1_SLOTS ? o + rank[k] : HM_T1 + (uint32_t)hm_lane();
        if (HM_L1_LATE_DEST) {
            ent[pos] = make_uint2(key[k], slot[k]);
        } else {
            const uint32_t dl = cw[HM_L1_CW + slot[k]];
            ent[pos] = make_uint2(key[k], dl + pos);
        }
    }
    if (HM_L1_LATE_DEST) deltas();
    hm_lds_barrier();
    HM_STAMP_M(4, 5);
    /* copy-out: a wave stores 64 consecutive staged keys -- cold keys in [0, C)
     * as OutT, hot keys in [C, total) as u16 (zb-relative); the kind tests
     * are wave-uniform except in the one wave straddling C or total */
    char* const outb = (char*)a.keys_out;
    char* const houtb = (char*)a.keys_hot;
    const uint32_t hm = (1u << hs) - 1u;
    auto put_cold = [&](uint2 e) { *(OutT*)(outb + (uint64_t)e.y * sizeof(OutT)) = (OutT)e.x; };
    const bool hot32 = a.hot_bytes == 4;   /* block-uniform */
    auto put_hot = [&](uint2 e) {
        /* (row offset, col offset) in the hot tile, from the cold key: u16 for
         * a last-level bucket tile, u32 for a mid-level one */
        const uint32_t hk = (((e.x >> hb) & hm) << hs) | (e.x & hm);
        if (hot32) *(uint32_t*)(houtb + (uint64_t)e.y * 4u) = hk;
        else *(uint16_t*)(houtb + (uint64_t)e.y * 2u) = (uint16_t)hk;
    };
    uint2 e[HM_P1_PPT];
#pragma unroll
    for (int j = 0; j < HM_P1_PPT; j++) {
        const uint32_t i = j * HM_P1_THREADS + tid;
        e[j] = ent[i];   /* past total: unused */
        if (HM_L1_LATE_DEST) e[j].y = i < total ? cw[HM_L1_CW + e[j].y] + i : 0u;
    }
    const uint32_t wofs = (uint32_t)tid & ~63u;
    if (!s_over) {
#pragma unroll
        for (int j = 0; j < HM_P1_PPT; j++) {
            const uint32_t wb = __builtin_amdgcn_readfirstlane(j * HM_P1_THREADS + wofs);
            const uint32_t i = j * HM_P1_THREADS + tid;
            if (wb + 64 <= C) {
                put_cold(e[j]);
            } else if (wb >= C && wb + 64 <= total) {
                put_hot(e[j]);
            } else if (wb < total) {
                if (i < C) put_cold(e[j]);
                else if (i < total) put_hot(e[j]);
            }
        }
    } else {
        /* a region overflowed (the host re-runs the level with exact sizes) */
#pragma unroll
        for (int j = 0; j < HM_P1_PPT; j++) {
            const uint32_t i = j * HM_P1_THREADS + tid;
            if (i < total && e[j].y < 0xFFF00000u) {
                if (i < C) put_cold(e[j]);
                else put_hot(e[j]);
            }
        }
    }
    HM_STAMP_M(4, 6);
}

/* ------------------------------------------------------------------------ */
/* level 1, persistent, with compute and writer waves (round 6): k_l1_ws     */
/* ------------------------------------------------------------------------ */
/* k_l1_fast keeps a tile's point loads, its reservation atomics and its key
 * stores in the same waves.  On gfx9 vmcnt retires in issue order, so a load
 * of the next tile issued by such a wave is waited for by each later atomic
 * or store of that wave: a block's points are in flight only while it waits
 * to project them, and a CU's point stream stops whenever both of its blocks
 * count, reserve, stage or copy out.
 *
 * k_l1_ws: one persistent 1024-thread block per CU walking tiles b, b + G, ...
 * of HM_TW = 12288 points, with two wave roles:
 *   compute waves 0-11 (768 threads x 16 points): project tile t, then issue
 *       the loads of tile t + G at once -- the only VMEM operations these
 *       waves issue, so nothing they do later waits behind them -- count +
 *       rank in LDS, take part in the slot scan, stage;
 *   writer waves 12-15 (256 threads): every global atomic and store: the
 *       reservations of tile t (issued as soon as its counts are complete,
 *       waited for a phase later) and the copy-out of tile t, which runs while
 *       the compute waves project tile t + G.
 * A round has five block barriers: count | scan (2) | offsets | stage.  The
 * polynomial and hot-tile tables stay in LDS for the block's life.  The keys,
 * regions, reservations and deferred points are k_l1_fast's.  LDS: 98.8 KB
 * stage + 31.8 KB tables + 21 KB slot words (one block per CU). */
#ifndef HM_L1_WS
#define HM_L1_WS 0                  /* 1: whole units of tiles through k_l1_ws (measured slower) */
#endif
#ifndef HM_WS_PREFETCH_LATE
#define HM_WS_PREFETCH_LATE 0       /* 1: the next tile's loads after the count (fewer live VGPRs) */
#endif
#ifndef HM_WS_PREFETCH_RING
#define HM_WS_PREFETCH_RING 0       /* 1: each point pair's next-tile load as soon as the pair is projected */
#endif
#ifndef HM_WS_C
#define HM_WS_C 768                 /* compute threads: 12 waves */
#endif
#define HM_WS_W (1024 - HM_WS_C)    /* writer threads: the rest of a 1024-thread block */
#define HM_WS_THREADS (HM_WS_C + HM_WS_W)
#define HM_TW (HM_WS_C * HM_P1_PPT) /* points per tile: 12288 at 12 compute waves */
#define HM_WS_NJ ((HM_TW + HM_WS_W - 1) / HM_WS_W)   /* staged entries per writer thread */
#define HM_WS_DLT 2048              /* delta words (slot index masked to 11 bits) */
/* tiles per unit: whole units of k_l1_ws tiles end on a k_l1_fast tile boundary */
#define HM_WS_UNIT (HM_TW % HM_T1 == 0 ? 1 : (2 * HM_TW) % HM_T1 == 0 ? 2 : 4)
static_assert(HM_P1_PPT == 16 && (HM_WS_UNIT * HM_TW) % HM_T1 == 0, "k_l1_ws: whole units end on a k_l1_fast tile");
static_assert(HM_WS_C % 64 == 0 && HM_WS_W >= 64, "whole waves of both roles");
static_assert(HM_L1_SLOTS == HM_WS_THREADS + HM_MAX_HOT && HM_MAX_HOT <= HM_WS_THREADS,
              "k_l1_ws scan: thread t owns slot t, and slot t + 1024 when t < HM_MAX_HOT");
static_assert(HM_L1_SLOTS % HM_WS_W == 0, "writer slots per thread");
static_assert(HM_L1_CW <= HM_WS_DLT, "slot indices fit the delta table");

template <typename OutT, bool KEEP>
__global__ __launch_bounds__(HM_WS_THREADS) void k_l1_ws(HmPart1Args a, uint32_t ntiles)
{
    /* staged (key, slot) + one pad entry per lane */
    __shared__ __attribute__((aligned(16))) uint2 ent[HM_TW + 64];
    constexpr int YROWS = HM_YTAB_ROWS + 1;   /* + the NaN poison row (k_l1_fast) */
    constexpr int YN = YROWS * HM_YTAB_STRIDE;
    __shared__ __attribute__((aligned(16))) double tab[YN];
    __shared__ __attribute__((aligned(16))) uint2 hot2[HM_HOT_SLOTS / 2];
    __shared__ uint32_t cnt[HM_L1_CW];    /* per slot: count + rank atomics (+ 64 dummies) */
    __shared__ uint32_t off[HM_L1_CW];    /* per slot: stage offset */
    __shared__ uint32_t dlt[HM_WS_DLT];   /* per slot: destination - stage offset (writer waves) */
    __shared__ uint32_t scr[HM_WS_THREADS / 64 + 1];
    __shared__ uint32_t s_over, s_sync;
    const int tid = threadIdx.x;
    const uint32_t wave = __builtin_amdgcn_readfirstlane((uint32_t)tid >> 6);
    const int F = 1 << a.dbits;
    const uint32_t H = a.hot_z >= 0 ? *a.hot_n : 0u;
    const uint32_t G = gridDim.x;
    const int wd = a.dbits >> 1;
    auto digit_of = [&](uint32_t sl) -> uint32_t {
        if (sl < HM_MAX_HOT) return HM_MAX_F1 + sl;
        const uint32_t u = sl - HM_MAX_HOT, m = (1u << wd) - 1u;
        return HM_SKEW_CUR ? ((u & ~m) | ((u - ((u >> wd) << 3)) & m)) : u;
    };
    auto live = [&](uint32_t sl) {
        return sl < HM_MAX_HOT ? sl < H : (sl - HM_MAX_HOT) < (uint32_t)F;
    };
    /* the slot scan, by all 1024 threads (the same three barriers in both
     * roles): thread t owns slot t and, t < HM_MAX_HOT, slot t + 1024; the
     * cold slots get the stage's front, the hot ones follow (k_l1_fast) */
    auto scan_slots = [&](uint32_t& Cc, uint32_t& total) {
        constexpr int NW = HM_WS_THREADS / 64;
        /* thread-derived LDS addresses recomputed here: hoisted out of the
         * tile loop they would hold registers across it */
        const uint32_t tt = hm_opaque((uint32_t)tid), ln = tt & 63u;
        const uint32_t s1 = tt + HM_WS_THREADS;
        const bool two = tt < HM_MAX_HOT;
        const uint32_t c0 = live(tt) ? cnt[tt] : 0u;
        const uint32_t c1 = (two && live(s1)) ? cnt[s1] : 0u;
        const uint32_t v = two ? (c1 | (c0 << 16)) : c0;
        const uint32_t inc = hm_wave_incl_scan(v);
        if (ln == 63) scr[wave] = inc;
        hm_lds_barrier();
        if (wave == 0) {
            const uint32_t s = ln < NW ? scr[ln] : 0u;
            const uint32_t si = hm_wave_incl_scan(s);
            if (ln < NW) scr[ln] = si - s;
            if (ln == NW - 1) scr[NW] = si;
        }
        hm_lds_barrier();
        const uint32_t pre = scr[wave] + inc - v, tot = scr[NW];
        Cc = tot & 0xFFFFu;
        total = Cc + (tot >> 16);
        const uint32_t oc = pre & 0xFFFFu;
        if (two) {
            off[tt] = Cc + (pre >> 16);
            off[s1] = oc;
        } else {
            off[tt] = oc;
        }
        hm_lds_barrier();
    };
    if (wave < HM_WS_C / 64) {
        /* ---------------- compute waves ---------------- */
        const uint32_t ct = (uint32_t)tid;
        double2 la[HM_P1_PPT / 2], lo[HM_P1_PPT / 2];
        uint32_t kp[HM_P1_PPT / 2];
        /* point pair kk of tile t (lanes interleaved: coalesced 16-B loads) */
        auto load_pair = [&](uint32_t t, int kk) {
            const int64_t b = (int64_t)t * HM_TW;
            const uint32_t o = hm_opaque(ct);
            if (KEEP) kp[kk] = ((const uint16_t*)(a.keep + b))[kk * HM_WS_C + o];
            la[kk] = hm_stream_load2((const double2*)(a.lat + b) + kk * HM_WS_C + o);
            lo[kk] = hm_stream_load2((const double2*)(a.lon + b) + kk * HM_WS_C + o);
        };
        auto load_tile = [&](uint32_t t) {
#pragma unroll
            for (int k = 0; k < HM_P1_PPT / 2; k++) load_pair(t, k);
        };
        if (!KEEP) {
#pragma unroll
            for (int k = 0; k < HM_P1_PPT / 2; k++) kp[k] = 0x0101;
        }
        load_tile(blockIdx.x);
        hm_lds_barrier();   /* the writer waves filled the tables and zeroed the counts */
        const int hb = a.restbits >> 1;
        const uint32_t lowm = (1u << hb) - 1u;
        const uint32_t keym = (uint32_t)((1ull << (2 * hb)) - 1ull);
        const uint32_t wm = (1u << wd) - 1u;
        const int hs = a.hot_z >= 0 ? a.Z - a.hot_z : 0;
#if defined(HM_STAMPS) && HM_STAMPS == 6
        /* phase cycles per block, summed over its tiles (tools/stamps.py stamps6) */
        unsigned long long sacc[6] = {0, 0, 0, 0, 0, 0}, sprev = __builtin_amdgcn_s_memtime();
        auto stamp = [&](int i) {
            const unsigned long long now = __builtin_amdgcn_s_memtime();
            sacc[i] += now - sprev;
            sprev = now;
        };
#else
        auto stamp = [&](int) {};
#endif
        for (uint32_t t = blockIdx.x; t < ntiles; t += G) {
            const int64_t base = (int64_t)t * HM_TW;
            /* the projection's f64 constants, k_l1_fast's values bit for bit,
             * built per tile from an opaque 52-bit exponent shift in SGPRs:
             * every one is a power-of-two multiple of a compile-time double
             * (2^Z scaling is exact), so no 64-bit literal is materialised
             * and hoisted into registers that live across the tile loop */
            uint64_t zb = (uint64_t)a.Z << 52;
            asm volatile("" : "+s"(zb));
            constexpr double C180 = 180.0 * HM_INV360;   /* 180 kz = RN(180 RN(1/360)) 2^Z */
            const double nscale = hm_u2d(hm_d2u(-1.0) + zb), hscale = hm_u2d(hm_d2u(0.5) + zb);
            const double kz = hm_u2d(hm_d2u(HM_INV360) + zb);
            const double c180 = hm_u2d(hm_d2u(C180) + zb);
            const double ghalf = 0.5 - hm_u2d(hm_d2u(HM_Y_EPS) + zb);
            const double ghalf2 = 0.5 - hm_u2d(hm_d2u(0x1p-49) + zb);
            const uint32_t lane = hm_opaque((uint32_t)tid) & 63u;
            const uint32_t dummy = HM_L1_SLOTS + lane;
            uint32_t slot[HM_P1_PPT], key[HM_P1_PPT];
            uint32_t redo = 0;
            /* the next tile (the last round reloads its own tile: straight-line
             * loads, no conditional register set) */
            const uint32_t tn = t + G < ntiles ? t + G : t;
#pragma unroll
            for (int k = 0; k < HM_P1_PPT; k++) {
                /* k_l1_fast's projection, statement for statement */
                const double pa = (k & 1) ? la[k >> 1].y : la[k >> 1].x;
                const double po = (k & 1) ? lo[k >> 1].y : lo[k >> 1].x;
                const double dd = 90.0 - fabs(pa);
                const uint32_t dh = (uint32_t)(hm_d2u(dd) >> 32);
                constexpr uint32_t I0 = (1023u + HM_YTAB_E0) << HM_YTAB_K;
                const uint32_t ii = min((dh >> (20 - HM_YTAB_K)) - I0, (uint32_t)HM_YTAB_ROWS);
                const double dlo = hm_u2d((uint64_t)(dh & ~((1u << (20 - HM_YTAB_K)) - 1u)) << 32);
                const double tt = dd - dlo;
                const double* cf = tab + ii * HM_YTAB_STRIDE;
                double p = cf[5];
                p = fma(p, tt, cf[4]);
                p = fma(p, tt, cf[3]);
                p = fma(p, tt, cf[2]);
                p = fma(p, tt, cf[1]);
                p = fma(p, tt, cf[0]);
                const double R = fma(copysign(p, pa), nscale, hscale);
                const double fr = __builtin_amdgcn_fract(R);
                const double y = fma(po, kz, c180);
                const double fc = __builtin_amdgcn_fract(y);
                const bool ok = (int)(dd >= 90.0 - HM_LAT_SQ) & (int)(fabs(fr - 0.5) < ghalf) &
                                (int)(fabs(po) < 180.0) & (int)(fabs(fc - 0.5) < ghalf2);
                const uint32_t r = (uint32_t)(int32_t)R;
                const uint32_t c = (uint32_t)(int32_t)y;
                const bool kept = ((kp[k >> 1] >> (8 * (k & 1))) & 0xFFu) != 0;
                redo |= (uint32_t)!ok << k;
                const uint32_t rd = r >> hb, cd = c >> hb;
                const uint32_t rdw = (rd << wd) + HM_MAX_HOT;
                uint32_t sl = HM_SKEW_CUR ? (((cd + (rd << 3)) & wm) | rdw) : (cd | rdw);
                if (H) sl = min(hm_hot_find(hot2, r >> hs, c >> hs), sl);
                key[k] = ((r << hb) | (c & lowm)) & keym;
                slot[k] = (ok & kept) ? sl : dummy;
                asm volatile("" : "+v"(slot[k]), "+v"(key[k]));
                /* ring: the pair's registers are free, its next-tile load goes
                 * out now (the loads stay ~one tile ahead, issued evenly over
                 * the projection instead of in one burst after it) */
                if (HM_WS_PREFETCH_RING && !HM_WS_PREFETCH_LATE && (k & 1)) load_pair(tn, k >> 1);
                __builtin_amdgcn_sched_barrier(0);
            }
            stamp(0);   /* wait for the points + projection */
            /* deferred points (rare; their returning atomic waits for every
             * load this wave has in flight, so they go before the prefetch) */
            if (__builtin_amdgcn_ballot_w64(redo != 0)) {
                /* scalar lane picks and an opaque thread index: nothing of this
                 * rare block is hoisted into registers that live across the loop */
                const uint32_t cto = hm_opaque(ct);
                uint32_t ws = 0;
#pragma unroll
                for (int k = 0; k < HM_P1_PPT; k++) {
                    const bool rd = (redo >> k) & 1u;
                    const uint64_t m = __builtin_amdgcn_ballot_w64(rd);
                    if (m) {
                        const int l = __builtin_ctzll(m);
                        uint64_t b = 0;
                        if (hm_lane() == l) b = atomicAdd(a.redo_count, (unsigned long long)__popcll(m));
                        b = ((uint64_t)__builtin_amdgcn_readlane((uint32_t)(b >> 32), l) << 32) |
                            __builtin_amdgcn_readlane((uint32_t)b, l);
                        const uint64_t q = b + hm_mbcnt(m);
                        if (rd && q < a.redo_cap)
                            a.redo_idx[q] = (uint32_t)(base + 2 * ((int64_t)(k >> 1) * HM_WS_C + cto) + (k & 1));
                        ws += (uint32_t)__popcll(m);
                    }
                }
                if (hm_lane() == 0) atomicAdd(a.slow_count, (unsigned long long)ws);
            }
            if (!HM_WS_PREFETCH_RING && !HM_WS_PREFETCH_LATE) load_tile(tn);
            /* count + rank (k_l1_fast) */
            uint32_t rank[HM_P1_PPT];
            uint32_t merged = 0;
#pragma unroll
            for (int k = 0; k < HM_P1_PPT; k++) {
                const uint32_t k0 = __builtin_amdgcn_readfirstlane(slot[k]);
                const uint64_t m = __builtin_amdgcn_ballot_w64(slot[k] == k0);
                const uint32_t pm = (uint32_t)__builtin_popcount((uint32_t)m) + (uint32_t)__builtin_popcount((uint32_t)(m >> 32));
                uint32_t idx = slot[k], inc = 1u;
                if (pm >= HM_L1_MERGE_MIN) {
                    merged |= 1u << k;
                    const bool in = (m >> lane) & 1ull;
                    idx = (in && lane != 0) ? dummy : idx;
                    inc = lane == 0 ? pm : inc;
                }
                rank[k] = atomicAdd(&cnt[idx], inc);
            }
            if (merged) {
#pragma unroll
                for (int k = 0; k < HM_P1_PPT; k++)
                    if ((merged >> k) & 1u) {
                        const uint32_t k0 = __builtin_amdgcn_readfirstlane(slot[k]);
                        const uint64_t m = __builtin_amdgcn_ballot_w64(slot[k] == k0);
                        const uint32_t r0 = __builtin_amdgcn_readfirstlane(rank[k]);
                        if ((m >> lane) & 1ull) rank[k] = r0 + hm_mbcnt(m);
                    }
            }
            /* slot (11 bits) and rank (< 2^14) share a register from here */
            uint32_t sr[HM_P1_PPT];
#pragma unroll
            for (int k = 0; k < HM_P1_PPT; k++) sr[k] = slot[k] | (rank[k] << 11);
            if (HM_WS_PREFETCH_LATE) load_tile(tn);
            stamp(1);   /* redo, prefetch issue, count + rank */
            hm_lds_barrier();   /* counts complete: the writer waves reserve */
            stamp(2);
            uint32_t Cc, total;
            scan_slots(Cc, total);
            stamp(3);
            /* staging, branch-free: a point that stages nothing writes its
             * lane's pad entry; the entry holds the point's slot (the writer
             * waves look the destination delta up per key) */
#pragma unroll
            for (int k = 0; k < HM_P1_PPT; k++) {
                const uint32_t s = sr[k] & 2047u;
                const uint32_t o = off[s];
                const uint32_t pos = s < HM_L1_SLOTS ? o + (sr[k] >> 11) : HM_TW + (uint32_t)lane;
                ent[pos] = make_uint2(key[k], s);
            }
            stamp(4);
            hm_lds_barrier();   /* staged: the writer waves copy out */
            stamp(5);
        }
        /* the last prefetch is a reload of a tile already counted: drain it */
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#if defined(HM_STAMPS) && HM_STAMPS == 6
        if (tid == 0 && blockIdx.x < HM_STAMP_BLOCKS) {
            for (int i = 0; i < 6; i++) g_stamps[blockIdx.x * 12 + i] = sacc[i];
            g_stamps[blockIdx.x * 12 + 11] = (ntiles - blockIdx.x + G - 1) / G;
        }
#endif
    } else {
        /* ---------------- writer waves ---------------- */
        const uint32_t wt = (uint32_t)tid - HM_WS_C;
        /* the tables (while the compute waves' first points are in flight) */
        for (int i = (int)wt; i < YN; i += HM_WS_W) tab[i] = i >= HM_YTAB_N ? __builtin_nan("") : c_ytab[i];
        if (H)
            for (int j = (int)wt; j < HM_HOT_SLOTS / 4; j += HM_WS_W) ((uint4*)hot2)[j] = ((const uint4*)a.hot_hash)[j];
        for (int i = (int)wt; i < HM_L1_CW; i += HM_WS_W) cnt[i] = 0;
        if (wt == 0) {
            s_over = 0;
            s_sync = 0;
        }
        /* reservation slots q * 256 + wt: their region (shard of this block) */
        constexpr int WQ = HM_L1_SLOTS / HM_WS_W;
        uint32_t fi[WQ], rc[WQ], rb[WQ];
#pragma unroll
        for (int q = 0; q < WQ; q++) {
            const uint32_t sl = q * HM_WS_W + wt;
            const uint32_t d = digit_of(sl);
            const bool lv = live(sl);
            const uint32_t sh = (lv && a.smask[d] != 0) ? (blockIdx.x & (HM_L1_SHARDS - 1)) : 0u;
            fi[q] = hm_l1i(d, sh);
            rc[q] = lv ? a.rcap[fi[q]] : 0u;
            rb[q] = lv ? a.rbase[fi[q]] : 0u;
        }
        hm_lds_barrier();
        char* const outb = (char*)a.keys_out;
        char* const houtb = (char*)a.keys_hot;
        const int hb = a.restbits >> 1;
        const int hs = a.hot_z >= 0 ? a.Z - a.hot_z : 0;
        const uint32_t hm = (1u << hs) - 1u;
        const bool hot32 = a.hot_bytes == 4;
        auto put_cold = [&](uint2 e) { *(OutT*)(outb + (uint64_t)e.y * sizeof(OutT)) = (OutT)e.x; };
        /* a hot key: (row offset, col offset) in the hot tile, from the cold
         * key -- u16 for a last-level bucket tile, u32 for a mid-level one */
        auto hot_key = [&](uint32_t x) { return (((x >> hb) & hm) << hs) | (x & hm); };
        uint32_t pc[WQ], gp[WQ];
#pragma unroll
        for (int q = 0; q < WQ; q++) pc[q] = gp[q] = 0;
        uint32_t pC = 0, ptot = 0, nsync = 0;
#if defined(HM_STAMPS) && HM_STAMPS == 6
        unsigned long long sacc[8] = {0, 0, 0, 0, 0, 0, 0, 0}, sprev = __builtin_amdgcn_s_memtime();
        auto stamp = [&](int i) {
            const unsigned long long now = __builtin_amdgcn_s_memtime();
            sacc[i] += now - sprev;
            sprev = now;
        };
#else
        auto stamp = [&](int) {};
#endif
        /* the previous tile: destination deltas once its reservations are
         * back, a writer-only rendezvous, then its keys leave lane-parallel */
        auto copy_out = [&]() {
            bool over = false;
#pragma unroll
            for (int q = 0; q < WQ; q++) {
                const uint32_t sl = q * HM_WS_W + wt;
                if (live(sl)) {
                    const bool fits = (uint64_t)gp[q] + pc[q] <= (uint64_t)rc[q];
                    over |= pc[q] && !fits;
                    dlt[sl] = (fits ? rb[q] + gp[q] : 0xFFF00000u) - off[sl];
                }
            }
            if (over) {
                atomicOr(a.overflow, 1ull);
                atomicOr(&s_over, 1u);
            }
            stamp(0);   /* deltas (the reservations waited for) */
            nsync += HM_WS_W / 64;
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
            if (hm_lane() == 0) atomicAdd(&s_sync, 1u);
            while (__atomic_load_n(&s_sync, __ATOMIC_RELAXED) < nsync) __builtin_amdgcn_s_sleep(1);
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
            const bool ov = __atomic_load_n(&s_over, __ATOMIC_RELAXED) != 0;   /* block-uniform */
            stamp(1);   /* writer rendezvous */
            /* the cold keys [0, pC) then the hot ones [pC, ptot), each range
             * lane-consecutive (a wave stores 64 consecutive staged keys), no
             * per-key kind test; a region that overflowed: destinations
             * >= 0xFFF00000, dropped (the host re-runs the level) */
            constexpr int JB = HM_WS_NJ < 16 ? HM_WS_NJ : 16;
            auto range = [&](uint32_t lo, uint32_t hi, auto put) {
#pragma unroll 1
                for (uint32_t b0 = lo; b0 < hi; b0 += JB * HM_WS_W) {   /* block-uniform */
                    uint2 e[JB];
#pragma unroll
                    for (int j = 0; j < JB; j++) {
                        const uint32_t i = b0 + j * HM_WS_W + wt;
                        e[j] = ent[min(i, (uint32_t)HM_TW)];
                        e[j].y = dlt[e[j].y & (HM_WS_DLT - 1)] + i;   /* past hi: unused */
                    }
#pragma unroll
                    for (int j = 0; j < JB; j++) {
                        const uint32_t i = b0 + j * HM_WS_W + wt;
                        if (i < hi && (!ov || e[j].y < 0xFFF00000u)) put(e[j]);
                    }
                }
            };
            range(0, pC, put_cold);
            if (hot32)
                range(pC, ptot, [&](uint2 e) { *(uint32_t*)(houtb + (uint64_t)e.y * 4u) = hot_key(e.x); });
            else
                range(pC, ptot, [&](uint2 e) { *(uint16_t*)(houtb + (uint64_t)e.y * 2u) = (uint16_t)hot_key(e.x); });
            stamp(2);   /* copy-out */
        };
        bool have = false;
        for (uint32_t t = blockIdx.x; t < ntiles; t += G) {
            if (have) copy_out();
            hm_lds_barrier();   /* this tile's counts are complete */
            stamp(3);
            if (wt == 0) s_over = 0;   /* every writer read it in copy_out */
#pragma unroll
            for (int q = 0; q < WQ; q++) {
                const uint32_t sl = q * HM_WS_W + wt;
                pc[q] = live(sl) ? cnt[sl] : 0u;
                gp[q] = 0;
                if (pc[q]) gp[q] = atomicAdd(&a.fill[fi[q]], pc[q]);   /* waited for in the next copy_out */
            }
            stamp(4);   /* reservations issued */
            scan_slots(pC, ptot);
            stamp(5);
            for (int i = (int)wt; i < HM_L1_CW; i += HM_WS_W) cnt[i] = 0;   /* the scan has read them */
            hm_lds_barrier();   /* staged */
            stamp(6);
            have = true;
        }
        if (have) copy_out();
#if defined(HM_STAMPS) && HM_STAMPS == 6
        if (wt == 0 && blockIdx.x < 4096)
            for (int i = 0; i < 8; i++) g_stamps[(4096 + blockIdx.x) * 12 + i] = sacc[i];
#endif
    }
}

/* Sampled digit histogram of level 1 (every stride-th point, fast projection
 * only): sizes the per-digit key regions k_project_partition fills. */
#define HM_SAMPLE_HSLOTS 4096   /* per-block hash of sampled hot-zoom tiles */
template <bool FROM_TILES, bool HOT>
__global__ __launch_bounds__(256) void k_sample_digits(HmPart1Args a, uint64_t stride_pts, uint32_t* hist,
                                                       uint32_t* hot_counts)
{
    __shared__ uint32_t h[HM_MAX_F1 + 64];
    __shared__ double tab[HM_YTAB_N];
    /* HOT: the block's samples per zoom-hot_z tile, pre-aggregated in LDS
     * (a hot tile gets one global atomic per block, not one per sample) */
    __shared__ uint32_t hk[HOT ? HM_SAMPLE_HSLOTS : 1], hc[HOT ? HM_SAMPLE_HSLOTS : 1];
    const int F = 1 << a.dbits;
    for (int i = threadIdx.x; i < F; i += 256) h[i] = 0;
    if (HOT)
        for (int i = threadIdx.x; i < HM_SAMPLE_HSLOTS; i += 256) {
            hk[i] = HM_HOT_EMPTY;
            hc[i] = 0;
        }
    if (!FROM_TILES) hm_load_ytab(tab);
    __syncthreads();
    uint32_t hlost = 0;   /* samples the (full) LDS hash could not take: counted directly */
    const double scale = hm_exp2i(a.Z);
    const double kz = HM_INV360 * scale;
    const uint32_t lim = 1u << a.Z;
    const int hb = a.restbits >> 1, wd = a.dbits >> 1;
    const uint64_t m = (uint64_t)(a.n + stride_pts - 1) / stride_pts;
    const uint64_t m_up = (m + 63) & ~63ull;
    const uint64_t step = (uint64_t)gridDim.x * 256;
    for (uint64_t j = (uint64_t)blockIdx.x * 256 + threadIdx.x; j < m_up; j += step) {
        const uint64_t i = j * stride_pts;
        bool v = j < m && (!a.keep || a.keep[i]);
        int64_t r = 0, c = 0;
        if (v) {
            if (FROM_TILES) {
                r = a.rows_in[i];
                c = a.cols_in[i];
            } else {
                int32_t r32, c32;
                v = hm_project_fast(a.lat[i], a.lon[i], scale, kz, &r32, &c32, tab);
                r = r32;
                c = c32;
            }
            v = v && (uint64_t)r < lim && (uint64_t)c < lim;
        }
        const uint32_t d = ((((uint32_t)r) >> hb) << wd) | (((uint32_t)c) >> hb);
        hm_lds_count(h, HM_MAX_F1, d, v);
        if (HOT && v) {
            const int hs = a.Z - a.hot_z;
            const uint32_t t = ((((uint32_t)r) >> hs) << a.hot_z) | (((uint32_t)c) >> hs);
            uint32_t sl = (t * 2654435761u) >> (32 - 12);
            static_assert(HM_SAMPLE_HSLOTS == 1 << 12, "sample hash slots");
            /* a few probes, then the global count: a spread-out cloud (4096+
             * distinct tiles per block) fills the table, and a full scan per
             * sample took uniform clouds 1.5 ms */
            int probes = 0;
            for (;;) {
                const uint32_t o = atomicCAS(&hk[sl], HM_HOT_EMPTY, t);
                if (o == HM_HOT_EMPTY || o == t) {
                    atomicAdd(&hc[sl], 1u);
                    break;
                }
                sl = (sl + 1) & (HM_SAMPLE_HSLOTS - 1);
                if (++probes == 16) {
                    atomicAdd(&hot_counts[t], 1u);
                    hlost++;
                    break;
                }
            }
        }
    }
    __syncthreads();
    for (int i = threadIdx.x; i < F; i += 256)
        if (h[i]) atomicAdd(&hist[i], h[i]);
    if (HOT)
        for (int i = threadIdx.x; i < HM_SAMPLE_HSLOTS; i += 256)
            if (hc[i]) atomicAdd(&hot_counts[hk[i]], hc[i]);
    (void)hlost;
}

/* Hot-tile candidates: every zoom-zb tile with >= thresh sampled points (at
 * most HM_HOT_CAND, first come), listed with its sampled count. */
__global__ __launch_bounds__(256) void k_hot_select(HmHotArgs a)
{
    const uint64_t ntiles = 1ull << (2 * a.zb);
    const uint64_t stride = (uint64_t)gridDim.x * 256;
    uint32_t* const ncand = a.cand + 2 * HM_HOT_CAND;
    for (uint64_t t = (uint64_t)blockIdx.x * 256 + threadIdx.x; t < ntiles; t += stride) {
        const uint32_t c = a.counts[t];
        if (c >= a.thresh) {
            const uint32_t j = atomicAdd(ncand, 1u);
            if (j < HM_HOT_CAND) {
                a.cand[2 * j] = (uint32_t)t;
                a.cand[2 * j + 1] = c;
            }
        }
    }
}

/* The hot tiles and the table image k_project_partition looks them up in.
 * The biggest candidates go first: a histogram of their sampled counts (8
 * bins per octave) gives the cutoff bin above which fewer than HM_MAX_HOT
 * candidates lie; those are placed, then the cutoff bin's first come.  A
 * candidate becomes hot tile h (< HM_MAX_HOT) when its bucket has a free way;
 * otherwise it stays cold (any set of hot tiles gives the same counts).  Hot
 * tile h: its sampled count as level-1 histogram entry HM_MAX_F1 + h, taken
 * off its z1 digit, which is flagged as a hot parent.  One block. */
__device__ __forceinline__ uint32_t hm_hot_bin(uint32_t c)
{
    const uint32_t e = 31u - __clz(c | 1u);
    return e < 3 ? c : (e << 3) | ((c >> (e - 3)) & 7u);   /* < 256 */
}

__global__ __launch_bounds__(1024) void k_hot_hash(HmHotArgs a)
{
    __shared__ uint32_t tab[HM_HOT_SLOTS];
    __shared__ uint32_t fill[HM_HOT_BUCKETS];
    __shared__ uint32_t bins[256];
    __shared__ uint32_t nh, cut;
    static_assert(HM_HOT_CAND <= 4 * 1024, "4 candidates a thread");
    const int tid = threadIdx.x;
    for (int i = tid; i < HM_HOT_SLOTS; i += 1024) tab[i] = HM_HOT_EMPTY;
    for (int i = tid; i < HM_HOT_BUCKETS; i += 1024) fill[i] = 0;
    for (int i = tid; i < 256; i += 1024) bins[i] = 0;
    if (tid == 0) nh = 0;
    /* the thread's candidates j = tid + 1024 u, read once for the three passes */
    const uint32_t nc = min(a.cand[2 * HM_HOT_CAND], (uint32_t)HM_HOT_CAND);
    uint32_t ct[4], cc[4];
#pragma unroll
    for (int u = 0; u < 4; u++) {
        const uint32_t j = tid + 1024u * u;
        const uint2 v = j < nc ? ((const uint2*)a.cand)[j] : make_uint2(0u, 0u);
        ct[u] = v.x;
        cc[u] = v.y;
    }
    __syncthreads();
#pragma unroll
    for (int u = 0; u < 4; u++)
        if (tid + 1024u * u < nc) atomicAdd(&bins[hm_hot_bin(cc[u])], 1u);
    __syncthreads();
    if (tid < 64) {
        /* cutoff: the highest bin b whose candidates from the top (bins >= b)
         * reach HM_HOT_LIMIT, 0 if none -- lane l holds bins 4l .. 4l+3, the
         * bins above them a reversed-lane scan */
        const int l = tid;
        uint32_t s = 0;
        uint32_t bv[4];
#pragma unroll
        for (int k = 0; k < 4; k++) s += (bv[k] = bins[4 * l + k]);
        const uint32_t rs = __shfl(s, 63 - l, 64);              /* lane l: the sum of lane 63 - l */
        const uint32_t incl = hm_wave_incl_scan(rs);              /* lanes 63-l .. 63 from the top */
        const uint32_t above = __shfl(incl, 62 - l < 0 ? 0 : 62 - l, 64);   /* bins of lanes > l */
        uint32_t acc = l == 63 ? 0u : above;
        int best = -1;
#pragma unroll
        for (int k = 3; k >= 0; k--) {
            acc += bv[k];
            if (best < 0 && acc >= HM_HOT_LIMIT) best = 4 * l + k;
        }
        for (int o = 32; o > 0; o >>= 1) best = max(best, __shfl_xor(best, o, 64));
        if (l == 0) cut = best < 0 ? 0u : (uint32_t)best;
    }
    __syncthreads();
    /* pass 0: above the cutoff bin; 1: at it; 2: below it (only while hot
     * digits are left: candidates whose bucket was full leave room) */
    for (int pass = 0; pass < 3; pass++) {
        if (pass == 2 && nh >= HM_HOT_LIMIT) break;   /* (block-uniform: read after the barrier) */
#pragma unroll
        for (int u = 0; u < 4; u++) {
            if (tid + 1024u * u >= nc) continue;
            const uint32_t t = ct[u], c = cc[u];
            const uint32_t bn = hm_hot_bin(c);
            if (pass == 0 ? bn <= cut : pass == 1 ? bn != cut : bn >= cut) continue;
            const uint32_t tr = t >> a.zb, tc = t & ((1u << a.zb) - 1u);
            const uint32_t b = hm_hot_bucket(tr, tc);
            const uint32_t w = atomicAdd(&fill[b], 1u);
            if (w >= HM_HOT_WAYS) continue;
            const uint32_t h = atomicAdd(&nh, 1u);
            if (h >= HM_HOT_LIMIT) continue;   /* its way stays empty */
            tab[b * HM_HOT_WAYS + w] = (tr << HM_HOT_TAG) | h;
            a.tiles[h] = t;
            a.hist[HM_MAX_F1 + h] = c;
            const int s = a.zb - a.z1;
            const uint32_t d = ((tr >> s) << a.z1) | (tc >> s);
            a.hotparent[d] = 1;
            atomicSub(&a.hist[d], c);   /* those samples' keys leave the cold digit */
        }
        __syncthreads();
    }
    for (int i = tid; i < HM_HOT_SLOTS; i += 1024) a.hash[i] = tab[i];
    if (tid == 0) *a.n = min(nh, (uint32_t)HM_HOT_LIMIT);
}

void hm_launch_hot_select(hipStream_t s, const HmHotArgs& a)
{
    const uint64_t ntiles = 1ull << (2 * a.zb);
    uint64_t blocks = (ntiles + 4095) / 4096;
    if (blocks > 1024) blocks = 1024;
    if (blocks < 1) blocks = 1;
    hipLaunchKernelGGL(k_hot_select, dim3((unsigned)blocks), dim3(256), 0, s, a);
    hipLaunchKernelGGL(k_hot_hash, dim3(1), dim3(1024), 0, s, a);
}

/* Level-1 region sizes from the sampled histogram, on the device (no host
 * round trip): per digit est = hist * stride; a digit above 64 tiles gets
 * HM_L1_SHARDS shards; per shard cap = e + e/16 + 8 sqrt(e * stride) + 2 T1
 * (e = est / shards); bases = exclusive prefix over (digit, shard), the F
 * cold digits first, then the hot tiles' digits HM_MAX_F1 + h (h < *hot_n),
 * one position space.  The same formula as the host's retry path.  One block
 * of 1024 threads: thread t sizes cold digit t and hot digit HM_MAX_F1 + t. */
__device__ __forceinline__ uint32_t hm_l1_cap(uint32_t hist, uint64_t stride, int* ns)
{
    const double est = (double)hist * (double)stride;
    *ns = est > (double)HM_L1_SHARD_TILES * HM_T1 ? HM_L1_SHARDS : 1;
    const double e = est / *ns;
    /* + HM_L1_ZERO_SAMPLES strides per digit: a digit with few or no samples
     * may still hold that many strides of points (P(0 samples | 24) = 4e-11);
     * the region's unused tail is never read */
    return (uint32_t)fmin(1.0e9, e + e / 16 + 8.0 * sqrt(e * (double)stride) +
                                     (double)HM_L1_ZERO_SAMPLES * (double)stride / *ns + 2.0 * HM_T1);
}

__global__ __launch_bounds__(1024) void k_l1_sizes(const uint32_t* __restrict__ hist, int F,
                                                   const uint32_t* __restrict__ hot_n, uint64_t stride,
                                                   uint32_t* __restrict__ rcap, uint32_t* __restrict__ rbase,
                                                   uint8_t* __restrict__ smask, unsigned long long* total)
{
    __shared__ unsigned long long wsum[1024 / 64];
    static_assert(HM_MAX_HOT <= 1024 && HM_MAX_F1 <= 1024, "one digit of each kind per thread");
    const int t = threadIdx.x;
    const int lane = t & 63, w = t >> 6;
    const uint32_t H = hot_n ? min(*hot_n, (uint32_t)HM_MAX_HOT) : 0u;
    unsigned long long base = 0;
    for (int kind = 0; kind < 2; kind++) {
        const int d = kind ? HM_MAX_F1 + t : t;
        const bool live = kind ? (uint32_t)t < H : t < F;
        uint32_t c = 0;
        int ns = 1;
        if (live) {
            c = hm_l1_cap(hist[d], stride, &ns);
            smask[d] = (uint8_t)(ns - 1);
        }
        const unsigned long long mine = live ? (unsigned long long)c * (unsigned long long)ns : 0ull;
        unsigned long long incl = mine;
        for (int o = 1; o < 64; o <<= 1) {
            const unsigned long long y = __shfl_up(incl, o, 64);
            if (lane >= o) incl += y;
        }
        __syncthreads();
        if (lane == 63) wsum[w] = incl;
        __syncthreads();
        unsigned long long before = 0, all = 0;
        for (int i = 0; i < 1024 / 64; i++) {
            before += i < w ? wsum[i] : 0ull;
            all += wsum[i];
        }
        unsigned long long pos = base + before + incl - mine;
        if (live)
            for (int sh = 0; sh < HM_L1_SHARDS; sh++) {
                const uint32_t cs = sh < ns ? c : 0u;
                rcap[hm_l1i(d, sh)] = cs;
                rbase[hm_l1i(d, sh)] = (uint32_t)pos;   /* total < 2^32: the host's bound */
                pos += cs;
            }
        base += all;
    }
    if (t == 0 && total) *total = base;
}

void hm_launch_l1_sizes(hipStream_t s, const uint32_t* hist, int F, const uint32_t* hot_n, uint64_t stride,
                        uint32_t* rcap, uint32_t* rbase, uint8_t* smask, unsigned long long* total)
{
    hipLaunchKernelGGL(k_l1_sizes, dim3(1), dim3(1024), 0, s, hist, F, hot_n, stride, rcap, rbase, smask, total);
}

void hm_launch_sample_digits(hipStream_t s, const HmPart1Args& a, uint64_t stride_pts, uint32_t* hist,
                             uint32_t* hot_counts)
{
    const uint64_t m = ((uint64_t)a.n + stride_pts - 1) / stride_pts;
    uint64_t blocks = (m + 1023) / 1024;
    /* with the hot-tile counts: fewer, fuller blocks (one global atomic per
     * block and tile) */
    const uint64_t cap = hot_counts ? 256 : 2048;
    if (blocks > cap) blocks = cap;
    if (blocks < 1) blocks = 1;
#define HM_SD(T, H) hipLaunchKernelGGL((k_sample_digits<T, H>), dim3((unsigned)blocks), dim3(256), 0, s, a, stride_pts, \
                                       hist, hot_counts)
    if (a.rows_in) {
        if (hot_counts) HM_SD(true, true);
        else HM_SD(true, false);
    } else {
        if (hot_counts) HM_SD(false, true);
        else HM_SD(false, false);
    }
#undef HM_SD
}

/* Level-1 buckets from the filled regions: one flat run per non-empty digit
 * (its whole region), the bucket list, work-item prefix and, when level 1 is
 * the last level, the merge slots of multi-item buckets.  One block. */
__global__ __launch_bounds__(1024) void k_level1_buckets(HmL1Args a)
{
    __shared__ uint32_t scr[1024 / 64 + 1];
    const int d = threadIdx.x;
    uint32_t f[HM_L1_SHARDS];
    uint32_t nk = 0, nr = 0;
    const int ns = d < a.F ? a.smask[d] + 1 : 0;
#pragma unroll
    for (int sh = 0; sh < HM_L1_SHARDS; sh++) {
        f[sh] = sh < ns ? a.fill[hm_l1i(d, sh)] : 0u;
        nk += f[sh];
        nr += f[sh] != 0;
    }
    /* a digit whose points all went to its hot tiles is still a bucket: the
     * parent of those tiles at level 2 (no keys, no items of its own) */
    const uint32_t ne = nk > 0 || (a.hotparent && d < a.F && a.hotparent[d]);
    const uint32_t nit = nk ? (nk <= a.sparse_max ? 0u : (nk + a.item_keys - 1) / a.item_keys) : 0u;
    uint32_t count, items, runs;
    const uint32_t idx = hm_block_excl_scan<1024>(ne, scr, &count);
    const uint32_t ib = hm_block_excl_scan<1024>(nit, scr, &items);
    const uint32_t r0 = hm_block_excl_scan<1024>(nr, scr, &runs);
    if (a.d2b && d < a.F) a.d2b[d] = ne ? idx : 0xFFFFFFFFu;
    if (ne) {
        /* logical key positions of the bucket: [region base, + nk), its
         * non-empty shards' keys one after the other */
        const uint32_t kb = a.rbase[hm_l1i(d, 0)];
        a.out.nkeys[idx] = nk;
        a.out.nruns[idx] = nr;
        a.out.rbase[idx] = r0;
        a.out.keybase[idx] = kb;
        a.out.item_begin[idx] = ib;
        a.out.digit[idx] = (uint32_t)d;
        const int wd = a.dbits >> 1;
        a.out.coord[idx] = ((uint64_t)(d >> wd) << 32) | (uint64_t)(d & ((1 << wd) - 1));
        uint32_t j = r0, at = kb;
#pragma unroll
        for (int sh = 0; sh < HM_L1_SHARDS; sh++) {
            if (f[sh]) {
                a.runs[j] = make_uint2(a.rbase[hm_l1i(d, sh)], f[sh]);
                a.excl[j] = at;
                at += f[sh];
                j++;
            }
        }
        if (a.slots) {
            int32_t sl = -1;
            if (nit > 1) {
                sl = (int32_t)atomicAdd(a.nslots, 1ull);
                a.slot_bucket[sl] = idx;
            }
            a.slots[idx] = sl;
        }
    }
    if (d == 0) {
        a.out.item_begin[count] = items;
        a.child_begin[0] = 0;
        a.child_begin[1] = count;
        *a.total = ((uint64_t)count << 32) | items;
    }
}

void hm_launch_level1_buckets(hipStream_t s, const HmL1Args& a)
{
    hipLaunchKernelGGL(k_level1_buckets, dim3(1), dim3(1024), 0, s, a);
}

/* ------------------------------------------------------------------------ */
/* work items and run streaming                                              */
/* ------------------------------------------------------------------------ */

template <typename T>
__device__ __forceinline__ uint32_t hm_upper_bound(const T* a, uint32_t n, T v)
{
    uint32_t lo = 0, hi = n;
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (a[mid] <= v)
            lo = mid + 1;
        else
            hi = mid;
    }
    return lo;
}

template <typename T>
__device__ __forceinline__ uint32_t hm_lower_bound(const T* a, uint32_t n, T v)
{
    uint32_t lo = 0, hi = n;
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (a[mid] < v)
            lo = mid + 1;
        else
            hi = mid;
    }
    return lo;
}

/* one 32-B descriptor load (written by k_items) per block */
__device__ __forceinline__ HmItem hm_item(const HmBuckets& B, uint32_t g)
{
    const uint4 d0 = B.desc[2 * g], d1 = B.desc[2 * g + 1];
    HmItem it;
    it.bucket = d0.x;
    it.j = d0.y;
    it.nitems = d0.z;
    it.r0 = d0.w;
    it.r1 = d1.x;
    it.a = d1.z;
    it.b = d1.w;
    return it;
}

/* Descriptor of work item g (T keys per item): its bucket (binary search over
 * item_begin), its logical positions [a, b) and the runs [r0, r1) that
 * overlap them.  One thread per item; the searches of all items overlap. */
__global__ __launch_bounds__(256) void k_items(HmBuckets B, HmRuns in, uint32_t items, uint32_t T, uint4* desc,
                                               uint32_t* seg)
{
    const uint32_t g = blockIdx.x * 256 + threadIdx.x;
    if (g >= items) return;
    const uint32_t bk = hm_upper_bound(B.item_begin, B.count + 1, g) - 1;
    const uint32_t j = g - B.item_begin[bk];
    const uint32_t nitems = B.item_begin[bk + 1] - B.item_begin[bk];
    const uint64_t kb = B.keybase[bk], nk = B.nkeys[bk];
    const uint64_t a = kb + (uint64_t)j * T;
    const uint64_t b = kb + min((uint64_t)(j + 1) * T, nk);
    const uint32_t rb = B.rbase[bk], nr = B.nruns[bk];
    const uint32_t r0 = rb + hm_upper_bound(in.excl + rb, nr, a) - 1;   /* last run starting <= a */
    const uint32_t r1 = rb + hm_lower_bound(in.excl + rb, nr, b);       /* first run starting >= b */
    desc[2 * g] = make_uint4(bk, j, nitems, r0);
    desc[2 * g + 1] = make_uint4(r1, 0u, (uint32_t)a, (uint32_t)b);
    if (seg) {
        /* the item's <= HM_L1_SHARDS runs as (logical start, source index)
         * pairs, unused entries repeating the last run (k_partition_fr) */
        uint4* sg = (uint4*)(seg + 16 * (size_t)g);
        uint32_t v[2 * HM_L1_SHARDS];
        const uint32_t last = r1 > r0 ? r1 - 1 : r0;
#pragma unroll
        for (int q = 0; q < HM_L1_SHARDS; q++) {
            const uint32_t r = min(r0 + q, last);
            v[2 * q] = (uint32_t)in.excl[r];
            v[2 * q + 1] = in.run[r].x;
        }
#pragma unroll
        for (int q = 0; q < HM_L1_SHARDS / 2; q++) sg[q] = make_uint4(v[4 * q], v[4 * q + 1], v[4 * q + 2], v[4 * q + 3]);
    }
}

void hm_launch_items(hipStream_t s, const HmBuckets& B, HmRuns in, uint32_t items, uint32_t T, uint4* desc,
                     uint32_t* seg)
{
    if (items) hipLaunchKernelGGL(k_items, dim3((items + 255) / 256), dim3(256), 0, s, B, in, items, T, desc, seg);
}

/* Run chunk staged in LDS, dense per run i of the chunk: its 16-B-aligned
 * body (first vector, vectors; zero unless long) and two pieces (head and
 * tail of a long run, or the whole short run), each with an exclusive prefix. */
template <int RCH>
struct HmRunLds {
    uint32_t bv[RCH], bn[RCH], pre[RCH + 1];
    uint32_t ps[2 * RCH], pn[2 * RCH], ppre[2 * RCH + 1];
};

/* one wave: pre[0..n] = exclusive prefix of in[0..n), pre[n] = total */
__device__ __forceinline__ void hm_wave_prefix(const uint32_t* in, uint32_t n, uint32_t* pre)
{
    const uint32_t lane = hm_lane();
    const uint32_t per = (n + 63) / 64;
    const uint32_t i0 = min(n, lane * per), i1 = min(n, i0 + per);
    uint32_t sum = 0;
    for (uint32_t i = i0; i < i1; i++) sum += in[i];
    const uint32_t incl = hm_wave_incl_scan(sum);
    uint32_t acc = incl - sum;
    for (uint32_t i = i0; i < i1; i++) {
        const uint32_t x = in[i];
        pre[i] = acc;
        acc += x;
    }
    if (lane == 63) pre[n] = incl;
}

#ifndef HM_SU
#define HM_SU 4
#endif

/* Calls f.vec(uint4 x, valid, pos) / f.key(key, valid, pos) for every key at
 * the item's logical positions [a, b): the keys of vector x are staged order
 * positions pos..pos+V-1, single keys pos; together the positions are a
 * permutation of [0, b - a) (deterministic: no append atomics).  The item's
 * runs are staged RCH at a time and clipped to [a, b).  The 16-B-aligned
 * bodies of runs with >= HM_LONG_RUN keys form one flat vector space, split
 * into contiguous per-wave spans; a lane keeps HM_SU 16-B loads in flight and
 * finds each vector's run by walking a monotone cursor over the body prefix.
 * Short runs and the bodies' unaligned heads and tails ("pieces") go either
 * one lane each (8 loads in flight) or, COOP, 64 pieces per wave expanded
 * into consecutive keys per lane.  Block-uniform: every thread calls. */
template <typename InT, int THREADS, int RCH, bool COOP, typename F>
__device__ __forceinline__ void hm_stream_runs(const HmItem& it, const InT* __restrict__ keys, const HmRuns& in,
                                               HmRunLds<RCH>& L, uint32_t* scr, F& f)
{
    constexpr int NW = THREADS / 64;
    constexpr uint32_t V = 16 / sizeof(InT);   /* keys per 16-B vector */
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int w = tid >> 6;
    const uint4* kv = (const uint4*)keys;
    if (it.r1 - it.r0 <= HM_L1_SHARDS) {
        /* a few long runs (level-1 regions): each a contiguous key range,
         * streamed directly -- head keys, 16-B body vectors HM_SU per lane in
         * flight, tail keys; positions in that order, run after run */
        uint32_t pos0 = 0;
        for (uint32_t r = it.r0; r < it.r1; r++) {
        const uint2 run = in.run[r];
        const uint64_t s0 = in.excl[r];
        const uint64_t s2 = max(s0, (uint64_t)it.a), e2 = min(s0 + run.y, (uint64_t)it.b);
        const uint32_t cnt = e2 > s2 ? (uint32_t)(e2 - s2) : 0u;
        const uint32_t src = run.x + (uint32_t)(s2 - s0);
        const uint32_t head = min(cnt, (V - (src & (V - 1))) & (V - 1));
        const uint32_t nv = (cnt - head) / V;
        const uint32_t tail = cnt - head - nv * V;
        const uint32_t vb = (src + head) / V;
        for (uint32_t v0 = 0; v0 < nv; v0 += THREADS * HM_SU) {
            uint4 x[HM_SU];
            bool ok[HM_SU];
#pragma unroll
            for (int u = 0; u < HM_SU; u++) {
                const uint32_t v = v0 + u * THREADS + tid;
                ok[u] = v < nv;
                x[u] = ok[u] ? kv[vb + v] : make_uint4(0, 0, 0, 0);
            }
#pragma unroll
            for (int u = 0; u < HM_SU; u++) f.vec(x[u], ok[u], pos0 + head + V * (v0 + u * THREADS + tid));
        }
        const uint32_t t = (uint32_t)tid;
        const uint32_t kh = t < head ? (uint32_t)keys[src + t] : 0u;
        const uint32_t kt = t < tail ? (uint32_t)keys[src + head + nv * V + t] : 0u;
        f.key(kh, t < head, pos0 + t);
        f.key(kt, t < tail, pos0 + head + nv * V + t);
        pos0 += cnt;
        }
        __syncthreads();
        return;
    }
    uint32_t carry = 0;                        /* keys staged by earlier chunks */
    for (uint32_t rc = it.r0; rc < it.r1; rc += RCH) {
        const uint32_t m = min((uint32_t)RCH, it.r1 - rc);
        for (uint32_t i = tid; i < m; i += THREADS) {
            const uint2 run = in.run[rc + i];
            const uint64_t s = in.excl[rc + i];
            const uint64_t e = s + run.y;
            const uint64_t s2 = max(s, (uint64_t)it.a), e2 = min(e, (uint64_t)it.b);
            const uint32_t cnt = e2 > s2 ? (uint32_t)(e2 - s2) : 0u;
            const uint32_t src = run.x + (uint32_t)(s2 - s);
            const uint32_t head = min(cnt, (V - (src & (V - 1))) & (V - 1));
            const uint32_t nv = (cnt - head) / V;
            const bool lg = cnt >= HM_LONG_RUN && nv > 0;
            L.bv[i] = (src + head) / V;
            L.bn[i] = lg ? nv : 0u;
            L.ps[2 * i] = src;
            L.pn[2 * i] = lg ? head : cnt;
            L.ps[2 * i + 1] = src + head + nv * V;
            L.pn[2 * i + 1] = lg ? cnt - head - nv * V : 0u;
        }
        __syncthreads();
        if (sizeof(InT) == 2 && rc == it.r0) HM_STAMP_M(5, 8);
        if (w == 0) hm_wave_prefix(L.bn, m, L.pre);
        if (w == 1 || NW == 1) hm_wave_prefix(L.pn, 2 * m, L.ppre);
        __syncthreads();
        if (sizeof(InT) == 2 && rc == it.r0) HM_STAMP_M(5, 9);
        const uint32_t nb = m, np = 2 * m;
        const uint32_t total = L.pre[nb];
        const uint32_t pbase = carry + V * total;
        /* bodies: contiguous wave spans of the flat vector space */
        const uint32_t span = ((total + NW - 1) / NW + 63) & ~63u;
        const uint32_t vb = min(total, span * w), ve = min(total, vb + span);
        if (vb < ve) {
            uint32_t r = hm_upper_bound(L.pre, nb + 1, vb) - 1;
            for (uint32_t v0 = vb; v0 < ve; v0 += 64 * HM_SU) {
                uint4 x[HM_SU];
                bool ok[HM_SU];
#pragma unroll
                for (int u = 0; u < HM_SU; u++) {
                    const uint32_t v = v0 + u * 64 + lane;
                    ok[u] = v < ve;
                    x[u] = make_uint4(0, 0, 0, 0);
                    if (ok[u]) {
                        while (L.pre[r + 1] <= v) r++;
                        x[u] = kv[L.bv[r] + (v - L.pre[r])];
                    }
                }
#pragma unroll
                for (int u = 0; u < HM_SU; u++) f.vec(x[u], ok[u], carry + V * (v0 + u * 64 + lane));
            }
        }
        if (sizeof(InT) == 4 && rc == it.r0) HM_STAMP(5);
        if (sizeof(InT) == 2 && rc == it.r0) HM_STAMP_M(5, 10);
        /* pieces: a wave takes 64 at a time, scans their lengths and hands
         * consecutive keys to consecutive lanes (piece found by a 6-step
         * shuffle search), 4 loads per lane in flight */
        if (COOP) {
        for (uint32_t q0 = (uint32_t)w * 64; q0 < np; q0 += NW * 64) {
            const uint32_t q = q0 + lane;
            const uint2 pc = q < np ? make_uint2(L.ps[q], L.pn[q]) : make_uint2(0, 0);
            const uint32_t pp = q < np ? pbase + L.ppre[q] : 0u;
            const uint32_t incl = hm_wave_incl_scan(pc.y);
            const uint32_t tot = __shfl(incl, 63, 64);
            for (uint32_t j0 = 0; j0 < tot; j0 += 256) {
                uint32_t kk[4], at[4];
                bool ok[4];
#pragma unroll
                for (int u = 0; u < 4; u++) {
                    const uint32_t j = j0 + u * 64 + lane;
                    uint32_t lo = 0;
#pragma unroll
                    for (int st = 32; st > 0; st >>= 1)
                        if (__shfl(incl, lo + st - 1, 64) <= j) lo += st;
                    lo = min(lo, 63u);
                    const uint32_t cnt = __shfl(pc.y, lo, 64);
                    const uint32_t off = j - (__shfl(incl, lo, 64) - cnt);
                    ok[u] = j < tot;
                    at[u] = __shfl(pp, lo, 64) + off;
                    /* every shuffle outside the ok-branch: a shuffle under a
                     * partial exec mask reads garbage from inactive lanes */
                    const uint32_t src = __shfl(pc.x, lo, 64) + off;
                    kk[u] = ok[u] ? (uint32_t)keys[src] : 0u;
                }
#pragma unroll
                for (int u = 0; u < 4; u++) f.key(kk[u], ok[u], at[u]);
            }
        }
        } else {
            for (uint32_t q = tid; q < np; q += THREADS) {
                const uint32_t cnt = L.pn[q], src = L.ps[q], pq = pbase + L.ppre[q];
                for (uint32_t k0 = 0; k0 < cnt; k0 += 8) {
                    uint32_t kk[8];
#pragma unroll
                    for (int u = 0; u < 8; u++) kk[u] = (k0 + u < cnt) ? (uint32_t)keys[src + k0 + u] : 0u;
#pragma unroll
                    for (int u = 0; u < 8; u++) f.key(kk[u], k0 + u < cnt, pq + k0 + u);
                }
            }
        }
        if (sizeof(InT) == 4 && rc == it.r0) HM_STAMP(6);
        if (sizeof(InT) == 2 && rc == it.r0) HM_STAMP_M(5, 11);
        carry = pbase + L.ppre[np];
        __syncthreads();
    }
}

/* ------------------------------------------------------------------------ */
/* levels >= 2: stream a parent item's runs, counting sort by the next digit */
/* ------------------------------------------------------------------------ */

template <typename OutT>
__global__ __launch_bounds__(HM_PN_THREADS, 8) void k_partition(HmPartNArgs a)
{
    /* streamed keys in staged order, then the digit-sorted output (OutT);
     * words [HM_TN, HM_TN + 64) absorb the writes of idle lanes */
    __shared__ __attribute__((aligned(16))) uint32_t stage[HM_TN + 64];
    __shared__ uint32_t cur[HM_MAX_FN + 64];   /* + 64 dummy words (hm_lds_count) */
    __shared__ uint32_t scr[HM_PN_THREADS / 64 + 1];
    __shared__ unsigned long long scr64[HM_PN_THREADS / 64 + 1];
    __shared__ HmRunLds<512> L;
    HM_STAMP(0);
    const int tid = threadIdx.x;
    const int F = 1 << a.dbits;
    for (int i = tid; i < F; i += HM_PN_THREADS) cur[i] = 0;
    __syncthreads();
    HM_STAMP(1);
    if (hm_block_id() >= a.items) return;
    const HmItem it = hm_item(a.parent, hm_block_id());
    /* parent key: (row << sp) | col, sp = s + w bits each; digit = top w bits
     * of both, rest = low s bits of both.  Streaming re-encodes every key as
     * (digit << 2s) | rest (still <= 32 bits), so the scatter only shifts. */
    const int sw = a.restbits >> 1, ww = a.dbits >> 1, sp = sw + ww;
    const uint32_t restmask = (a.restbits >= 32) ? 0xFFFFFFFFu : ((1u << a.restbits) - 1u);
    struct {
        uint32_t* cur;
        uint32_t dummy;
        uint32_t* stage;
        int s, w, sp;
        __device__ __forceinline__ uint32_t pack(uint32_t k) const
        {
            const uint32_t r = k >> sp, c = k & ((1u << sp) - 1u), m = (1u << s) - 1u;
            const uint32_t d = ((r >> s) << w) | (c >> s);
            return (d << (2 * s)) | ((r & m) << s) | (c & m);
        }
        __device__ __forceinline__ void key(uint32_t k, bool v, uint32_t pos)
        {
            const uint32_t x = pack(k);
            hm_lds_count_m(cur, dummy, hm_cur_slot(x >> (2 * s), w), v);
            stage[v ? pos : HM_TN + hm_lane()] = x;
        }
        __device__ __forceinline__ void vec(const uint4& k, bool v, uint32_t pos)
        {
            const uint4 x = make_uint4(pack(k.x), pack(k.y), pack(k.z), pack(k.w));
            hm_lds_count_m(cur, dummy, hm_cur_slot(x.x >> (2 * s), w), v);
            hm_lds_count_m(cur, dummy, hm_cur_slot(x.y >> (2 * s), w), v);
            hm_lds_count_m(cur, dummy, hm_cur_slot(x.z >> (2 * s), w), v);
            hm_lds_count_m(cur, dummy, hm_cur_slot(x.w >> (2 * s), w), v);
            *(uint4*)&stage[v ? pos : HM_TN] = x;
        }
    } f{cur, HM_MAX_FN, stage, sw, ww, sp};
    HM_STAMP(2);
    hm_stream_runs<uint32_t, HM_PN_THREADS, 512, true>(it, a.keys_in, a.in, L, scr, f);
    HM_STAMP(7);
    const uint32_t total = it.b - it.a;
    constexpr int PER = HM_MAX_FN / HM_PN_THREADS;
    static_assert(HM_TN < (1 << (64 / PER)), "packed digit counts");
    uint32_t cnt[PER];
#pragma unroll
    for (int q = 0; q < PER; q++) {
        const int d = q * HM_PN_THREADS + tid;
        cnt[q] = d < F ? cur[hm_cur_slot(d, ww)] : 0u;
    }
    uint32_t offq[PER];
    hm_digit_offsets<HM_PN_THREADS, PER>(cnt, offq, scr64);
    HM_STAMP(8);
    const uint32_t tile0 = a.parent.item_begin[it.bucket];
    const uint32_t sh = it.j & ((1u << a.shard_bits) - 1u);
    const uint64_t cap = ((uint64_t)it.nitems + (1u << a.shard_bits) - 1) >> a.shard_bits;
    /* run-slot atomics are issued here and their results consumed only after
     * the scatter, so their latency hides behind it */
    uint32_t idx[PER];
#pragma unroll
    for (int q = 0; q < PER; q++) {
        const int d = q * HM_PN_THREADS + tid;
        idx[q] = 0;
        if (d < F && cnt[q])
            idx[q] = atomicAdd(&a.nruns_out[((((uint64_t)it.bucket << a.dbits) + d) << a.shard_bits) + sh], 1u);
    }
#pragma unroll
    for (int q = 0; q < PER; q++) {
        const int d = q * HM_PN_THREADS + tid;
        if (d < F) cur[hm_cur_slot(d, ww)] = offq[q];
    }
    constexpr int KPT = HM_TN / HM_PN_THREADS;
    uint32_t kv[KPT];
#pragma unroll
    for (int k = 0; k < KPT; k++) {
        const uint32_t i = k * HM_PN_THREADS + tid;
        kv[k] = i < total ? stage[i] : 0u;
    }
    __syncthreads();
    HM_STAMP(9);
    OutT* so = (OutT*)stage;
    /* claim: every slot atomic issued before any result is consumed (the
     * helper's logic of hm_lds_claim, unrolled over the KPT keys) */
    {
        uint32_t old[KPT];
        HmMerge g[KPT];
        bool v[KPT];
#pragma unroll
        for (int k = 0; k < KPT; k++) {
            v[k] = k * HM_PN_THREADS + tid < total;
            g[k] = hm_merge_prep(hm_cur_slot(kv[k] >> a.restbits, ww), v[k], HM_MAX_FN);
            old[k] = atomicAdd(&cur[g[k].idx], g[k].inc);
        }
#pragma unroll
        for (int k = 0; k < KPT; k++)
            so[v[k] ? hm_merge_pos(g[k], old[k]) : HM_TN + tid % 64] = (OutT)(kv[k] & restmask);
    }
    __syncthreads();
    HM_STAMP(10);
    OutT* out = (OutT*)a.keys_out + it.a;
    for (uint32_t i = tid; i < total; i += HM_PN_THREADS) out[i] = so[i];
#pragma unroll
    for (int q = 0; q < PER; q++) {
        const int d = q * HM_PN_THREADS + tid;
        if (d < F && cnt[q]) {
            const uint64_t rb = hm_run_base(tile0, it.nitems, it.bucket, d, a.dbits, a.shard_bits);
            a.runs_out[rb + sh * cap + idx[q]] = make_uint2(it.a + offq[q], cnt[q]);
        }
    }
    HM_STAMP(11);
}

/* Level 2 from the level-1 regions: every parent item spans at most
 * HM_L1_SHARDS contiguous runs, so each thread loads its HM_FR_KPT keys
 * straight into registers (key i of the item at thread i % T) -- no LDS
 * staging of the streamed keys.  One returning LDS atomic per key gives both
 * the digit histogram and the key's rank within its digit; after the scan a
 * key's slot is offset[digit] + rank.  Small blocks (512 threads, ~34 KB of
 * LDS) so that 4 blocks share a CU and one block's loads overlap the others'
 * LDS phases.  Output contract identical to k_partition. */
template <typename OutT>
__global__ __launch_bounds__(HM_FR_THREADS, 8) void k_partition_fr(HmPartNArgs a)
{
    constexpr int T = HM_FR_THREADS;
    constexpr int KPT = HM_TN / T;
    constexpr int PER = HM_MAX_FN / T;
    __shared__ uint32_t cur[HM_MAX_FN + 64];   /* + 64 dummy words */
    constexpr uint32_t V = 16 / sizeof(OutT);   /* keys per 16-B vector */
    /* key e of the item at stage[sh + e], sh = it.a mod V: the copy-out then
     * moves 16-B vectors aligned on both sides */
    __shared__ __attribute__((aligned(16))) OutT stage[HM_TN + 64 + V];
    __shared__ unsigned long long scr[T / 64 + 1];
    const int tid = threadIdx.x;
    const int F = 1 << a.dbits;
    const uint32_t g = hm_block_id();
    if (g >= a.items) return;
    HM_STAMP_M(3, 0);
    const HmItem it = hm_item(a.parent, g);
    /* the item's runs (<= HM_L1_SHARDS, block-uniform): logical start and
     * source index of each, from k_items' per-item table -- one 64-B load
     * next to the descriptor's, not a chain of dependent loads */
    const uint4* sg = (const uint4*)(a.seg + 16 * (size_t)g);
    const uint4 s0 = sg[0], s1 = sg[1], s2 = sg[2], s3 = sg[3];
    const uint32_t rpos[HM_L1_SHARDS] = {s0.x, s0.z, s1.x, s1.z, s2.x, s2.z, s3.x, s3.z};
    const uint32_t rsrc[HM_L1_SHARDS] = {s0.y, s0.w, s1.y, s1.w, s2.y, s2.w, s3.y, s3.w};
    const uint32_t nr = min(it.r1 - it.r0, (uint32_t)HM_L1_SHARDS);
    const uint32_t total = it.b - it.a;
    uint32_t kv[KPT];
#pragma unroll
    for (int k = 0; k < KPT; k++) {
        const uint32_t i = (uint32_t)(k * T + tid);
        const uint32_t p = it.a + i;
        uint32_t src = rsrc[0] + (p - rpos[0]);
#pragma unroll
        for (int j = 1; j < HM_L1_SHARDS; j++)
            src = ((uint32_t)j < nr && rpos[j] <= p) ? rsrc[j] + (p - rpos[j]) : src;
        kv[k] = i < total ? a.keys_in[src] : 0u;
    }
    for (int i = tid; i < F; i += T) cur[i] = 0;
    __syncthreads();
    HM_STAMP_M(3, 1);
    const int sw = a.restbits >> 1, ww = a.dbits >> 1, sp = sw + ww;
    const uint32_t m = (1u << sw) - 1u;
    /* re-encode each key as (digit slot << 2s) | rest (the slot: the digit's
     * hm_cur_slot, a bijection), then count and rank */
    uint32_t rank[KPT];
    const uint32_t dummy = HM_MAX_FN + (uint32_t)hm_lane();
    /* HM_FR_GROUP atomics in flight per thread (more costs registers) */
#pragma unroll
    for (int k0 = 0; k0 < KPT; k0 += HM_FR_GROUP) {
        HmClaim gm[HM_FR_GROUP];
        uint32_t old[HM_FR_GROUP];
#pragma unroll
        for (int u = 0; u < HM_FR_GROUP; u++) {
            const int k = k0 + u;
            const uint32_t r = kv[k] >> sp, c = kv[k] & ((1u << sp) - 1u);
            const uint32_t ds = hm_cur_slot(((r >> sw) << ww) | (c >> sw), ww);
            kv[k] = (ds << (2 * sw)) | ((r & m) << sw) | (c & m);
            const bool v = (uint32_t)(k * T + tid) < total;
            gm[u] = hm_claim_prep(ds, v, dummy);
            old[u] = atomicAdd(&cur[gm[u].idx], gm[u].inc);
        }
#pragma unroll
        for (int u = 0; u < HM_FR_GROUP; u++) rank[k0 + u] = hm_claim_pos(gm[u], old[u]);
    }
    HM_STAMP_M(3, 2);
    __syncthreads();
    HM_STAMP_M(3, 3);
    static_assert(HM_TN < (1 << (64 / PER)), "packed digit counts");
    uint32_t cnt[PER];
#pragma unroll
    for (int q = 0; q < PER; q++) {
        const int d = q * T + tid;
        cnt[q] = d < F ? cur[hm_cur_slot(d, ww)] : 0u;
    }
    if (a.mode == HM_PN_HIST) {
        /* the bucket's child totals (a pass before the partition proper) */
#pragma unroll
        for (int q = 0; q < PER; q++) {
            const int d = q * T + tid;
            if (d < F && cnt[q])
                atomicAdd(&a.ctot[((uint64_t)it.bucket << a.dbits) + d], (unsigned long long)cnt[q]);
        }
        return;
    }
    const bool contig = a.mode == HM_PN_CONTIG;
    uint32_t offq[PER];
    hm_digit_offsets<T, PER>(cnt, offq, scr);
    const uint32_t tile0 = a.parent.item_begin[it.bucket];
    const uint32_t sh = it.j & ((1u << a.shard_bits) - 1u);
    const uint64_t cap = ((uint64_t)it.nitems + (1u << a.shard_bits) - 1) >> a.shard_bits;
    /* lanes own consecutive digits: with one run counter per child
     * (shard_bits 0) a wave's run-slot atomics coalesce */
    uint32_t idx[PER];
#pragma unroll
    for (int q = 0; q < PER; q++) {
        const int d = q * T + tid;
        idx[q] = 0;
        if (d < F && cnt[q]) {
            const uint64_t child = ((uint64_t)it.bucket << a.dbits) + d;
            if (contig) {
                /* idx: the key position of this item's range of the child */
                idx[q] = a.cbase_off + (uint32_t)a.cbase[child] + atomicAdd(&a.ccur[child], cnt[q]);
                if (atomicCAS(&a.nruns_out[child], 0u, 1u) == 0u) {
                    const uint64_t rb = hm_run_base(tile0, it.nitems, it.bucket, d, a.dbits, 0);
                    a.runs_out[rb] = make_uint2(a.cbase_off + (uint32_t)a.cbase[child], (uint32_t)a.ctot[child]);
                }
            } else {
                idx[q] = atomicAdd(&a.nruns_out[(child << a.shard_bits) + sh], 1u);
            }
        }
    }
#pragma unroll
    for (int q = 0; q < PER; q++) {
        const int d = q * T + tid;
        if (d < F) cur[hm_cur_slot(d, ww)] = offq[q];
    }
    __syncthreads();
    HM_STAMP_M(3, 4);
    const uint32_t restmask = (a.restbits >= 32) ? 0xFFFFFFFFu : ((1u << a.restbits) - 1u);
    const uint32_t sh0 = contig ? 0u : it.a & (V - 1);
#pragma unroll
    for (int k = 0; k < KPT; k++) {
        const bool v = (uint32_t)(k * T + tid) < total;
        const uint32_t ds = kv[k] >> a.restbits;   /* digit slot */
        const uint32_t pos = v ? sh0 + cur[v ? ds : 0u] + rank[k] : (uint32_t)HM_TN + V + (uint32_t)(tid & 63);
        /* (a child-contiguous level stages the digit slot with the key: the
         * copy-out finds each key's destination from it) */
        stage[pos] = (OutT)(contig ? kv[k] : kv[k] & restmask);
    }
    __syncthreads();
    HM_STAMP_M(3, 5);
    if (contig) {
        /* a digit's keys [offq, offq + cnt) of the stage go to idx.. */
#pragma unroll
        for (int q = 0; q < PER; q++) {
            const int d = q * T + tid;
            if (d < F) cur[hm_cur_slot(d, ww)] = idx[q] - offq[q];
        }
        __syncthreads();
        OutT* out = (OutT*)a.keys_out;
        for (uint32_t e = tid; e < total; e += T) {
            const uint32_t x = (uint32_t)stage[e];
            out[cur[x >> a.restbits] + e] = (OutT)(x & restmask);
        }
        return;
    }
    {
        /* 16-B vectors [V t, V t + V) of stage map to out[it.a - sh0 + V t ..) */
        OutT* out = (OutT*)a.keys_out + (it.a - sh0);
        const uint32_t end = sh0 + total, nv = (end + V - 1) / V;
        for (uint32_t t = tid; t < nv; t += T) {
            const uint32_t e0 = t * V;
            if (e0 >= sh0 && e0 + V <= end) {
                *(uint4*)(out + e0) = *(const uint4*)(stage + e0);
            } else {
                for (uint32_t e = max(e0, sh0); e < min(e0 + V, end); e++) out[e] = stage[e];
            }
        }
    }
#pragma unroll
    for (int q = 0; q < PER; q++) {
        const int d = q * T + tid;
        if (d < F && cnt[q]) {
            const uint64_t rb = hm_run_base(tile0, it.nitems, it.bucket, d, a.dbits, a.shard_bits);
            a.runs_out[rb + sh * cap + idx[q]] = make_uint2(it.a + offq[q], cnt[q]);
        }
    }
    HM_STAMP_M(3, 6);
}

/* Child totals of a child-contiguous level (HM_PN_HIST): a block takes
 * HM_HIST_G consecutive items (items are in bucket order, so they mostly
 * share a bucket), counts their keys' children in LDS and adds each bucket's
 * non-zero counts once per block -- HM_HIST_G times fewer global atomics than
 * one flush per item. */
#define HM_HIST_G 8
__global__ __launch_bounds__(HM_FR_THREADS) void k_partition_hist(HmPartNArgs a)
{
    constexpr int T = HM_FR_THREADS;
    constexpr int KPT = HM_TN / T;
    __shared__ uint32_t cur[HM_MAX_FN];
    const int tid = threadIdx.x;
    const int F = 1 << a.dbits;
    const uint32_t g0 = hm_block_id() * HM_HIST_G;
    if (g0 >= a.items) return;
    const uint32_t g1 = min(g0 + HM_HIST_G, a.items);
    const int sw = a.restbits >> 1, ww = a.dbits >> 1, sp = sw + ww;
    for (int i = tid; i < F; i += T) cur[i] = 0;
    __syncthreads();
    uint32_t bucket = hm_item(a.parent, g0).bucket;
    for (uint32_t g = g0; g < g1; g++) {
        const HmItem it = hm_item(a.parent, g);   /* block-uniform */
        if (it.bucket != bucket) {
            /* flush the previous bucket's counts */
            __syncthreads();
            for (int d = tid; d < F; d += T) {
                const uint32_t c = cur[hm_cur_slot(d, ww)];
                if (c) atomicAdd(&a.ctot[((uint64_t)bucket << a.dbits) + d], (unsigned long long)c);
            }
            __syncthreads();
            for (int i = tid; i < F; i += T) cur[i] = 0;
            __syncthreads();
            bucket = it.bucket;
        }
        const uint4* sg = (const uint4*)(a.seg + 16 * (size_t)g);
        const uint4 s0 = sg[0], s1 = sg[1], s2 = sg[2], s3 = sg[3];
        const uint32_t rpos[HM_L1_SHARDS] = {s0.x, s0.z, s1.x, s1.z, s2.x, s2.z, s3.x, s3.z};
        const uint32_t rsrc[HM_L1_SHARDS] = {s0.y, s0.w, s1.y, s1.w, s2.y, s2.w, s3.y, s3.w};
        const uint32_t nr = min(it.r1 - it.r0, (uint32_t)HM_L1_SHARDS);
        const uint32_t total = it.b - it.a;
        uint32_t kv[KPT];
#pragma unroll
        for (int k = 0; k < KPT; k++) {
            const uint32_t i = (uint32_t)(k * T + tid);
            const uint32_t p = it.a + i;
            uint32_t src = rsrc[0] + (p - rpos[0]);
#pragma unroll
            for (int j = 1; j < HM_L1_SHARDS; j++)
                src = ((uint32_t)j < nr && rpos[j] <= p) ? rsrc[j] + (p - rpos[j]) : src;
            kv[k] = i < total ? a.keys_in[src] : 0u;
        }
#pragma unroll
        for (int k = 0; k < KPT; k++) {
            if ((uint32_t)(k * T + tid) < total) {
                const uint32_t r = kv[k] >> sp, c = kv[k] & ((1u << sp) - 1u);
                atomicAdd(&cur[hm_cur_slot(((r >> sw) << ww) | (c >> sw), ww)], 1u);
            }
        }
    }
    __syncthreads();
    for (int d = tid; d < F; d += T) {
        const uint32_t c = cur[hm_cur_slot(d, ww)];
        if (c) atomicAdd(&a.ctot[((uint64_t)bucket << a.dbits) + d], (unsigned long long)c);
    }
}

void hm_launch_partition_hist(hipStream_t s, const HmPartNArgs& a)
{
    const uint32_t blocks = (a.items + HM_HIST_G - 1) / HM_HIST_G;
    if (blocks) hipLaunchKernelGGL(k_partition_hist, hm_grid2(blocks), dim3(HM_FR_THREADS), 0, s, a);
}

/* ------------------------------------------------------------------------ */
/* run scan: sharded run counters -> one flat, child-ordered run list        */
/* ------------------------------------------------------------------------ */

/* per (child, shard) counter: exclusive offset within the child, and per
 * child its run total.  Lanes read consecutive counters (coalesced); a
 * child's S = 2^shard_bits shards are S consecutive lanes, scanned with
 * shuffles.  Every lane of a wave runs every step. */
__global__ __launch_bounds__(256) void k_rs_count(HmRsArgs a)
{
    const uint32_t S = 1u << a.shard_bits;
    const uint64_t npairs = a.nchildren << a.shard_bits;
    const uint64_t stride = (uint64_t)gridDim.x * 256;
    const uint32_t sl = (uint32_t)hm_lane() & (S - 1);
    for (uint64_t k = (uint64_t)blockIdx.x * 256 + threadIdx.x; k - (uint64_t)hm_lane() < npairs; k += stride) {
        const bool in = k < npairs;
        const uint32_t n = in ? a.nruns[k] : 0u;
        uint32_t v = n;
        for (uint32_t o = 1; o < S; o <<= 1) {
            const uint32_t t = __shfl_up(v, o, 64);
            if (sl >= o) v += t;
        }
        if (in) {
            a.shoff[k] = v - n;
            if (sl == S - 1) a.nr[k >> a.shard_bits] = v;
        }
    }
}

/* sharded run list of child c -> flat[runbase[c] .. + nr[c]), one wave per
 * child: lanes 0..S-1 hold the child's shards (count, flat offset, source),
 * and the wave copies the child's runs HM_RS_SLICE at a time, 8 loads per lane
 * in flight, each run's shard found by a shuffle search over the S lanes.
 * A child of more than a.big_min runs (HM_RS_BIG by default; one run per
 * parent work item: the hot tile of a skewed cloud has 10^5) is listed instead, and k_rs_copy_big
 * spreads its slices over every wave of the grid. */
#define HM_RS_SLICE 512
#ifndef HM_RS_LANE_MAX
#define HM_RS_LANE_MAX 256  /* children of at most this many runs: copied 64 / S at a time */
#endif

struct HmRsChild {
    uint32_t n, incl;
    uint64_t src;
};

/* lanes 0..S-1: shard counts and sources of child c (loads only) */
__device__ __forceinline__ HmRsChild hm_rs_child_load(const HmRsArgs& a, uint64_t c)
{
    const uint32_t S = 1u << a.shard_bits;
    const uint32_t lane = (uint32_t)hm_lane();
    const uint64_t k = (c << a.shard_bits) + lane;
    HmRsChild h;
    h.n = 0;
    h.src = 0;
    h.incl = 0;
    if (lane < S) {
        h.n = a.nruns[k];
        const uint64_t p = c >> a.dbits;
        const uint64_t d = c & ((1ull << a.dbits) - 1);
        const uint32_t t0 = a.parent_item_begin[p];
        const uint32_t tp = a.parent_item_begin[p + 1] - t0;
        const uint32_t cap = (tp + S - 1) >> a.shard_bits;
        h.src = hm_run_base(t0, tp, p, d, a.dbits, a.shard_bits) + (uint64_t)lane * cap;
    }
    return h;
}

__device__ __forceinline__ HmRsChild hm_rs_child(const HmRsArgs& a, uint64_t c)
{
    HmRsChild h = hm_rs_child_load(a, c);
    h.incl = hm_wave_incl_scan(h.n);   /* shard offsets within the child */
    return h;
}

/* runs j0 .. j0 + 64 U of the child (each lane's shard: a shuffle search) */
template <int U = HM_RS_SLICE / 64>
__device__ __forceinline__ void hm_rs_slice(const HmRsArgs& a, const HmRsChild& h, uint64_t nr, uint64_t rb,
                                            uint64_t j0)
{
    const uint32_t lane = (uint32_t)hm_lane();
    uint2 r[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
        const uint64_t x = j0 + (uint64_t)u * 64 + lane;
        const uint32_t xc = (uint32_t)min(x, nr - 1);
        uint32_t l = 0;
#pragma unroll
        for (int st = 32; st > 0; st >>= 1)
            if (__shfl(h.incl, l + st - 1, 64) <= xc) l += st;
        l = min(l, 63u);
        const uint32_t off = xc - (__shfl(h.incl, l, 64) - __shfl(h.n, l, 64));
        const uint64_t sj = __shfl(h.src, l, 64) + off;
        r[u] = x < nr ? a.runs[sj] : make_uint2(0, 0);
    }
#pragma unroll
    for (int u = 0; u < U; u++) {
        const uint64_t x = j0 + (uint64_t)u * 64 + lane;
        if (x < nr) {
            a.flat[rb + x] = r[u];
            a.cnt[rb + x] = r[u].y;
        }
    }
}

/* a wave takes 64 consecutive children at a time: their run counts and
 * bases in one lane-per-child load, then the non-empty ones in turn (most
 * children of a sparse level are empty or hold a few runs: the per-child
 * chain of dependent loads is what this kernel waits on) */
__global__ __launch_bounds__(256) void k_rs_copy(HmRsArgs a)
{
    const uint64_t nw = (uint64_t)gridDim.x * 4;
    const uint32_t lane = (uint32_t)hm_lane();
    for (uint64_t c0 = ((uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * 64; c0 < a.nchildren; c0 += nw * 64) {
        const uint64_t cl = c0 + lane;
        const uint64_t nrl = cl < a.nchildren ? a.nr[cl] : 0ull;
        const uint64_t rbl = nrl ? a.runbase[cl] : 0ull;
        /* the copied children in order; the next one's shard table loads
         * are issued before the current one's run copy */
        uint64_t m = __ballot((nrl != 0) & (nrl <= a.big_min));
        uint64_t mb = __ballot(nrl > a.big_min);
        while (mb) {
            const int i = __builtin_ctzll(mb);
            mb &= mb - 1;
            uint32_t slot = 0;
            if (lane == 0) slot = atomicAdd(a.nbig, 1u);
            slot = __shfl(slot, 0, 64);
            if (slot < HM_RS_BIG_MAX) {
                if (lane == 0) a.big[slot] = (uint32_t)(c0 + (uint64_t)i);
            } else {
                m |= 1ull << i;   /* list full: copied here */
            }
        }
        {
            /* children of <= HM_RS_LANE_MAX runs (not big, not hot) are copied
             * 64 / S at a time, one (child, shard) per lane: a shard's runs
             * are one contiguous source range, a child's one contiguous flat
             * range, so element x of the group's concatenation finds its
             * (child, shard) by a search over the lanes' inclusive run counts;
             * consecutive children have adjacent flat ranges, so the stores
             * coalesce (one child at a time left the wave waiting on each
             * child's chain of dependent loads) */
            const uint32_t S = 1u << a.shard_bits, G = 64u / S;   /* (shard_bits <= 6, as below) */
            const bool mine_l = ((m >> lane) & 1ull) && nrl <= HM_RS_LANE_MAX && G > 0;
            const uint64_t mineb = __ballot(mine_l);
            m &= ~mineb;
            const uint64_t gmask = G >= 64 ? ~0ull : ((1ull << G) - 1ull);
            for (uint32_t g0 = 0; mineb && g0 < 64; g0 += G) {
                if (!((mineb >> g0) & gmask)) continue;   /* wave-uniform */
                const uint32_t ci = g0 + lane / S, sh = lane & (S - 1u);
                const bool cm = (mineb >> ci) & 1ull;
                const uint64_t rbc = __shfl(rbl, (int)ci, 64);
                uint32_t n = 0;
                uint64_t src = 0;
                if (cm) {
                    const uint64_t c = c0 + ci;
                    n = a.nruns[(c << a.shard_bits) + sh];   /* 0 for a hot tile (k_hot_runs lists its runs) */
                    const uint64_t p = c >> a.dbits, d = c & ((1ull << a.dbits) - 1);
                    const uint32_t t0 = a.parent_item_begin[p];
                    const uint32_t tp = a.parent_item_begin[p + 1] - t0;
                    const uint64_t cap = ((uint64_t)tp + S - 1) >> a.shard_bits;
                    src = hm_run_base(t0, tp, p, d, a.dbits, a.shard_bits) + (uint64_t)sh * cap;
                }
                const uint32_t incl = hm_wave_incl_scan(n);
                const int fl = (int)(lane & ~(S - 1u));   /* the child's first lane */
                const uint32_t cfirst = __shfl(incl, fl, 64) - __shfl(n, fl, 64);
                const uint64_t dst = rbc + (incl - n - cfirst);
                const uint32_t tot = __shfl(incl, 63, 64);
                for (uint32_t x0 = 0; x0 < tot; x0 += 64) {
                    const uint32_t x = x0 + lane;
                    const uint32_t xc = min(x, tot - 1u);
                    uint32_t l = 0;
#pragma unroll
                    for (int st = 32; st > 0; st >>= 1)
                        if (__shfl(incl, (int)(l + st - 1), 64) <= xc) l += st;
                    l = min(l, 63u);
                    const uint32_t j = xc - (__shfl(incl, (int)l, 64) - __shfl(n, (int)l, 64));
                    const uint64_t sj = __shfl(src, (int)l, 64) + j, dj = __shfl(dst, (int)l, 64) + j;
                    if (x < tot) {
                        const uint2 r = a.runs[sj];
                        a.flat[dj] = r;
                        a.cnt[dj] = r.y;
                    }
                }
            }
        }
        if (!m) continue;
        int i = __builtin_ctzll(m);
        m &= m - 1;
        HmRsChild h = hm_rs_child_load(a, c0 + (uint64_t)i);
        for (;;) {
            const int inext = m ? __builtin_ctzll(m) : -1;
            HmRsChild hn;
            if (inext >= 0) {
                m &= m - 1;
                hn = hm_rs_child_load(a, c0 + (uint64_t)inext);
            }
            h.incl = hm_wave_incl_scan(h.n);
            const uint64_t nr = __shfl(nrl, i, 64);
            const uint64_t rb = __shfl(rbl, i, 64);
            /* a sparse level's children hold a few runs: one 64-run step;
             * a hot tile has runs but no sharded ones (k_hot_runs lists them) */
            if (__shfl(h.incl, 63, 64) == 0)
                ;
            else if (nr <= 64)
                hm_rs_slice<1>(a, h, nr, rb, 0);
            else if (nr <= 256)
                hm_rs_slice<4>(a, h, nr, rb, 0);
            else
                for (uint64_t j0 = 0; j0 < nr; j0 += HM_RS_SLICE) hm_rs_slice(a, h, nr, rb, j0);
            if (inext < 0) break;
            i = inext;
            h = hn;
        }
    }
}

/* the listed children: wave w copies slices w, w + waves, ... of each */
__global__ __launch_bounds__(256) void k_rs_copy_big(HmRsArgs a)
{
    const uint32_t nb = min(*a.nbig, (uint32_t)HM_RS_BIG_MAX);
    const uint64_t nw = (uint64_t)gridDim.x * 4;
    const uint64_t w = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const uint32_t lane = (uint32_t)hm_lane();
    for (uint32_t e0 = 0; e0 < nb; e0 += 64) {
        /* 64 listed children per lane-parallel load */
        const bool in = e0 + lane < nb;
        const uint32_t cl = in ? a.big[e0 + lane] : 0u;
        const uint64_t nrl = in ? a.nr[cl] : 0ull;
        const uint64_t rbl = in ? a.runbase[cl] : 0ull;
        const uint32_t ne = min(64u, nb - e0);
        for (uint32_t j = 0; j < ne; j++) {
            const uint64_t nr = __shfl(nrl, (int)j, 64);
            /* rotate the starting wave per child so short tails spread out */
            const uint64_t w0 = (w + (uint64_t)(e0 + j) * 97) % nw;
            if (w0 * HM_RS_SLICE >= nr) continue;
            const uint64_t c = __shfl(cl, (int)j, 64);
            const uint64_t rb = __shfl(rbl, (int)j, 64);
            const HmRsChild h = hm_rs_child(a, c);
            for (uint64_t j0 = w0 * HM_RS_SLICE; j0 < nr; j0 += nw * HM_RS_SLICE) hm_rs_slice(a, h, nr, rb, j0);
        }
    }
}

/* per child: global key range of its runs and work items of the next stage */
__global__ __launch_bounds__(256) void k_rs_keys(HmRsArgs a)
{
    const uint64_t stride = (uint64_t)gridDim.x * 256;
    for (uint64_t c = (uint64_t)blockIdx.x * 256 + threadIdx.x; c < a.nchildren; c += stride) {
        const uint64_t nr = a.nr[c];
        if (nr == 0) {
            a.nkeys[c] = 0;
            a.keybase[c] = 0;
            /* a forced child is a bucket without keys or items (a hot tile's
             * ancestor: the tile joins it as a child one level down) */
            a.vals[c] = (a.force && a.force[c]) ? (1ull << 32) : 0ull;
            continue;
        }
        const uint64_t rb = a.runbase[c];
        const uint64_t kb = a.excl[rb];
        const uint64_t nflat = a.nflat_dev ? *a.nflat_dev : a.nflat;
        const uint64_t ke = (rb + nr < nflat) ? a.excl[rb + nr] : *a.total_keys;
        const uint32_t nk = (uint32_t)(ke - kb);
        a.nkeys[c] = nk;
        a.keybase[c] = (uint32_t)kb;
        /* last level: buckets of <= HM_SP_MAX keys get no dense work items
         * (one wavefront each: k_small_sort / k_small_emit) */
        const uint32_t nit = nk <= a.sparse_max ? 0u : (nk + a.item_keys - 1) / a.item_keys;
        a.vals[c] = (1ull << 32) | (uint64_t)nit;
    }
}

/* Hot tiles as level-2 children: child (bucket of its z1 digit, its digit
 * below it); its runs are its non-empty level-1 region shards, whose keys K1
 * wrote in the final (u16) form into the level-2 key array.  k_hot_nr sets
 * the children's run counts before the run scan, k_hot_runs lists the runs at
 * their flat positions after it (k_rs_copy skips the children). */
__device__ __forceinline__ uint64_t hm_hot_parent(const HmHotRunArgs& a, uint32_t tr, uint32_t tc, int* s)
{
    const int s1 = a.zb - a.z1;
    uint64_t p = a.d2b[((tr >> s1) << a.z1) | (tc >> s1)];   /* the z1 bucket */
    *s = s1;
    if (a.c2b) {
        /* level 3: the zoom-zp ancestor's bucket among the z1 bucket's children */
        const int sp = a.zb - a.zp, w = a.zp - a.z1;
        const uint32_t m = (1u << w) - 1u;
        p = a.c2b[(p << (2 * w)) | (((tr >> sp) & m) << w) | ((tc >> sp) & m)];
        *s = sp;
    }
    return p;
}

/* the last-level child index of hot tile t */
__device__ __forceinline__ uint64_t hm_hot_child(const HmHotRunArgs& a, uint32_t t)
{
    const uint32_t tr = t >> a.zb, tc = t & ((1u << a.zb) - 1u);
    int s;
    const uint64_t p = hm_hot_parent(a, tr, tc, &s);
    const uint32_t m = (1u << s) - 1u;
    return (p << a.dbits) | (((tr & m) << s) | (tc & m));
}

/* 3-level plan: flag each hot tile's zoom-zp ancestor among the level-2
 * children (child = z1 bucket << dbits | ancestor digit), so it stays a bucket */
__global__ __launch_bounds__(256) void k_hot_force(HmHotRunArgs a, uint8_t* force)
{
    const uint32_t H = *a.n;
    for (uint32_t h = blockIdx.x * 256 + threadIdx.x; h < H; h += gridDim.x * 256) {
        const uint32_t t = a.tiles[h];
        const uint32_t tr = t >> a.zb, tc = t & ((1u << a.zb) - 1u);
        const int s1 = a.zb - a.z1, sp = a.zb - a.zp, w = a.zp - a.z1;
        const uint64_t p = a.d2b[((tr >> s1) << a.z1) | (tc >> s1)];
        const uint32_t m = (1u << w) - 1u;
        force[(p << a.dbits) | (((tr >> sp) & m) << w) | ((tc >> sp) & m)] = 1;
    }
}

__global__ __launch_bounds__(256) void k_hot_nr(HmHotRunArgs a)
{
    const uint32_t H = *a.n;
    for (uint32_t h = blockIdx.x * 256 + threadIdx.x; h < H; h += gridDim.x * 256) {
        uint32_t nr = 0;
#pragma unroll
        for (int sh = 0; sh < HM_L1_SHARDS; sh++) nr += a.fill[hm_l1i(HM_MAX_F1 + h, sh)] != 0;
        if (nr) a.nr[hm_hot_child(a, a.tiles[h])] = nr;
    }
}

__global__ __launch_bounds__(256) void k_hot_runs(HmHotRunArgs a)
{
    const uint32_t H = *a.n;
    for (uint32_t h = blockIdx.x * 256 + threadIdx.x; h < H; h += gridDim.x * 256) {
        uint64_t j = 0;
        bool any = false;
#pragma unroll
        for (int sh = 0; sh < HM_L1_SHARDS; sh++) any |= a.fill[hm_l1i(HM_MAX_F1 + h, sh)] != 0;
        if (!any) continue;
        const uint64_t rb = a.runbase[hm_hot_child(a, a.tiles[h])];
#pragma unroll
        for (int sh = 0; sh < HM_L1_SHARDS; sh++) {
            const uint32_t k = hm_l1i(HM_MAX_F1 + h, sh);
            const uint32_t f = a.fill[k];
            if (f) {
                a.flat[rb + j] = make_uint2(a.rbase[k], f);
                a.cnt[rb + j] = f;
                j++;
            }
        }
    }
}

void hm_launch_hot_force(hipStream_t s, const HmHotRunArgs& a, uint8_t* force)
{
    hipLaunchKernelGGL(k_hot_force, dim3(HM_MAX_HOT / 256), dim3(256), 0, s, a, force);
}

void hm_launch_hot_nr(hipStream_t s, const HmHotRunArgs& a)
{
    hipLaunchKernelGGL(k_hot_nr, dim3(HM_MAX_HOT / 256), dim3(256), 0, s, a);
}

void hm_launch_hot_runs(hipStream_t s, const HmHotRunArgs& a)
{
    hipLaunchKernelGGL(k_hot_runs, dim3(HM_MAX_HOT / 256), dim3(256), 0, s, a);
}

/* ------------------------------------------------------------------------ */
/* device-wide exclusive scan of u64 (any length)                            */
/* ------------------------------------------------------------------------ */

#define HM_SCAN_ITEMS 4096
#define HM_SCAN_THREADS 256
#define HM_SCAN_MAXB 4096

__global__ __launch_bounds__(HM_SCAN_THREADS) void k_scan_reduce(const uint64_t* v, uint64_t n, uint64_t chunk,
                                                                 uint64_t* partial, const uint64_t* ndev)
{
    __shared__ uint64_t red[HM_SCAN_THREADS / 64];
    if (ndev) n = min(n, *ndev);   /* the live length, read on the device */
    const uint64_t b0 = (uint64_t)blockIdx.x * chunk;
    const uint64_t b1 = min(b0 + chunk, n);
    uint64_t s = 0;
    for (uint64_t i = b0 + threadIdx.x; i < b1; i += HM_SCAN_THREADS) s += v[i];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
    if (hm_lane() == 0) red[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint64_t t = 0;
        for (int w = 0; w < HM_SCAN_THREADS / 64; w++) t += red[w];
        partial[blockIdx.x] = t;
    }
}

/* single block: exclusive scan of up to 1024 * PER values v -> out (may be
 * v itself: a thread reads its PER values before writing them); total ->
 * *total.  PER = 4: the partials of a multi-block scan; PER = 16: a whole
 * scan of <= 16384 values in one dispatch (small calls are dispatch-bound). */
template <int PER>
__global__ __launch_bounds__(1024) void k_scan_one(const uint64_t* v, uint32_t n, uint64_t* out, uint64_t* total,
                                                   const uint64_t* ndev)
{
    __shared__ uint64_t ws[17];
    if (ndev) n = (uint32_t)min((uint64_t)n, *ndev);
    const int tid = threadIdx.x;
    uint64_t x[PER];
    uint64_t s = 0;
#pragma unroll
    for (int q = 0; q < PER; q++) {
        const uint32_t i = tid * PER + q;
        x[q] = i < n ? v[i] : 0;
        s += x[q];
    }
    const uint64_t inc = hm_wave_incl_scan64(s);
    const int w = tid >> 6;
    if (hm_lane() == 63) ws[w] = inc;
    __syncthreads();
    if (tid == 0) {
        uint64_t acc = 0;
        for (int k = 0; k < 16; k++) {
            const uint64_t t = ws[k];
            ws[k] = acc;
            acc += t;
        }
        ws[16] = acc;
    }
    __syncthreads();
    uint64_t off = ws[w] + inc - s;
#pragma unroll
    for (int q = 0; q < PER; q++) {
        const uint32_t i = tid * PER + q;
        if (i < n) out[i] = off;
        off += x[q];
    }
    if (tid == 0) *total = ws[16];
}

/* block b: its chunk in sub-chunks of HM_SCAN_ITEMS, carrying the prefix.
 * The sub-chunk passes through LDS both ways (padded one word per 16), so
 * global loads and stores are lane-consecutive while each thread scans 16
 * consecutive values.  SUM (grids of <= HM_SCAN_THREADS blocks): the block
 * sums the partials before it itself, and the last block writes the total --
 * no k_scan_one dispatch between the two passes */
#define HM_SCAN_PAD(i) ((i) + ((i) >> 4))
template <bool SUM>
__global__ __launch_bounds__(HM_SCAN_THREADS) void k_scan_down(const uint64_t* v, uint64_t n, uint64_t chunk,
                                                               const uint64_t* partial, uint64_t* out,
                                                               const uint64_t* ndev, uint64_t* total)
{
    __shared__ uint64_t ws[HM_SCAN_THREADS / 64 + 1];
    __shared__ uint64_t buf[HM_SCAN_PAD(HM_SCAN_ITEMS)];
    if (ndev) n = min(n, *ndev);
    constexpr int PER = HM_SCAN_ITEMS / HM_SCAN_THREADS;
    const uint32_t tid = threadIdx.x;
    const uint64_t c0 = (uint64_t)blockIdx.x * chunk;
    const uint64_t c1 = min(c0 + chunk, n);
    uint64_t carry;
    if (SUM) {
        uint64_t p = tid < blockIdx.x ? partial[tid] : 0ull;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) p += __shfl_xor(p, o, 64);
        if (hm_lane() == 0) ws[tid >> 6] = p;
        __syncthreads();
        carry = 0;
#pragma unroll
        for (int k = 0; k < HM_SCAN_THREADS / 64; k++) carry += ws[k];
        __syncthreads();
    } else {
        carry = partial[blockIdx.x];
    }
    for (uint64_t s0 = c0; s0 < c1; s0 += HM_SCAN_ITEMS) {
        const uint64_t m = min<uint64_t>(c1 - s0, HM_SCAN_ITEMS);
#pragma unroll
        for (int q = 0; q < PER; q++) {
            const uint32_t i = (uint32_t)q * HM_SCAN_THREADS + tid;
            buf[HM_SCAN_PAD(i)] = i < m ? v[s0 + i] : 0ull;
        }
        __syncthreads();
        uint64_t x[PER];
        uint64_t s = 0;
#pragma unroll
        for (int q = 0; q < PER; q++) {
            x[q] = buf[HM_SCAN_PAD(tid * PER + q)];
            s += x[q];
        }
        const uint64_t inc = hm_wave_incl_scan64(s);
        const int w = tid >> 6;
        if (hm_lane() == 63) ws[w] = inc;
        __syncthreads();
        if (tid == 0) {
            uint64_t acc = 0;
            for (int k = 0; k < HM_SCAN_THREADS / 64; k++) {
                const uint64_t t = ws[k];
                ws[k] = acc;
                acc += t;
            }
            ws[HM_SCAN_THREADS / 64] = acc;
        }
        __syncthreads();
        uint64_t off = carry + ws[w] + inc - s;
#pragma unroll
        for (int q = 0; q < PER; q++) {
            buf[HM_SCAN_PAD(tid * PER + q)] = off;
            off += x[q];
        }
        carry += ws[HM_SCAN_THREADS / 64];
        __syncthreads();
#pragma unroll
        for (int q = 0; q < PER; q++) {
            const uint32_t i = (uint32_t)q * HM_SCAN_THREADS + tid;
            if (i < m) out[s0 + i] = buf[HM_SCAN_PAD(i)];
        }
        __syncthreads();
    }
    if (SUM && blockIdx.x == gridDim.x - 1 && tid == 0) *total = carry;
}

/* compaction of non-empty children into the bucket list B_l (parent-major) */
__global__ __launch_bounds__(256) void k_compact(HmCompactArgs a)
{
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    const uint64_t F = 1ull << a.dbits;
    const uint32_t count = (uint32_t)(*a.total >> 32);
    const uint32_t items = (uint32_t)(*a.total & 0xFFFFFFFFull);
    for (uint64_t c = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; c < a.nchildren; c += stride) {
        const uint64_t pre = a.prefix[c];
        const uint32_t idx = (uint32_t)(pre >> 32);
        const uint32_t ib = (uint32_t)(pre & 0xFFFFFFFFull);
        const uint64_t p = c >> a.dbits;
        const uint64_t d = c & (F - 1);
        if (d == 0) a.child_begin[p] = idx;
        if (a.vals[c] >> 32) {
            if (a.c2b) a.c2b[c] = idx;
            a.out.nkeys[idx] = a.nkeys[c];
            a.out.nruns[idx] = (uint32_t)a.nr[c];
            a.out.rbase[idx] = (uint32_t)a.runbase[c];
            a.out.keybase[idx] = a.keybase[c];
            a.out.item_begin[idx] = ib;
            a.out.digit[idx] = (uint32_t)d;
            const uint64_t pc = a.parent_coord[p];
            const int wd = a.dbits >> 1;
            const uint64_t rr = ((pc >> 32) << wd) | (d >> wd);
            const uint64_t cc = ((pc & 0xFFFFFFFFull) << wd) | (d & ((1ull << wd) - 1));
            a.out.coord[idx] = (rr << 32) | cc;
            if (a.slots) {
                const uint32_t nit = (uint32_t)(a.vals[c] & 0xFFFFFFFFull);
                int32_t sl = -1;
                if (nit > 1) {
                    sl = (int32_t)atomicAdd(a.nslots, 1ull);
                    a.slot_bucket[sl] = idx;
                }
                a.slots[idx] = sl;
            }
        }
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        a.out.item_begin[count] = items;
        a.child_begin[a.nparents] = count;
    }
}
/* ------------------------------------------------------------------------ */
/* emission helpers                                                          */
/* ------------------------------------------------------------------------ */

/* Emit the non-zero cells v[0..n) of zoom z: the row-major (2^lg)^2 block
 * whose corner tile at zoom z - lg is `prefix` (a coord).  All threads of the
 * block must call. */
template <typename T, int THREADS>
__device__ void hm_emit_level(const T* v, uint32_t n, int z, uint64_t prefix, int lg, const HmOut& o,
                              uint32_t* scr, unsigned long long* sbase)
{
    const uint32_t per = (n + THREADS - 1) / THREADS;
    const uint32_t i0 = threadIdx.x * per;
    const uint32_t i1 = min(i0 + per, n);
    uint32_t c = 0;
    for (uint32_t i = i0; i < i1; i++) c += v[i] != 0;
    uint32_t tot;
    uint32_t off = hm_block_excl_scan<THREADS>(c, scr, &tot);
    if (tot == 0) return;
    if (threadIdx.x == 0) *sbase = atomicAdd(o.cursor, (unsigned long long)tot);
    __syncthreads();
    const uint64_t base = *sbase;
    __syncthreads();
    for (uint32_t i = i0; i < i1; i++) {
        const T x = v[i];
        if (x != 0) {
            const uint64_t pos = base + off;
            if (pos < o.capacity) {
                o.keys[pos] = hm_cell_key(z, prefix, lg, i);
                o.counts[pos] = (uint64_t)x;
            }
            off++;
        }
    }
}

/* In-LDS 4:1 pyramid over the row-major v[0..4^lg): emits zooms z_top ..
 * z_top-lg+1 (those in [zmin, zmax]) and leaves the total in v[0]. */
template <typename T, int THREADS>
__device__ void hm_pyramid(T* v, int lg, int z_top, uint64_t prefix, const HmOut& o, uint32_t* scr,
                           unsigned long long* sbase)
{
    uint32_t n = 1u << (2 * lg);
    for (int k = 0; k < lg; k++) {
        const int z = z_top - k;
        if (z >= o.zmin && z <= o.zmax) hm_emit_level<T, THREADS>(v, n, z, prefix, lg - k, o, scr, sbase);
        __syncthreads();
        n >>= 2;
        constexpr int MAXPER = (HM_AG_CELLS / 4 + THREADS - 1) / THREADS;
        T acc[MAXPER];
#pragma unroll
        for (int m = 0; m < MAXPER; m++) {
            const uint32_t i = threadIdx.x + m * THREADS;
            acc[m] = i < n ? hm_sum4<T>(v, i, lg - k - 1) : (T)0;
        }
        __syncthreads();
#pragma unroll
        for (int m = 0; m < MAXPER; m++) {
            const uint32_t i = threadIdx.x + m * THREADS;
            if (i < n) v[i] = acc[m];
        }
        __syncthreads();
    }
}

/* Emit the non-empty cells i in [0, n) of v (cells with zoom outside [zmin,
 * zmax] skipped) with ONE output reservation per block, coalesced: wave w
 * takes the 64-cell chunks w, w + NW, ...; a chunk's non-empty cells go to
 * consecutive output positions (ballot + mbcnt), so one store instruction
 * writes one contiguous run of keys and one of counts.  cell(i) -> (zoom,
 * key) of cell i; the cells may be written in any order.  Every thread of
 * the block must call. */
template <int THREADS, typename CellF>
__device__ void hm_emit_cells(const uint32_t* v, uint32_t n, CellF cell, const HmOut& o, uint32_t* scr,
                              unsigned long long* sbase)
{
    constexpr int NW = THREADS / 64;
    const int lane = hm_lane(), w = threadIdx.x >> 6;
    uint32_t c = 0;
    for (uint32_t i0 = (uint32_t)w * 64; i0 < n; i0 += NW * 64) {
        const uint32_t i = i0 + lane;
        int z = 0;
        uint64_t k = 0;
        if (i < n) cell(i, z, k);
        const bool nz = i < n && v[i] != 0 && z >= o.zmin && z <= o.zmax;
        c += (uint32_t)__builtin_popcountll(__builtin_amdgcn_ballot_w64(nz));
    }
    if (lane == 0) scr[w] = c;
    __syncthreads();
    if (w == 0) {
        const uint32_t x = lane < NW ? scr[lane] : 0u;
        const uint32_t incl = hm_wave_incl_scan(x);
        if (lane < NW) scr[lane] = incl - x;
        if (lane == NW - 1) *sbase = incl ? atomicAdd(o.cursor, (unsigned long long)incl) : 0ull;
    }
    __syncthreads();
    uint64_t base = *sbase + scr[w];
    __syncthreads();
    for (uint32_t i0 = (uint32_t)w * 64; i0 < n; i0 += NW * 64) {
        const uint32_t i = i0 + lane;
        int z = 0;
        uint64_t k = 0;
        uint32_t x = 0;
        if (i < n) {
            cell(i, z, k);
            x = v[i];
        }
        const bool nz = x != 0 && z >= o.zmin && z <= o.zmax;
        const uint64_t m = __builtin_amdgcn_ballot_w64(nz);
        const uint64_t pos = base + hm_mbcnt(m);
        if (nz && pos < o.capacity) {
            o.keys[pos] = k;
            o.counts[pos] = x;
        }
        base += (uint32_t)__builtin_popcountll(m);
    }
}

/* Bucket pyramid with two output reservations per block: level z_top (4^lg
 * cells in v) is emitted first; then levels z_top-1 .. z_top-lg+1 are built as
 * consecutive regions of v (the first in place), counted together, reserved
 * with one atomic and emitted.  v[0] ends up holding nothing useful; the
 * bucket total is returned (block-uniform). */
template <int THREADS>
__device__ uint64_t hm_bucket_pyramid(uint32_t* v, int lg, int z_top, uint64_t prefix, const HmOut& o,
                                      uint32_t* scr, unsigned long long* sbase)
{
    const uint32_t n0 = 1u << (2 * lg);
    if (lg == 0) return v[0];   /* the bucket is the zoom-z_top cell; k_pool emits it */
    hm_emit_cells<THREADS>(v, n0, [&](uint32_t i, int& z, uint64_t& k) {
        z = z_top;
        k = hm_cell_key(z_top, prefix, lg, i);
    }, o, scr, sbase);
    __syncthreads();
    /* level z_top-1 in place into v[0 .. n0/4) */
    uint32_t n = n0 >> 2;
    {
        constexpr int MAXPER = (HM_AG_CELLS / 4 + THREADS - 1) / THREADS;
        uint32_t acc[MAXPER];
#pragma unroll
        for (int m = 0; m < MAXPER; m++) {
            const uint32_t i = threadIdx.x + m * THREADS;
            acc[m] = i < n ? hm_sum4<uint32_t>(v, i, lg - 1) : 0u;
        }
        __syncthreads();
#pragma unroll
        for (int m = 0; m < MAXPER; m++) {
            const uint32_t i = threadIdx.x + m * THREADS;
            if (i < n) v[i] = acc[m];
        }
        __syncthreads();
    }
    /* remaining levels appended: level k (k = 1 .. lg-1) at off[k], 4^(lg-k) cells */
    uint32_t off[HM_AG_LG + 1];
    off[1] = 0;
    uint32_t end = n;
    for (int k = 2; k <= lg; k++) {
        const uint32_t src = off[k - 1];
        const uint32_t m = n >> 2;
        off[k] = end;
        for (uint32_t i = threadIdx.x; i < m; i += THREADS)
            v[end + i] = hm_sum4<uint32_t>(v + src, i, lg - k);
        __syncthreads();
        end += m;
        n = m;
    }
    /* v[off[lg]] is the bucket total (zoom z_top - lg); emit levels 1..lg-1 */
    const uint64_t total = v[off[lg]];
    hm_emit_cells<THREADS>(v, off[lg], [&](uint32_t i, int& z, uint64_t& key) {
        int k = 1;
        while (k < lg - 1 && i >= off[k + 1]) k++;
        z = z_top - k;
        key = hm_cell_key(z, prefix, lg - k, i - off[k]);
    }, o, scr, sbase);
    __syncthreads();
    return total;
}

/* Final level, dense buckets: one block per <= HM_TA-key work item counts the
 * item's u16 keys in an LDS 2^lg x 2^lg histogram.  The rows are padded to
 * 2^lg + 8 words (cell (r, c) at r (2^lg + 8) + c: a cluster's cells in one
 * column fall in different banks, the row stride no longer being a multiple
 * of the 64 banks).  A single-item bucket emits its pyramid, at lg = 7 from
 * registers straight off the padded rows (hm_reg_pyramid7), below that from
 * the squeezed histogram; an item of a multi-item bucket adds its squeezed
 * histogram into the bucket's slot and k_aggregate_merged emits it. */
#ifndef HM_AG_PADW
#define HM_AG_PADW 8u   /* pad words per histogram row (a multiple of 4: hm_reg_pyramid7 reads 16-B vectors) */
#endif
#define HM_AG_ROW(lg) ((1u << (lg)) + HM_AG_PADW)
#define HM_AG_PADDED (128u * (128u + HM_AG_PADW))
#ifndef HM_AG_STAGE
#define HM_AG_STAGE 1   /* hm_reg_pyramid7: cells staged in the dead histogram, written a whole line per store */
#endif
static_assert(HM_AG_LG == 7 && HM_AG_CELLS == 128 * 128, "padded histogram");

/* The lg = 7 bucket pyramid from registers (k_aggregate's single-item
 * buckets): thread t holds the 4 x 4 block (t >> 5, t & 31) of the padded
 * 128 x 128 histogram, so zooms z_top-1 and z_top-2 are in-register sums; wave
 * 0 takes the 32 x 32 level (through s19) on to the bucket total, its lanes'
 * 4 x 4 blocks giving z_top-3 and z_top-4 and lane shuffles z_top-5, z_top-6
 * and the total.  Two barriers and one output reservation (hm_bucket_pyramid:
 * a barrier per level and LDS passes over every level twice); each level's
 * non-empty cells are ballot-compacted per wave, so the stores stay
 * coalesced.  Emits zooms z_top .. z_top-6 within [zmin, zmax] and returns the
 * bucket total (zoom z_top-7) in wave 0.  Every thread calls; the histogram's
 * rows are ROW words apart; s19 is 1024 words of 16-B-aligned scratch LDS. */
template <uint32_t ROW>
__device__ __forceinline__ uint64_t hm_reg_pyramid7(uint32_t* grid, int z_top, uint64_t prefix, const HmOut& o,
                                                    uint32_t* s19, uint32_t* scr, unsigned long long* sbase)
{
    constexpr int NW = HM_AG_THREADS / 64;
    static_assert(HM_AG_THREADS == 1024, "one 4 x 4 block per thread");
    const int tid = threadIdx.x, lane = hm_lane(), w = tid >> 6;
    const uint32_t br = (uint32_t)tid >> 5, bc = (uint32_t)tid & 31u;
    auto in = [&](int z) { return z >= o.zmin && z <= o.zmax; };
    auto nnz = [](bool nz) { return (uint32_t)__builtin_popcountll(__builtin_amdgcn_ballot_w64(nz)); };
    uint32_t c[16], d[4];
#pragma unroll
    for (int y = 0; y < 4; y++) {
        const uint4 q = *(const uint4*)&grid[(4u * br + y) * ROW + 4u * bc];
        c[4 * y] = q.x;
        c[4 * y + 1] = q.y;
        c[4 * y + 2] = q.z;
        c[4 * y + 3] = q.w;
    }
#pragma unroll
    for (int j = 0; j < 4; j++) {
        const int r = 8 * (j >> 1) + 2 * (j & 1);
        d[j] = c[r] + c[r + 1] + c[r + 4] + c[r + 5];
    }
    const uint32_t e = d[0] + d[1] + d[2] + d[3];
    s19[tid] = e;
    const bool i0 = in(z_top), i1 = in(z_top - 1), i2 = in(z_top - 2);
    uint32_t n = 0;
    if (i0)
#pragma unroll
        for (int j = 0; j < 16; j++) n += nnz(c[j] != 0);
    if (i1)
#pragma unroll
        for (int j = 0; j < 4; j++) n += nnz(d[j] != 0);
    if (i2) n += nnz(e != 0);
    if (lane == 0) scr[w] = n;
    __syncthreads();
    /* wave 0: lane l the 4 x 4 block (l >> 3, l & 7) of the 32 x 32 level */
    const uint32_t R = (uint32_t)lane >> 3, C = (uint32_t)lane & 7u;
    const bool l5 = (lane & 9) == 0, l6 = (lane & 27) == 0;
    const bool i3 = in(z_top - 3), i4 = in(z_top - 4), i5 = in(z_top - 5), i6 = in(z_top - 6);
    uint32_t g[4] = {0u, 0u, 0u, 0u}, h = 0, h5 = 0, h6 = 0, tot = 0;
    if (w == 0) {
        uint32_t f[16];
#pragma unroll
        for (int y = 0; y < 4; y++) {
            const uint4 q = *(const uint4*)&s19[(4u * R + y) * 32u + 4u * C];
            f[4 * y] = q.x;
            f[4 * y + 1] = q.y;
            f[4 * y + 2] = q.z;
            f[4 * y + 3] = q.w;
        }
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const int r = 8 * (j >> 1) + 2 * (j & 1);
            g[j] = f[r] + f[r + 1] + f[r + 4] + f[r + 5];
        }
        h = g[0] + g[1] + g[2] + g[3];                 /* z_top-4: (R, C) of 8 x 8 */
        uint32_t s = h + __shfl_xor(h, 1, 64);
        h5 = s + __shfl_xor(s, 8, 64);                 /* z_top-5: (R/2, C/2), lanes & 9 == 0 */
        s = h5 + __shfl_xor(h5, 2, 64);
        h6 = s + __shfl_xor(s, 16, 64);                /* z_top-6: (R/4, C/4), lanes & 27 == 0 */
        s = h6 + __shfl_xor(h6, 4, 64);
        tot = s + __shfl_xor(s, 32, 64);
        uint32_t ns = 0;
        if (i3)
#pragma unroll
            for (int j = 0; j < 4; j++) ns += nnz(g[j] != 0);
        if (i4) ns += nnz(h != 0);
        if (i5) ns += nnz(l5 && h5 != 0);
        if (i6) ns += nnz(l6 && h6 != 0);
        /* the waves' counts, then the small levels (slot NW) */
        const uint32_t x = lane < NW ? scr[lane] : lane == NW ? ns : 0u;
        const uint32_t incl = hm_wave_incl_scan(x);
        if (lane <= NW) scr[lane] = incl - x;
        if (lane == NW) *sbase = incl ? atomicAdd(o.cursor, (unsigned long long)incl) : 0ull;
    }
    __syncthreads();
    uint64_t base = *sbase + scr[w];
#if HM_AG_STAGE
    /* the wave's cells staged in its share of the (now dead) histogram as
     * (level << 14 | cell, count) pairs and written out a whole line per
     * store (HM_AG_STAGE; as k_small_pairs' hm_sp_flush) */
    constexpr uint32_t SC = HM_AG_PADDED / NW / 2 / 64 * 64;   /* cells per wave */
    uint2* stg = (uint2*)grid + (uint32_t)w * SC;
    uint32_t fill = 0;
    const auto flush = [&]() {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        for (uint32_t q0 = 0; q0 < fill; q0 += 64) {
            const uint32_t q = q0 + (uint32_t)lane;
            const uint2 x = stg[q < fill ? q : 0u];
            const int l = (int)(x.x >> 14);
            const uint64_t pos = base + q;
            if (q < fill && pos < o.capacity) {
                o.keys[pos] = hm_cell_key(z_top - l, prefix, 7 - l, x.x & 0x3FFFu);
                o.counts[pos] = x.y;
            }
        }
        base += fill;
        fill = 0;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    };
    auto put = [&](bool nz, int z, int lg, uint32_t i, uint32_t v) {
        if (fill + 64u > SC) flush();   /* wave-uniform */
        const uint64_t m = __builtin_amdgcn_ballot_w64(nz);
        if (nz) stg[fill + hm_mbcnt(m)] = make_uint2(((uint32_t)(z_top - z) << 14) | i, v);
        fill += (uint32_t)__builtin_popcountll(m);
    };
#else
    auto put = [&](bool nz, int z, int lg, uint32_t i, uint32_t v) {
        const uint64_t m = __builtin_amdgcn_ballot_w64(nz);
        const uint64_t pos = base + hm_mbcnt(m);
        if (nz && pos < o.capacity) {
            o.keys[pos] = hm_cell_key(z, prefix, lg, i);
            o.counts[pos] = v;
        }
        base += (uint32_t)__builtin_popcountll(m);
    };
    const auto flush = [&]() {};
#endif
    if (i0)
#pragma unroll
        for (int j = 0; j < 16; j++)
            put(c[j] != 0, z_top, 7, (4u * br + (j >> 2)) * 128u + 4u * bc + (j & 3), c[j]);
    if (i1)
#pragma unroll
        for (int j = 0; j < 4; j++) put(d[j] != 0, z_top - 1, 6, (2u * br + (j >> 1)) * 64u + 2u * bc + (j & 1), d[j]);
    if (i2) put(e != 0, z_top - 2, 5, br * 32u + bc, e);
    flush();
    if (w == 0) {
        base = *sbase + scr[NW];
        if (i3)
#pragma unroll
            for (int j = 0; j < 4; j++) put(g[j] != 0, z_top - 3, 4, (2u * R + (j >> 1)) * 16u + 2u * C + (j & 1), g[j]);
        if (i4) put(h != 0, z_top - 4, 3, R * 8u + C, h);
        if (i5) put(l5 && h5 != 0, z_top - 5, 2, (R >> 1) * 4u + (C >> 1), h5);
        if (i6) put(l6 && h6 != 0, z_top - 6, 1, (R >> 2) * 2u + (C >> 2), h6);
        flush();
    }
    return tot;
}
__global__ __launch_bounds__(HM_AG_THREADS, 8) void k_aggregate(HmAggArgs a)
{
    __shared__ alignas(16) uint32_t grid[HM_AG_PADDED + 64];   /* + 64 dummy words (hm_lds_count) */
    __shared__ uint32_t scr[HM_AG_THREADS / 64 + 1];
    __shared__ unsigned long long sbase;
    __shared__ alignas(16) HmRunLds<256> L;                     /* after the count: hm_reg_pyramid7's s19 */
    static_assert(sizeof(HmRunLds<256>) >= 1024 * sizeof(uint32_t), "s19 in the run chunk");
    const int tid = threadIdx.x;
    const uint32_t side = 1u << a.lg, ncell = side * side, npad = side * HM_AG_ROW(a.lg);
    HM_STAMP_M(5, 0);
    for (uint32_t i = tid; i < npad; i += HM_AG_THREADS) grid[i] = 0;
    __syncthreads();
    if (hm_block_id() >= a.items) return;   /* block-uniform */
    const HmItem it = hm_item(a.B, hm_block_id());
    HM_STAMP_M(5, 1);
    struct {
        uint32_t* grid;
        uint32_t dummy;
        int lg;
        __device__ __forceinline__ uint32_t sl(uint32_t k) { return k + (k >> lg) * HM_AG_PADW; }   /* padded row */
        __device__ __forceinline__ void cnt(uint32_t k, bool v)
        {
            if (HM_AG_FAST)
                hm_lds_count_fast(grid, dummy + (uint32_t)hm_lane(), sl(k), v);
            else
                hm_lds_count(grid, dummy, sl(k), v);
        }
        __device__ __forceinline__ void key(uint32_t k, bool v, uint32_t) { cnt(k, v); }
        __device__ __forceinline__ void add(uint32_t k, bool v) { atomicAdd(&grid[v ? sl(k) : dummy + (uint32_t)hm_lane()], 1u); }
        /* 8 keys: the wave tests its first key only -- more than HM_MERGE_MIN
         * lanes on lane 0's key (a skewed cloud's hot cell) sends all 8 through
         * the merging count, otherwise they are 8 plain atomics (1e9 hotspots:
         * aggregation 762-770 -> 710-723 us at zooms 0-18, 3.58 -> 3.48 ms at
         * 6-21; skew unchanged; plain atomics on every vector took the skewed
         * cloud's aggregation 6.1 -> 8.6 ms) */
        __device__ __forceinline__ void vec(const uint4& x, bool v, uint32_t)
        {
            const uint32_t k0 = x.x & 0xFFFFu;
            const uint64_t m = __builtin_amdgcn_ballot_w64(v && k0 == __builtin_amdgcn_readfirstlane(k0));
            if (!HM_AG_FAST || (uint32_t)__builtin_popcount((uint32_t)m) + (uint32_t)__builtin_popcount((uint32_t)(m >> 32)) >
                                   HM_MERGE_MIN) {
                cnt(x.x & 0xFFFFu, v);
                cnt(x.x >> 16, v);
                cnt(x.y & 0xFFFFu, v);
                cnt(x.y >> 16, v);
                cnt(x.z & 0xFFFFu, v);
                cnt(x.z >> 16, v);
                cnt(x.w & 0xFFFFu, v);
                cnt(x.w >> 16, v);
            } else {
                add(x.x & 0xFFFFu, v);
                add(x.x >> 16, v);
                add(x.y & 0xFFFFu, v);
                add(x.y >> 16, v);
                add(x.z & 0xFFFFu, v);
                add(x.z >> 16, v);
                add(x.w & 0xFFFFu, v);
                add(x.w >> 16, v);
            }
        }
    } f{grid, HM_AG_PADDED, a.lg};
    hm_stream_runs<uint16_t, HM_AG_THREADS, 256, false>(it, a.keys, a.in, L, scr, f);
    HM_STAMP_M(5, 2);
    HM_STAMP_V(5, 5, (unsigned long long)(it.b - it.a));
    HM_STAMP_V(5, 6, (unsigned long long)(it.r1 - it.r0));
    HM_STAMP_V(5, 7, (unsigned long long)it.nitems);
    if (it.nitems == 1 && a.lg == HM_AG_LG) {   /* block-uniform */
        const uint64_t t = hm_reg_pyramid7<HM_AG_ROW(7)>(grid, a.Z, a.B.coord[it.bucket], a.out, (uint32_t*)&L, scr,
                                                         &sbase);
        if (tid == 0) a.totals[it.bucket] = t;
        HM_STAMP_M(5, 3);
        HM_STAMP_M(5, 4);
        return;
    }
    /* squeeze the padding out: cell i back at i */
    constexpr int CPT = HM_AG_CELLS / HM_AG_THREADS;
    uint32_t x[CPT];
#pragma unroll
    for (int k = 0; k < CPT; k++) {
        const uint32_t i = k * HM_AG_THREADS + tid;
        x[k] = i < ncell ? grid[i + (i >> a.lg) * HM_AG_PADW] : 0u;
    }
    if (it.nitems > 1) {
        /* added into the bucket's slot (coalesced: consecutive threads,
         * consecutive words).  Measured against a slot per item summed by
         * k_aggregate_merged: the same on hotspots, and the skew cloud's one
         * 3400-item bucket made that sum a 3.7 ms single-block tail */
        uint32_t* g = a.gslots + (uint64_t)a.B.slots[it.bucket] * HM_AG_CELLS;
        uint32_t s = 0;
#pragma unroll
        for (int k = 0; k < CPT; k++) {
            const uint32_t i = k * HM_AG_THREADS + tid;
            if (i < ncell && x[k]) atomicAdd(&g[i], x[k]);
            s += x[k];
        }
        s = hm_wave_sum(s);
        if (hm_lane() == 0 && s) atomicAdd(&a.totals[it.bucket], (unsigned long long)s);
        HM_STAMP_M(5, 3);
        HM_STAMP_M(5, 4);
        return;
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < CPT; k++) {
        const uint32_t i = k * HM_AG_THREADS + tid;
        if (i < ncell) grid[i] = x[k];
    }
    __syncthreads();
    HM_STAMP_M(5, 3);
    const uint64_t t = hm_bucket_pyramid<HM_AG_THREADS>(grid, a.lg, a.Z, a.B.coord[it.bucket], a.out, scr, &sbase);
    if (tid == 0) a.totals[it.bucket] = t;
    HM_STAMP_M(5, 4);
}
/* one block per multi-item bucket: its summed histogram, then its pyramid */
__global__ __launch_bounds__(HM_AG_THREADS) void k_aggregate_merged(HmAggArgs a)
{
    __shared__ alignas(16) uint32_t grid[HM_AG_CELLS];
    __shared__ alignas(16) uint32_t s19[1024];
    __shared__ uint32_t scr[HM_AG_THREADS / 64 + 1];
    __shared__ unsigned long long sbase;
    const uint32_t ncell = 1u << (2 * a.lg);
    if (hm_block_id() >= a.nslots) return;
    const uint32_t b = a.slot_bucket[hm_block_id()];
    const uint4* g = (const uint4*)(a.gslots + (uint64_t)hm_block_id() * HM_AG_CELLS);
    for (uint32_t v = threadIdx.x; v < ncell / 4; v += HM_AG_THREADS) ((uint4*)grid)[v] = g[v];
    __syncthreads();
    if (a.lg == HM_AG_LG)
        hm_reg_pyramid7<1u << HM_AG_LG>(grid, a.Z, a.B.coord[b], a.out, s19, scr, &sbase);
    else
        hm_bucket_pyramid<HM_AG_THREADS>(grid, a.lg, a.Z, a.B.coord[b], a.out, scr, &sbase);
}

/* ------------------------------------------------------------------------ */
/* final level, small buckets (<= HM_SPW_MAX keys): one wavefront per bucket  */
/* ------------------------------------------------------------------------ */

__device__ __forceinline__ uint32_t hm_spread7(uint32_t x)
{
    x = (x | (x << 4)) & 0x0F0Fu;
    x = (x | (x << 2)) & 0x3333u;
    return (x | (x << 1)) & 0x5555u;
}
__device__ __forceinline__ uint32_t hm_compact7(uint32_t x)
{
    x &= 0x5555u;
    x = (x | (x >> 1)) & 0x3333u;
    x = (x | (x >> 2)) & 0x0F0Fu;
    return (x | (x >> 4)) & 0x00FFu;
}

/* the value of lane (lane ^ M): DPP quad permutes for M = 1, 2 (no LDS
 * instruction), ds_swizzle's xor mode below 32 (no address), a bpermute for
 * 32 (HIP's __shfl_xor is a bpermute with a computed address for every M) */
template <int M>
__device__ __forceinline__ uint32_t hm_xor_lane(uint32_t v)
{
    if constexpr (M == 1)
        return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xF, 0xF, false);   /* quad_perm [1,0,3,2] */
    else if constexpr (M == 2)
        return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x4E, 0xF, 0xF, false);   /* quad_perm [2,3,0,1] */
    else if constexpr (M < 32)
        return (uint32_t)__builtin_amdgcn_ds_swizzle((int)v, (M << 10) | 0x1F);           /* xor within 32 lanes */
    else
        return __shfl_xor(v, M, 64);
}

/* Ascending bitonic sort of the wave's 64*K values, element e = lane*K + u in
 * v[u]: distances < K swap registers, larger ones exchange across lanes.
 * Compile-time recursion over (size, stride), so every lane exchange has a
 * constant distance (hm_xor_lane). */
template <int K, int SIZE, int STRIDE>
__device__ __forceinline__ void hm_bitonic_step(uint32_t (&v)[K], uint32_t lane)
{
    if constexpr (STRIDE >= K) {
#pragma unroll
        for (int u = 0; u < K; u++) {
            const uint32_t e = lane * K + u;
            const uint32_t o = hm_xor_lane<STRIDE / K>(v[u]);
            const bool take_min = ((e & STRIDE) == 0) == ((e & SIZE) == 0);
            v[u] = take_min ? min(v[u], o) : max(v[u], o);
        }
    } else {
#pragma unroll
        for (int u = 0; u < K; u++) {
            if ((u & STRIDE) == 0) {
                const int w = u | STRIDE;
                const bool up = ((lane * K + u) & SIZE) == 0;
                const uint32_t lo = min(v[u], v[w]), hi = max(v[u], v[w]);
                v[u] = up ? lo : hi;
                v[w] = up ? hi : lo;
            }
        }
    }
    if constexpr (STRIDE > 1) hm_bitonic_step<K, SIZE, STRIDE / 2>(v, lane);
}
template <int K, int SIZE>
__device__ __forceinline__ void hm_bitonic_size(uint32_t (&v)[K], uint32_t lane)
{
    hm_bitonic_step<K, SIZE, SIZE / 2>(v, lane);
    if constexpr (SIZE < 64 * K) hm_bitonic_size<K, SIZE * 2>(v, lane);
}
template <int K>
__device__ __forceinline__ void hm_wave_bitonic(uint32_t (&v)[K])
{
    hm_bitonic_size<K, 2>(v, hm_lane());
}

/* Two 32-lane ascending bitonic sorts side by side (lanes 0-31 and 32-63,
 * one value per lane): the 64-lane network's stages up to size 32, with the
 * direction of size 32 taken inside each half */
template <int SIZE, int STRIDE>
__device__ __forceinline__ void hm_seg32_step(uint32_t& v, uint32_t lane)
{
    const uint32_t o = hm_xor_lane<STRIDE>(v);
    const bool take_min = ((lane & STRIDE) == 0) == ((lane & SIZE & 31u) == 0);
    v = take_min ? min(v, o) : max(v, o);
    if constexpr (STRIDE > 1) hm_seg32_step<SIZE, STRIDE / 2>(v, lane);
}
template <int SIZE>
__device__ __forceinline__ void hm_seg32_size(uint32_t& v, uint32_t lane)
{
    hm_seg32_step<SIZE, SIZE / 2>(v, lane);
    if constexpr (SIZE < 32) hm_seg32_size<SIZE * 2>(v, lane);
}

/* Buckets of <= 32 keys (a sparse cloud's common case: the skew background
 * averages ~24 per zoom-11 bucket) two per wave, one 32-lane segment each:
 * the bucket of segment g is the g-th of a pair picked from the wave's
 * ballot.  hm_pair_lane: the wave lane holding this lane's bucket (-1: the
 * segment has none). */
__device__ __forceinline__ int hm_pair_lane(uint64_t& mt)
{
    const int i0 = __builtin_ctzll(mt);
    mt &= mt - 1;
    const int i1 = mt ? __builtin_ctzll(mt) : -1;
    if (mt) mt &= mt - 1;
    return (hm_lane() >> 5) ? i1 : i0;
}

/* Small buckets run in two passes so that the output needs no per-bucket
 * cursor atomic (4M buckets would serialise on it at ~12 ns each):
 *   pass 1 (k_small_sort): a wave gathers a bucket's keys, re-codes them in
 *     Morton order inside the bucket, sorts them (Morton parents preserve the
 *     order, so the cells of level l are the runs of equal code >> 2l), stores
 *     the sorted codes at the bucket's own key range and counts its cells;
 *   an exclusive scan of the counts places every bucket's cells;
 *   pass 2 (k_small_emit): re-reads the sorted codes (coalesced) and writes
 *     each cell at its place; a cell is written by its last element, its count
 *     is that position minus the segment start (a wave max-scan). */

template <int K>
__device__ __forceinline__ void hm_small_load(const uint16_t* src, uint32_t nk, uint32_t (&v)[K])
{
    const uint32_t lane = hm_lane();
#pragma unroll
    for (int u = 0; u < K; u++) {
        const uint32_t e = lane * K + u;
        v[u] = e < nk ? (uint32_t)src[e] : 0xFFFFFFFFu;
    }
}

/* last element of its level-l cell (valid elements only); nx = the next
 * lane's v[0] */
template <int K>
__device__ __forceinline__ void hm_small_ends(const uint32_t (&v)[K], uint32_t nk, int l, bool (&end)[K], uint32_t nx)
{
    const uint32_t lane = hm_lane();
#pragma unroll
    for (int u = 0; u < K; u++) {
        const uint32_t e = lane * K + u;
        const uint32_t next = (u + 1 < K) ? v[u + 1] : nx;
        end[u] = (e < nk) & ((e + 1 == nk) | ((next >> (2 * l)) != (v[u] >> (2 * l))));
    }
}

template <int K>
__device__ __forceinline__ void hm_small_sort(const HmAggArgs& a, const uint16_t* ks, uint32_t nk, uint32_t kb,
                                              uint32_t zmask, uint32_t b)
{
    const uint32_t lane = hm_lane();
    const int lg = a.lg;
    const uint32_t cm = (1u << lg) - 1;
    uint32_t v[K];
    hm_small_load<K>(ks, nk, v);
#pragma unroll
    for (int u = 0; u < K; u++)
        if (v[u] != 0xFFFFFFFFu) v[u] = hm_spread7(v[u] & cm) | (hm_spread7(v[u] >> lg) << 1);
    hm_wave_bitonic<K>(v);
#pragma unroll
    for (int u = 0; u < K; u++) {
        const uint32_t e = lane * K + u;
        if (e < nk) a.codes[kb + e] = (uint16_t)v[u];
    }
    /* cells: element e ends a level-l cell iff its code and the next one's
     * differ above bit 2l, i.e. for the levels below half the bit length of
     * their xor (the last element ends every level): one count per element,
     * not a ballot per (level, element) */
    const uint32_t nx = __shfl_down(v[0], 1, 64);
    const uint32_t zall = (uint32_t)__popc(zmask);
    uint32_t cnt = 0;
#pragma unroll
    for (int u = 0; u < K; u++) {
        const uint32_t e = lane * K + u;
        const uint32_t next = (u + 1 < K) ? v[u + 1] : nx;
        const uint32_t x = v[u] ^ next;
        const uint32_t hl = (33u - (uint32_t)__clz((int)x)) >> 1;   /* x = 0: 0 */
        const uint32_t c = e + 1 == nk ? zall : (uint32_t)__popc(zmask & ((1u << hl) - 1u));
        cnt += e < nk ? c : 0u;
    }
    const uint32_t total = hm_wave_sum(cnt);
    if (lane == 0) a.spcnt[b] = total;
}

template <int K>
__device__ __forceinline__ void hm_small_emit(const HmAggArgs& a, uint32_t nk, uint32_t kb, uint64_t coord,
                                              uint32_t zmask, uint64_t base, uint32_t* hw)
{
    const uint32_t lane = hm_lane();
    const int lg = a.lg;
    uint32_t v[K];
    hm_small_load<K>(a.codes + kb, nk, v);
    /* the four coarsest levels (<= 256 cells each) from a 256-slot LDS
     * histogram of the codes' top 8 bits: one LDS atomic per key; the
     * coarsest-but-three level has 4 slots per lane, the next ones are sums
     * of 4 (in the lane, then across quads of lanes): one store per level and
     * slot group instead of a pass over every key per level */
    /* (buckets of <= 128 keys: the three coarsest levels, 64 slots -- the
     * fourth costs them more as 256 slots than as a pass over their keys) */
    constexpr int NC = K >= 4 ? 4 : 3;
    const int lc = lg >= NC ? lg - NC : 0;
    if (zmask >> lc) {
        uint4* hw4 = (uint4*)hw;
        if (NC == 4) hw4[lane] = make_uint4(0u, 0u, 0u, 0u);
        else hw[lane] = 0u;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int u = 0; u < K; u++)
            if (lane * K + u < nk) atomicAdd(&hw[v[u] >> (2 * lc)], 1u);
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
        __builtin_amdgcn_wave_barrier();
        uint64_t q = base;
        auto put = [&](bool mine, uint64_t bal, uint32_t code, int l, uint32_t c) {
            if (mine) {
                const int sl = lg - l;
                const uint32_t idx = (hm_compact7(code >> 1) << sl) | hm_compact7(code);
                const uint64_t p = q + hm_mbcnt(bal);
                if (p < a.out.capacity) {
                    a.out.keys[p] = hm_cell_key(a.Z - l, coord, sl, idx);
                    a.out.counts[p] = (uint64_t)c;
                }
            }
            q += (uint64_t)__popcll(bal);
        };
        uint32_t c;   /* the count of prefix = lane at level l1 */
        int l1 = lc;
        if constexpr (NC == 4) {
            const uint4 c4 = hw4[lane];   /* prefixes 4 lane + j (slots past 4^(lg - lc) stay 0) */
            if ((zmask >> lc) & 1u) {
                const uint32_t cj[4] = {c4.x, c4.y, c4.z, c4.w};
#pragma unroll
                for (int j = 0; j < 4; j++) {
                    const bool mine = cj[j] != 0u;
                    put(mine, __ballot(mine), lane * 4u + (uint32_t)j, lc, cj[j]);
                }
            }
            c = c4.x + c4.y + c4.z + c4.w;
            l1 = lc + 1;
        } else {
            c = hw[lane];
        }
        for (int l = l1; l < lg; l++) {
            const int g = 2 * (l - l1);   /* this level's prefix: lane >> g on lanes with those bits clear */
            if (g) {
                /* sum the 4 finer cells: lanes lane + {0, 1, 2, 3} 2^(g-2) */
                const int st = 1 << (g - 2);
                c += __shfl_down(c, st, 64);
                c += __shfl_down(c, 2 * st, 64);
            }
            const bool mine = (lane & ((1u << g) - 1u)) == 0u && c != 0u && ((zmask >> l) & 1u);
            put(mine, __ballot(mine), lane >> g, l, c);
        }
        base = q;
        __builtin_amdgcn_wave_barrier();   /* hw is free for the next bucket */
    }
    /* the neighbours' codes are level-independent: read once per bucket */
    const uint32_t nx = __shfl_down(v[0], 1, 64);
    const uint32_t pv = __shfl_up(v[K - 1], 1, 64);
    for (int l = 0; l < lc; l++) {
        if (!((zmask >> l) & 1u)) continue;
        bool end[K];
        hm_small_ends<K>(v, nk, l, end, nx);
        /* segment start of every element: running max of head positions */
        uint32_t hs[K];
        uint32_t run = 0;
#pragma unroll
        for (int u = 0; u < K; u++) {
            const uint32_t e = lane * K + u;
            const uint32_t prev = u > 0 ? v[u - 1] : pv;
            run = ((e == 0) | ((prev >> (2 * l)) != (v[u] >> (2 * l)))) ? e : run;
            hs[u] = run;
        }
        /* the last head before this lane's elements: heads' positions grow
         * with the lane, so it is the run of the highest lower lane holding a
         * head (lane 0 always does: element 0) -- one ballot and one
         * cross-lane read instead of a 6-step max-scan */
        const uint64_t hmask = __ballot((run != 0u) | (lane == 0u));
        const uint64_t below = hmask & ((1ull << lane) - 1ull);
        uint32_t ex = __shfl(run, below ? 63 - __clzll((long long)below) : 0, 64);
        ex = lane ? ex : 0u;
        const int zl = a.Z - l;
        const int s = lg - l;
#pragma unroll
        for (int u = 0; u < K; u++) {
            const uint64_t bal = __ballot(end[u]);
            if (end[u]) {
                const uint32_t e = lane * K + u;
                const uint32_t code = v[u] >> (2 * l);
                const uint32_t idx = (hm_compact7(code >> 1) << s) | hm_compact7(code);
                const uint64_t q = base + hm_mbcnt(bal);
                if (q < a.out.capacity) {
                    a.out.keys[q] = hm_cell_key(zl, coord, s, idx);
                    a.out.counts[q] = (uint64_t)(e - max(hs[u], ex) + 1);
                }
            }
            base += __popcll(bal);
        }
    }
}

__device__ __forceinline__ uint32_t hm_small_zmask(const HmAggArgs& a)
{
    uint32_t zmask = 0;
    for (int l = 0; l < a.lg; l++) {
        const int z = a.Z - l;
        zmask |= (uint32_t)(z >= a.out.zmin && z <= a.out.zmax) << l;
    }
    return zmask;
}

/* The register sort of bucket size nk runs with K = ceil(nk / 64) rounded up
 * to a power of two, for K in the instantiation's range only: a kernel's VGPR
 * budget is its widest K's (K = 32 needs ~200, two waves per SIMD), so buckets
 * of <= HM_SPW_SPLIT keys get their own narrow, high-occupancy instantiation
 * and LO < nk <= HI selects a kernel's share. */
template <uint32_t LO, uint32_t HI, typename F>
__device__ __forceinline__ void hm_small_dispatch(uint32_t nk, F&& f)
{
    if constexpr (LO < 64) if (nk <= 64) { f(std::integral_constant<int, 1>{}); return; }
    if constexpr (LO < 128 && HI >= 128) if (nk <= 128) { f(std::integral_constant<int, 2>{}); return; }
    if constexpr (LO < 256 && HI >= 256) if (nk <= 256) { f(std::integral_constant<int, 4>{}); return; }
    if constexpr (LO < 512 && HI >= 512) if (nk <= 512) { f(std::integral_constant<int, 8>{}); return; }
    if constexpr (LO < 1024 && HI >= 1024) if (nk <= 1024) { f(std::integral_constant<int, 16>{}); return; }
    if constexpr (LO < 2048 && HI >= 2048) if (nk <= 2048) { f(std::integral_constant<int, 32>{}); return; }
    if constexpr (HI >= 4096) f(std::integral_constant<int, 64>{});
}

/* Which buckets a wave looks at.  LO == 0 (the narrow instantiation, most
 * buckets): wave w takes the batches of spbatch consecutive buckets w, w +
 * waves, ...  LO > 0 (the wide one: buckets of > HM_SPW_SPLIT keys, few and
 * clustered in space, i.e. in bucket order): lane j of wave w at step s looks
 * at bucket (64 s + j) waves + w, so neighbouring big buckets go to different
 * waves (consecutive batches left one wave sorting several of them while the
 * others idled: the tail of a stream batch's 513-2048-key pass). */
template <uint32_t LO>
struct HmSmallMap {
    static __device__ __forceinline__ uint32_t first(uint32_t wid, uint32_t spb) { return LO ? 0u : wid * spb; }
    static __device__ __forceinline__ uint32_t step(uint32_t nw, uint32_t spb) { return LO ? 64u : nw * spb; }
    static __device__ __forceinline__ uint64_t bucket(uint32_t s0, uint32_t lane, uint32_t wid, uint32_t nw)
    {
        return LO ? (uint64_t)(s0 + lane) * nw + wid : (uint64_t)s0 + lane;
    }
    static __device__ __forceinline__ bool lane_in(uint32_t lane, uint32_t spb) { return LO ? true : lane < spb; }
};

/* the small buckets k_small_pairs takes (HM_SP_FUSED): <= 32 keys in <= 32
 * runs (two a wave pass) or 33-64 keys in <= 64 runs (one) */
__device__ __forceinline__ bool hm_sp_fused_ok(uint32_t nk, uint32_t nr)
{
    return HM_SP_FUSED && nk <= 64 && nr <= (nk <= 32 ? 32u : 64u);
}

/* Persistent: a bucket is this instantiation's when LO < nkeys <= HI (larger
 * ones are k_aggregate's). The LO == 0 instantiation runs first and zeroes the
 * cell count of every bucket that is not its own. */
template <uint32_t LO, uint32_t HI>
__global__ __launch_bounds__(HM_SPW_THREADS) void k_small_sort(HmAggArgs a)
{
    __shared__ uint16_t kss[HM_SPW_THREADS / 64][HI];
    const uint32_t lane = hm_lane();
    uint16_t* ks = kss[threadIdx.x >> 6];
    const uint32_t nw = gridDim.x * (HM_SPW_THREADS / 64);
    const uint32_t zmask = hm_small_zmask(a);
    const uint32_t wid = blockIdx.x * (HM_SPW_THREADS / 64) + (threadIdx.x >> 6);
    const uint32_t step = HmSmallMap<LO>::step(nw, a.spbatch);
    for (uint32_t s0 = HmSmallMap<LO>::first(wid, a.spbatch); HmSmallMap<LO>::bucket(s0, 0, wid, nw) < a.B.count;
         s0 += step) {
        const uint64_t bl64 = HmSmallMap<LO>::bucket(s0, lane, wid, nw);
        const bool in = HmSmallMap<LO>::lane_in(lane, a.spbatch) & (bl64 < a.B.count);
        const uint32_t bl = in ? (uint32_t)bl64 : 0u;
        const uint32_t nkl = in ? a.B.nkeys[bl] : 0u;
        const bool small = in & (LO == 0 || nkl > LO) & (nkl <= HI);
        const uint32_t rbl = small ? a.B.rbase[bl] : 0u, nrl = small ? a.B.nruns[bl] : 0u;
        const uint32_t kbl = small ? a.B.keybase[bl] : 0u;
        /* (HM_SP_FUSED: the <= 32-key, <= 4-run buckets are k_small_pairs') */
        const bool pairb = LO == 0 && small && hm_sp_fused_ok(nkl, nrl);
        if (LO == 0 && in && (!small || pairb)) a.spcnt[bl] = 0;
        if (small && !pairb) a.totals[bl] = nkl;
        uint64_t m = __ballot(small && !pairb);
        if constexpr (LO == 0 && !HM_SP_FUSED) {
            /* buckets of <= 32 keys in <= 4 runs: two per pass of the wave */
            uint64_t mt = __ballot(small && nkl <= 32 && nrl <= 4);
            m &= ~mt;
            const uint32_t j = lane & 31;
            while (mt) {
                const int sl = hm_pair_lane(mt);
                const bool seg = sl >= 0;
                const int sr = seg ? sl : 0;
                /* (every shuffle with the whole wave active: a bpermute reads
                 * garbage from a lane outside the exec mask) */
                const uint32_t nk0 = __shfl(nkl, sr, 64);
                const uint32_t b = __shfl(bl, sr, 64), nk = seg ? nk0 : 0u;
                const uint32_t r0 = __shfl(rbl, sr, 64), nr = __shfl(nrl, sr, 64), kb = __shfl(kbl, sr, 64);
                /* this lane's key: its run among the bucket's <= 4 */
                uint32_t src = 0, acc = 0;
                bool found = false;
#pragma unroll
                for (int q = 0; q < 4; q++) {
                    const uint2 run = (seg && (uint32_t)q < nr) ? a.in.run[r0 + q] : make_uint2(0, 0);
                    if (!found && j < acc + run.y) {
                        src = run.x + (j - acc);
                        found = true;
                    }
                    acc += run.y;
                }
                const bool v_ok = seg && j < nk;
                uint32_t v = 0xFFFFFFFFu;
                if (v_ok) {
                    const uint32_t key = (uint32_t)a.keys[src];
                    const uint32_t cm = (1u << a.lg) - 1;
                    v = hm_spread7(key & cm) | (hm_spread7(key >> a.lg) << 1);
                }
                hm_seg32_size<2>(v, lane);
                if (v_ok) a.codes[kb + j] = (uint16_t)v;
                const uint32_t nx = __shfl_down(v, 1, 64);
                /* cells ended by this element (as in hm_small_sort), summed
                 * over the 32-lane segment */
                const uint32_t hl = (33u - (uint32_t)__clz((int)(v ^ nx))) >> 1;
                uint32_t total = !v_ok ? 0u
                                       : (j + 1 == nk) ? (uint32_t)__popc(zmask)
                                                       : (uint32_t)__popc(zmask & ((1u << hl) - 1u));
#pragma unroll
                for (int o = 16; o > 0; o >>= 1) total += __shfl_xor(total, o, 64);
                if (seg && j == 0) a.spcnt[b] = total;
            }
        }
        while (m) {
            const int i = __builtin_ctzll(m);
            m &= m - 1;
            const uint32_t b = __shfl(bl, i, 64);
            const uint32_t nk = __shfl(nkl, i, 64), r0 = __shfl(rbl, i, 64), nr = __shfl(nrl, i, 64);
            const uint32_t kb = __shfl(kbl, i, 64);
            /* gather: runs 64 at a time, consecutive keys to consecutive lanes */
            uint32_t fill = 0;
            if (nr <= 4) {
                /* few runs (the common case: one per parent item): their
                 * bounds in scalar registers, a key's run by three compares
                 * instead of a 6-step shuffle search */
                const uint2 run = lane < nr ? a.in.run[r0 + lane] : make_uint2(0, 0);
                const uint32_t x0 = __builtin_amdgcn_readlane(run.x, 0), x1 = __builtin_amdgcn_readlane(run.x, 1);
                const uint32_t x2 = __builtin_amdgcn_readlane(run.x, 2), x3 = __builtin_amdgcn_readlane(run.x, 3);
                const uint32_t p1 = __builtin_amdgcn_readlane(run.y, 0);
                const uint32_t p2 = p1 + __builtin_amdgcn_readlane(run.y, 1);
                const uint32_t p3 = p2 + __builtin_amdgcn_readlane(run.y, 2);
                const uint32_t tot = p3 + __builtin_amdgcn_readlane(run.y, 3);
                for (uint32_t j = lane; j < tot; j += 64) {
                    const uint32_t src = j < p1 ? x0 + j : j < p2 ? x1 + (j - p1) : j < p3 ? x2 + (j - p2) : x3 + (j - p3);
                    ks[j] = a.keys[src];
                }
            } else
            for (uint32_t c0 = 0; c0 < nr; c0 += 64) {
                const uint32_t q = c0 + lane;
                const uint2 run = q < nr ? a.in.run[r0 + q] : make_uint2(0, 0);
                const uint32_t incl = hm_wave_incl_scan(run.y);
                const uint32_t tot = __shfl(incl, 63, 64);
                for (uint32_t j0 = 0; j0 < tot; j0 += 64) {
                    const uint32_t j = j0 + lane;
                    uint32_t lo = 0;
#pragma unroll
                    for (int st = 32; st > 0; st >>= 1)
                        if (__shfl(incl, lo + st - 1, 64) <= j) lo += st;
                    lo = min(lo, 63u);
                    const uint32_t cnt = __shfl(run.y, lo, 64);
                    const uint32_t off = j - (__shfl(incl, lo, 64) - cnt);
                    const uint32_t src = __shfl(run.x, lo, 64) + off;
                    if (j < tot) ks[fill + j] = a.keys[src];
                }
                fill += tot;
            }
            __builtin_amdgcn_wave_barrier();
            hm_small_dispatch<LO, HI>(nk, [&](auto kc) { hm_small_sort<decltype(kc)::value>(a, ks, nk, kb, zmask, b); });
            __builtin_amdgcn_wave_barrier();
        }
    }
}

/* k_small_pairs (HM_SP_FUSED, round 6): the small buckets of <= 64 keys --
 * the skew cloud's background, ~24 keys per zoom-11 bucket, 4M of them --
 * gathered, sorted, counted AND emitted in one pass.  A wave pass ("row")
 * takes two buckets of <= 32 keys in <= 32 runs (one 32-lane segment each) or
 * one of 33-64 keys in <= 64 runs; a wave sorts up to 32 rows of its batch of
 * 64 buckets into 4 KB of LDS, reserves their cells with ONE cursor atomic
 * (~1.5K cells on the skew cloud: ~65K atomics for 4M buckets, not one per
 * bucket) and emits them from LDS as k_small_emit does: no sorted codes
 * through HBM, no per-bucket count array, no scan or reservation launch. */

/* One row's bucket(s) in three steps, so a wave can keep the next rows'
 * loads in flight while it sorts: W = 32 (a pair: each 32-lane half holds its
 * own bucket) or 64 (one bucket); every lane active; the loads are
 * unconditional (inactive lanes read element 0), so the compiler counts them.
 *   hm_sp_run:  the segment's runs, one a lane;
 *   hm_sp_key:  lane j's key: in the first run whose inclusive key count
 *               passes j (segmented scan + binary search), 0xFFFF if none;
 *   hm_sp_sort: Morton code, segmented sort, the segment's cell count. */
__device__ __forceinline__ uint2 hm_sp_run(const HmAggArgs& a, bool seg, uint32_t r0, uint32_t nr, uint32_t j)
{
    const bool v = seg && j < nr;
    const uint2 r = a.in.run[v ? r0 + j : 0u];
    return v ? r : make_uint2(0, 0);
}
template <int W>
__device__ __forceinline__ uint32_t hm_sp_key(const HmAggArgs& a, uint2 run, bool seg, uint32_t nk, uint32_t lane,
                                              uint2* sc)
{
    const uint32_t j = lane & (W - 1);
    /* each non-empty run r marks its first key position excl_r in the wave's
     * 64-slot scratch with x_r - excl_r; lane j's run starts at the last mark
     * at or below j (a ballot), so its key is at that mark's value + j: a DPP
     * scan and three LDS round trips instead of a shuffle search */
    uint32_t incl = run.y;
    HM_DPP_ADD(incl, 0x111, 0xF);   /* row_shr:1 */
    HM_DPP_ADD(incl, 0x112, 0xF);   /* row_shr:2 */
    HM_DPP_ADD(incl, 0x114, 0xF);   /* row_shr:4 */
    HM_DPP_ADD(incl, 0x118, 0xF);   /* row_shr:8 */
    HM_DPP_ADD(incl, 0x142, 0xA);   /* row_bcast:15: rows 0 -> 1, 2 -> 3 (each 32-lane half scanned) */
    if constexpr (W == 64) HM_DPP_ADD(incl, 0x143, 0xC);   /* row_bcast:31: the whole wave */
    const uint32_t excl = incl - run.y;
    sc[lane] = make_uint2(0u, 0u);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    if (run.y) sc[(lane & ~(uint32_t)(W - 1)) + excl] = make_uint2(run.x - excl, 1u);   /* (run.y = 0 past nr) */
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const uint64_t marks = __ballot(sc[lane].y != 0u);
    const uint64_t below = marks & ((2ull << lane) - 1ull);
    const uint32_t h = below ? 63u - (uint32_t)__clzll((long long)below) : lane;
    const uint32_t d = sc[h].x;
    const bool v_ok = seg && j < nk;
    const uint32_t k = (uint32_t)a.keys[v_ok ? d + j : 0u];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();   /* sc is free for the next row */
    return v_ok ? k : 0xFFFFFFFFu;
}
template <int W>
__device__ __forceinline__ uint32_t hm_sp_sort(const HmAggArgs& a, uint32_t key, uint32_t nk, uint32_t lane,
                                               uint32_t zmask, uint32_t& v)
{
    const uint32_t j = lane & (W - 1);
    const uint32_t cm = (1u << a.lg) - 1;
    const bool v_ok = key != 0xFFFFFFFFu;
    v = v_ok ? hm_spread7(key & cm) | (hm_spread7(key >> a.lg) << 1) : 0xFFFFFFFFu;
    if constexpr (W == 32) {
        hm_seg32_size<2>(v, lane);
    } else {
        uint32_t vv[1] = {v};
        hm_wave_bitonic<1>(vv);
        v = vv[0];
    }
    /* cells ended by this element (hm_small_sort), summed over the segment */
    const uint32_t nx = __shfl_down(v, 1, 64);
    const uint32_t hl = (33u - (uint32_t)__clz((int)(v ^ nx))) >> 1;
    uint32_t total = !v_ok ? 0u
                           : (j + 1 == nk) ? (uint32_t)__popc(zmask) : (uint32_t)__popc(zmask & ((1u << hl) - 1u));
#pragma unroll
    for (int o = W / 2; o > 0; o >>= 1) total += __shfl_xor(total, o, 64);
    return total;
}

/* the cells of one sorted row segment at q: a cell is written by its last
 * element, its count = that position - the segment's last head at or below */
template <int W>
__device__ __forceinline__ void hm_sp_emit(const HmAggArgs& a, uint32_t v, bool v_ok, uint32_t nk, uint64_t coord,
                                           uint64_t q, uint32_t zmask, uint32_t lane)
{
    const uint32_t j = lane & (W - 1);
    const uint64_t segm = W == 64 ? ~0ull : (lane >> 5) ? 0xFFFFFFFF00000000ull : 0x00000000FFFFFFFFull;
    const uint32_t nx = __shfl_down(v, 1, 64), pv = __shfl_up(v, 1, 64);
    /* the element's row and column offsets in the bucket, de-interleaved
     * once: a level-l cell's are these >> l (hm_cell_key's layout) */
    const uint32_t cr = hm_compact7(v >> 1), cc = hm_compact7(v);
    const uint32_t crow = (uint32_t)(coord >> 32), ccol = (uint32_t)coord;
    for (int l = 0; l < a.lg; l++) {
        if (!((zmask >> l) & 1u)) continue;
        const bool head = v_ok && ((j == 0) | ((pv >> (2 * l)) != (v >> (2 * l))));
        const bool end = v_ok && ((j + 1 == nk) | ((nx >> (2 * l)) != (v >> (2 * l))));
        /* the cell's first element: the last head at or below this lane (the
         * segment's element 0 is one), as a position in the segment */
        const uint64_t hm = __ballot(head) & ((2ull << lane) - 1ull);
        const uint32_t start = (hm ? 63u - (uint32_t)__clzll((long long)hm) : 0u) & (uint32_t)(W - 1);
        const uint64_t bal = __ballot(end) & segm;
        if (end) {
            const int s = a.lg - l;
            const uint32_t row = (crow << s) | (cr >> l), col = (ccol << s) | (cc >> l);
            const uint64_t pos = q + hm_mbcnt(bal);
            if (pos < a.out.capacity) {
                a.out.keys[pos] = ((uint64_t)(a.Z - l) << 58) | ((uint64_t)row << 29) | col;
                a.out.counts[pos] = (uint64_t)(j - start + 1);
            }
        }
        q += (uint64_t)__popcll(bal);
    }
}

/* HM_SPP_STAGE: the same cells staged in the wave's LDS buffer as one u32
 * each -- bucket lane (6 bits) | level (3) | row (7) | column (7) | count (7)
 * -- at q (per lane, relative to the buffer), for hm_sp_flush to write out */
template <int W>
__device__ __forceinline__ void hm_sp_stage(const HmAggArgs& a, uint32_t v, bool v_ok, uint32_t nk, uint32_t b,
                                            uint32_t q, uint32_t zmask, uint32_t lane, uint32_t* sb)
{
    const uint32_t j = lane & (W - 1);
    const uint64_t segm = W == 64 ? ~0ull : (lane >> 5) ? 0xFFFFFFFF00000000ull : 0x00000000FFFFFFFFull;
    const uint32_t nx = __shfl_down(v, 1, 64);
    const uint32_t cr = hm_compact7(v >> 1), cc = hm_compact7(v);
    const uint32_t bl = b << 24;
    /* the element ends its level-l cell for the levels below half the bit
     * length of (its code ^ the next one's), every level if it is the last;
     * a cell starts after the previous end in the segment: one ballot a level */
    const uint32_t hl = !v_ok ? 0u : (j + 1 == nk) ? 32u : (33u - (uint32_t)__clz((int)(v ^ nx))) >> 1;
    const uint64_t below = segm & ((1ull << lane) - 1ull);
    const uint32_t s0 = lane & ~(uint32_t)(W - 1);   /* the segment's first lane */
    for (int l = 0; l < a.lg; l++) {
        if (!((zmask >> l) & 1u)) continue;
        const bool end = (uint32_t)l < hl;
        const uint64_t bal = __ballot(end) & segm;
        if (end) {
            const uint64_t pe = bal & below;
            const uint32_t start = pe ? 64u - (uint32_t)__clzll((long long)pe) : s0;
            sb[q + (uint32_t)__popcll(pe)] = bl | ((uint32_t)l << 21) | ((cr >> l) << 14) | ((cc >> l) << 7) | (lane - start + 1);
        }
        q += (uint32_t)__popcll(bal);
    }
}

/* n staged cells to keys / counts [g, g + n): every lane two 8-B stores of
 * consecutive cells, so each 64-B line is written whole by one instruction
 * (the per-level stores of hm_sp_emit leave lines written in pieces by
 * several instructions; skew aggregation 3.88-3.92 -> 3.53-3.77 ms,
 * profiles/r6/small_pairs_block_res_ab.jsonl) */
__device__ __forceinline__ void hm_sp_flush(const HmAggArgs& a, const uint32_t* sb, uint32_t n, uint64_t g,
                                            uint64_t cl, uint32_t lane)
{
    const uint32_t clo = (uint32_t)cl, chi = (uint32_t)(cl >> 32);
    for (uint32_t i0 = 0; i0 < n; i0 += 64) {
        const uint32_t i = i0 + lane;
        const uint32_t c = sb[i < n ? i : 0u];
        const int b = (int)((c >> 24) & 63u), l = (int)((c >> 21) & 7u);
        const uint32_t crow = (uint32_t)__shfl((int)chi, b, 64), ccol = (uint32_t)__shfl((int)clo, b, 64);
        const int s = a.lg - l;
        const uint32_t row = (crow << s) | ((c >> 14) & 127u), col = (ccol << s) | ((c >> 7) & 127u);
        const uint64_t p = g + i;
        if (i < n && p < a.out.capacity) {
            a.out.keys[p] = ((uint64_t)(a.Z - l) << 58) | ((uint64_t)row << 29) | col;
            a.out.counts[p] = (uint64_t)(c & 127u);
        }
    }
}

/* The waves of a block reserve their cells together: one cursor atomic per
 * block and round (HM_SPP_WAVES waves' sub-batches of <= 32 rows) instead of
 * one per wave sub-batch (~65K on the skew cloud, on ONE word; skew
 * aggregation -0.3 ms.  The "no atomic" timing builds of
 * profiles/r6/small_pairs_atomics_ab.jsonl overstate the atomics' cost: their
 * made-up positions overlapped, and WRITE_SIZE showed them writing 0.57 of
 * the 6.1 GB of cells, profiles/r6/small_pairs_pmc_bytes.txt).  Block
 * batches (HM_SPP_WAVES x spbatch consecutive buckets) come from a counter,
 * one atomic per block batch.  Rounds are block-synchronous: pass 1 of every
 * wave, a barrier, the reservation (wave 0), a barrier, pass 2.  (An extra
 * wave for the atomics, so that they do not queue behind wave 0's cell
 * stores, measured slower: 9-wave blocks fit 2 to a CU, not 3.) */
template <int NWB>
__global__ __launch_bounds__(64 * NWB) void k_small_pairs(HmAggArgs a)
{
    __shared__ uint16_t cds[NWB][HM_SPP_ROWS][64];   /* a round's rows of sorted codes per wave */
    __shared__ uint2 gsc[NWB][64];          /* hm_sp_key's run marks */
#if HM_SPP_STAGE
    __shared__ uint32_t sbuf[NWB][HM_SPP_STAGE_CELLS];   /* staged cells (hm_sp_stage) */
#endif
    __shared__ uint32_t s_wtot[NWB];        /* the round's cells per wave */
    __shared__ unsigned long long s_base;   /* the round's reservation */
    __shared__ uint32_t s_batch;            /* the block's next batch */
    __shared__ uint32_t s_more[2];          /* a wave has rows for the next round (by round parity) */
    const uint32_t lane = hm_lane();
    const uint32_t wl = threadIdx.x >> 6;
    const bool alloc = wl == 0;   /* the wave of the atomics (wave-uniform) */
    const uint32_t wc = wl;
    const uint32_t zmask = hm_small_zmask(a);
    const uint32_t per_block = NWB * a.spbatch;
    /* (block barriers are LDS-only: a __syncthreads would also wait for the
     * waves' cell stores) */
    if (alloc && lane == 0) {
        s_batch = atomicAdd(a.spq, 1u);
        s_more[0] = s_more[1] = 0u;
    }
    hm_lds_barrier();
    uint32_t rr = 0;   /* round parity */
#if defined(HM_STAMPS) && HM_STAMPS == 7
    /* cycles summed per block: worker 0's pass 1, first-barrier wait, second-
     * barrier wait, pass 2; the atomics (wave 0); rounds; block batches */
    unsigned long long st7[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    unsigned long long t7 = __builtin_amdgcn_s_memtime();
#define HM_ST7(k) do { const unsigned long long n7 = __builtin_amdgcn_s_memtime(); st7[k] += n7 - t7; t7 = n7; } while (0)
#else
#define HM_ST7(k) do { } while (0)
#endif
    for (;;) {
        const uint32_t kb = s_batch;   /* block-uniform */
        if ((uint64_t)kb * per_block >= a.B.count) break;
        uint32_t kn = 0;   /* (thread 0) the block's batch after this one */
        const uint64_t bl64 = (uint64_t)kb * per_block + wc * a.spbatch + lane;
        const bool in = lane < a.spbatch && bl64 < a.B.count;
        const uint32_t bl = in ? (uint32_t)bl64 : 0u;
        const uint32_t nkl = in ? a.B.nkeys[bl] : 0u;
        const bool small = in & (nkl <= HM_SPW_SPLIT);
        const uint32_t nrl = small ? a.B.nruns[bl] : 0u;
        const bool mine = small && hm_sp_fused_ok(nkl, nrl);
        uint64_t mp = __ballot(mine && nkl <= 32), ms = __ballot(mine && nkl > 32);
        const uint32_t rbl = mine ? a.B.rbase[bl] : 0u;
        const uint64_t cl = mine ? a.B.coord[bl] : 0ull;
        if (mine) a.totals[bl] = nkl;
        for (bool first = true;; first = false) {
            /* pass 1: up to 32 rows (pairs first) sorted into LDS; lane 2p + g
             * keeps row p's segment-g cell count.  Software-pipelined: while
             * row p sorts, row p+1's key and row p+2's runs are loading */
            uint32_t segcnt = 0;
            uint64_t mp1 = mp, ms1 = ms;
            const uint32_t nrows = min((uint32_t)HM_SPP_ROWS, (uint32_t)(__popcll(mp) + 1) / 2 + (uint32_t)__popcll(ms));
            if (mp | ms) {   /* wave-uniform */
                struct Row {
                    bool paired, seg;
                    uint32_t nk, r0, nr;
                };
                auto take = [&](bool any) -> Row {
                    Row r;
                    r.paired = !any || mp1 != 0;
                    int src = 0;
                    r.seg = false;
                    if (any && mp1) {
                        const int sl = hm_pair_lane(mp1);
                        r.seg = sl >= 0;
                        src = r.seg ? sl : 0;
                    } else if (any && ms1) {
                        src = __builtin_ctzll(ms1);
                        ms1 &= ms1 - 1;
                        r.seg = true;
                    }
                    const uint32_t nk0 = __shfl(nkl, src, 64), r00 = __shfl(rbl, src, 64), nr0 = __shfl(nrl, src, 64);
                    r.nk = r.seg ? nk0 : 0u;
                    r.r0 = r00;
                    r.nr = r.seg ? nr0 : 0u;
                    return r;
                };
                auto key_of = [&](const Row& r, uint2 run) {
                    return r.paired ? hm_sp_key<32>(a, run, r.seg, r.nk, lane, gsc[wc])
                                    : hm_sp_key<64>(a, run, r.seg, r.nk, lane, gsc[wc]);
                };
                const uint32_t jl = lane & 31u;
                Row A = take(true);
                uint2 runA = hm_sp_run(a, A.seg, A.r0, A.nr, A.paired ? jl : lane);
                Row B = take(nrows > 1);
                uint2 runB = hm_sp_run(a, B.seg, B.r0, B.nr, B.paired ? jl : lane);
                uint32_t keyA = key_of(A, runA);
                for (uint32_t p = 0; p < nrows; p++) {
                    const Row C = take(p + 2 < nrows);
                    const uint2 runC = hm_sp_run(a, C.seg, C.r0, C.nr, C.paired ? jl : lane);
                    const uint32_t keyB = key_of(B, runB);
                    uint32_t v, tot;
                    if (A.paired) tot = hm_sp_sort<32>(a, keyA, A.nk, lane, zmask, v);
                    else tot = hm_sp_sort<64>(a, keyA, A.nk, lane, zmask, v);
                    cds[wc][p][lane] = (uint16_t)v;
                    /* (a single's segment is the whole wave: lane 32 repeats its total) */
                    const uint32_t t0 = __builtin_amdgcn_readlane(tot, 0);
                    const uint32_t t1 = A.paired ? __builtin_amdgcn_readlane(tot, 32) : 0u;
                    segcnt = lane == 2 * p ? t0 : lane == 2 * p + 1 ? t1 : segcnt;
                    A = B;
                    keyA = keyB;
                    B = C;
                    runB = runC;
                }
            }
            HM_ST7(0);
            const uint32_t incl = hm_wave_incl_scan(segcnt);
            const uint32_t excl = incl - segcnt;
            if (lane == 0) {
                s_wtot[wl] = __builtin_amdgcn_readlane(incl, 63);
                if (mp1 | ms1) s_more[rr] = 1u;
            }
            hm_lds_barrier();
            HM_ST7(1);
            const bool more = s_more[rr] != 0u;
            /* one reservation for the block's rows (and, in the first round,
             * the block's next batch, both atomics in flight together) */
            uint32_t wpre = 0, btotal = 0;
#pragma unroll
            for (int w = 0; w < NWB; w++) {
                const uint32_t t = s_wtot[w];
                wpre += (uint32_t)w < wl ? t : 0u;
                btotal += t;
            }
            if (alloc && lane == 0) {
                s_more[rr ^ 1u] = 0u;   /* (last read before the previous round's second barrier) */
                if (first) kn = atomicAdd(a.spq, 1u);
                s_base = btotal ? atomicAdd(a.out.cursor, (unsigned long long)btotal) : 0ull;
            }
            HM_ST7(4);
            hm_lds_barrier();
            HM_ST7(2);
            const uint64_t base = s_base + wpre;
            /* pass 2: the same rows in the same order, codes from LDS */
            uint64_t mp2 = mp, ms2 = ms;
#if HM_SPP_STAGE
            /* the cells go through the wave's LDS buffer (rows in order: the
             * wave's cells are written in order), flushed before a row that
             * does not fit and at the end */
            uint32_t* sb = sbuf[wc];
            uint32_t flushed = 0;   /* this round's cells written so far */
            const auto sync_sb = [&]() {
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            };
#endif
            for (uint32_t p = 0; p < ((mp | ms) ? nrows : 0u); p++) {
                const uint32_t v = cds[wc][p][lane];
#if HM_SPP_STAGE
                const uint32_t rlo = __shfl(excl, (int)(2 * p), 64), rhi = __shfl(incl, (int)(2 * p + 1), 64);
                if (rhi - flushed > HM_SPP_STAGE_CELLS) {
                    sync_sb();
                    hm_sp_flush(a, sb, rlo - flushed, base + flushed, cl, lane);
                    sync_sb();
                    flushed = rlo;
                }
#endif
                if (mp2) {
                    const int sl = hm_pair_lane(mp2);
                    const bool seg = sl >= 0;
                    const int sr = seg ? sl : 0;
                    const uint32_t nk0 = __shfl(nkl, sr, 64);
                    const uint32_t nk = seg ? nk0 : 0u;
#if HM_SPP_STAGE
                    const uint32_t q = __shfl(excl, (int)(2 * p + (lane >> 5)), 64) - flushed;
                    hm_sp_stage<32>(a, v == 0xFFFFu ? 0xFFFFFFFFu : v, seg && (lane & 31u) < nk, nk, (uint32_t)sr, q, zmask,
                                    lane, sb);
#else
                    const uint64_t coord = __shfl(cl, sr, 64);
                    const uint64_t q = base + __shfl(excl, (int)(2 * p + (lane >> 5)), 64);
                    hm_sp_emit<32>(a, v == 0xFFFFu ? 0xFFFFFFFFu : v, seg && (lane & 31u) < nk, nk, coord, q, zmask, lane);
#endif
                } else {
                    const int i = __builtin_ctzll(ms2);
                    ms2 &= ms2 - 1;
                    const uint32_t nk = __shfl(nkl, i, 64);
#if HM_SPP_STAGE
                    const uint32_t q = __shfl(excl, (int)(2 * p), 64) - flushed;
                    hm_sp_stage<64>(a, v == 0xFFFFu ? 0xFFFFFFFFu : v, lane < nk, nk, (uint32_t)i, q, zmask, lane, sb);
#else
                    const uint64_t coord = __shfl(cl, i, 64);
                    const uint64_t q = base + __shfl(excl, (int)(2 * p), 64);
                    hm_sp_emit<64>(a, v == 0xFFFFu ? 0xFFFFFFFFu : v, lane < nk, nk, coord, q, zmask, lane);
#endif
                }
            }
#if HM_SPP_STAGE
            {
                const uint32_t wt = __builtin_amdgcn_readlane(incl, 63);
                sync_sb();
                hm_sp_flush(a, sb, wt - flushed, base + flushed, cl, lane);
                sync_sb();
            }
#endif
            mp = mp1;
            ms = ms1;
            rr ^= 1u;
            HM_ST7(3);
#if defined(HM_STAMPS) && HM_STAMPS == 7
            st7[6]++;
#endif
            /* every wave has read s_base and s_wtot before it reaches the next
             * round's first barrier, and writes them again only after it */
            __builtin_amdgcn_wave_barrier();   /* cds is free for the next round */
            if (!more) break;
        }
        if (alloc && lane == 0) s_batch = kn;   /* (read at this batch's start, before its first round's barriers) */
        hm_lds_barrier();
#if defined(HM_STAMPS) && HM_STAMPS == 7
        st7[7]++;
#endif
    }
#if defined(HM_STAMPS) && HM_STAMPS == 7
    /* wave 0 (which also makes the atomics) in row b, wave 1 in row 4096 + b */
    if (lane == 0 && wl < 2 && blockIdx.x < 4096)
        for (int q = 0; q < 8; q++) g_stamps[(blockIdx.x + wl * 4096u) * 12 + q] = st7[q];
#endif
#undef HM_ST7
}

/* one reservation for every small bucket's cells */
__global__ void k_small_reserve(HmAggArgs a)
{
    if (threadIdx.x == 0) *a.spbase = atomicAdd(a.out.cursor, (unsigned long long)*a.sptotal);
}

template <uint32_t LO, uint32_t HI>
__global__ __launch_bounds__(HM_SPW_THREADS) void k_small_emit(HmAggArgs a)
{
    __shared__ __attribute__((aligned(16))) uint32_t hist[HM_SPW_THREADS / 64][256];
    uint32_t* hw = hist[threadIdx.x >> 6];
    const uint32_t lane = hm_lane();
    const uint32_t nw = gridDim.x * (HM_SPW_THREADS / 64);
    const uint32_t zmask = hm_small_zmask(a);
    const uint64_t base = *a.spbase;
    const uint32_t wid = blockIdx.x * (HM_SPW_THREADS / 64) + (threadIdx.x >> 6);
    const uint32_t step = HmSmallMap<LO>::step(nw, a.spbatch);
    for (uint32_t s0 = HmSmallMap<LO>::first(wid, a.spbatch); HmSmallMap<LO>::bucket(s0, 0, wid, nw) < a.B.count;
         s0 += step) {
        const uint64_t bl64 = HmSmallMap<LO>::bucket(s0, lane, wid, nw);
        const bool in = HmSmallMap<LO>::lane_in(lane, a.spbatch) & (bl64 < a.B.count);
        const uint32_t bl = in ? (uint32_t)bl64 : 0u;
        const uint32_t nkl = in ? a.B.nkeys[bl] : 0u;
        const bool small = in & (LO == 0 || nkl > LO) & (nkl <= HI);
        const uint32_t kbl = small ? a.B.keybase[bl] : 0u;
        const uint64_t cl = small ? a.B.coord[bl] : 0ull;
        const uint64_t ol = small ? a.spoff[bl] : 0ull;
        uint64_t m = __ballot(small);
        if constexpr (LO == 0 && HM_SP_FUSED) {
            const uint32_t nrl = small ? a.B.nruns[bl] : 0u;
            m &= ~__ballot(small && hm_sp_fused_ok(nkl, nrl));   /* k_small_pairs' */
        }
        if constexpr (LO == 0 && !HM_SP_FUSED) {
            /* the <= 32-key buckets in pairs, as k_small_sort took them */
            const uint32_t nrl = small ? a.B.nruns[bl] : 0u;
            uint64_t mt = __ballot(small && nkl <= 32 && nrl <= 4);
            m &= ~mt;
            const uint32_t j = lane & 31;
            const uint64_t segm = (lane >> 5) ? 0xFFFFFFFF00000000ull : 0x00000000FFFFFFFFull;
            while (mt) {
                const int sl = hm_pair_lane(mt);
                const bool seg = sl >= 0;
                const int sr = seg ? sl : 0;
                const uint32_t nk0 = __shfl(nkl, sr, 64);   /* whole wave active (see k_small_sort) */
                const uint32_t nk = seg ? nk0 : 0u, kb = __shfl(kbl, sr, 64);
                const uint64_t coord = __shfl(cl, sr, 64);
                uint64_t q = base + __shfl(ol, sr, 64);
                const bool v_ok = seg && j < nk;
                const uint32_t v = v_ok ? (uint32_t)a.codes[kb + j] : 0xFFFFFFFFu;
                const uint32_t nx = __shfl_down(v, 1, 64), pv = __shfl_up(v, 1, 64);
                for (int l = 0; l < a.lg; l++) {
                    if (!((zmask >> l) & 1u)) continue;
                    const bool head = v_ok && ((j == 0) | ((pv >> (2 * l)) != (v >> (2 * l))));
                    const bool end = v_ok && ((j + 1 == nk) | ((nx >> (2 * l)) != (v >> (2 * l))));
                    /* the segment's last head at or below this lane (its j = 0
                     * lane is one): the cell's first element */
                    const uint64_t hm = __ballot(head) & ((2ull << lane) - 1ull);
                    const uint32_t hl = hm ? 63u - (uint32_t)__clzll((long long)hm) : 0u;
                    const uint32_t start = (uint32_t)__shfl((int)j, (int)hl, 64);
                    const uint64_t bal = __ballot(end) & segm;
                    if (end) {
                        const uint32_t code = v >> (2 * l);
                        const int s = a.lg - l;
                        const uint32_t idx = (hm_compact7(code >> 1) << s) | hm_compact7(code);
                        const uint64_t p = q + hm_mbcnt(bal);
                        if (p < a.out.capacity) {
                            a.out.keys[p] = hm_cell_key(a.Z - l, coord, s, idx);
                            a.out.counts[p] = (uint64_t)(j - start + 1);
                        }
                    }
                    q += (uint64_t)__popcll(bal);
                }
            }
        }
        while (m) {
            const int i = __builtin_ctzll(m);
            m &= m - 1;
            const uint32_t nk = __shfl(nkl, i, 64), kb = __shfl(kbl, i, 64);
            const uint64_t coord = __shfl(cl, i, 64), q = base + __shfl(ol, i, 64);
            hm_small_dispatch<LO, HI>(nk, [&](auto kc) { hm_small_emit<decltype(kc)::value>(a, nk, kb, coord, zmask, q, hw); });
        }
    }
}
/* ------------------------------------------------------------------------ */
/* pooling of bucket totals: zooms z_l .. z_{l-1}+1 (root: down to 0)        */
/* ------------------------------------------------------------------------ */

__global__ __launch_bounds__(HM_POOL_THREADS) void k_pool(HmPoolArgs a)
{
    __shared__ unsigned long long v[HM_MAX_FN];
    __shared__ uint32_t scr[HM_POOL_THREADS / 64 + 1];
    __shared__ unsigned long long sbase;
    const uint32_t p = hm_block_id();
    if (p >= a.nparents) return;
    const uint32_t F = 1u << a.dbits;
    for (uint32_t i = threadIdx.x; i < F; i += HM_POOL_THREADS) v[i] = 0;
    __syncthreads();
    const uint32_t c0 = a.child_begin[p], c1 = a.child_begin[p + 1];
    for (uint32_t c = c0 + threadIdx.x; c < c1; c += HM_POOL_THREADS) v[a.child_digit[c]] = a.child_totals[c];
    __syncthreads();
    const uint64_t pm = a.parent_coord ? a.parent_coord[p] : 0ull;
    hm_pyramid<unsigned long long, HM_POOL_THREADS>(v, a.dbits / 2, a.z_child, pm, a.out, scr, &sbase);
    if (threadIdx.x == 0) {
        if (a.parent_totals) a.parent_totals[p] = v[0];
        if (a.emit_root && v[0] && a.out.zmin == 0) {
            const uint64_t pos = atomicAdd(a.out.cursor, 1ull);
            if (pos < a.out.capacity) {
                a.out.keys[pos] = hm_key(0, 0, 0);
                a.out.counts[pos] = v[0];
            }
        }
    }
}

/* k_pool for levels of <= 64 children per parent (dbits <= 6): one wavefront
 * per parent, HM_POOLW_WAVES parents per block and ONE output reservation per
 * block.  (A block per parent took one same-address cursor atomic per emitted
 * zoom -- 196K of them on the uniform cloud's z8 -> z11 level, ~2.2 ms at the
 * L2's ~88 same-address atomics per microsecond.) */
#define HM_POOLW_WAVES 16
__global__ __launch_bounds__(64 * HM_POOLW_WAVES) void k_pool_waves(HmPoolArgs a)
{
    __shared__ unsigned long long lv[HM_POOLW_WAVES][64 + 16 + 4 + 1];
    __shared__ uint32_t wtot[HM_POOLW_WAVES];
    __shared__ unsigned long long sbase;
    const uint32_t lane = hm_lane(), w = threadIdx.x >> 6;
    const uint32_t p = hm_block_id() * HM_POOLW_WAVES + w;
    const bool live = p < a.nparents;
    const int lg = a.dbits / 2;
    const uint32_t F = 1u << a.dbits;
    unsigned long long* cur = lv[w];
    if (lane < F) cur[lane] = 0;
    __builtin_amdgcn_wave_barrier();
    const uint32_t c0 = live ? a.child_begin[p] : 0u, c1 = live ? a.child_begin[p + 1] : 0u;
    if (c0 + lane < c1) cur[a.child_digit[c0 + lane]] = a.child_totals[c0 + lane];
    __builtin_amdgcn_wave_barrier();
    const uint64_t pm = (live && a.parent_coord) ? a.parent_coord[p] : 0ull;
    /* levels k = 0 .. lg-1 (zooms z_child - k), each 4^(lg-k) row-major cells,
     * stored one after another in the wave's LDS row */
    unsigned long long val[3];
    uint64_t bal[3];
    uint32_t cnt = 0;
#pragma unroll
    for (int k = 0; k < 3; k++) {
        val[k] = 0;
        bal[k] = 0;
        if (k < lg) {
            const uint32_t nk = 1u << (2 * (lg - k));
            const unsigned long long x = lane < nk ? cur[lane] : 0ull;
            const int z = a.z_child - k;
            val[k] = x;
            bal[k] = __ballot(live && z >= a.out.zmin && z <= a.out.zmax && x != 0ull);
            cnt += (uint32_t)__popcll(bal[k]);
            unsigned long long* nxt = cur + nk;
            if (lane < nk / 4) nxt[lane] = hm_sum4<unsigned long long>(cur, lane, lg - k - 1);
            __builtin_amdgcn_wave_barrier();
            cur = nxt;
        }
    }
    if (live && lane == 0 && a.parent_totals) a.parent_totals[p] = cur[0];
    if (lane == 0) wtot[w] = cnt;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t t = 0;
        for (int i = 0; i < HM_POOLW_WAVES; i++) t += wtot[i];
        sbase = t ? atomicAdd(a.out.cursor, (unsigned long long)t) : 0ull;
    }
    __syncthreads();
    uint64_t base = sbase;
    for (uint32_t i = 0; i < w; i++) base += wtot[i];
#pragma unroll
    for (int k = 0; k < 3; k++) {
        if (k < lg) {
            if ((bal[k] >> lane) & 1ull) {
                const uint64_t pos = base + hm_mbcnt(bal[k]);
                if (pos < a.out.capacity) {
                    a.out.keys[pos] = hm_cell_key(a.z_child - k, pm, lg - k, lane);
                    a.out.counts[pos] = val[k];
                }
            }
            base += (uint64_t)__popcll(bal[k]);
        }
    }
}

/* ------------------------------------------------------------------------ */
/* host launchers                                                            */
/* ------------------------------------------------------------------------ */

__global__ __launch_bounds__(256) void k_fill(HmFill f)
{
    const uint64_t stride = (uint64_t)gridDim.x * 256, t = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    for (int e = 0; e < f.k; e++) {
        const uint32_t w = f.word[e];
        if (f.unit[e] == 16) {
            uint4* p = (uint4*)f.p[e];
            const uint4 v = make_uint4(w, w, w, w);
            for (uint64_t i = t; i < f.bytes[e] / 16; i += stride) p[i] = v;
        } else if (f.unit[e] == 4) {
            uint32_t* p = (uint32_t*)f.p[e];
            for (uint64_t i = t; i < f.bytes[e] / 4; i += stride) p[i] = w;
        } else {
            uint8_t* p = (uint8_t*)f.p[e];
            for (uint64_t i = t; i < f.bytes[e]; i += stride) p[i] = (uint8_t)w;
        }
    }
}

void hm_fill_add(HmFill& f, void* p, int value, uint64_t bytes)
{
    if (!bytes) return;
    const uint32_t b = (uint32_t)value & 0xFFu;
    const uintptr_t a = (uintptr_t)p;
    f.p[f.k] = p;
    f.bytes[f.k] = bytes;
    f.word[f.k] = b * 0x01010101u;
    f.unit[f.k] = (a % 16 == 0 && bytes % 16 == 0) ? 16u : (a % 4 == 0 && bytes % 4 == 0) ? 4u : 1u;
    f.k++;
}

void hm_launch_fill(hipStream_t s, const HmFill& f)
{
    if (!f.k) return;
    uint64_t most = 0;
    for (int e = 0; e < f.k; e++) most = std::max<uint64_t>(most, f.bytes[e] / f.unit[e]);
    const uint64_t blocks = std::min<uint64_t>(2048, std::max<uint64_t>(1, (most + 255) / 256));
    hipLaunchKernelGGL(k_fill, dim3((unsigned)blocks), dim3(256), 0, s, f);
}

void hm_launch_project(hipStream_t s, const double* lat, const double* lon, int64_t n, int zoom, int64_t* row,
                       int64_t* col, uint8_t* status, unsigned long long* err_word, unsigned long long* slow)
{
    int64_t blocks = (n + 255) / 256;
    if (blocks > 256 * 16) blocks = 256 * 16;
    if (blocks < 1) blocks = 1;
    hipLaunchKernelGGL(k_project, dim3((unsigned)blocks), dim3(256), 0, s, lat, lon, n, zoom, row, col, status,
                       err_word, slow);
}

static uint32_t hm_cu_count()
{
    static int cus = 0;   /* every device of a node is the same part */
    if (cus <= 0) {
        int dev = 0, c = 0;
        if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
            c <= 0)
            c = 256;
        cus = c;
    }
    return (uint32_t)cus;
}

void hm_launch_part1(hipStream_t s, const HmPart1Args& a0, uint32_t grid, bool out16, int mode)
{
    if (grid == 0) return;
    dim3 b(HM_P1_THREADS);
    /* lat/lon input: the whole tiles in one launch (FULL), the partial last
     * tile in another; tile input (mode 1) reads its length on the device */
    const uint32_t full = mode == 1 ? 0u : (uint32_t)std::min<int64_t>(grid, a0.n / HM_T1);
    HmPart1Args a = a0;
    a.tile0 = 0;
#define HM_P1_CASE(T, M, FL, G) hipLaunchKernelGGL((k_project_partition<T, M, FL>), dim3(G), b, 0, s, a)
#define HM_P1_MODES(T, FL, G)                      \
    do {                                           \
        if (mode == 0) HM_P1_CASE(T, 0, FL, G);    \
        else if (mode == 1) HM_P1_CASE(T, 1, FL, G); \
        else HM_P1_CASE(T, 2, FL, G);              \
    } while (0)
    /* whole pairs of 12288-point tiles through the persistent k_l1_ws (one
     * block per CU); they end on a k_l1_fast tile boundary, t0 */
    uint32_t t0 = 0;
    /* (keep-less calls only: with the keep bytes prefetched too the compute
     * waves pass 128 VGPRs and spill) */
    if (HM_L1_WS && HM_L1_FAST && mode == 0 && !a0.keep && full && (int64_t)full == a0.n / HM_T1) {
        const uint32_t m = HM_WS_UNIT * (uint32_t)(a0.n / (HM_WS_UNIT * (int64_t)HM_TW));
        if (m) {
            /* a multiple of HM_L1_SHARDS blocks (or one block per tile): the
             * shard of a tile, block & 7 = tile & 7, is then fixed by the tile,
             * as a region overflow's exact re-run needs */
            const uint32_t cus = std::max<uint32_t>(hm_cu_count() & ~(uint32_t)(HM_L1_SHARDS - 1), HM_L1_SHARDS);
            const dim3 g(m <= cus ? m : cus);
            const dim3 bw(HM_WS_THREADS);
            if (out16) hipLaunchKernelGGL((k_l1_ws<uint16_t, false>), g, bw, 0, s, a, m);
            else hipLaunchKernelGGL((k_l1_ws<uint32_t, false>), g, bw, 0, s, a, m);
            t0 = (uint32_t)((uint64_t)m * HM_TW / HM_T1);
        }
    }
    if (full > t0) {
        a.tile0 = t0;
        const uint32_t nf = full - t0;
        if (mode == 0 && HM_L1_FAST) {
            if (out16) {
                if (a.keep) hipLaunchKernelGGL((k_l1_fast<uint16_t, true>), dim3(nf), b, 0, s, a);
                else hipLaunchKernelGGL((k_l1_fast<uint16_t, false>), dim3(nf), b, 0, s, a);
            } else {
                if (a.keep) hipLaunchKernelGGL((k_l1_fast<uint32_t, true>), dim3(nf), b, 0, s, a);
                else hipLaunchKernelGGL((k_l1_fast<uint32_t, false>), dim3(nf), b, 0, s, a);
            }
        } else if (out16) HM_P1_MODES(uint16_t, true, nf);
        else HM_P1_MODES(uint32_t, true, nf);
    }
    if (grid > full) {
        a.tile0 = full;
        if (out16) HM_P1_MODES(uint16_t, false, grid - full);
        else HM_P1_MODES(uint32_t, false, grid - full);
    }
#undef HM_P1_MODES
#undef HM_P1_CASE
}

/* exact resolution of the points k_project_partition (mode 0) deferred */
__global__ __launch_bounds__(256) void k_redo(HmRedoArgs a)
{
    const uint64_t n = min((uint64_t)*a.redo_count, a.cap);   /* the list holds at most cap */
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t q = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; q < n; q += stride) {
        const uint32_t i = a.redo_idx[q];
        int64_t r = 0, c = 0;
        int st = hm_row_exact(a.lat[i], a.Z, &r);
        if (st == HM_OK) st = hm_col_exact(a.lon[i], a.Z, &c);
        const bool kept = !a.keep || a.keep[i];
        const uint64_t lim = 1ull << a.Z;
        if (st != HM_OK) atomicMin(a.err_word, ((unsigned long long)i << 8) | (unsigned long long)st);
        const bool good = (st == HM_OK) & kept;
        const bool outside = good & (((uint64_t)r >= lim) | ((uint64_t)c >= lim));
        hm_exotic_append(a.x, outside, r, c, (int64_t)i);
        if (good & !outside) {
            const unsigned long long o = atomicAdd(a.out_count, 1ull);
            a.rows_out[o] = r;
            a.cols_out[o] = c;
        }
    }
}

void hm_launch_redo(hipStream_t s, const HmRedoArgs& a, uint64_t n)
{
    uint64_t blocks = (n + 255) / 256;
    if (blocks > 1024) blocks = 1024;   /* grid-stride: most calls have a handful of points */
    if (blocks < 1) blocks = 1;
    hipLaunchKernelGGL(k_redo, dim3((unsigned)blocks), dim3(256), 0, s, a);
}

/* the exotic list overflowed its first capacity: rebuild it over every point */
template <bool FROM_TILES>
__global__ __launch_bounds__(256) void k_collect_exotic(const double* lat, const double* lon, const int64_t* rows,
                                                        const int64_t* cols, const uint8_t* keep, int64_t n, int Z,
                                                        HmExotic x)
{
    __shared__ double tab[HM_YTAB_N];
    if (!FROM_TILES) hm_load_ytab(tab);
    __syncthreads();
    const uint64_t lim = 1ull << Z;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    const int64_t n_up = (n + 63) & ~63ll;   /* whole waves stay in the loop */
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n_up; i += stride) {
        int64_t r = 0, c = 0;
        int st = HM_E_ARG;
        if (i < n) {
            if (FROM_TILES) {
                r = rows[i];
                c = cols[i];
                st = HM_OK;
            } else {
                int slow = 0;
                st = hm_project_point(lat[i], lon[i], Z, &r, &c, &slow, tab);
            }
        }
        const bool kept = i < n && (!keep || keep[i]);
        hm_exotic_append(x, kept & (st == HM_OK) & (((uint64_t)r >= lim) | ((uint64_t)c >= lim)), r, c, i);
    }
}

void hm_launch_collect_exotic(hipStream_t s, const double* lat, const double* lon, const int64_t* rows,
                              const int64_t* cols, const uint8_t* keep, int64_t n, int Z, HmExotic x)
{
    int64_t blocks = (n + 255) / 256;
    if (blocks > 4096) blocks = 4096;
    if (blocks < 1) blocks = 1;
    if (rows)
        hipLaunchKernelGGL(k_collect_exotic<true>, dim3((unsigned)blocks), dim3(256), 0, s, lat, lon, rows, cols, keep,
                           n, Z, x);
    else
        hipLaunchKernelGGL(k_collect_exotic<false>, dim3((unsigned)blocks), dim3(256), 0, s, lat, lon, rows, cols, keep,
                           n, Z, x);
}

/* grouped counts: exact tile of every point (errors in input order), and a
 * list of the kept ones with their group and input index */
/* Kept points as a (row, col, group, index) list for the general path.  A
 * block takes HM_PL_PPT * 256 consecutive points per step: projections in
 * registers, one block scan, ONE output reservation per step (one reservation
 * per wave on a single counter saturated it: ~88 per us, 18.8 ms per 1e8
 * points).  The list is in no particular order. */
#define HM_PL_PPT 16
__global__ __launch_bounds__(256) void k_project_list(const double* lat, const double* lon, const uint8_t* keep,
                                                      const uint32_t* group, int64_t n, int Z, int64_t* row,
                                                      int64_t* col, uint32_t* grp, int64_t* idx,
                                                      unsigned long long* count, unsigned long long* err_word)
{
    __shared__ double tab[HM_YTAB_N];
    __shared__ uint32_t scr[256 / 64 + 1];
    __shared__ unsigned long long base_s;
    hm_load_ytab(tab);
    __syncthreads();
    constexpr int64_t TILE = 256 * HM_PL_PPT;
    for (int64_t t0 = (int64_t)blockIdx.x * TILE; t0 < n; t0 += (int64_t)gridDim.x * TILE) {
        int64_t r[HM_PL_PPT], c[HM_PL_PPT];
        uint32_t pm = 0;
#pragma unroll
        for (int k = 0; k < HM_PL_PPT; k++) {
            const int64_t i = t0 + (int64_t)k * 256 + threadIdx.x;
            r[k] = 0;
            c[k] = 0;
            int st = HM_E_ARG;
            if (i < n) {
                int slow = 0;
                st = hm_project_point(lat[i], lon[i], Z, &r[k], &c[k], &slow, tab);
                if (st != HM_OK) atomicMin(err_word, ((unsigned long long)i << 8) | (unsigned long long)st);
            }
            pm |= (uint32_t)(i < n && st == HM_OK && (!keep || keep[i])) << k;
        }
        uint32_t tot;
        uint32_t pos = hm_block_excl_scan<256>((uint32_t)__popc(pm), scr, &tot);
        if (threadIdx.x == 0) base_s = tot ? atomicAdd(count, (unsigned long long)tot) : 0ull;
        __syncthreads();
        const unsigned long long b = base_s;
        __syncthreads();
#pragma unroll
        for (int k = 0; k < HM_PL_PPT; k++) {
            if ((pm >> k) & 1u) {
                const int64_t i = t0 + (int64_t)k * 256 + threadIdx.x;
                const uint64_t q = b + pos++;
                row[q] = r[k];
                col[q] = c[k];
                grp[q] = group ? group[i] : 0u;
                idx[q] = i;
            }
        }
    }
}

void hm_launch_project_list(hipStream_t s, const double* lat, const double* lon, const uint8_t* keep,
                            const uint32_t* group, int64_t n, int Z, int64_t* row, int64_t* col, uint32_t* grp,
                            int64_t* idx, unsigned long long* count, unsigned long long* err_word)
{
    int64_t blocks = (n + 256 * HM_PL_PPT - 1) / (256 * HM_PL_PPT);
    if (blocks > 4096) blocks = 4096;
    if (blocks < 1) blocks = 1;
    hipLaunchKernelGGL(k_project_list, dim3((unsigned)blocks), dim3(256), 0, s, lat, lon, keep, group, n, Z, row, col,
                       grp, idx, count, err_word);
}

/* The same list as general-path keys (hm_genkey.h), built while projecting:
 * the kept points' 128-bit (group, super tile, Morton) keys, compacted, and
 * the OR / AND of all keys (the radix sort skips digits they agree on).
 * Errors (projection, or a tile beyond the key's fields) by input index. */
__global__ __launch_bounds__(256) void k_project_keys(const double* lat, const double* lon, const uint8_t* keep,
                                                      const uint32_t* group, int64_t n, int Z, uint64_t* klo,
                                                      uint64_t* khi, unsigned long long* count,
                                                      unsigned long long* err_word, unsigned long long* orand)
{
    __shared__ double tab[HM_YTAB_N];
    __shared__ uint32_t scr[256 / 64 + 1];
    __shared__ unsigned long long base_s;
    hm_load_ytab(tab);
    __syncthreads();
    unsigned long long o_lo = 0, o_hi = 0, n_lo = ~0ull, n_hi = ~0ull;
    constexpr int64_t TILE = 256 * HM_PL_PPT;
    for (int64_t t0 = (int64_t)blockIdx.x * TILE; t0 < n; t0 += (int64_t)gridDim.x * TILE) {
        hm_u128 k[HM_PL_PPT];
        uint32_t pm = 0;
#pragma unroll
        for (int j = 0; j < HM_PL_PPT; j++) {
            const int64_t i = t0 + (int64_t)j * 256 + threadIdx.x;
            k[j] = 0;
            bool ok = false;
            if (i < n) {
                /* every point projects (and raises) first, kept or not */
                int64_t r = 0, c = 0;
                int slow = 0;
                int st = hm_project_point(lat[i], lon[i], Z, &r, &c, &slow, tab);
                if (st == HM_OK && (!keep || keep[i])) {
                    k[j] = hm_gen_key(r, c, group ? group[i] : 0u, Z, &ok);
                    if (!ok) st = HM_E_RANGE;   /* representable by the reference, beyond this path's key */
                }
                if (st != HM_OK) atomicMin(err_word, ((unsigned long long)i << 8) | (unsigned long long)st);
            }
            pm |= (uint32_t)ok << j;
            if (ok) {
                o_lo |= (unsigned long long)k[j];
                o_hi |= (unsigned long long)(k[j] >> 64);
                n_lo &= (unsigned long long)k[j];
                n_hi &= (unsigned long long)(k[j] >> 64);
            }
        }
        uint32_t tot;
        uint32_t pos = hm_block_excl_scan<256>((uint32_t)__popc(pm), scr, &tot);
        if (threadIdx.x == 0) base_s = tot ? atomicAdd(count, (unsigned long long)tot) : 0ull;
        __syncthreads();
        const unsigned long long b = base_s;
        __syncthreads();
#pragma unroll
        for (int j = 0; j < HM_PL_PPT; j++)
            if ((pm >> j) & 1u) {
                klo[b + pos] = (uint64_t)k[j];
                khi[b + pos] = (uint64_t)(k[j] >> 64);
                pos++;
            }
    }
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

/* The keys' fast form: hm_project_fast (no transcendental, no call) for
 * every point; the points it cannot settle (guard band, |lat| > 85.05, a tile
 * outside the square, non-finite input: a few per million) are listed for
 * k_project_keys_slow, which takes them through k_project_keys' exact code --
 * the keys are a multiset (sorted next), so where a key lands in the
 * compacted list is free, and errors go by input index (atomicMin) either
 * way.  (k_project_keys with the exact chain inline ran at 2 waves a SIMD:
 * 2.1 ms for 1e8 points.)  Dense (no keep mask): every point's key goes to
 * its own index -- no compaction, no per-tile cursor atomic (one address:
 * 49K of them took ~0.5 ms for 1e8 points).  write_hi = 0: the high halves
 * are not stored (the caller runs the pass again with them when the keys
 * turn out wide; narrow keys share one high half, which the sort and the
 * cascade take as a constant). */
#define HM_PK_PPT 8
__global__ __launch_bounds__(256) void k_project_keys_fast(HmPkArgs a)
{
    __shared__ double tab[HM_YTAB_N];
    __shared__ uint32_t scr[256 / 64 + 1];
    __shared__ unsigned long long base_s;
    hm_load_ytab(tab);
    __syncthreads();
    const double scale = hm_exp2i(a.Z), kz = HM_INV360 * scale;
    unsigned long long o_lo = 0, o_hi = 0, n_lo = ~0ull, n_hi = ~0ull;
    constexpr int64_t TILE = 256 * HM_PK_PPT;
    for (int64_t t0 = (int64_t)blockIdx.x * TILE; t0 < a.n; t0 += (int64_t)gridDim.x * TILE) {
        hm_u128 k[HM_PK_PPT];
        uint32_t pm = 0, sm = 0;
#pragma unroll
        for (int j = 0; j < HM_PK_PPT; j++) {
            const int64_t i = t0 + (int64_t)j * 256 + threadIdx.x;
            k[j] = 0;
            if (i < a.n) {
                int32_t r, c;
                const int fast = hm_project_fast(a.lat[i], a.lon[i], scale, kz, &r, &c, tab);
                sm |= (uint32_t)(!fast) << j;
                if (fast && (!a.keep || a.keep[i])) {
                    bool ok = false;
                    k[j] = hm_gen_key(r, c, a.group ? a.group[i] : 0u, a.Z, &ok);
                    if (!ok) atomicMin(a.err_word, ((unsigned long long)i << 8) | (unsigned long long)HM_E_RANGE);
                    pm |= (uint32_t)ok << j;
                    if (ok) {
                        o_lo |= (unsigned long long)k[j];
                        o_hi |= (unsigned long long)(k[j] >> 64);
                        n_lo &= (unsigned long long)k[j];
                        n_hi &= (unsigned long long)(k[j] >> 64);
                    }
                }
            }
        }
        /* the unsettled points, one list reservation a wave */
#pragma unroll
        for (int j = 0; j < HM_PK_PPT; j++) {
            const bool sl = (sm >> j) & 1u;
            const uint64_t m = __ballot(sl);
            if (!m) continue;
            unsigned long long at = 0;
            if (hm_lane() == 0) at = atomicAdd(a.redo_count, (unsigned long long)__popcll(m));
            at = __shfl(at, 0, 64) + hm_mbcnt(m);
            if (sl && at < a.redo_cap) a.redo_idx[at] = (uint32_t)(t0 + (int64_t)j * 256 + threadIdx.x);
        }
        if (a.dense) {
            /* no keep mask: every point has a key (or the call fails), at its index */
#pragma unroll
            for (int j = 0; j < HM_PK_PPT; j++)
                if ((pm >> j) & 1u) {
                    const int64_t i = t0 + (int64_t)j * 256 + threadIdx.x;
                    a.klo[i] = (uint64_t)k[j];
                    if (a.write_hi) a.khi[i] = (uint64_t)(k[j] >> 64);
                }
            continue;
        }
        uint32_t tot;
        uint32_t pos = hm_block_excl_scan<256>((uint32_t)__popc(pm), scr, &tot);
        if (threadIdx.x == 0) base_s = tot ? atomicAdd(a.count, (unsigned long long)tot) : 0ull;
        __syncthreads();
        const unsigned long long b = base_s;
        __syncthreads();
#pragma unroll
        for (int j = 0; j < HM_PK_PPT; j++)
            if ((pm >> j) & 1u) {
                a.klo[b + pos] = (uint64_t)k[j];
                if (a.write_hi) a.khi[b + pos] = (uint64_t)(k[j] >> 64);
                pos++;
            }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        o_lo |= __shfl_xor(o_lo, o, 64);
        o_hi |= __shfl_xor(o_hi, o, 64);
        n_lo &= __shfl_xor(n_lo, o, 64);
        n_hi &= __shfl_xor(n_hi, o, 64);
    }
    /* one OR / AND per block: these four words take every block's atomics
     * (per wave they were 32K same-address atomics a word for 1e8 points) */
    __shared__ unsigned long long red[4][4];
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
        atomicOr(&a.orand[0], o_lo);
        atomicOr(&a.orand[1], o_hi);
        atomicAnd(&a.orand[2], n_lo);
        atomicAnd(&a.orand[3], n_hi);
    }
}

/* the listed points through the exact chain (k_project_keys' per-point code);
 * a list that overflowed its capacity: every point the fast form cannot
 * settle, found again by a sweep of the whole input */
__global__ __launch_bounds__(256) void k_project_keys_slow(HmPkArgs a)
{
    __shared__ double tab[HM_YTAB_N];
    hm_load_ytab(tab);
    __syncthreads();
    const uint64_t listed = *a.redo_count;
    const bool sweep = listed > a.redo_cap;
    const uint64_t m = sweep ? (uint64_t)a.n : listed;
    const double scale = hm_exp2i(a.Z), kz = HM_INV360 * scale;
    unsigned long long o_lo = 0, o_hi = 0, n_lo = ~0ull, n_hi = ~0ull;
    for (uint64_t v = (uint64_t)blockIdx.x * 256 + threadIdx.x; v < m; v += (uint64_t)gridDim.x * 256) {
        const int64_t i = sweep ? (int64_t)v : (int64_t)a.redo_idx[v];
        if (sweep) {
            int32_t r, c;
            if (hm_project_fast(a.lat[i], a.lon[i], scale, kz, &r, &c, tab)) continue;
        }
        int64_t r = 0, c = 0;
        int slow = 0;
        int st = hm_project_point(a.lat[i], a.lon[i], a.Z, &r, &c, &slow, tab);
        bool ok = false;
        hm_u128 k = 0;
        if (st == HM_OK && (!a.keep || a.keep[i])) {
            k = hm_gen_key(r, c, a.group ? a.group[i] : 0u, a.Z, &ok);
            if (!ok) st = HM_E_RANGE;
        }
        if (st != HM_OK) atomicMin(a.err_word, ((unsigned long long)i << 8) | (unsigned long long)st);
        if (ok) {
            const unsigned long long q = a.dense ? (unsigned long long)i : atomicAdd(a.count, 1ull);
            a.klo[q] = (uint64_t)k;
            if (a.write_hi) a.khi[q] = (uint64_t)(k >> 64);
            o_lo |= (unsigned long long)k;
            o_hi |= (unsigned long long)(k >> 64);
            n_lo &= (unsigned long long)k;
            n_hi &= (unsigned long long)(k >> 64);
        }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        o_lo |= __shfl_xor(o_lo, o, 64);
        o_hi |= __shfl_xor(o_hi, o, 64);
        n_lo &= __shfl_xor(n_lo, o, 64);
        n_hi &= __shfl_xor(n_hi, o, 64);
    }
    if (hm_lane() == 0 && (o_lo | o_hi)) {
        atomicOr(&a.orand[0], o_lo);
        atomicOr(&a.orand[1], o_hi);
        atomicAnd(&a.orand[2], n_lo);
        atomicAnd(&a.orand[3], n_hi);
    }
}

void hm_launch_project_keys(hipStream_t s, const HmPkArgs& a)
{
    int64_t blocks = (a.n + 256 * HM_PK_PPT - 1) / (256 * HM_PK_PPT);
    if (blocks > 2048) blocks = 2048;
    if (blocks < 1) blocks = 1;
    hipLaunchKernelGGL(k_project_keys_fast, dim3((unsigned)blocks), dim3(256), 0, s, a);
    hipLaunchKernelGGL(k_project_keys_slow, dim3(1024), dim3(256), 0, s, a);
}

void hm_launch_partN(hipStream_t s, const HmPartNArgs& a, uint32_t items, bool out16, bool few_runs)
{
    if (items == 0) return;
    if (few_runs && HM_K2_FR) {
        if (out16)
            hipLaunchKernelGGL(k_partition_fr<uint16_t>, hm_grid2(items), dim3(HM_FR_THREADS), 0, s, a);
        else
            hipLaunchKernelGGL(k_partition_fr<uint32_t>, hm_grid2(items), dim3(HM_FR_THREADS), 0, s, a);
        return;
    }
    if (out16)
        hipLaunchKernelGGL(k_partition<uint16_t>, hm_grid2(items), dim3(HM_PN_THREADS), 0, s, a);
    else
        hipLaunchKernelGGL(k_partition<uint32_t>, hm_grid2(items), dim3(HM_PN_THREADS), 0, s, a);
}

static unsigned hm_grid(uint64_t n, unsigned per, unsigned cap)
{
    uint64_t b = (n + per - 1) / per;
    if (b > cap) b = cap;
    return (unsigned)(b ? b : 1);
}

void hm_launch_rs_count(hipStream_t s, const HmRsArgs& a)
{
    hipLaunchKernelGGL(k_rs_count, dim3(hm_grid(a.nchildren << a.shard_bits, 256, 16384)), dim3(256), 0, s, a);
}

void hm_launch_rs_copy(hipStream_t s, const HmRsArgs& a)
{
    const uint64_t pairs = a.nchildren << a.shard_bits;
    if (pairs == 0) return;   /* a level with no parent buckets (nothing kept) */
    hipLaunchKernelGGL(k_rs_copy, dim3(hm_grid((a.nchildren + 63) / 64, 4, 16384)), dim3(256), 0, s, a);
    hipLaunchKernelGGL(k_rs_copy_big, dim3(1024), dim3(256), 0, s, a);
}

void hm_launch_rs_keys(hipStream_t s, const HmRsArgs& a)
{
    hipLaunchKernelGGL(k_rs_keys, dim3(hm_grid(a.nchildren, 256, 16384)), dim3(256), 0, s, a);
}

/* exclusive scan of v[0, n) -> out, total -> *total.  ndev: the length is
 * min(n, *ndev), read on the device (n: the host's bound, which sizes the
 * grid) -- no read-back before the scan */
void hm_launch_scan(hipStream_t s, const uint64_t* v, uint64_t n, uint64_t* partial, uint64_t* out, uint64_t* total,
                    const uint64_t* ndev)
{
    uint64_t chunk = HM_SCAN_ITEMS;
    while ((n + chunk - 1) / chunk > HM_SCAN_MAXB) chunk += HM_SCAN_ITEMS;
    if (n <= 16 * 1024) {
        hipLaunchKernelGGL(k_scan_one<16>, dim3(1), dim3(1024), 0, s, v, (uint32_t)n, out, total, ndev);
        return;
    }
    const uint32_t nb = (uint32_t)((n + chunk - 1) / chunk);
    const uint32_t g = nb ? nb : 1;
    hipLaunchKernelGGL(k_scan_reduce, dim3(g), dim3(HM_SCAN_THREADS), 0, s, v, n, chunk, partial, ndev);
    if (g <= HM_SCAN_THREADS) {
        hipLaunchKernelGGL(k_scan_down<true>, dim3(g), dim3(HM_SCAN_THREADS), 0, s, v, n, chunk, partial, out, ndev,
                           total);
        return;
    }
    hipLaunchKernelGGL(k_scan_one<4>, dim3(1), dim3(1024), 0, s, partial, g, partial, total, nullptr);
    hipLaunchKernelGGL(k_scan_down<false>, dim3(g), dim3(HM_SCAN_THREADS), 0, s, v, n, chunk, partial, out, ndev,
                       total);
}

void hm_launch_compact(hipStream_t s, const HmCompactArgs& a)
{
    hipLaunchKernelGGL(k_compact, dim3(hm_grid(a.nchildren, 256, 8192)), dim3(256), 0, s, a);
}

void hm_launch_aggregate(hipStream_t s, const HmAggArgs& a, uint32_t items, uint32_t nslots)
{
    if (items) hipLaunchKernelGGL(k_aggregate, hm_grid2(items), dim3(HM_AG_THREADS), 0, s, a);
    if (nslots) hipLaunchKernelGGL(k_aggregate_merged, hm_grid2(nslots), dim3(HM_AG_THREADS), 0, s, a);
}
/* HM_SPW_GRID blocks is 8 waves per SIMD, more than is resident of the
 * kernels holding > 96 SGPRs or > 64 VGPRs (k_small_pairs 7, k_small_sort 5,
 * k_small_emit 4).  HM_SPW_RESIDENT=1 launches only the blocks that fit at
 * once; measured slower (profiles/r6/small_grid_ab.jsonl: hotspot aggregation
 * +50 us, z6-21 +150 us, skew no better): k_small_sort / k_small_emit map
 * buckets to waves statically, and the blocks of the second round that start
 * as the first ones drain even out their uneven shares. */
template <typename K>
static uint32_t hm_spw_grid(K kernel, int& cache, uint32_t wb)
{
    uint32_t g = HM_SPW_GRID;
    if (HM_SPW_RESIDENT) {
        if (cache <= 0) {
            int per = 0;
            if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, kernel, HM_SPW_THREADS, 0) != hipSuccess || per <= 0)
                per = HM_SPW_GRID / 256;
            cache = per;
        }
        g = (uint32_t)cache * hm_cu_count();
    }
    return wb < g ? wb : g;
}

void hm_launch_small(hipStream_t s, const HmAggArgs& a, uint64_t* partial)
{
    if (!a.B.count) return;
    /* batches of <= 64 consecutive buckets per wave, small enough that every
     * wave of the grid gets one when buckets are few (a wave walks its batch
     * serially) */
    HmAggArgs b = a;
    const uint32_t waves = HM_SPW_GRID * (HM_SPW_THREADS / 64);
    b.spbatch = 1;
    while (b.spbatch < 64 && (uint64_t)b.spbatch * waves < a.B.count) b.spbatch <<= 1;
    const uint32_t per_block = b.spbatch * (HM_SPW_THREADS / 64);
    const uint32_t wb = (a.B.count + per_block - 1) / per_block;
    static int occ[5];
    const dim3 t(HM_SPW_THREADS);
    if (HM_SP_FUSED) {
        /* block batches from a counter: a grid of what fits, plus spare blocks
         * that find the counter spent */
        const uint32_t bb = b.spbatch * HM_SPP_WAVES;
        const uint32_t nbb = (a.B.count + bb - 1) / bb;
        const uint32_t gp = HM_SPW_GRID * (HM_SPW_THREADS / 64) / HM_SPP_WAVES;
        hipLaunchKernelGGL(k_small_pairs<HM_SPP_WAVES>, dim3(nbb < gp ? nbb : gp), dim3(64 * HM_SPP_WAVES), 0, s, b);
    }
    hipLaunchKernelGGL((k_small_sort<0, HM_SPW_SPLIT>), dim3(hm_spw_grid(k_small_sort<0, HM_SPW_SPLIT>, occ[1], wb)), t,
                       0, s, b);
    if (HM_SPW_MAX > HM_SPW_SPLIT)
        hipLaunchKernelGGL((k_small_sort<HM_SPW_SPLIT, HM_SPW_MAX>),
                           dim3(hm_spw_grid(k_small_sort<HM_SPW_SPLIT, HM_SPW_MAX>, occ[2], wb)), t, 0, s, b);
    hm_launch_scan(s, b.spcnt, b.B.count, partial, (uint64_t*)b.spoff, b.sptotal);
    hipLaunchKernelGGL(k_small_reserve, dim3(1), dim3(64), 0, s, b);
    hipLaunchKernelGGL((k_small_emit<0, HM_SPW_SPLIT>), dim3(hm_spw_grid(k_small_emit<0, HM_SPW_SPLIT>, occ[3], wb)), t,
                       0, s, b);
    if (HM_SPW_MAX > HM_SPW_SPLIT)
        hipLaunchKernelGGL((k_small_emit<HM_SPW_SPLIT, HM_SPW_MAX>),
                           dim3(hm_spw_grid(k_small_emit<HM_SPW_SPLIT, HM_SPW_MAX>, occ[4], wb)), t, 0, s, b);
}
void hm_launch_pool(hipStream_t s, const HmPoolArgs& a, uint32_t nparents)
{
    if (!nparents) return;
    if (!a.emit_root && a.dbits <= 6)
        hipLaunchKernelGGL(k_pool_waves, hm_grid2((nparents + HM_POOLW_WAVES - 1) / HM_POOLW_WAVES),
                           dim3(64 * HM_POOLW_WAVES), 0, s, a);
    else
        hipLaunchKernelGGL(k_pool, hm_grid2(nparents), dim3(HM_POOL_THREADS), 0, s, a);
}

/* ------------------------------------------------------------------------ */
/* synthetic point clouds (bit-identical to heatmap_amd/synth.py)            */
/* ------------------------------------------------------------------------ */

__device__ __forceinline__ uint64_t hm_splitmix(uint64_t x)
{
    uint64_t z = x + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

__device__ __forceinline__ double hm_u01(uint64_t seed, uint64_t idx, uint32_t lane, uint32_t lanes)
{
    const uint64_t ctr = seed * 0x100000001B3ull + idx * lanes + lane;
    return (double)(hm_splitmix(ctr) >> 11) * 0x1p-53;
}

__global__ __launch_bounds__(256) void k_synth(int kind, uint64_t seed, int64_t start, int64_t n, double* lat,
                                               double* lon, const double* tab, int k)
{
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const uint64_t idx = (uint64_t)(start + i);
        double la, lo;
        if (kind == 0) {
            const double u1 = hm_u01(seed, idx, 0, 2), u2 = hm_u01(seed, idx, 1, 2);
            la = (u1 * 2.0 - 1.0) * 85.0511287798066;
            lo = u2 * 360.0 - 180.0;
        } else if (kind == 1) {
            const double u0 = hm_u01(seed, idx, 0, 9);
            int c = 0;
            while (c < k - 1 && !(tab[3 * k + c] > u0)) c++;
            double sy = hm_u01(seed, idx, 1, 9) + hm_u01(seed, idx, 2, 9);
            sy = sy + hm_u01(seed, idx, 3, 9);
            sy = sy + hm_u01(seed, idx, 4, 9);
            double sx = hm_u01(seed, idx, 5, 9) + hm_u01(seed, idx, 6, 9);
            sx = sx + hm_u01(seed, idx, 7, 9);
            sx = sx + hm_u01(seed, idx, 8, 9);
            const double gy = (sy - 2.0) * 1.7320508075688772;
            const double gx = (sx - 2.0) * 1.7320508075688772;
            la = tab[c] + tab[2 * k + c] * gy;
            lo = tab[k + c] + tab[2 * k + c] * gx;
        } else {
            const double u0 = hm_u01(seed, idx, 0, 3), u1 = hm_u01(seed, idx, 1, 3), u2 = hm_u01(seed, idx, 2, 3);
            const double w = 360.0 / 262144.0;
            if (u0 < 0.9) {
                la = 47.60014 + (u1 - 0.5) * 0.0008;
                lo = (42015.0 + 0.0625 + u2 * 0.875) * w - 180.0;
            } else {
                la = (u1 * 2.0 - 1.0) * 85.0511287798066;
                lo = u2 * 360.0 - 180.0;
            }
        }
        lat[i] = la;
        lon[i] = lo;
    }
}

void hm_launch_synth(hipStream_t s, int kind, uint64_t seed, int64_t start, int64_t n, double* lat, double* lon,
                     const double* tab, int k)
{
    int64_t blocks = (n + 255) / 256;
    if (blocks > 256 * 32) blocks = 256 * 32;
    if (blocks < 1) blocks = 1;
    hipLaunchKernelGGL(k_synth, dim3((unsigned)blocks), dim3(256), 0, s, kind, seed, start, n, lat, lon, tab, k);
}

/* ------------------------------------------------------------------------ */
/* HBM read-stream peak (bench.py's measured_peak): K1's access shape without  */
/* its arithmetic -- two fp64 arrays read once, 16 B per lane per load (the   */
/* double2 loads of k_project_partition), HM_RS_INFLIGHT loads in flight per */
/* lane, one XOR per block written so nothing is dead.                       */
/* ------------------------------------------------------------------------ */
#define HM_RS_THREADS 512
#define HM_RS_V 4   /* 16-B loads in flight per lane and array (8 in all, K1 has 16) */
__global__ __launch_bounds__(HM_RS_THREADS) void k_read_stream(const uint4* __restrict__ a, const uint4* __restrict__ b,
                                                            uint64_t n16, uint64_t* __restrict__ sink)
{
    constexpr uint64_t TILE = (uint64_t)HM_RS_THREADS * HM_RS_V;   /* vectors of each array per tile */
    uint32_t acc = 0;
    for (uint64_t t0 = (uint64_t)blockIdx.x * TILE; t0 < n16; t0 += (uint64_t)gridDim.x * TILE) {
        uint4 va[HM_RS_V], vb[HM_RS_V];
        if (t0 + TILE <= n16) {
#pragma unroll
            for (int k = 0; k < HM_RS_V; k++) {
                va[k] = a[t0 + (uint64_t)k * HM_RS_THREADS + threadIdx.x];
                vb[k] = b[t0 + (uint64_t)k * HM_RS_THREADS + threadIdx.x];
            }
        } else {
#pragma unroll
            for (int k = 0; k < HM_RS_V; k++) {
                const uint64_t i = t0 + (uint64_t)k * HM_RS_THREADS + threadIdx.x;
                va[k] = i < n16 ? a[i] : make_uint4(0u, 0u, 0u, 0u);
                vb[k] = i < n16 ? b[i] : make_uint4(0u, 0u, 0u, 0u);
            }
        }
#pragma unroll
        for (int k = 0; k < HM_RS_V; k++)
            acc ^= va[k].x ^ va[k].y ^ va[k].z ^ va[k].w ^ vb[k].x ^ vb[k].y ^ vb[k].z ^ vb[k].w;
    }
    acc = hm_wave_sum(acc);
    if (hm_lane() == 0 && acc == 0x9E3779B9u) sink[blockIdx.x] = acc;   /* data-dependent: the loads stay live */
}

void hm_launch_read_stream(hipStream_t s, const void* a, const void* b, uint64_t bytes_each, uint64_t* sink)
{
    const uint64_t n16 = bytes_each / 16;
    const uint64_t tile = (uint64_t)HM_RS_THREADS * HM_RS_V;
    uint64_t blocks = (n16 + tile - 1) / tile;
    if (blocks > 256ull * 16) blocks = 256ull * 16;
    if (blocks < 1) blocks = 1;
    hipLaunchKernelGGL(k_read_stream, dim3((unsigned)blocks), dim3(HM_RS_THREADS), 0, s, (const uint4*)a,
                       (const uint4*)b, n16, sink);
}
