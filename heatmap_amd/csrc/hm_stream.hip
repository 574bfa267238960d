/* Resident multi-zoom heatmap for streaming micro-batches (BASELINE config 5,
 * SURVEY.md 8f item 2).
 *
 * The reference recomputes its whole pyramid per Spark job (heatmap.py:152-158)
 * and keys every bin by user group and timespan label (heatmap.py:54-55,62-75).
 * A stream instead folds each micro-batch's cells into tables that stay in HBM:
 *
 *   bucket table  u64 keys {group u32 | period u32}, open addressing; a
 *                 bucket's id is its SLOT INDEX, so interning needs one CAS on
 *                 the key word and no value word (no second write another
 *                 thread would have to wait for).  Periods: an epoch hour
 *                 relative to the stream's base, "undated", or (rollup outputs)
 *                 a day / month / year / alltime label.
 *   cell table    16-B slots {u64 key, u64 count}: key = bucket << cb | cell,
 *                 cell = the pyramid index (4^z - 1)/3 + row * 2^z + col of a
 *                 tile of zoom z (cb bits: 43 at zmax 21).  One insert per
 *                 batch cell; every label (alltime, year, month, day) is a
 *                 rollup of the hour buckets at query time.
 *
 * Per batch: k_stream_buckets interns each kept point's (group, hour) and
 * writes its bucket id; one count pass (hm_count when the batch has one
 * bucket, else the grouped general path with the bucket as group) gives the
 * batch's cells; k_stream_convert checks them (tiles outside the square are
 * refused before anything is inserted) and k_stream_insert folds them in.
 * Rollups (k_stream_rollup) re-key every cell slot to (group or all groups,
 * label) in a scratch table and k_stream_emit lists it.
 */
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/heatmap_amd.h"
#include "hm_device.h"
#include "hm_pipeline.h"
#include "hm_table.h"

__device__ __forceinline__ uint64_t hms_pyr_off(int z) { return ((1ull << (2 * z)) - 1ull) / 3ull; }

/* hm_count key (zoom<<58 | row<<29 | col) -> pyramid cell index */
__device__ __forceinline__ uint64_t hms_cell(uint64_t k)
{
    const int z = (int)(k >> 58);
    const uint64_t r = (k >> 29) & 0x1FFFFFFFull, c = k & 0x1FFFFFFFull;
    return hms_pyr_off(z) + (r << z) + c;
}

__device__ __forceinline__ uint64_t hms_cell_key(uint64_t id, int zmin, int zmax)
{
    int z = zmin;
    while (z < zmax && id >= hms_pyr_off(z + 1)) z++;
    const uint64_t m = id - hms_pyr_off(z);
    return ((uint64_t)z << 58) | ((m >> z) << 29) | (m & ((1ull << z) - 1ull));
}

/* bucket id of key k (interning it), or HMS_NO_BUCKET when the table is full */
__device__ __forceinline__ uint32_t hms_intern(const HmsBuckets& b, uint64_t k, uint32_t* claimed)
{
    uint64_t h = hms_hash(k) & b.mask;
    for (uint64_t probe = 0; probe <= b.mask; probe++) {
        /* a plain (L1-cacheable) read: a key word changes once, EMPTY -> key,
         * so a stale EMPTY only sends us to the CAS, which returns the truth */
        uint64_t cur = b.keys[h];
        if (cur == HMS_EMPTY) {
            const unsigned long long prev =
                atomicCAS((unsigned long long*)&b.keys[h], (unsigned long long)HMS_EMPTY, (unsigned long long)k);
            if (prev == HMS_EMPTY) {
                *claimed += 1;
                return (uint32_t)h;
            }
            cur = prev;
        }
        if (cur == k) return (uint32_t)h;
        h = (h + 1) & b.mask;
    }
    return HMS_NO_BUCKET;
}

/* a bucket met by a wave: flagged with the batch epoch (a plain store -- the
 * waves of a batch start together, so a flag read-then-atomic would put
 * thousands of same-address atomics on one L2 channel); k_stream_collect
 * lists the flagged buckets afterwards */
__device__ __forceinline__ void hms_seen(const HmsBucketArgs& a, uint32_t b)
{
    if (b != HMS_NO_BUCKET && a.bflag[b] != a.epoch) a.bflag[b] = a.epoch;
}

/* Bucket of every kept point: (group or HMS_NOGROUP, hour - base or
 * HMS_UNDATED).  Each wave walks a contiguous range of the batch, HMS_WC
 * (key, bucket) pairs cached in registers (wave-uniform): a point whose key
 * is cached costs no probe and no atomic (a time-ordered batch is one key, a
 * batch of a few hours a few); a miss interns the key once for the wave
 * (ballot match) and evicts round-robin.  Also the list of the batch's
 * distinct buckets and their min/max.  Hours outside [base, base + 2^28) are
 * input errors (first index wins). */
#define HMS_WC 4
__global__ __launch_bounds__(256) void k_stream_buckets(HmsBucketArgs a)
{
    constexpr int U = 4;   /* points per lane per step, loads issued together */
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t wave = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const uint64_t waves = ((uint64_t)gridDim.x * blockDim.x) >> 6;
    const uint64_t per = ((a.n + waves - 1) / waves + 64 * U - 1) / (64 * U) * (64 * U);
    const uint64_t w0 = wave * per, w1 = min(w0 + per, a.n);
    uint32_t claimed = 0, full = 0;
    uint64_t ck[HMS_WC];
    uint32_t cb[HMS_WC];
#pragma unroll
    for (int c = 0; c < HMS_WC; c++) {
        ck[c] = HMS_EMPTY;
        cb[c] = HMS_NO_BUCKET;
    }
    uint32_t victim = 0;
    for (uint64_t i0 = w0; i0 < w1; i0 += 64 * U) {
        uint64_t key[U];
        bool kept[U];
#pragma unroll
        for (int u = 0; u < U; u++) {
            const uint64_t i = i0 + (uint64_t)u * 64 + lane;
            kept[u] = i < w1 && (!a.keep || a.keep[i]);
            const uint32_t h = (a.hour && i < w1) ? a.hour[i] : a.base;
            const uint32_t g = (a.group && i < w1) ? a.group[i] : HMS_NOGROUP;
            if (kept[u] && a.hour && (h < a.base || h - a.base >= HMS_MAX_HOUR_OFFSET)) {
                atomicMin(a.err_word, ((unsigned long long)i << 8) | (unsigned long long)HM_E_RANGE);
                kept[u] = false;
            }
            key[u] = ((uint64_t)g << 32) | (a.hour ? h - a.base : HMS_UNDATED);
        }
#pragma unroll
        for (int u = 0; u < U; u++) {
            uint32_t mine = HMS_NO_BUCKET;
            bool hit = false;
#pragma unroll
            for (int c = 0; c < HMS_WC; c++)
                if (key[u] == ck[c]) {
                    mine = cb[c];
                    hit = true;
                }
            uint64_t pending = __ballot(kept[u] && !hit);
            while (pending) {
                const int leader = __ffsll((unsigned long long)pending) - 1;
                const uint64_t k0 = __shfl((unsigned long long)key[u], leader, 64);
                const uint64_t match = __ballot(kept[u] && key[u] == k0) & pending;
                uint32_t b = 0;
                if ((int)lane == leader) b = hms_intern(a.buckets, k0, &claimed);
                b = __shfl(b, leader, 64);
                if (lane == 0) hms_seen(a, b);
                full |= b == HMS_NO_BUCKET;
#pragma unroll
                for (int c = 0; c < HMS_WC; c++)
                    if (c == (int)victim) {
                        ck[c] = k0;
                        cb[c] = b;
                    }
                victim = (victim + 1) % HMS_WC;
                if ((match >> lane) & 1ull) mine = b;
                pending &= ~match;
            }
            const uint64_t i = i0 + (uint64_t)u * 64 + lane;
            if (kept[u] && a.out) a.out[i] = mine;
        }
    }
    const uint64_t cl = hms_wave_sum(claimed);
    if (lane == 0) {
        if (cl) atomicAdd(&a.state[HMS_ST_BUCKETS], (unsigned long long)cl);
        if (full) atomicAdd(&a.state[HMS_ST_BFULL], 1ull);
    }
}

/* the buckets flagged with this batch's epoch -> the batch's list (one
 * atomic per wave that finds any); HMS_ST_BMM receives one of them (THE one
 * when the batch has a single bucket) */
__global__ __launch_bounds__(256) void k_stream_collect(const uint32_t* __restrict__ bflag, uint64_t nb, uint32_t epoch,
                                                        uint32_t* __restrict__ list, unsigned long long* state)
{
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i0 = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) & ~63ull; i0 < nb; i0 += stride) {
        const uint64_t i = i0 + lane;
        const bool m = i < nb && bflag[i] == epoch;
        const uint64_t bal = __ballot(m);
        if (!bal) continue;
        unsigned long long first = 0;
        if (lane == 0) first = atomicAdd(&state[HMS_ST_NLIST], (unsigned long long)__popcll(bal));
        first = __shfl(first, 0, 64);
        if (m) {
            list[first + hm_mbcnt(bal)] = (uint32_t)i;
            if (hm_mbcnt(bal) == 0) state[HMS_ST_BMM] = i;
        }
    }
}

/* the batch's distinct buckets -> their run index j (loc[bucket]) */
__global__ __launch_bounds__(256) void k_stream_batch_list(const uint32_t* __restrict__ list, uint32_t nlist,
                                                           uint32_t* __restrict__ loc)
{
    const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j < nlist) loc[list[j]] = j;
}

/* points per run: the kept points of each of the batch's buckets, and (run
 * nparts) the points not kept; a block histogram, one atomic per run */
__global__ __launch_bounds__(256) void k_stream_part_count(HmsScatterArgs a)
{
    __shared__ uint32_t h[HMS_MAX_PARTS + 1 + 64];
    const int tid = threadIdx.x;
    const uint32_t np = a.nparts + 1;
    if (tid < (int)np) h[tid] = 0;
    __syncthreads();
    const uint64_t stride = (uint64_t)gridDim.x * 256;
    const uint64_t n_up = (a.n + 255) & ~255ull;
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + tid; i < n_up; i += stride) {
        const bool in = i < a.n;
        const bool kept = in && (!a.keep || a.keep[i]);
        const uint32_t part = in ? (kept ? a.loc[a.bids[i]] : a.nparts) : 0u;
        hm_lds_count(h, HMS_MAX_PARTS + 1, part, in);
    }
    __syncthreads();
    if (tid < (int)np && h[tid]) atomicAdd(&a.cursor[tid], (unsigned long long)h[tid]);
}

/* Gather a batch into bucket-contiguous runs (the partition path for batches
 * of a few buckets): run j = the kept points of the batch's j-th bucket, run
 * nparts = the points not kept (projected for their errors only).  Per block
 * chunk: LDS histogram, one global reservation per run, LDS slot claims. */
__global__ __launch_bounds__(256) void k_stream_scatter(HmsScatterArgs a)
{
    __shared__ uint32_t cur[HMS_MAX_PARTS + 1 + 64];   /* + 64 dummy words */
    __shared__ uint64_t base[HMS_MAX_PARTS + 1];
    const int tid = threadIdx.x;
    const uint32_t np = a.nparts + 1;
    const uint64_t chunk = 256 * 16;
    for (uint64_t c0 = (uint64_t)blockIdx.x * chunk; c0 < a.n; c0 += (uint64_t)gridDim.x * chunk) {
        if (tid < (int)np) cur[tid] = 0;
        __syncthreads();
        uint32_t part[16];
#pragma unroll
        for (int k = 0; k < 16; k++) {
            const uint64_t i = c0 + (uint64_t)k * 256 + tid;
            const bool in = i < a.n;
            const bool kept = in && (!a.keep || a.keep[i]);
            part[k] = in ? (kept ? a.loc[a.bids[i]] : a.nparts) : 0xFFFFFFFFu;
            hm_lds_count(cur, HMS_MAX_PARTS + 1, part[k], in);
        }
        __syncthreads();
        if (tid < (int)np) {
            const uint32_t c = cur[tid];
            base[tid] = a.start[tid] + (c ? atomicAdd(&a.cursor[tid], (unsigned long long)c) : 0ull);
            cur[tid] = 0;
        }
        __syncthreads();
#pragma unroll
        for (int k = 0; k < 16; k++) {
            const uint64_t i = c0 + (uint64_t)k * 256 + tid;
            const bool in = i < a.n;
            const uint32_t pos = hm_lds_claim(cur, HMS_MAX_PARTS + 1, part[k], in);
            if (in) {
                const uint64_t q = base[part[k]] + pos;
                a.lat_out[q] = a.lat[i];
                a.lon_out[q] = a.lon[i];
            }
        }
        __syncthreads();
    }
}

/* hm_count keys of one bucket's cells -> cell-table keys, in place */
__global__ __launch_bounds__(256) void k_stream_rekey(uint64_t* __restrict__ keys, uint64_t m, uint64_t prefix)
{
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < m; i += stride)
        keys[i] = prefix | hms_cell(keys[i]);
}

/* grouped-path records (bucket, zoom, row, col, count) -> cell-table keys;
 * records of tiles outside [0, 2^z)^2 are counted, not converted */
__global__ __launch_bounds__(256) void k_stream_convert(const int64_t* __restrict__ rec, uint64_t m, int cb,
                                                        uint64_t* __restrict__ keys, uint64_t* __restrict__ counts,
                                                        unsigned long long* state)
{
    uint32_t bad = 0;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < m; i += stride) {
        const int64_t* r = rec + 5 * i;
        const int z = (int)r[1];
        const int64_t row = r[2], col = r[3];
        const bool in = row >= 0 && col >= 0 && row < (1ll << z) && col < (1ll << z);
        bad += !in;
        keys[i] = in ? ((uint64_t)r[0] << cb) | (hms_pyr_off(z) + ((uint64_t)row << z) + (uint64_t)col) : HMS_EMPTY;
        counts[i] = (uint64_t)r[4];
    }
    uint64_t v[1] = {bad};
    hms_block_sums(v);
    if (threadIdx.x == 0 && v[0]) atomicAdd(&state[HMS_ST_EXOTIC], (unsigned long long)v[0]);
}

/* Fold n cells into the table.  FROM_COUNT: hm_count keys of one bucket
 * (prefix = bucket << cb); else cell-table keys as k_stream_convert made them. */
template <bool FROM_COUNT>
__global__ __launch_bounds__(256) void k_stream_insert(const uint64_t* __restrict__ keys,
                                                       const uint64_t* __restrict__ counts, uint64_t n,
                                                       uint64_t prefix, HmsTable t)
{
    uint64_t claimed = 0;
    uint32_t overflow = 0;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const uint64_t k = FROM_COUNT ? prefix | hms_cell(keys[i]) : keys[i];
        claimed += hms_insert_unique(t, k, counts[i], &overflow);   /* a batch's cells are distinct */
    }
    uint64_t v[2] = {claimed, overflow};
    hms_block_sums(v);
    if (threadIdx.x == 0) {
        if (v[0]) atomicAdd(&t.state[HMS_ST_OCCUPIED], (unsigned long long)v[0]);
        if (v[1]) atomicAdd(&t.state[HMS_ST_OVERFLOW], (unsigned long long)v[1]);
    }
}

/* Re-insert every occupied slot of `from` into `to` (table growth). */
__global__ __launch_bounds__(256) void k_stream_rehash(HmsTable from, HmsTable to)
{
    uint64_t claimed = 0;
    uint32_t overflow = 0;
    const uint64_t n = from.mask + 1;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const ulonglong2 sl = ((const ulonglong2*)from.slots)[i];
        if (sl.x != HMS_EMPTY) claimed += hms_insert_unique(to, sl.x, sl.y, &overflow);
    }
    uint64_t v[2] = {claimed, overflow};
    hms_block_sums(v);
    if (threadIdx.x == 0) {
        if (v[0]) atomicAdd(&to.state[HMS_ST_OCCUPIED], (unsigned long long)v[0]);
        if (v[1]) atomicAdd(&to.state[HMS_ST_OVERFLOW], (unsigned long long)v[1]);
    }
}

__global__ __launch_bounds__(256) void k_stream_init(HmsTable t)
{
    const uint64_t n = t.mask + 1;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
        ((ulonglong2*)t.slots)[i] = make_ulonglong2(HMS_EMPTY, 0ull);
}

__global__ __launch_bounds__(256) void k_stream_fill(uint64_t* p, uint64_t n, uint64_t v)
{
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) p[i] = v;
}

/* days since 1970-01-01 -> (year, month 1..12): the proleptic Gregorian
 * civil-from-days conversion (400-year eras of 146097 days, March-based years) */
__device__ __forceinline__ void hms_civil(uint32_t days, uint32_t* y, uint32_t* m)
{
    const uint32_t z = days + 719468u;
    const uint32_t era = z / 146097u;
    const uint32_t doe = z - era * 146097u;
    const uint32_t yoe = (doe - doe / 1460u + doe / 36524u - doe / 146096u) / 365u;
    const uint32_t doy = doe - (365u * yoe + yoe / 4u - yoe / 100u);
    const uint32_t mp = (5u * doy + 2u) / 153u;
    const uint32_t mm = mp < 10u ? mp + 3u : mp - 9u;
    *y = yoe + era * 400u + (mm <= 2u);
    *m = mm;
}

/* label period word of an hour bucket for a span; HMS_SKIP: not in the span */
__device__ __forceinline__ uint32_t hms_label(uint32_t pw, uint32_t base, int span)
{
    if (span == HM_SPAN_ALLTIME) return HMS_TYPE_ALLTIME << 28;
    if (pw == HMS_UNDATED) return HMS_SKIP;
    const uint32_t hour = base + pw;
    if (span == HM_SPAN_HOUR) return pw;
    const uint32_t day = hour / 24u;
    if (span == HM_SPAN_DAY) return (HMS_TYPE_DAY << 28) | day;
    uint32_t y, m;
    hms_civil(day, &y, &m);
    if (span == HM_SPAN_MONTH) return (HMS_TYPE_MONTH << 28) | (y * 12u + m - 1u);
    return (HMS_TYPE_YEAR << 28) | y;
}

/* the period a caller sees: epoch hour, days since 1970, year*12 + month-1, year, 0 */
__device__ __forceinline__ uint32_t hms_period_value(uint32_t pw, uint32_t base)
{
    const uint32_t type = pw >> 28;
    if (type == 0) return base + pw;
    if (type == HMS_TYPE_ALLTIME) return 0;
    return pw & 0x0FFFFFFFu;
}

__global__ __launch_bounds__(256) void k_stream_rollup(HmsRollupArgs a)
{
    uint64_t claimed = 0;
    uint32_t overflow = 0, bclaimed = 0, full = 0;
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t n = a.from.mask + 1;
    const uint64_t cmask = (1ull << a.cb) - 1ull;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const ulonglong2 sl = ((const ulonglong2*)a.from.slots)[i];
        if (sl.x == HMS_EMPTY) continue;
        const uint64_t bk = a.buckets.keys[sl.x >> a.cb];
        const uint32_t pw = (uint32_t)bk;
        if ((pw >> 28) != 0 && pw != HMS_UNDATED) continue;   /* not a raw bucket (cannot happen) */
        const uint32_t lp = hms_label(pw, a.base, a.span);
        if (lp == HMS_SKIP) continue;
        if (a.select >= 0 && (int64_t)hms_period_value(lp, a.base) != a.select) continue;
        const uint32_t g = a.merge ? HMS_ALLGROUPS : (uint32_t)(bk >> 32);
        const uint64_t key = ((uint64_t)g << 32) | lp;
        /* the lanes sharing the first lane's label bucket intern it once (a
         * merged rollup is one label for the whole wave); the rest probe alone */
        const uint64_t k0 = __builtin_amdgcn_readfirstlane(key);
        const uint64_t same = __ballot(key == k0);
        uint32_t b = 0;
        if (lane == (uint32_t)(__ffsll((unsigned long long)same) - 1)) b = hms_intern(a.buckets, k0, &bclaimed);
        b = __shfl(b, __ffsll((unsigned long long)same) - 1, 64);
        if (key != k0) b = hms_intern(a.buckets, key, &bclaimed);
        if (b == HMS_NO_BUCKET) {
            full = 1;
            continue;
        }
        claimed += hms_insert(a.to, ((uint64_t)b << a.cb) | (sl.x & cmask), sl.y, &overflow);
    }
    uint64_t v[4] = {claimed, overflow, bclaimed, full};
    hms_block_sums(v);
    if (threadIdx.x == 0) {
        if (v[0]) atomicAdd(&a.to.state[HMS_ST_OCCUPIED], (unsigned long long)v[0]);
        if (v[1]) atomicAdd(&a.to.state[HMS_ST_OVERFLOW], (unsigned long long)v[1]);
        if (v[2]) atomicAdd(&a.state[HMS_ST_BUCKETS], (unsigned long long)v[2]);
        if (v[3]) atomicAdd(&a.state[HMS_ST_BFULL], (unsigned long long)v[3]);
    }
}

/* occupied slots of a rollup table -> (group, period, hm_count key, count).
 * Each wave owns chunks of HMS_XCHUNK slots: it counts the occupied ones,
 * reserves its output with ONE atomic per chunk, then re-reads the (cache-hot)
 * chunk and writes in slot order.  Past `cap`: counted, not written. */
#define HMS_XCHUNK (64 * 64)
__global__ __launch_bounds__(256) void k_stream_emit(HmsEmitArgs a)
{
    const uint64_t n = a.t.mask + 1;   /* power of two >= 1024 */
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t cmask = (1ull << a.cb) - 1ull;
    const uint64_t wave = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const uint64_t waves = ((uint64_t)gridDim.x * blockDim.x) >> 6;
    const ulonglong2* slots = (const ulonglong2*)a.t.slots;
    for (uint64_t c0 = wave * HMS_XCHUNK; c0 < n; c0 += waves * HMS_XCHUNK) {
        const uint64_t c1 = c0 + HMS_XCHUNK < n ? c0 + HMS_XCHUNK : n;
        uint64_t cnt = 0;
        for (uint64_t i = c0 + lane; i < c1; i += 64) cnt += slots[i].x != HMS_EMPTY;
        cnt = hms_wave_sum(cnt);
        if (!cnt) continue;
        unsigned long long first = 0;
        if (lane == 0) first = atomicAdd(a.cursor, (unsigned long long)cnt);
        first = __shfl(first, 0, 64);
        for (uint64_t j0 = c0; j0 < c1; j0 += 64) {
            const ulonglong2 sl = slots[j0 + lane];
            const bool m = sl.x != HMS_EMPTY;
            const uint64_t bal = __ballot(m);
            if (m) {
                const uint64_t pos = first + hm_mbcnt(bal);
                if (pos < a.cap) {
                    const uint64_t bk = a.buckets.keys[sl.x >> a.cb];
                    a.keys_out[pos] = hms_cell_key(sl.x & cmask, a.zmin, a.zmax);
                    a.counts_out[pos] = sl.y;
                    if (a.groups_out) a.groups_out[pos] = (uint32_t)(bk >> 32);
                    if (a.periods_out) a.periods_out[pos] = hms_period_value((uint32_t)bk, a.base);
                }
            }
            first += __popcll(bal);
        }
    }
}

static dim3 hms_grid(uint64_t n)
{
    uint64_t b = (n + 255) / 256;
    if (b > 2048) b = 2048;   /* 8 blocks per CU; one state atomic per block */
    return dim3((unsigned)(b ? b : 1));
}

void hm_launch_stream_buckets(hipStream_t s, const HmsBucketArgs& a)
{
    /* ~8+ steps of 256 points per wave: runs of one key stay in registers */
    uint64_t b = (a.n + 8192 - 1) / 8192;
    if (b > 2048) b = 2048;
    if (a.n) hipLaunchKernelGGL(k_stream_buckets, dim3((unsigned)(b ? b : 1)), dim3(256), 0, s, a);
}

void hm_launch_stream_collect(hipStream_t s, const uint32_t* bflag, uint64_t nb, uint32_t epoch, uint32_t* list,
                              unsigned long long* state)
{
    uint64_t b = (nb + 4095) / 4096;
    if (b > 1024) b = 1024;
    hipLaunchKernelGGL(k_stream_collect, dim3((unsigned)(b ? b : 1)), dim3(256), 0, s, bflag, nb, epoch, list, state);
}

void hm_launch_stream_batch_list(hipStream_t s, const uint32_t* list, uint32_t nlist, uint32_t* loc)
{
    if (nlist) hipLaunchKernelGGL(k_stream_batch_list, dim3((nlist + 255) / 256), dim3(256), 0, s, list, nlist, loc);
}

void hm_launch_stream_part_count(hipStream_t s, const HmsScatterArgs& a)
{
    uint64_t b = (a.n + 32767) / 32768;
    if (b > 512) b = 512;
    if (a.n) hipLaunchKernelGGL(k_stream_part_count, dim3((unsigned)(b ? b : 1)), dim3(256), 0, s, a);
}

void hm_launch_stream_scatter(hipStream_t s, const HmsScatterArgs& a)
{
    uint64_t b = (a.n + 4095) / 4096;
    if (b > 2048) b = 2048;
    if (a.n) hipLaunchKernelGGL(k_stream_scatter, dim3((unsigned)(b ? b : 1)), dim3(256), 0, s, a);
}

void hm_launch_stream_rekey(hipStream_t s, uint64_t* keys, uint64_t m, uint64_t prefix)
{
    if (m) hipLaunchKernelGGL(k_stream_rekey, hms_grid(m), dim3(256), 0, s, keys, m, prefix);
}

void hm_launch_stream_convert(hipStream_t s, const int64_t* rec, uint64_t m, int cb, uint64_t* keys, uint64_t* counts,
                              unsigned long long* state)
{
    if (m) hipLaunchKernelGGL(k_stream_convert, hms_grid(m), dim3(256), 0, s, rec, m, cb, keys, counts, state);
}

void hm_launch_stream_insert(hipStream_t s, const uint64_t* keys, const uint64_t* counts, uint64_t n, bool from_count,
                             uint64_t prefix, const HmsTable& t)
{
    if (!n) return;
    if (from_count)
        hipLaunchKernelGGL(k_stream_insert<true>, hms_grid(n), dim3(256), 0, s, keys, counts, n, prefix, t);
    else
        hipLaunchKernelGGL(k_stream_insert<false>, hms_grid(n), dim3(256), 0, s, keys, counts, n, prefix, t);
}

void hm_launch_stream_init(hipStream_t s, const HmsTable& t)
{
    hipLaunchKernelGGL(k_stream_init, hms_grid(t.mask + 1), dim3(256), 0, s, t);
}

void hm_launch_stream_fill(hipStream_t s, uint64_t* p, uint64_t n, uint64_t v)
{
    if (n) hipLaunchKernelGGL(k_stream_fill, hms_grid(n), dim3(256), 0, s, p, n, v);
}

void hm_launch_stream_rehash(hipStream_t s, const HmsTable& from, const HmsTable& to)
{
    hipLaunchKernelGGL(k_stream_rehash, hms_grid(from.mask + 1), dim3(256), 0, s, from, to);
}

void hm_launch_stream_rollup(hipStream_t s, const HmsRollupArgs& a)
{
    hipLaunchKernelGGL(k_stream_rollup, hms_grid(a.from.mask + 1), dim3(256), 0, s, a);
}

void hm_launch_stream_emit(hipStream_t s, const HmsEmitArgs& a)
{
    const uint64_t chunks = (a.t.mask + HMS_XCHUNK) / HMS_XCHUNK, blocks = (chunks + 3) / 4;
    hipLaunchKernelGGL(k_stream_emit, dim3((unsigned)(blocks < 4096 ? blocks : 4096)), dim3(256), 0, s, a);
}
