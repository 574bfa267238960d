/* Resident multi-zoom heatmap for streaming micro-batches (BASELINE config 5,
 * SURVEY.md 8f item 2).
 *
 * The reference recomputes its whole pyramid per Spark job (heatmap.py:152-158)
 * and keys every bin by user group and timespan label (heatmap.py:54-55,62-75).
 * A stream instead keeps every micro-batch's cells in HBM, log-structured:
 *
 *   bucket table  u64 keys {group u32 | period u32}, open addressing; a
 *                 bucket's id is its SLOT INDEX, so interning needs one CAS on
 *                 the key word and no value word.  Periods: an epoch hour
 *                 relative to the stream's base, "undated", or (rollup outputs)
 *                 a day / month / year / alltime label.
 *   cell log      {u64 key, u64 count} arrays: key = bucket << cb | cell, cell =
 *                 the pyramid index (4^z - 1)/3 + row * 2^z + col of a tile of
 *                 zoom z (cb bits: 43 at zmax 21).  A batch's count pass writes
 *                 its cells straight at the log's tail and k_stream_rekey adds
 *                 the bucket: ingest is an append (no hash-table probe per cell;
 *                 a 4 GB table insert took 0.4 ms per 10M-point batch).
 *
 * Per batch: k_stream_buckets interns each kept point's (group, hour) and
 * writes its bucket id; one count pass (hm_count when the batch has one
 * bucket, one per bucket for a few, else the grouped general path with the
 * bucket as group) writes the batch's cells at the tail.  Queries (rollups:
 * hour, day, month, year, alltime) relabel the log's cells to (group or all
 * groups, label) buckets (k_stream_relabel), sum equal keys with the bucketed
 * LDS merge (hm_cells_merge) and list them (k_stream_emit).  The log is
 * compacted (the same merge) when it fills up or its exact size is asked for.
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
 * nparts) the points not kept; a block histogram over 4096-point chunks (a
 * thread's 16 bucket ids and keep bytes loaded before their run lookups),
 * one atomic per run */
__global__ __launch_bounds__(256) void k_stream_part_count(HmsScatterArgs a)
{
    __shared__ uint32_t h[HMS_MAX_PARTS + 1 + 64];
    const int tid = threadIdx.x;
    const uint32_t np = a.nparts + 1;
    if (tid < (int)np) h[tid] = 0;
    __syncthreads();
    const uint64_t chunk = 256 * 16;
    for (uint64_t c0 = (uint64_t)blockIdx.x * chunk; c0 < a.n; c0 += (uint64_t)gridDim.x * chunk) {
        uint32_t bid[16];
        bool kept[16];
#pragma unroll
        for (int k = 0; k < 16; k++) {
            const uint64_t i = c0 + (uint64_t)k * 256 + tid;
            bid[k] = i < a.n ? a.bids[i] : 0u;
            kept[k] = i < a.n && (!a.keep || a.keep[i]);
        }
#pragma unroll
        for (int k = 0; k < 16; k++) {
            const bool in = c0 + (uint64_t)k * 256 + tid < a.n;
            const uint32_t part = in ? (kept[k] ? a.loc[bid[k]] : a.nparts) : 0u;
            hm_lds_count(h, HMS_MAX_PARTS + 1, part, in);
        }
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

__global__ __launch_bounds__(256) void k_stream_rekey_dev(uint64_t* __restrict__ keys,
                                                          const unsigned long long* __restrict__ m_dev, uint64_t cap,
                                                          const unsigned long long* __restrict__ state, int cb)
{
    const uint64_t m = min((uint64_t)*m_dev, cap);
    const uint64_t prefix = state[HMS_ST_NLIST] ? (uint64_t)(uint32_t)state[HMS_ST_BMM] << cb : 0ull;
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

/* log key -> rollup label key (group or HMS_ALLGROUPS, label period word),
 * or ~0: not in the rollup */
__device__ __forceinline__ uint64_t hms_relabel_key(const HmsRelabelArgs& a, uint64_t k)
{
    const uint64_t bk = a.buckets.keys[k >> a.cb];
    const uint32_t pw = (uint32_t)bk;
    if ((pw >> 28) != 0 && pw != HMS_UNDATED) return ~0ull;   /* not a raw bucket (cannot happen) */
    const uint32_t lp = hms_label(pw, a.base, a.span);
    if (lp == HMS_SKIP) return ~0ull;
    if (a.select >= 0 && (int64_t)hms_period_value(lp, a.base) != a.select) return ~0ull;
    const uint32_t g = a.merge ? HMS_ALLGROUPS : (uint32_t)(bk >> 32);
    return ((uint64_t)g << 32) | lp;
}

/* The log's cells of a rollup, re-keyed to their label buckets (interned) and
 * compacted: a block takes 256 * HMS_RL_PPT cells at a time, counts the ones
 * in the rollup, reserves their room with one atomic and writes them.  The
 * lanes sharing lane 0's label intern it once (a merged rollup is one label
 * per period); the rest probe alone. */
#define HMS_RL_PPT 32
__global__ __launch_bounds__(256) void k_stream_relabel(HmsRelabelArgs a)
{
    __shared__ uint32_t scr[256 / 64 + 1];
    __shared__ unsigned long long sbase;
    const int tid = threadIdx.x;
    const uint64_t cmask = (1ull << a.cb) - 1ull;
    uint32_t bclaimed = 0, full = 0;
    constexpr uint64_t CH = 256 * HMS_RL_PPT;
    for (uint64_t c0 = (uint64_t)blockIdx.x * CH; c0 < a.n; c0 += (uint64_t)gridDim.x * CH) {
        uint32_t cnt = 0;
        for (int j = 0; j < HMS_RL_PPT; j++) {
            const uint64_t i = c0 + (uint64_t)j * 256 + tid;
            if (i < a.n) cnt += hms_relabel_key(a, a.keys[i]) != ~0ull;
        }
        uint32_t tot;
        uint32_t pos = hm_block_excl_scan<256>(cnt, scr, &tot);
        if (tid == 0) sbase = tot ? atomicAdd(a.cursor, (unsigned long long)tot) : 0ull;
        __syncthreads();
        const uint64_t base = sbase;
        __syncthreads();
        if (!tot) continue;
        for (int j = 0; j < HMS_RL_PPT; j++) {
            const uint64_t i = c0 + (uint64_t)j * 256 + tid;
            const uint64_t k = i < a.n ? a.keys[i] : 0ull;
            const uint64_t lk = i < a.n ? hms_relabel_key(a, k) : ~0ull;
            const bool in = lk != ~0ull;
            const uint64_t k0 = ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(lk >> 32)) << 32) |
                                __builtin_amdgcn_readfirstlane((uint32_t)lk);
            const bool same = in & (lk == k0);
            const uint64_t sm = __ballot(same);
            uint32_t b = 0;
            if (sm && hm_lane() == 0) b = hms_intern(a.buckets, k0, &bclaimed);   /* lane 0 is in the group */
            b = __shfl(b, 0, 64);
            if (in && !same) b = hms_intern(a.buckets, lk, &bclaimed);
            if (in) {
                full |= b == HMS_NO_BUCKET;   /* the caller discards the rollup */
                const uint64_t q = base + pos++;
                a.keys_out[q] = ((uint64_t)(b == HMS_NO_BUCKET ? 0u : b) << a.cb) | (k & cmask);
                a.counts_out[q] = a.counts[i];
            }
        }
    }
    uint64_t v[2] = {bclaimed, full};
    hms_block_sums(v);
    if (tid == 0) {
        if (v[0]) atomicAdd(&a.state[HMS_ST_BUCKETS], (unsigned long long)v[0]);
        if (v[1]) atomicAdd(&a.state[HMS_ST_BFULL], (unsigned long long)v[1]);
    }
}

/* merged label cells -> (hm_count key, count, group, period) */
__global__ __launch_bounds__(256) void k_stream_emit(HmsEmitArgs a)
{
    const uint64_t cmask = (1ull << a.cb) - 1ull;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < a.n; j += stride) {
        const uint64_t k = a.keys[j];
        const uint64_t bk = a.buckets.keys[k >> a.cb];
        a.keys_out[j] = hms_cell_key(k & cmask, a.zmin, a.zmax);
        a.counts_out[j] = a.counts[j];
        if (a.groups_out) a.groups_out[j] = (uint32_t)(bk >> 32);
        if (a.periods_out) a.periods_out[j] = hms_period_value((uint32_t)bk, a.base);
    }
}

static dim3 hms_grid(uint64_t n)
{
    uint64_t b = (n + 255) / 256;
    if (b > 2048) b = 2048;   /* 8 blocks per CU; one state atomic per block */
    return dim3((unsigned)(b ? b : 1));
}

/* The keys of the batch's first and last kept-looking points, interned by one
 * thread ahead of k_stream_buckets: a time-ordered batch brings a NEW hour, and
 * every wave of the main kernel would otherwise find it missing at once and
 * CAS the same key word (~5000 same-address atomics per 10M points, 55 us) */
__global__ void k_stream_prime(HmsBucketArgs a)
{
    if (threadIdx.x != 0 || !a.hour) return;
    uint32_t claimed = 0;
    for (int e = 0; e < 2; e++) {
        const uint64_t i = e ? a.n - 1 : 0;
        if (a.keep && !a.keep[i]) continue;
        const uint32_t h = a.hour[i];
        if (h < a.base || h - a.base >= HMS_MAX_HOUR_OFFSET) continue;   /* k_stream_buckets reports it */
        const uint32_t g = a.group ? a.group[i] : HMS_NOGROUP;
        hms_intern(a.buckets, ((uint64_t)g << 32) | (h - a.base), &claimed);
    }
    if (claimed) atomicAdd(&a.state[HMS_ST_BUCKETS], (unsigned long long)claimed);
}

void hm_launch_stream_buckets(hipStream_t s, const HmsBucketArgs& a)
{
    /* ~8+ steps of 256 points per wave: runs of one key stay in registers */
    uint64_t b = (a.n + 8192 - 1) / 8192;
    if (b > 2048) b = 2048;
    if (a.n && a.hour) hipLaunchKernelGGL(k_stream_prime, dim3(1), dim3(64), 0, s, a);
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
    uint64_t b = (a.n + 4095) / 4096;
    if (b > 2048) b = 2048;
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

void hm_launch_stream_rekey_dev(hipStream_t s, uint64_t* keys, const unsigned long long* m_dev, uint64_t cap,
                                const unsigned long long* state, int cb)
{
    if (cap) hipLaunchKernelGGL(k_stream_rekey_dev, dim3(1024), dim3(256), 0, s, keys, m_dev, cap, state, cb);
}

void hm_launch_stream_convert(hipStream_t s, const int64_t* rec, uint64_t m, int cb, uint64_t* keys, uint64_t* counts,
                              unsigned long long* state)
{
    if (m) hipLaunchKernelGGL(k_stream_convert, hms_grid(m), dim3(256), 0, s, rec, m, cb, keys, counts, state);
}

void hm_launch_stream_init(hipStream_t s, const HmsTable& t)
{
    hipLaunchKernelGGL(k_stream_init, hms_grid(t.mask + 1), dim3(256), 0, s, t);
}

void hm_launch_stream_fill(hipStream_t s, uint64_t* p, uint64_t n, uint64_t v)
{
    if (n) hipLaunchKernelGGL(k_stream_fill, hms_grid(n), dim3(256), 0, s, p, n, v);
}

void hm_launch_stream_relabel(hipStream_t s, const HmsRelabelArgs& a)
{
    const uint64_t chunks = (a.n + 256 * HMS_RL_PPT - 1) / (256 * HMS_RL_PPT);
    if (a.n) hipLaunchKernelGGL(k_stream_relabel, dim3((unsigned)(chunks < 1024 ? chunks : 1024)), dim3(256), 0, s, a);
}

void hm_launch_stream_emit(hipStream_t s, const HmsEmitArgs& a)
{
    if (a.n) hipLaunchKernelGGL(k_stream_emit, hms_grid(a.n), dim3(256), 0, s, a);
}
