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
        uint64_t cur = __atomic_load_n(&b.keys[h], __ATOMIC_RELAXED);
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

/* Bucket of every kept point: (group or HMS_NOGROUP, hour - base or
 * HMS_UNDATED).  A wave whose kept points share one key interns it once.
 * Hours outside [base, base + 2^28) are input errors (first index wins). */
__global__ __launch_bounds__(256) void k_stream_buckets(HmsBucketArgs a)
{
    const uint32_t lane = threadIdx.x & 63;
    uint32_t lo = 0xFFFFFFFFu, hi = 0, claimed = 0, full = 0;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    const uint64_t n_up = (a.n + 63) & ~63ull;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n_up; i += stride) {
        bool kept = i < a.n && (!a.keep || a.keep[i]);
        uint64_t key = 0;
        if (kept) {
            uint32_t pw = HMS_UNDATED;
            if (a.hour) {
                const uint32_t h = a.hour[i];
                if (h < a.base || h - a.base >= HMS_MAX_HOUR_OFFSET) {
                    atomicMin(a.err_word, ((unsigned long long)i << 8) | (unsigned long long)HM_E_RANGE);
                    kept = false;
                }
                pw = h - a.base;
            }
            key = ((uint64_t)(a.group ? a.group[i] : HMS_NOGROUP) << 32) | pw;
        }
        const uint64_t km = __ballot(kept);
        if (!km) continue;
        const int leader = __ffsll((unsigned long long)km) - 1;
        const uint64_t k0 = __shfl((unsigned long long)key, leader, 64);
        uint32_t b = 0;
        if (__ballot(kept && key != k0) == 0) {
            if ((int)lane == leader) b = hms_intern(a.buckets, k0, &claimed);
            b = __shfl(b, leader, 64);
        } else if (kept) {
            b = hms_intern(a.buckets, key, &claimed);
        }
        if (kept) {
            full |= b == HMS_NO_BUCKET;
            lo = b < lo ? b : lo;
            hi = b > hi ? b : hi;
            a.out[i] = b;
        }
    }
    for (int o = 32; o > 0; o >>= 1) {
        const uint32_t x = __shfl_xor(lo, o, 64), y = __shfl_xor(hi, o, 64);
        lo = x < lo ? x : lo;
        hi = y > hi ? y : hi;
    }
    const uint64_t cl = hms_wave_sum(claimed);
    const uint64_t fl = hms_wave_sum(full);
    if (lane == 0) {
        unsigned int* mm = (unsigned int*)(a.state + HMS_ST_BMM);
        if (lo <= hi) {
            atomicMin(&mm[0], lo);
            atomicMax(&mm[1], hi);
        }
        if (cl) atomicAdd(&a.state[HMS_ST_BUCKETS], (unsigned long long)cl);
        if (fl) atomicAdd(&a.state[HMS_ST_BFULL], (unsigned long long)fl);
    }
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
    const uint64_t b = hms_wave_sum(bad);
    if ((threadIdx.x & 63) == 0 && b) atomicAdd(&state[HMS_ST_EXOTIC], (unsigned long long)b);
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
        claimed += hms_insert(t, k, counts[i], &overflow);
    }
    claimed = hms_wave_sum(claimed);
    const uint64_t of = hms_wave_sum(overflow);
    if ((threadIdx.x & 63) == 0) {
        if (claimed) atomicAdd(&t.state[HMS_ST_OCCUPIED], (unsigned long long)claimed);
        if (of) atomicAdd(&t.state[HMS_ST_OVERFLOW], (unsigned long long)of);
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
        if (sl.x != HMS_EMPTY) claimed += hms_insert(to, sl.x, sl.y, &overflow);
    }
    claimed = hms_wave_sum(claimed);
    const uint64_t of = hms_wave_sum(overflow);
    if ((threadIdx.x & 63) == 0) {
        if (claimed) atomicAdd(&to.state[HMS_ST_OCCUPIED], (unsigned long long)claimed);
        if (of) atomicAdd(&to.state[HMS_ST_OVERFLOW], (unsigned long long)of);
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
        const uint32_t b = hms_intern(a.buckets, ((uint64_t)g << 32) | lp, &bclaimed);
        if (b == HMS_NO_BUCKET) {
            full = 1;
            continue;
        }
        claimed += hms_insert(a.to, ((uint64_t)b << a.cb) | (sl.x & cmask), sl.y, &overflow);
    }
    claimed = hms_wave_sum(claimed);
    const uint64_t of = hms_wave_sum(overflow);
    const uint64_t bc = hms_wave_sum(bclaimed);
    const uint64_t fl = hms_wave_sum(full);
    if ((threadIdx.x & 63) == 0) {
        if (claimed) atomicAdd(&a.to.state[HMS_ST_OCCUPIED], (unsigned long long)claimed);
        if (of) atomicAdd(&a.to.state[HMS_ST_OVERFLOW], (unsigned long long)of);
        if (bc) atomicAdd(&a.state[HMS_ST_BUCKETS], (unsigned long long)bc);
        if (fl) atomicAdd(&a.state[HMS_ST_BFULL], (unsigned long long)fl);
    }
}

/* occupied slots of a rollup table -> (group, period, hm_count key, count);
 * one output reservation per wave and 64 slots; past `cap`: counted only */
__global__ __launch_bounds__(256) void k_stream_emit(HmsEmitArgs a)
{
    const uint64_t n = a.t.mask + 1;
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t cmask = (1ull << a.cb) - 1ull;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    const ulonglong2* slots = (const ulonglong2*)a.t.slots;
    for (uint64_t i0 = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) & ~63ull; i0 < n; i0 += stride) {
        const uint64_t i = i0 + lane;
        const ulonglong2 sl = i < n ? slots[i] : make_ulonglong2(HMS_EMPTY, 0ull);
        const bool m = sl.x != HMS_EMPTY;
        const uint64_t bal = __ballot(m);
        if (!bal) continue;
        unsigned long long first = 0;
        if (lane == 0) first = atomicAdd(a.cursor, (unsigned long long)__popcll(bal));
        first = __shfl(first, 0, 64);
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
    }
}

static dim3 hms_grid(uint64_t n)
{
    uint64_t b = (n + 255) / 256;
    if (b > 8192) b = 8192;
    return dim3((unsigned)(b ? b : 1));
}

void hm_launch_stream_buckets(hipStream_t s, const HmsBucketArgs& a)
{
    if (a.n) hipLaunchKernelGGL(k_stream_buckets, hms_grid(a.n), dim3(256), 0, s, a);
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
    hipLaunchKernelGGL(k_stream_emit, hms_grid(a.t.mask + 1), dim3(256), 0, s, a);
}
