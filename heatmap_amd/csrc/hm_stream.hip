/* Resident multi-zoom heatmap for streaming micro-batches (BASELINE config 5,
 * SURVEY.md 8f item 2).
 *
 * The reference recomputes its whole pyramid per Spark job (heatmap.py:152-158);
 * a streaming caller instead folds each micro-batch's hm_count cells into a
 * heatmap that stays in HBM.  The resident heatmap is an open-addressing hash
 * table of 16-B slots (u64 key, u64 count in one slot, so a probe hit and its
 * count add touch one cache line; linear probing, EMPTY key = all ones):
 *   - merge cost is O(cells of the batch), independent of the resident size
 *     (a sorted resident set would re-stream every resident cell per batch);
 *   - a batch cell is one probe sequence + one 64-bit atomic add, so the
 *     kernel is bound by random 64-B HBM transactions, not by arithmetic.
 * Table key = hour bucket (17 bits) | zoom (5) | row (21) | col (21); the hour
 * bucket HM_STREAM_ALLTIME_TAG holds the alltime heatmap, every other value
 * an epoch hour relative to the stream's base hour.
 */
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "hm_pipeline.h"
#include "hm_table.h"

/* hm_count key (zoom<<58 | row<<29 | col) -> 42-bit cell field of a table key */
__device__ __forceinline__ uint64_t hms_pack(uint64_t k)
{
    const uint64_t z = k >> 58, r = (k >> 29) & 0x1FFFFFFFull, c = k & 0x1FFFFFFFull;
    return (z << 42) | (r << 21) | c;
}

__device__ __forceinline__ uint64_t hms_unpack(uint64_t p)
{
    const uint64_t z = (p >> 42) & 31ull, r = (p >> 21) & 0x1FFFFFull, c = p & 0x1FFFFFull;
    return (z << 58) | (r << 29) | c;
}

/* Fold n cells (hm_count layout) into the table under tag_a and, if
 * tag_b != 0, again under tag_b (the alltime bucket). */
__global__ __launch_bounds__(256) void k_stream_insert(const uint64_t* __restrict__ keys,
                                                       const uint64_t* __restrict__ counts, uint64_t n,
                                                       uint64_t tag_a, uint64_t tag_b, HmsTable t)
{
    uint64_t claimed = 0;
    uint32_t overflow = 0;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const uint64_t p = hms_pack(keys[i]);
        const uint64_t c = counts[i];
        claimed += hms_insert(t, tag_a | p, c, &overflow);
        if (tag_b) claimed += hms_insert(t, tag_b | p, c, &overflow);
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

/* Min / max epoch hour over the kept points of a batch. */
__global__ __launch_bounds__(256) void k_stream_hour_range(const uint32_t* __restrict__ hour,
                                                           const uint8_t* __restrict__ keep, uint64_t n,
                                                           unsigned int* mm)
{
    uint32_t lo = 0xFFFFFFFFu, hi = 0;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        if (keep && !keep[i]) continue;
        const uint32_t h = hour[i];
        lo = h < lo ? h : lo;
        hi = h > hi ? h : hi;
    }
    for (int o = 32; o > 0; o >>= 1) {
        const uint32_t a = __shfl_xor(lo, o, 64), b = __shfl_xor(hi, o, 64);
        lo = a < lo ? a : lo;
        hi = b > hi ? b : hi;
    }
    __shared__ uint32_t wlo[4], whi[4];
    if ((threadIdx.x & 63) == 0) {
        wlo[threadIdx.x >> 6] = lo;
        whi[threadIdx.x >> 6] = hi;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int w = 1; w < 4; w++) {
            lo = wlo[w] < lo ? wlo[w] : lo;
            hi = whi[w] > hi ? whi[w] : hi;
        }
        if (lo <= hi) { /* one pair of atomics per block */
            atomicMin(&mm[0], lo);
            atomicMax(&mm[1], hi);
        }
    }
}

/* present[h - lo] = 1 for every hour of a kept point (benign same-value races). */
__global__ __launch_bounds__(256) void k_stream_hour_presence(const uint32_t* __restrict__ hour,
                                                              const uint8_t* __restrict__ keep, uint64_t n,
                                                              uint32_t lo, uint8_t* present)
{
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        if (keep && !keep[i]) continue;
        present[hour[i] - lo] = 1;
    }
}

/* mask[i] = keep[i] && hour[i] == h */
__global__ __launch_bounds__(256) void k_stream_hour_mask(const uint32_t* __restrict__ hour,
                                                          const uint8_t* __restrict__ keep, uint64_t n, uint32_t h,
                                                          uint8_t* __restrict__ mask)
{
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
        mask[i] = (uint8_t)((!keep || keep[i]) && hour[i] == h);
}

/* Dump the slots whose hour bucket matches `sel` (sel == HMS_SEL_EVERY_HOUR:
 * every bucket but alltime) as hm_count keys + counts (+ absolute epoch hour).
 * Each wave owns chunks of HMS_XCHUNK slots: it counts its matches (ballots),
 * reserves output with ONE atomic per chunk, then re-reads the (cache-hot)
 * chunk and writes in slot order.  Matches past `cap` are counted, not written. */
#define HMS_XCHUNK (64 * 64)
__device__ __forceinline__ bool hms_sel(uint64_t k, uint64_t sel)
{
    const uint64_t tag = k >> HMS_TAG_SHIFT;
    return k != HMS_EMPTY && (sel == HMS_SEL_EVERY_HOUR ? tag != HM_STREAM_ALLTIME_TAG : tag == sel);
}

__global__ __launch_bounds__(256) void k_stream_extract(HmsTable t, uint64_t sel, uint64_t* __restrict__ keys_out,
                                                        uint64_t* __restrict__ counts_out,
                                                        uint32_t* __restrict__ hours_out, uint32_t base_hour,
                                                        uint64_t cap, unsigned long long* cursor)
{
    const uint64_t n = t.mask + 1; /* power of two >= 1024 */
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t wave = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const uint64_t waves = ((uint64_t)gridDim.x * blockDim.x) >> 6;
    const ulonglong2* slots = (const ulonglong2*)t.slots;
    for (uint64_t c0 = wave * HMS_XCHUNK; c0 < n; c0 += waves * HMS_XCHUNK) {
        const uint64_t c1 = c0 + HMS_XCHUNK < n ? c0 + HMS_XCHUNK : n;
        uint64_t cnt = 0;
        for (uint64_t i = c0 + lane; i < c1; i += 64) cnt += hms_sel(slots[i].x, sel);
        cnt = hms_wave_sum(cnt);
        if (!cnt) continue;
        unsigned long long first = 0;
        if (lane == 0) first = atomicAdd(cursor, (unsigned long long)cnt);
        first = __shfl(first, 0, 64);
        for (uint64_t j0 = c0; j0 < c1; j0 += 64) {
            const uint64_t i = j0 + lane;
            ulonglong2 sl = make_ulonglong2(HMS_EMPTY, 0ull);
            if (i < c1) sl = slots[i];
            const bool m = hms_sel(sl.x, sel);
            const uint64_t bal = __ballot(m);
            if (m) {
                const uint64_t pos = first + __popcll(bal & ((1ull << lane) - 1));
                if (pos < cap) {
                    keys_out[pos] = hms_unpack(sl.x);
                    counts_out[pos] = sl.y;
                    if (hours_out) hours_out[pos] = base_hour + (uint32_t)(sl.x >> HMS_TAG_SHIFT);
                }
            }
            first += __popcll(bal);
        }
    }
}

static dim3 hms_grid(uint64_t n)
{
    uint64_t b = (n + 255) / 256;
    if (b > 8192) b = 8192;
    return dim3((unsigned)(b ? b : 1));
}

void hm_launch_stream_insert(hipStream_t s, const uint64_t* keys, const uint64_t* counts, uint64_t n, uint64_t tag_a,
                             uint64_t tag_b, const HmsTable& t)
{
    if (n) hipLaunchKernelGGL(k_stream_insert, hms_grid(n), dim3(256), 0, s, keys, counts, n, tag_a, tag_b, t);
}

void hm_launch_stream_init(hipStream_t s, const HmsTable& t)
{
    hipLaunchKernelGGL(k_stream_init, hms_grid(t.mask + 1), dim3(256), 0, s, t);
}

void hm_launch_stream_rehash(hipStream_t s, const HmsTable& from, const HmsTable& to)
{
    hipLaunchKernelGGL(k_stream_rehash, hms_grid(from.mask + 1), dim3(256), 0, s, from, to);
}

void hm_launch_stream_hour_range(hipStream_t s, const uint32_t* hour, const uint8_t* keep, uint64_t n,
                                 unsigned int* mm)
{
    const uint64_t b = (n + 255) / 256;
    if (n) hipLaunchKernelGGL(k_stream_hour_range, dim3((unsigned)(b < 1024 ? b : 1024)), dim3(256), 0, s, hour, keep, n, mm);
}

void hm_launch_stream_hour_presence(hipStream_t s, const uint32_t* hour, const uint8_t* keep, uint64_t n,
                                    uint32_t lo, uint8_t* present)
{
    if (n) hipLaunchKernelGGL(k_stream_hour_presence, hms_grid(n), dim3(256), 0, s, hour, keep, n, lo, present);
}

void hm_launch_stream_hour_mask(hipStream_t s, const uint32_t* hour, const uint8_t* keep, uint64_t n, uint32_t h,
                                uint8_t* mask)
{
    if (n) hipLaunchKernelGGL(k_stream_hour_mask, hms_grid(n), dim3(256), 0, s, hour, keep, n, h, mask);
}

void hm_launch_stream_extract(hipStream_t s, const HmsTable& t, uint64_t sel, uint64_t* keys_out,
                              uint64_t* counts_out, uint32_t* hours_out, uint32_t base, uint64_t cap,
                              unsigned long long* cursor)
{
    const uint64_t chunks = (t.mask + HMS_XCHUNK) / HMS_XCHUNK, blocks = (chunks + 3) / 4;
    hipLaunchKernelGGL(k_stream_extract, dim3((unsigned)(blocks < 4096 ? blocks : 4096)), dim3(256), 0, s, t, sel, keys_out, counts_out,
                       hours_out, base, cap, cursor);
}
