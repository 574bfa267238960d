/* Open-addressing hash table of 16-B slots {u64 key, u64 count} on the
 * device: the resident streaming heatmap (hm_stream.hip) and the multi-GPU
 * cell merge (hm_merge.hip).  Linear probing; EMPTY key = all ones (never a
 * cell key: zoom field 63). */
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "hm_pipeline.h"


__device__ __forceinline__ uint64_t hms_hash(uint64_t k)
{
    /* 64-bit finaliser (MurmurHash3 fmix64) */
    k ^= k >> 33;
    k *= 0xFF51AFD7ED558CCDull;
    k ^= k >> 33;
    k *= 0xC4CEB9FE1A85EC53ull;
    k ^= k >> 33;
    return k;
}

__device__ __forceinline__ uint64_t hms_wave_sum(uint64_t v)
{
    for (int o = 32; o > 0; o >>= 1) v += (uint64_t)__shfl_xor((unsigned long long)v, o, 64);
    return v;
}

/* Sums of NV per-thread values over a 256-thread block, valid in thread 0
 * (every thread calls): the kernels' state counters then take one atomic per
 * block, not one per wave (a few thousand same-address atomics already cost
 * ~0.1 ms: one word takes ~88 per us) */
template <int NV>
__device__ __forceinline__ void hms_block_sums(uint64_t (&v)[NV])
{
    __shared__ unsigned long long s[NV][4];
#pragma unroll
    for (int q = 0; q < NV; q++) v[q] = hms_wave_sum(v[q]);
    if ((threadIdx.x & 63) == 0)
#pragma unroll
        for (int q = 0; q < NV; q++) s[q][threadIdx.x >> 6] = v[q];
    __syncthreads();
    if (threadIdx.x == 0)
#pragma unroll
        for (int q = 0; q < NV; q++) v[q] = s[q][0] + s[q][1] + s[q][2] + s[q][3];
}

/* Insert-or-add; returns 1 if this call claimed a new slot. */
__device__ __forceinline__ uint32_t hms_insert(const HmsTable& t, uint64_t k, uint64_t c, uint32_t* overflow)
{
    uint64_t h = hms_hash(k) & t.mask;
    for (uint64_t probe = 0; probe <= t.mask; probe++) {
        /* plain read: a key word changes once (EMPTY -> key); a stale EMPTY
         * only sends us to the CAS, which returns the current key */
        uint64_t cur = t.slots[2 * h];
        uint32_t claimed = 0;
        if (cur == HMS_EMPTY) {
            const unsigned long long prev =
                atomicCAS((unsigned long long*)&t.slots[2 * h], (unsigned long long)HMS_EMPTY, (unsigned long long)k);
            claimed = prev == HMS_EMPTY;
            cur = claimed ? k : prev;
        }
        if (cur == k) {
            atomicAdd((unsigned long long*)&t.slots[2 * h + 1], (unsigned long long)c);
            return claimed;
        }
        h = (h + 1) & t.mask;
    }
    *overflow = 1;
    return 0;
}


/* Insert-or-add of a key no other thread of the launch inserts (the stream's
 * batch cells are distinct keys): only the key claim needs an atomic; the
 * count is a plain store (fresh slot) or a plain read-modify-write. */
__device__ __forceinline__ uint32_t hms_insert_unique(const HmsTable& t, uint64_t k, uint64_t c, uint32_t* overflow)
{
    uint64_t h = hms_hash(k) & t.mask;
    for (uint64_t probe = 0; probe <= t.mask; probe++) {
        uint64_t cur = t.slots[2 * h];
        if (cur == HMS_EMPTY) {
            const unsigned long long prev =
                atomicCAS((unsigned long long*)&t.slots[2 * h], (unsigned long long)HMS_EMPTY, (unsigned long long)k);
            if (prev == HMS_EMPTY) {
                t.slots[2 * h + 1] = c;
                return 1;
            }
            cur = prev;
        }
        if (cur == k) {
            t.slots[2 * h + 1] += c;
            return 0;
        }
        h = (h + 1) & t.mask;
    }
    *overflow = 1;
    return 0;
}
