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
