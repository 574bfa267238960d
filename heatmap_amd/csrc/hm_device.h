/* Device-side helpers for gfx950 (wave64): Morton codes, wave aggregation,
 * block scans.  Wave width is hard-coded to 64 (CDNA). */
#pragma once
#include "hm_common.h"

#define HM_WAVE 64

/* ---- Morton (row bit above col bit) ---- */
__device__ __forceinline__ uint64_t hm_spread32(uint64_t v)
{
    v &= 0xFFFFFFFFull;
    v = (v | (v << 16)) & 0x0000FFFF0000FFFFull;
    v = (v | (v << 8)) & 0x00FF00FF00FF00FFull;
    v = (v | (v << 4)) & 0x0F0F0F0F0F0F0F0Full;
    v = (v | (v << 2)) & 0x3333333333333333ull;
    v = (v | (v << 1)) & 0x5555555555555555ull;
    return v;
}

__device__ __forceinline__ uint32_t hm_compact64(uint64_t v)
{
    v &= 0x5555555555555555ull;
    v = (v | (v >> 1)) & 0x3333333333333333ull;
    v = (v | (v >> 2)) & 0x0F0F0F0F0F0F0F0Full;
    v = (v | (v >> 4)) & 0x00FF00FF00FF00FFull;
    v = (v | (v >> 8)) & 0x0000FFFF0000FFFFull;
    v = (v | (v >> 16)) & 0x00000000FFFFFFFFull;
    return (uint32_t)v;
}

/* 16-bit -> even bits of 32 */
__device__ __forceinline__ uint32_t hm_spread16(uint32_t v)
{
    v &= 0xFFFFu;
    v = (v | (v << 8)) & 0x00FF00FFu;
    v = (v | (v << 4)) & 0x0F0F0F0Fu;
    v = (v | (v << 2)) & 0x33333333u;
    v = (v | (v << 1)) & 0x55555555u;
    return v;
}

/* Morton of two values < 2^16 (row bit above col bit) */
__device__ __forceinline__ uint32_t hm_morton16(uint32_t row, uint32_t col)
{
    return (hm_spread16(row) << 1) | hm_spread16(col);
}

__device__ __forceinline__ uint64_t hm_morton(uint32_t row, uint32_t col)
{
    return (hm_spread32(row) << 1) | hm_spread32(col);
}

/* output key of cell `m` (Morton index at zoom z) */
__device__ __forceinline__ uint64_t hm_out_key(int z, uint64_t m)
{
    return ((uint64_t)z << 58) | ((uint64_t)hm_compact64(m >> 1) << 29) | (uint64_t)hm_compact64(m);
}

/* ---- wave helpers ---- */
__device__ __forceinline__ int hm_lane() { return (int)__lane_id(); }

__device__ __forceinline__ uint32_t hm_mbcnt(uint64_t mask)
{
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0u));
}

/* inclusive wave prefix sum */
__device__ __forceinline__ uint32_t hm_wave_incl_scan(uint32_t v)
{
    const int lane = hm_lane();
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        uint32_t t = __shfl_up(v, o, 64);
        if (lane >= o) v += t;
    }
    return v;
}

__device__ __forceinline__ uint64_t hm_wave_incl_scan64(uint64_t v)
{
    const int lane = hm_lane();
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        uint64_t t = __shfl_up(v, o, 64);
        if (lane >= o) v += t;
    }
    return v;
}

__device__ __forceinline__ uint32_t hm_wave_sum(uint32_t v)
{
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

/* Block-wide exclusive scan of one value per thread; returns the block total
 * in *total.  `scratch` needs (blockDim/64 + 1) u32 of LDS. */
template <int THREADS>
__device__ __forceinline__ uint32_t hm_block_excl_scan(uint32_t v, uint32_t* scratch, uint32_t* total)
{
    constexpr int NW = THREADS / 64;
    const int lane = hm_lane();
    const int w = threadIdx.x >> 6;
    uint32_t inc = hm_wave_incl_scan(v);
    if (lane == 63) scratch[w] = inc;
    __syncthreads();
    if (w == 0) {
        uint32_t s = lane < NW ? scratch[lane] : 0u;
        uint32_t si = hm_wave_incl_scan(s);
        if (lane < NW) scratch[lane] = si - s;
        if (lane == NW - 1) scratch[NW] = si;
    }
    __syncthreads();
    uint32_t r = scratch[w] + inc - v;
    *total = scratch[NW];
    __syncthreads();
    return r;
}

/* LDS histogram increment.  Duplicate addresses within one ds_add are
 * serialised by the LDS unit, which is cheaper than software aggregation for
 * the usual mix; only a wave whose valid lanes ALL share one key (the skew
 * case, SURVEY.md section 7 hard part 3) is collapsed into a single add.
 * (Measured: 4 rounds of leader aggregation made k_project_partition
 * SALU-bound.) */
__device__ __forceinline__ void hm_lds_count(uint32_t* hist, uint32_t key, bool valid)
{
    const uint64_t vm = __ballot(valid);
    if (vm == 0) return;
    const int leader = __ffsll((unsigned long long)vm) - 1;
    const uint32_t kl = __builtin_amdgcn_readlane(key, leader);
    if (__ballot(valid && key == kl) == vm) {
        if (hm_lane() == leader) atomicAdd(&hist[kl], (uint32_t)__popcll(vm));
    } else if (valid) {
        atomicAdd(&hist[key], 1u);
    }
}

/* Slot reservation in bucket `key` (cursor array `cur`), same policy. */
__device__ __forceinline__ uint32_t hm_lds_claim(uint32_t* cur, uint32_t key, bool valid)
{
    const uint64_t vm = __ballot(valid);
    if (vm == 0) return 0;
    const int leader = __ffsll((unsigned long long)vm) - 1;
    const uint32_t kl = __builtin_amdgcn_readlane(key, leader);
    uint32_t pos = 0;
    if (__ballot(valid && key == kl) == vm) {
        uint32_t base = 0;
        if (hm_lane() == leader) base = atomicAdd(&cur[kl], (uint32_t)__popcll(vm));
        pos = __builtin_amdgcn_readlane(base, leader) + hm_mbcnt(vm);
    } else if (valid) {
        pos = atomicAdd(&cur[key], 1u);
    }
    return pos;
}
