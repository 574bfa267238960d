/* 128-bit cell keys of the general path (hm_general.hip), shared with the
 * list kernels that build them while projecting (hm_kernels.hip):
 *     sr + 16 (5) | sc + 2^47 (48) | group (32) | morton(ro, co) (2Z)
 * sr = row >> Z, sc = col >> Z (arithmetic) name the zoom-0 "super tile";
 * ro, co are the tile's offsets inside it.  The group sits right above the
 * Morton bits so that a few thousand groups and a single super tile vary in
 * one contiguous low range of the key (fewest radix digits).  The zoom-(Z-k)
 * cell of a key is the key with its low 2k bits cleared. */
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef unsigned __int128 hm_u128;

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

/* the key of zoom-Z tile (r, c) of group g; *ok = false when the super tile
 * is beyond the key's fields (the key is then 0) */
__device__ __forceinline__ hm_u128 hm_gen_key(int64_t r, int64_t c, uint32_t g, int Z, bool* ok)
{
    const int64_t sr = r >> Z, sc = c >> Z;
    const uint64_t m = (hm_spread21((uint64_t)r & ((1ull << Z) - 1)) << 1) | hm_spread21((uint64_t)c & ((1ull << Z) - 1));
    *ok = sr >= -HM_GEN_SR_BIAS && sr < HM_GEN_SR_BIAS && sc >= -HM_GEN_SC_BIAS && sc < HM_GEN_SC_BIAS;
    if (!*ok) return 0;
    const hm_u128 root = ((hm_u128)(uint64_t)(sr + HM_GEN_SR_BIAS) << 80) |
                         ((hm_u128)(uint64_t)(sc + HM_GEN_SC_BIAS) << 32) | (hm_u128)g;
    return (root << (2 * Z)) | (hm_u128)m;
}

/* decode of a zoom-z cell key (low 2(Z-z) bits clear) */
__device__ __forceinline__ void hm_gen_decode(hm_u128 k, int Z, int z, uint32_t* g, int64_t* row, int64_t* col)
{
    const hm_u128 root = k >> (2 * Z);
    const uint64_t m = (uint64_t)(k >> (2 * (Z - z))) & ((1ull << (2 * z)) - 1);
    const int64_t sr = (int64_t)(uint64_t)((root >> 80) & 31) - HM_GEN_SR_BIAS;
    const int64_t sc = (int64_t)((uint64_t)(root >> 32) & ((1ull << HM_GEN_SC_BITS) - 1)) - HM_GEN_SC_BIAS;
    *g = (uint32_t)root;
    /* sr * 2^z, sc * 2^z as unsigned shifts (two's complement) */
    *row = (int64_t)(((uint64_t)sr << z) + hm_compact21(m >> 1));
    *col = (int64_t)(((uint64_t)sc << z) + hm_compact21(m));
}
