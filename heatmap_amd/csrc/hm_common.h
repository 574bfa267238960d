/* Shared definitions for the heatmap_amd device code.
 *
 * Every header under csrc/ that holds projection arithmetic is written so it
 * compiles two ways:
 *   - by hipcc for gfx950, where the functions are __device__ code of the
 *     product kernels;
 *   - by gcc as plain C for the CPU tests (tests/test_math_host.py), which
 *     check the exact same statements against the oracle and the live libm.
 * Floating-point contraction is forbidden in both: an a*b+c that the
 * compiler silently fused would change results in the last bit.  Every FMA in
 * these files is an explicit fma() call.
 */
#pragma once

#include <stdint.h>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define HM_EMUL_FN __device__ static inline
#define HM_EMUL_TABLE __device__ static const
#define HM_FN __device__ static inline
#define HM_SLOW_FN __device__ static __attribute__((noinline))
#define HM_UNLIKELY(x) __builtin_expect(!!(x), 0)
#else
#include <math.h>
#include <string.h>
#define HM_EMUL_FN static inline
#define HM_EMUL_TABLE static const
#define HM_FN static inline
#define HM_SLOW_FN static
#define HM_UNLIKELY(x) __builtin_expect(!!(x), 0)
#endif

#define HM_EMUL_BEGIN _Pragma("clang fp contract(off)")
#define HM_EMUL_END

#if defined(__clang__)
#pragma clang fp contract(off)
#endif

typedef union {
    double d;
    uint64_t u;
} hm_x64;

HM_FN double hm_u2d(uint64_t u)
{
    hm_x64 x;
    x.u = u;
    return x.d;
}

HM_FN uint64_t hm_d2u(double d)
{
    hm_x64 x;
    x.d = d;
    return x.u;
}
