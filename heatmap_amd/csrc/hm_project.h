/* Per-point Web-Mercator projection, bit-exact with reference tile.py:15-21.
 *
 * row = floor((1 - log(tan(x) + 1/cos(x)) / pi) / 2 * 2^z),  x = lat*pi/180
 * col = floor((lon + 180.0) / 360.0 * 2^z)
 *
 * Column: three IEEE operations (add, correctly rounded divide, exact power of
 * two scale) -- reproduced exactly by construction.
 *
 * Row: two paths.
 *   fast  |lat| <= HM_LAT_FAST: Y = 0.5 - sign(lat) g(90 - |lat|), g a
 *         piecewise degree-5 polynomial on log-spaced intervals of the polar
 *         distance (hm_ytab.h, tools/gen_ytab.py): ~20 VALU per point, no
 *         transcendental.  |Y_fast - Y_ref| is bounded by HM_Y_EPS
 *         (calibrated on the CPU against the reference arithmetic by
 *         tests/test_math_host.py with a >= 8x margin), so if Y_fast * 2^z is
 *         more than HM_Y_EPS * 2^z away from an integer the floor is the
 *         reference's floor.
 *   exact everything else (guard band, |lat| > 85.06, non-finite input):
 *         the reference's literal evaluation chain, with tan/cos/log replaced
 *         by hm_glibc_{tan,cos,log}, a restatement of glibc 2.35's own
 *         arithmetic (hm_glibc_emul.h).  Bit-exact with CPython on glibc, the
 *         reference's runtime.  Guard-band traffic is ~2 * HM_Y_EPS * 2^z of
 *         the points (1e-8 at z18): a few lanes per million waves.
 *
 * Error kinds follow CPython (math_1, m_log, math.floor): see heatmap_amd.h.
 */
#pragma once
#include "hm_common.h"
#include "hm_glibc_emul.h"
#include "hm_ytab.h"
#include "../../include/heatmap_amd.h"

#define HM_PI 0x1.921fb54442d18p+1          /* math.pi */
#define HM_INV360 0x1.6c16c16c16c17p-9      /* RN(1/360) */
#define HM_LAT_FAST 85.06
#define HM_Y_EPS 1.5e-13

HM_FN double hm_exp2i(int z)
{
    return hm_u2d((uint64_t)(1023 + z) << 52);   /* 2^z, 0 <= z <= 1023 */
}

/* g(90 - |lat|) = ln(tan(x) + sec(x)) / (2 pi) for |lat| <= HM_LAT_FAST
 * (tab = HM_YTAB_INIT).  Interval = exponent and top HM_YTAB_K mantissa bits
 * of d = 90 - |lat|; t = d - d_lo is exact.  The index is clamped, so any
 * input (NaN, |lat| > 90) reads inside the table; callers reject those. */
HM_FN double hm_fast_g(double lat, const double* tab)
{
    const double d = 90.0 - fabs(lat);
    const uint32_t hi = (uint32_t)(hm_d2u(d) >> 32);
    uint32_t idx = (hi >> (20 - HM_YTAB_K)) - ((1023u + HM_YTAB_E0) << HM_YTAB_K);
    idx = idx < (uint32_t)HM_YTAB_ROWS ? idx : (uint32_t)HM_YTAB_ROWS - 1u;
    const double dlo = hm_u2d((uint64_t)(hi & ~((1u << (20 - HM_YTAB_K)) - 1u)) << 32);
    const double t = d - dlo;
    const double* c = tab + idx * HM_YTAB_STRIDE;
    double p = c[5];
    p = fma(p, t, c[4]);
    p = fma(p, t, c[3]);
    p = fma(p, t, c[2]);
    p = fma(p, t, c[1]);
    return fma(p, t, c[0]);
}

/* Y(lat) of the fast path (for the CPU error-bound test). */
HM_FN double hm_fast_Y(double lat, const double* tab)
{
    return 0.5 - copysign(hm_fast_g(lat, tab), lat);
}

/* R = Y * 2^z, rounded once */
HM_FN double hm_fast_R(double lat, double scale, const double* tab)
{
    return fma(-copysign(hm_fast_g(lat, tab), lat), scale, 0.5 * scale);
}

/* Reference chain, literally: tile.py:17 with CPython error semantics. */
HM_SLOW_FN int hm_row_exact(double lat, int zoom, int64_t* row)
{
    const double x = lat * HM_PI / 180.0;
    if (x != x) return HM_E_NAN;                  /* NaN flows to floor() */
    if (x - x != 0.0) return HM_E_DOMAIN;         /* tan(+-inf): math domain error */
    int un = 0;
    const double t = hm_glibc_tan(x, &un);
    if (un) return HM_E_RANGE;
    const double c = hm_glibc_cos(x, &un);
    if (un) return HM_E_RANGE;
    const double u = t + 1.0 / c;
    if (!(u > 0.0)) return HM_E_DOMAIN;           /* log(0), log(<0) */
    const double L = hm_glibc_log(u, &un);
    if (un) return HM_E_DOMAIN;
    const double R = (1.0 - L / HM_PI) / 2.0 * hm_exp2i(zoom);
    if (R != R) return HM_E_NAN;
    if (R - R != 0.0) return HM_E_INF;
    *row = (int64_t)floor(R);
    return HM_OK;
}

/* Returns status; *slow = 1 when the exact chain was used. */
HM_FN int hm_row(double lat, int zoom, int64_t* row, int* slow, const double* tab)
{
    if (fabs(lat) <= HM_LAT_FAST) {
        const double scale = hm_exp2i(zoom);
        const double R = hm_fast_R(lat, scale, tab);
        const double f = floor(R);
        const double fr = R - f;
        const double g = HM_Y_EPS * scale;
        if (fr > g && fr < 1.0 - g) {
            *row = (int64_t)f;
            *slow = 0;
            return HM_OK;
        }
    }
    *slow = 1;
    return hm_row_exact(lat, zoom, row);
}

/* Column: the reference's (lon + 180.0) / 360.0 * 2^z (tile.py:21).  Fast path
 * multiplies by RN(1/360) instead of dividing: |y_fast - y_ref| < |y| 2^-51,
 * so a fraction farther than |y| 2^-49 from an integer floors identically;
 * anything else (and NaN/inf) takes the literal division. */
HM_SLOW_FN int hm_col_exact(double lon, int zoom, int64_t* col)
{
    const double R = (lon + 180.0) / 360.0 * hm_exp2i(zoom);
    if (R != R) return HM_E_NAN;
    if (R - R != 0.0) return HM_E_INF;
    const double f = floor(R);
    if (!(f >= -9223372036854775808.0 && f < 9223372036854775808.0)) return HM_E_RANGE;
    *col = (int64_t)f;
    return HM_OK;
}

HM_FN int hm_col(double lon, int zoom, int64_t* col)
{
    const double y = (lon + 180.0) * HM_INV360 * hm_exp2i(zoom);
    const double ay = fabs(y);
    if (ay < 0x1p52) {
        const double f = floor(y);
        const double fr = y - f;
        const double g = ay * 0x1p-49;
        if (fr > g && fr < 1.0 - g) {
            *col = (int64_t)f;
            return HM_OK;
        }
    }
    return hm_col_exact(lon, zoom, col);
}

/* Branch-free fast projection for the streaming kernels: returns 1 and the
 * tile (int32) when both fast paths are conclusive and the tile lies inside
 * [0, 2^z)^2; 0 means "resolve this point with the exact chain" (guard band,
 * |lat| > HM_LAT_SQ, non-finite input, a column outside [0, 2^z)).
 * Identical results to hm_project_point whenever it returns 1 (then 0 <=
 * row, col < 2^z: |lat| <= 85.05 < 85.0511 keeps Y inside (0, 1), so callers
 * need no range test).  Per-launch constants: scale = 2^z, kz = RN(1/360) 2^z
 * (exact). */
#define HM_LAT_SQ 85.05
HM_FN int hm_project_fast(double lat, double lon, double scale, double kz, int32_t* row, int32_t* col,
                          const double* tab)
{
    const double R = hm_fast_R(lat, scale, tab);
    const double f = floor(R);
    const double g = HM_Y_EPS * scale;
    const double y = (lon + 180.0) * kz;
    const double f2 = floor(y);
    const double g2 = scale * 0x1p-49;   /* >= |y| 2^-49 on the accepted range 0 <= y < 2^z */
    const int ok = (int)(fabs(lat) <= HM_LAT_SQ) & (int)(fabs((R - f) - 0.5) < 0.5 - g) & (int)(y >= 0.0) &
                   (int)(y < scale) & (int)(fabs((y - f2) - 0.5) < 0.5 - g2);   /* branch-free */
    *row = (int32_t)(ok ? f : 0.0);
    *col = (int32_t)(ok ? f2 : 0.0);
    return ok;
}

/* tile_id_from_lat_long order: row first, its error wins (tile.py:10-11). */
HM_FN int hm_project_point(double lat, double lon, int zoom, int64_t* row, int64_t* col, int* slow,
                           const double* tab)
{
    int st = hm_row(lat, zoom, row, slow, tab);
    if (st != HM_OK) return st;
    return hm_col(lon, zoom, col);
}
