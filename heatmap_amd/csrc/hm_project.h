/* Per-point Web-Mercator projection, bit-exact with reference tile.py:15-21.
 *
 * row = floor((1 - log(tan(x) + 1/cos(x)) / pi) / 2 * 2^z),  x = lat*pi/180
 * col = floor((lon + 180.0) / 360.0 * 2^z)
 *
 * Column: three IEEE operations (add, correctly rounded divide, exact power of
 * two scale) -- reproduced exactly by construction.
 *
 * Row: two paths.
 *   fast  |lat| <= HM_LAT_FAST: Y = 0.5 - ln((1+s)/(1-s)) / (4 pi), s = sin(x),
 *         with sin and ln as fixed polynomials (no table, no libm).  |Y_fast -
 *         Y_ref| is bounded by HM_Y_EPS (calibrated on the CPU against the
 *         reference arithmetic by tests/test_math_host.py with a >= 8x margin),
 *         so if Y_fast * 2^z is more than HM_Y_EPS * 2^z away from an integer
 *         the floor is the reference's floor.
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
#include "hm_logtab.h"
#include "../../include/heatmap_amd.h"

#define HM_PI 0x1.921fb54442d18p+1          /* math.pi */
#define HM_DEG2RAD 0x1.1df46a2529d39p-6     /* pi/180 rounded */
#define HM_INV4PI 0x1.45f306dc9c883p-4      /* 1/(4 pi) rounded */
#define HM_LN2 0x1.62e42fefa39efp-1
#define HM_INV360 0x1.6c16c16c16c17p-9      /* RN(1/360) */
#define HM_LAT_FAST 85.06
#define HM_Y_EPS 1.5e-13

HM_FN double hm_exp2i(int z)
{
    return hm_u2d((uint64_t)(1023 + z) << 52);   /* 2^z, 0 <= z <= 1023 */
}

/* ln(x), x positive normal: x = 2^e m, m in [1,2); interval i = top 7 mantissa
 * bits; ln m = -ln(invc_i) + log1p(m*invc_i - 1), |m*invc_i - 1| < 2^-8, log1p
 * by its Taylor series to r^8 (truncation < 2^-75).  Division-free, so the
 * host build and gfx950 produce identical bits.  tab = HM_LOGTAB_INIT. */
HM_FN double hm_fast_ln(double x, const double* tab)
{
    const uint64_t b = hm_d2u(x);
    const int e = (int)(b >> 52) - 1023;
    const uint32_t i = (uint32_t)(b >> 45) & 127u;
    const double m = hm_u2d((b & 0x000fffffffffffffull) | 0x3ff0000000000000ull);
    const double r = fma(m, tab[2 * i], -1.0);
    double q = -0x1p-3;
    q = fma(q, r, 0x1.2492492492492p-3);   /*  1/7 */
    q = fma(q, r, -0x1.5555555555555p-3);  /* -1/6 */
    q = fma(q, r, 0x1.999999999999ap-3);   /*  1/5 */
    q = fma(q, r, -0x1p-2);                /* -1/4 */
    q = fma(q, r, 0x1.5555555555555p-2);   /*  1/3 */
    q = fma(q, r, -0x1p-1);                /* -1/2 */
    const double l1p = fma(r * r, q, r);
    return fma((double)e, HM_LN2, tab[2 * i + 1] + l1p);
}

/* Y(lat) = 0.5 - (ln(1+s) - ln(1-s)) / (4 pi), s = sin(lat*pi/180), |lat| <= 85.06.
 * 1 +- s is exact where it could cancel (Sterbenz), so no division is needed. */
HM_FN double hm_fast_Y(double lat, const double* tab)
{
    const double p = lat * HM_DEG2RAD;
    const double p2 = p * p;
    /* sin p = p + p^3 * S(p^2): Taylor to p^25 (|p| <= 1.4846: truncation < 1e-20) */
    double s = 0x1.3f3ccdd165fa9p-84;        /*  1/25! */
    s = fma(s, p2, -0x1.761b41316381ap-75);  /* -1/23! */
    s = fma(s, p2, 0x1.71b8ef6dcf572p-66);   /*  1/21! */
    s = fma(s, p2, -0x1.2f49b46814157p-57);  /* -1/19! */
    s = fma(s, p2, 0x1.952c77030ad4ap-49);   /*  1/17! */
    s = fma(s, p2, -0x1.ae7f3e733b81fp-41);  /* -1/15! */
    s = fma(s, p2, 0x1.6124613a86d09p-33);   /*  1/13! */
    s = fma(s, p2, -0x1.ae64567f544e4p-26);  /* -1/11! */
    s = fma(s, p2, 0x1.71de3a556c734p-19);   /*  1/9!  */
    s = fma(s, p2, -0x1.a01a01a01a01ap-13);  /* -1/7!  */
    s = fma(s, p2, 0x1.1111111111111p-7);    /*  1/5!  */
    s = fma(s, p2, -0x1.5555555555555p-3);   /* -1/3!  */
    s = fma(p * p2, s, p);
    const double L = hm_fast_ln(1.0 + s, tab) - hm_fast_ln(1.0 - s, tab);
    return fma(-L, HM_INV4PI, 0.5);
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
        const double R = hm_fast_Y(lat, tab) * scale;
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
 * tile when both fast paths are conclusive; 0 means "resolve this point with
 * hm_project_point" (guard band, |lat| > 85.06, non-finite input, huge lon).
 * Identical results to hm_project_point whenever it returns 1. */
HM_FN int hm_project_fast(double lat, double lon, int zoom, int64_t* row, int64_t* col, const double* tab)
{
    const double scale = hm_exp2i(zoom);
    const double R = hm_fast_Y(lat, tab) * scale;
    const double f = floor(R);
    const double fr = R - f;
    const double g = HM_Y_EPS * scale;
    const double y = (lon + 180.0) * HM_INV360 * scale;
    const double ay = fabs(y);
    const double f2 = floor(y);
    const double fr2 = y - f2;
    const double g2 = ay * 0x1p-49;
    const int ok = (fabs(lat) <= HM_LAT_FAST) & (fr > g) & (fr < 1.0 - g) & (ay < 0x1p52) & (fr2 > g2) &
                   (fr2 < 1.0 - g2);
    *row = (int64_t)(ok ? f : 0.0);
    *col = (int64_t)(ok ? f2 : 0.0);
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
