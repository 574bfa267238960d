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
#include "../../include/heatmap_amd.h"

#define HM_PI 0x1.921fb54442d18p+1          /* math.pi */
#define HM_DEG2RAD 0x1.1df46a2529d39p-6     /* pi/180 rounded */
#define HM_INV4PI 0x1.45f306dc9c883p-4      /* 1/(4 pi) rounded */
#define HM_LN2 0x1.62e42fefa39efp-1
#define HM_SQRT2 0x1.6a09e667f3bcdp+0
#define HM_LAT_FAST 85.06
#define HM_Y_EPS 1.5e-13

HM_FN double hm_exp2i(int z)
{
    return hm_u2d((uint64_t)(1023 + z) << 52);   /* 2^z, 0 <= z <= 1023 */
}

/* Y(lat) = 0.5 - atanh(sin(lat*pi/180)) / (2 pi), |lat| <= 85.06. */
HM_FN double hm_fast_Y(double lat)
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
    /* q = (1+s)/(1-s) > 0;  ln q = e ln2 + 2 atanh(t), t = (m-1)/(m+1) */
    const double q = (1.0 + s) / (1.0 - s);
    const uint64_t qb = hm_d2u(q);
    int e = (int)((qb >> 52) & 0x7ff) - 1023;
    double m = hm_u2d((qb & 0x000fffffffffffffull) | 0x3ff0000000000000ull);
    if (m > HM_SQRT2) {
        m = m * 0.5;
        e = e + 1;
    }
    const double t = (m - 1.0) / (m + 1.0);   /* |t| <= 0.1716 */
    const double t2 = t * t;
    double a = 0x1.8618618618618p-5;          /* 1/21 */
    a = fma(a, t2, 0x1.af286bca1af28p-5);     /* 1/19 */
    a = fma(a, t2, 0x1.e1e1e1e1e1e1ep-5);     /* 1/17 */
    a = fma(a, t2, 0x1.1111111111111p-4);     /* 1/15 */
    a = fma(a, t2, 0x1.3b13b13b13b14p-4);     /* 1/13 */
    a = fma(a, t2, 0x1.745d1745d1746p-4);     /* 1/11 */
    a = fma(a, t2, 0x1.c71c71c71c71cp-4);     /* 1/9  */
    a = fma(a, t2, 0x1.2492492492492p-3);     /* 1/7  */
    a = fma(a, t2, 0x1.999999999999ap-3);     /* 1/5  */
    a = fma(a, t2, 0x1.5555555555555p-2);     /* 1/3  */
    const double lnm = 2.0 * fma(t * t2, a, t);
    const double L = fma((double)e, HM_LN2, lnm);
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
HM_FN int hm_row(double lat, int zoom, int64_t* row, int* slow)
{
    if (fabs(lat) <= HM_LAT_FAST) {
        const double scale = hm_exp2i(zoom);
        const double R = hm_fast_Y(lat) * scale;
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

HM_FN int hm_col(double lon, int zoom, int64_t* col)
{
    const double R = (lon + 180.0) / 360.0 * hm_exp2i(zoom);
    if (R != R) return HM_E_NAN;
    if (R - R != 0.0) return HM_E_INF;
    const double f = floor(R);
    if (!(f >= -9223372036854775808.0 && f < 9223372036854775808.0)) return HM_E_RANGE;
    *col = (int64_t)f;
    return HM_OK;
}

/* tile_id_from_lat_long order: row first, its error wins (tile.py:10-11). */
HM_FN int hm_project_point(double lat, double lon, int zoom, int64_t* row, int64_t* col, int* slow)
{
    int st = hm_row(lat, zoom, row, slow);
    if (st != HM_OK) return st;
    return hm_col(lon, zoom, col);
}
