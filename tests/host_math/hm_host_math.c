/* Test-only host build of the product's projection arithmetic.
 *
 * Compiles heatmap_amd/csrc/hm_project.h -- the exact statements the gfx950
 * kernels execute -- with gcc so the CPU test suite can (a) check the
 * glibc-restating slow path against the live libm, (b) calibrate and verify
 * the fast path's error bound HM_Y_EPS, and (c) compare full projections with
 * the oracle on millions of points, without a GPU.  Built by
 * tests/conftest.py into tests/host_math/_build/ (never shipped).
 */
#include <math.h>
#include "hm_project.h"

static const double TAB[HM_YTAB_ROWS * HM_YTAB_STRIDE] = HM_YTAB_INIT;

int hmh_project(const double* lat, const double* lon, int64_t n, int zoom, int64_t* row,
                int64_t* col, uint8_t* st, uint8_t* slow)
{
    int64_t nslow = 0;
    for (int64_t i = 0; i < n; i++) {
        int64_t r = 0, c = 0;
        int s = 0;
        int k = hm_project_point(lat[i], lon[i], zoom, &r, &c, &s, TAB);
        row[i] = k == HM_OK ? r : 0;
        col[i] = k == HM_OK ? c : 0;
        st[i] = (uint8_t)k;
        slow[i] = (uint8_t)s;
        nslow += s;
    }
    return (int)(nslow > 2147483647 ? 2147483647 : nslow);
}

/* max |Y_fast - Y_ref| over the inputs, Y_ref by the literal chain on libm */
double hmh_fast_Y_maxerr(const double* lat, int64_t n, double* worst_lat)
{
    double m = 0.0;
    for (int64_t i = 0; i < n; i++) {
        double x = lat[i] * M_PI / 180;
        double yr = (1 - log(tan(x) + 1 / cos(x)) / M_PI) / 2;
        double e = fabs(hm_fast_Y(lat[i], TAB) - yr);
        if (e > m) {
            m = e;
            *worst_lat = lat[i];
        }
    }
    return m;
}

double hmh_glibc(int fn, double x, int* unsupported)
{
    if (fn == 0) return hm_glibc_tan(x, unsupported);
    if (fn == 1) return hm_glibc_cos(x, unsupported);
    return hm_glibc_log(x, unsupported);
}

/* counts of mismatches of hm_glibc_* vs libm over n inputs */
int64_t hmh_glibc_check(int fn, const double* x, int64_t n, int64_t* unsupported_count)
{
    int64_t bad = 0, un = 0;
    for (int64_t i = 0; i < n; i++) {
        int u = 0;
        double a = hmh_glibc(fn, x[i], &u);
        if (u) {
            un++;
            continue;
        }
        double b = fn == 0 ? tan(x[i]) : fn == 1 ? cos(x[i]) : log(x[i]);
        if (hm_d2u(a) != hm_d2u(b)) bad++;
    }
    *unsupported_count = un;
    return bad;
}

/* the streaming kernels' branch-free fast path (ok[i] = 1 where conclusive) */
int64_t hmh_project_fast(const double* lat, const double* lon, int64_t n, int zoom, int32_t* row, int32_t* col,
                         uint8_t* ok)
{
    const double scale = hm_exp2i(zoom);
    const double kz = HM_INV360 * scale;
    int64_t m = 0;
    for (int64_t i = 0; i < n; i++) {
        ok[i] = (uint8_t)hm_project_fast(lat[i], lon[i], scale, kz, &row[i], &col[i], TAB);
        m += ok[i];
    }
    return m;
}
