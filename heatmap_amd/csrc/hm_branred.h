/* Payne-Hanek reduction of glibc 2.35 libm, ``__branred`` (sysdeps/ieee754/
 * dbl-64/branred.c), restated for the device: x = n pi/2 + (a + aa) with
 * |a + aa| <= pi/4, returns n mod 4.  glibc's tan/cos call it for
 * |x| >= 105414350 (hm_glibc_emul.h), i.e. latitudes beyond ~6e9 degrees.
 * The routine is plain IEEE binary64 arithmetic (no FMA in libm's build of
 * it): x is scaled by 2^-600 and split into two 26-bit halves, each half times
 * six 24-bit digits of 2/pi (the ones that matter at its exponent) gives exact
 * partial products, whose integer parts (mod 4) are the quadrant and whose
 * fractions sum to the remainder in double-double; the remainder is then
 * multiplied by pi/2 in double-double.  Operation order is the C source's.
 * glibc is LGPL-2.1.  Checked bit for bit against the live libm's tan and cos
 * by tests/test_math_host.py::test_glibc_restatement_bit_exact (huge
 * arguments). */
#pragma once
#include "hm_common.h"

HM_EMUL_BEGIN

/* 2/pi in base 2^24: digit i = floor(2/pi * 2^(24(i+1))) mod 2^24 */
HM_EMUL_TABLE double hm_toverp[75] = {
    10680707.0, 7228996.0, 1387004.0, 2578385.0, 16069853.0, 12639074.0, 9804092.0, 4427841.0,
    16666979.0, 11263675.0, 12935607.0, 2387514.0, 4345298.0, 14681673.0, 3074569.0, 13734428.0,
    16653803.0, 1880361.0, 10960616.0, 8533493.0, 3062596.0, 8710556.0, 7349940.0, 6258241.0,
    3772886.0, 3769171.0, 3798172.0, 8675211.0, 12450088.0, 3874808.0, 9961438.0, 366607.0,
    15675153.0, 9132554.0, 7151469.0, 3571407.0, 2607881.0, 12013382.0, 4155038.0, 6285869.0,
    7677882.0, 13102053.0, 15825725.0, 473591.0, 9065106.0, 15363067.0, 6271263.0, 9264392.0,
    5636912.0, 4652155.0, 7056368.0, 13614112.0, 10155062.0, 1944035.0, 9527646.0, 15080200.0,
    6658437.0, 6231200.0, 6832269.0, 16767104.0, 5075751.0, 3212806.0, 1398474.0, 7579849.0,
    6349435.0, 12618859.0, 4703257.0, 12806093.0, 14477321.0, 2786137.0, 12875403.0, 9837734.0,
    14528324.0, 13719321.0, 343717.0,
};

HM_EMUL_FN int hm_branred_half(double x1, double* b_out, double* bb_out, double* sum_out)
{
    const double big = 6755399441055744.0;      /* 2^52 + 2^51 */
    const double big1 = 27021597764222976.0;    /* 2^54 + 2^53 */
    const double tm24 = 5.9604644775390625e-08; /* 2^-24 */
    hm_x64 u, gor;
    double r[6], s, t, sum, b, bb;
    int k;
    sum = 0.0;
    u.d = x1;
    k = (int)((u.u >> 52) & 2047);
    k = (k - 450) / 24;
    if (k < 0) k = 0;
    gor.u = 0x63F0000000000000ull - ((uint64_t)(k * 24) << 52);   /* 2^(576 - 24k) */
    for (int i = 0; i < 6; i++) {
        r[i] = x1 * hm_toverp[k + i] * gor.d;
        gor.d *= tm24;
    }
    for (int i = 0; i < 3; i++) {
        s = (r[i] + big) - big;
        sum += s;
        r[i] -= s;
    }
    t = 0.0;
    for (int i = 0; i < 6; i++) t += r[5 - i];
    bb = (((((r[0] - t) + r[1]) + r[2]) + r[3]) + r[4]) + r[5];
    s = (t + big) - big;
    sum += s;
    t -= s;
    b = t + bb;
    bb = (t - b) + bb;
    s = (sum + big1) - big1;
    sum -= s;
    *b_out = b;
    *bb_out = bb;
    *sum_out = sum;
    return 0;
}

HM_EMUL_FN int hm_branred(double x, double* a, double* aa)
{
    const double tm600 = 2.409919865102884e-181;   /* 2^-600 */
    const double split = 134217729.0;              /* 2^27 + 1 */
    const double hp0 = 0x1.921fb54442d18p+0;       /* pi/2 = hp0 + hp1 */
    const double hp1 = 0x1.1a62633145c07p-54;
    const double mp1 = 0x1.921fb58p+0;             /* pi/2 = mp1 + mp2 (28 bits each) */
    const double mp2 = -0x1.dde974p-27;
    double t, x1, x2, sum, sum1, sum2, b, bb, b1, bb1, b2, bb2, s, t1, t2;
    x *= tm600;
    t = x * split;
    x1 = t - (t - x);
    x2 = x - x1;
    hm_branred_half(x1, &b1, &bb1, &sum1);
    hm_branred_half(x2, &b2, &bb2, &sum2);
    sum = sum1 + sum2;
    b = b1 + b2;
    bb = (fabs(b1) > fabs(b2)) ? (b1 - b) + b2 : (b2 - b) + b1;
    if (b > 0.5) {
        b -= 1.0;
        sum += 1.0;
    } else if (b < -0.5) {
        b += 1.0;
        sum -= 1.0;
    }
    s = b + (bb + bb1 + bb2);
    t = ((b - s) + bb) + (bb1 + bb2);
    b = s * split;
    t1 = b - (b - s);
    t2 = s - t1;
    b = s * hp0;
    bb = (((t1 * mp1 - b) + t1 * mp2) + t2 * mp1) + (t2 * mp2 + s * hp1 + t * hp0);
    s = b + bb;
    t = (b - s) + bb;
    *a = s;
    *aa = t;
    return ((int)sum) & 3;
}

HM_EMUL_END
