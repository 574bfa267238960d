"""CPU: the product's projection arithmetic (heatmap_amd/csrc/hm_project.h, the
statements the gfx950 kernels execute) compiled with gcc, against the
reference's known answers and the oracle.

  * fast path + exact slow path == reference on every KAT (boundary pairs incl.)
  * == oracle on millions of random points at zooms 0..30
  * the fast path's |Y_fast - Y_ref| stays >= 8x below the guard band HM_Y_EPS
  * the glibc restatement (hm_glibc_emul.h) == the live libm bit-for-bit
"""
import ctypes
import os

import numpy as np
import pytest

from oracle import oracle
from heatmap_amd import synth

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")
HM_Y_EPS = 1.5e-13       # hm_project.h
HM_LAT_FAST = 85.06
HM_E_RANGE = 8


def _dp(a):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_double))


def _host_project(L, lat, lon, zoom):
    lat = np.ascontiguousarray(lat, np.float64)
    lon = np.ascontiguousarray(lon, np.float64)
    n = lat.size
    row = np.zeros(n, np.int64)
    col = np.zeros(n, np.int64)
    st = np.zeros(n, np.uint8)
    slow = np.zeros(n, np.uint8)
    P = ctypes.POINTER
    L.hmh_project(_dp(lat), _dp(lon), n, int(zoom), row.ctypes.data_as(P(ctypes.c_int64)),
                  col.ctypes.data_as(P(ctypes.c_int64)), st.ctypes.data_as(P(ctypes.c_uint8)),
                  slow.ctypes.data_as(P(ctypes.c_uint8)))
    return row, col, st, slow


def test_product_math_vs_kat(host_math):
    d = np.load(os.path.join(GOLDEN, "projection_kat.npz"))
    bad = 0
    slow_total = 0
    for z in np.unique(d["zoom"]):
        m = d["zoom"] == z
        r, c, st, slow = _host_project(host_math, d["lat"][m], d["lon"][m], int(z))
        re_, ce = d["row_err"][m], d["col_err"][m]
        exp = np.where(re_ != 0, re_, ce)
        ok = (st == exp) & ((exp != 0) | ((r == d["row"][m]) & (c == d["col"][m])))
        bad += int((~ok).sum())
        slow_total += int(slow.sum())
    assert bad == 0
    assert slow_total > 1000       # the bisected boundary pairs take the exact path


@pytest.mark.parametrize("kind", ["uniform", "hotspots", "skew"])
def test_product_math_vs_oracle_random(host_math, kind):
    lat, lon = synth.generate(kind, 1_000_000, seed=7)
    for z in (0, 5, 12, 18, 21, 26, 30):
        r, c, st, slow = _host_project(host_math, lat, lon, z)
        ro, co, so, _ = oracle.project(lat, lon, z)
        assert np.array_equal(st, so)
        assert np.array_equal(r, ro) and np.array_equal(c, co), z
        if z <= 21:
            assert slow.mean() < 1e-4


@pytest.mark.parametrize("kind", ["uniform", "hotspots", "skew", "kat"])
def test_streaming_fast_path_vs_oracle(host_math, kind):
    """hm_project_fast (k_project_partition's branch-free path): wherever it
    claims a result, the result is the reference's; it declines only rarely."""
    if kind == "kat":
        d = np.load(os.path.join(GOLDEN, "projection_kat.npz"))
        lat, lon, zs = d["lat"], d["lon"], sorted(set(int(z) for z in d["zoom"]) & set(range(0, 22)))
    else:
        lat, lon = synth.generate(kind, 1_000_000, seed=8)
        zs = (0, 3, 11, 14, 18, 21)
    P = ctypes.POINTER
    for z in zs:
        n = lat.size
        row = np.zeros(n, np.int32)
        col = np.zeros(n, np.int32)
        ok = np.zeros(n, np.uint8)
        m = host_math.hmh_project_fast(_dp(np.ascontiguousarray(lat)), _dp(np.ascontiguousarray(lon)), n, z,
                                       row.ctypes.data_as(P(ctypes.c_int32)), col.ctypes.data_as(P(ctypes.c_int32)),
                                       ok.ctypes.data_as(P(ctypes.c_uint8)))
        ro, co, so, _ = oracle.project(lat, lon, z)
        k = ok.astype(bool)
        assert np.all(so[k] == 0)
        assert np.array_equal(row[k], ro[k]) and np.array_equal(col[k], co[k]), z
        if kind != "kat":
            assert m >= n - max(50, n // 10000), (z, n - m)


def test_fast_Y_error_bound(host_math):
    """HM_Y_EPS carries a >= 8x margin over the worst fast-path error seen."""
    rng = np.random.default_rng(1)
    lat = np.concatenate([rng.uniform(-HM_LAT_FAST, HM_LAT_FAST, 3_000_000),
                          rng.uniform(84.0, HM_LAT_FAST, 200_000), rng.uniform(-HM_LAT_FAST, -84.0, 200_000),
                          rng.uniform(-1e-3, 1e-3, 100_000), np.array([0.0, -0.0, HM_LAT_FAST, -HM_LAT_FAST])])
    worst = ctypes.c_double(0)
    e = host_math.hmh_fast_Y_maxerr(_dp(lat), lat.size, ctypes.byref(worst))
    assert e * 8 <= HM_Y_EPS, (e, worst.value)


@pytest.mark.parametrize("fn,lo,hi", [(0, -2.0, 2.0), (1, -2.0, 2.0), (2, 1e-3, 1e3), (0, -1e4, 1e4),
                                       (1, -1e6, 1e6), (2, 1e-300, 1e300)])
def test_glibc_restatement_bit_exact(host_math, fn, lo, hi):
    """hm_glibc_{tan,cos,log} == this host's glibc (the reference's libm)."""
    rng = np.random.default_rng(fn * 10 + int(abs(lo)) % 7)
    if fn == 2 and hi / lo > 1e6:
        x = np.exp(rng.uniform(np.log(lo), np.log(hi), 400_000))
    else:
        x = rng.uniform(lo, hi, 400_000)
    un = ctypes.c_int64(0)
    bad = host_math.hmh_glibc_check(fn, _dp(x), x.size, ctypes.byref(un))
    assert bad == 0
    assert un.value == 0


@pytest.mark.parametrize("fn", [0, 1])
def test_glibc_branred_bit_exact(host_math, fn):
    """tan/cos beyond 105414350, where glibc reduces with __branred
    (hm_branred.h): log-uniform magnitudes up to DBL_MAX, both signs, plus the
    threshold's neighbourhood and multiples of pi/2 (hard cases)."""
    rng = np.random.default_rng(77 + fn)
    x = np.exp(rng.uniform(np.log(1.0e8), np.log(1.79e308), 300_000)) * rng.choice([-1.0, 1.0], 300_000)
    near = 105414350.0 + rng.uniform(-64.0, 64.0, 20_000)
    k = rng.integers(1, 1 << 52, 20_000).astype(np.float64) * (np.pi / 2)
    x = np.concatenate([x, near, -near, k, np.nextafter(k, np.inf), np.nextafter(k, -np.inf)])
    un = ctypes.c_int64(0)
    bad = host_math.hmh_glibc_check(fn, _dp(x), x.size, ctypes.byref(un))
    assert un.value == 0
    assert bad == 0


def test_product_math_huge_latitudes(host_math):
    """Latitudes beyond ~6e9 degrees reach glibc's __branred (hm_branred.h):
    rows, statuses and columns equal the oracle's (live libm) at every zoom."""
    rng = np.random.default_rng(11)
    n = 200_000
    lat = np.exp(rng.uniform(np.log(6.1e9), np.log(1e300), n)) * rng.choice([-1.0, 1.0], n)
    lon = rng.uniform(-180.0, 180.0, n)
    for z in (0, 7, 18, 21, 30):
        r, c, st, _ = _host_project(host_math, lat, lon, z)
        ro, co, so, _ = oracle.project(lat, lon, z)
        assert np.array_equal(st, so), z
        ok = so == 0
        assert ok.sum() > n // 4
        assert np.array_equal(r[ok], ro[ok]) and np.array_equal(c[ok], co[ok]), z
