"""Synthetic point clouds for tests and the benchmark (BASELINE.json configs).

Every generator here uses only IEEE add/multiply on doubles derived from a
splitmix64 counter stream, so numpy, the C oracle and the HIP generator
kernel (k_synth in csrc/hm_kernels.hip) produce bit-identical coordinates for the same
(seed, index).  That lets a GPU box regenerate a 1e9-point cloud in HBM and
still check it against host-side fixtures.

Distributions
-------------
uniform   lat ~ U(-85.0511287798066, 85.0511287798066), lon ~ U(-180, 180)
          
hotspots  K = 64 "city" centres, Zipf(1.1) weights, per-city sigma in
          [0.02, 0.2] degrees; offsets are Irwin-Hall(4) approximations of a
          normal deviate (sum of four uniforms, re-centred and scaled), which
          keeps every operation exact and bounds offsets at 3.47 sigma
          (config 2 / 3).
skew      90% of points uniform inside the zoom-18 tile containing
          (47.6, -122.3), 10% uniform world (config 4).
"""
from __future__ import annotations

import math

import numpy as np

LAT_MAX = 85.0511287798066
_M64 = (1 << 64) - 1
GOLDEN = 0x9E3779B97F4A7C15


def splitmix64(x: np.ndarray) -> np.ndarray:
    """splitmix64 finaliser of (x + golden); x is uint64."""
    with np.errstate(over="ignore"):
        z = x + np.uint64(GOLDEN)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def _stream(seed: int, idx: np.ndarray, lane: int, lanes: int) -> np.ndarray:
    """U[0,1) doubles: draw `lane` of `lanes` per point from one counter stream."""
    with np.errstate(over="ignore"):
        ctr = np.uint64(seed & _M64) * np.uint64(0x100000001B3) + idx.astype(np.uint64) * np.uint64(lanes) + np.uint64(lane)
    return (splitmix64(ctr) >> np.uint64(11)).astype(np.float64) * (2.0 ** -53)


def uniform(n: int, seed: int = 0, start: int = 0):
    idx = np.arange(start, start + n, dtype=np.uint64)
    u1 = _stream(seed, idx, 0, 2)
    u2 = _stream(seed, idx, 1, 2)
    lat = (u1 * 2.0 - 1.0) * LAT_MAX
    lon = u2 * 360.0 - 180.0
    return lat, lon


def hotspot_centres(seed: int = 0, k: int = 64):
    """City centres, sigmas and Zipf(1.1) cumulative weights (host constants).

    Computed once on the host with Python floats; the device generator takes
    the resulting table as an argument, so it never evaluates a pow/log.
    """
    idx = np.arange(k, dtype=np.uint64)
    clat = _stream(seed ^ 0x5EED, idx, 0, 3) * 130.0 - 60.0      # [-60, 70)
    clon = _stream(seed ^ 0x5EED, idx, 1, 3) * 350.0 - 175.0     # [-175, 175)
    sig = 0.02 + _stream(seed ^ 0x5EED, idx, 2, 3) * 0.18        # [0.02, 0.2)
    w = [1.0 / math.pow(i + 1, 1.1) for i in range(k)]
    tot = math.fsum(w)
    cdf, acc = [], 0.0
    for x in w:
        acc += x
        cdf.append(acc / tot)
    cdf[-1] = 1.0
    return clat, clon, sig, np.array(cdf, dtype=np.float64)


def _irwin_hall4(seed, idx, lane0, lanes):
    s = (_stream(seed, idx, lane0, lanes) + _stream(seed, idx, lane0 + 1, lanes))
    s = s + _stream(seed, idx, lane0 + 2, lanes)
    s = s + _stream(seed, idx, lane0 + 3, lanes)
    return (s - 2.0) * 1.7320508075688772   # unit variance, |g| <= 3.4641


def hotspots(n: int, seed: int = 0, start: int = 0, k: int = 64):
    clat, clon, sig, cdf = hotspot_centres(seed, k)
    idx = np.arange(start, start + n, dtype=np.uint64)
    lanes = 9
    u0 = _stream(seed, idx, 0, lanes)
    city = np.searchsorted(cdf, u0, side="right")
    city = np.minimum(city, k - 1)
    gy = _irwin_hall4(seed, idx, 1, lanes)
    gx = _irwin_hall4(seed, idx, 5, lanes)
    lat = clat[city] + sig[city] * gy
    lon = clon[city] + sig[city] * gx
    return lat, lon


# zoom-18 tile containing (47.6, -122.3): "18_91558_42015" (tile.py:9-13);
# its north/south edges are 47.60060732292068 / 47.59968131206439.
SKEW_Z18 = (91558, 42015)


def skew(n: int, seed: int = 0, start: int = 0):
    """90% inside one zoom-18 tile, 10% uniform world (config 4)."""
    idx = np.arange(start, start + n, dtype=np.uint64)
    u0 = _stream(seed, idx, 0, 3)
    u1 = _stream(seed, idx, 1, 3)
    u2 = _stream(seed, idx, 2, 3)
    row, col = SKEW_Z18
    # tile interior in lon is exact: col/2^18*360-180 .. (col+1)/2^18*360-180
    w = 360.0 / 262144.0
    lon_in = (col + 0.0625 + u2 * 0.875) * w - 180.0
    # interior latitude band around the tile centre (47.600144...), +-0.0004
    lat_c = 47.60014
    lat_in = lat_c + (u1 - 0.5) * 0.0008
    lat_w = (u1 * 2.0 - 1.0) * LAT_MAX
    lon_w = u2 * 360.0 - 180.0
    hot = u0 < 0.9
    return np.where(hot, lat_in, lat_w), np.where(hot, lon_in, lon_w)


GENERATORS = {"uniform": uniform, "hotspots": hotspots, "skew": skew}


def generate(kind: str, n: int, seed: int = 0, start: int = 0):
    return GENERATORS[kind](n, seed=seed, start=start)
