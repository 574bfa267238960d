"""Streaming micro-batches into a resident heatmap (hm_stream_*, BASELINE config 5)
vs the oracle: after any sequence of add() calls, the alltime bucket equals one
oracle count over every kept point so far, and each hour bucket equals the
oracle count over that hour's kept points.  Parity anchor: the oracle is pinned
to the reference's goldens (tests/test_oracle.py); the hour buckets have no
reference counterpart (its timespan labels other than 'alltime' are dead code,
heatmap.py:62-63), so they are checked for consistency with the same oracle."""
import numpy as np
import pytest

from oracle import oracle
from heatmap_amd import _lib, synth
from heatmap_amd.stream import ALLTIME, StreamingHeatmap

pytestmark = pytest.mark.gpu
BASE = 480000  # epoch hour (2024-10-04)


def _same(got, ref):
    got = got.sorted()
    assert ref["status"] == 0
    assert np.array_equal(got.zoom, ref["zoom"])
    assert np.array_equal(got.row, ref["row"])
    assert np.array_equal(got.col, ref["col"])
    assert np.array_equal(got.count, ref["count"])


def _batches(kind, nb, n, seed):
    out = []
    for b in range(nb):
        lat, lon = synth.generate(kind, n, seed=seed, start=b * n)
        rng = np.random.default_rng(seed * 100 + b)
        hour = (BASE + 3 * b + rng.integers(0, 3, n)).astype(np.uint32)  # batches overlap hours
        keep = (rng.random(n) > 0.1).astype(np.uint8)
        out.append((lat, lon, keep, hour))
    return out


@pytest.mark.parametrize("kind,zmin,zmax,initial", [("hotspots", 0, 18, 1 << 10), ("uniform", 3, 14, 1 << 22),
                                                    ("skew", 0, 21, 5000)])
def test_stream_matches_oracle(gpu, kind, zmin, zmax, initial):
    bs = _batches(kind, 4, 40000, seed=7)
    s = StreamingHeatmap(zmin, zmax, base_hour=BASE, initial_cells=initial)
    for lat, lon, keep, hour in bs:
        s.add(lat, lon, keep, hour)
    lat = np.concatenate([b[0] for b in bs])
    lon = np.concatenate([b[1] for b in bs])
    keep = np.concatenate([b[2] for b in bs])
    hour = np.concatenate([b[3] for b in bs])
    _same(s.counts(ALLTIME), oracle.count(lat, lon, keep, zmin, zmax))
    hourly = s.hourly()
    assert sorted(hourly) == sorted(np.unique(hour[keep == 1]).tolist())
    for h, c in hourly.items():
        _same(c, oracle.count(lat, lon, keep & (hour == h).astype(np.uint8), zmin, zmax))
    h0 = int(np.unique(hour)[0])
    _same(s.counts(h0), oracle.count(lat, lon, keep & (hour == h0).astype(np.uint8), zmin, zmax))
    cells, cap = s.cells()
    assert cells == sum(len(c.count) for c in hourly.values()) + len(s.counts(ALLTIME).count)
    assert cells * 8 <= cap * 5
    s.close()


def test_stream_alltime_only_and_errors(gpu):
    lat, lon = synth.generate("hotspots", 30000, seed=2)
    s = StreamingHeatmap(0, 16, base_hour=BASE)
    s.add(lat[:10000], lon[:10000])
    s.add(lat[10000:], lon[10000:])
    _same(s.counts(), oracle.count(lat, lon, None, 0, 16))
    bad = lat[:100].copy()
    bad[37] = np.nan
    with pytest.raises(ValueError):
        s.add(bad, lon[:100])
    with pytest.raises(Exception):  # hour before the stream's base hour
        s.add(lat[:10], lon[:10], hour=np.full(10, BASE - 1, np.uint32))
    # a failed add leaves the resident heatmap unchanged
    _same(s.counts(), oracle.count(lat, lon, None, 0, 16))
    s.close()


def test_stream_empty_and_unkept(gpu):
    s = StreamingHeatmap(0, 12, base_hour=BASE)
    s.add(np.zeros(0), np.zeros(0))
    lat, lon = synth.generate("uniform", 1000, seed=4)
    s.add(lat, lon, keep=np.zeros(1000, np.uint8), hour=np.full(1000, BASE, np.uint32))
    assert s.counts().count.size == 0
    assert s.cells()[0] == 0
    s.close()


def test_stream_single_hour_batches(gpu):
    """Time-ordered batches, one hour each (the fast path that folds `keep` directly)."""
    lat, lon = synth.generate("hotspots", 60000, seed=9)
    rng = np.random.default_rng(9)
    keep = (rng.random(60000) > 0.2).astype(np.uint8)
    hour = (BASE + np.arange(60000) // 20000).astype(np.uint32)  # 3 batches, 1 hour each
    s = StreamingHeatmap(2, 17, base_hour=BASE, initial_cells=2000)
    for b in range(3):
        sl = slice(b * 20000, (b + 1) * 20000)
        s.add(lat[sl], lon[sl], keep[sl], hour[sl])
    s.add(lat[:5000], lon[:5000], keep[:5000], hour[:5000])  # a late batch for an older hour
    lat2, lon2 = np.concatenate([lat, lat[:5000]]), np.concatenate([lon, lon[:5000]])
    keep2, hour2 = np.concatenate([keep, keep[:5000]]), np.concatenate([hour, hour[:5000]])
    _same(s.counts(ALLTIME), oracle.count(lat2, lon2, keep2, 2, 17))
    for h, c in s.hourly().items():
        _same(c, oracle.count(lat2, lon2, keep2 & (hour2 == h).astype(np.uint8), 2, 17))
    s.close()
