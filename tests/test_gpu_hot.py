"""Hot tiles (hm_pipeline.h): zoom-(Z-7) tiles that a
sample shows to hold >= 1/4096 of the points get their own level-1 digit and
go straight to the final aggregation, skipping the level-2 partition.  The
counts must not change: every case is compared with the oracle (the per-zoom
reduceByKey of heatmap.py:109-111) cell for cell, or, at tens of millions of
points, through the order-free cell digest.  HM_HOT_MIN_KEYS = 0 (through
hm_ctx_tune) lets parity-size clouds have hot tiles; hm_last_stats slot 6
reports how many a call found.
"""
import numpy as np
import pytest

from conftest import cells_digest
from oracle import oracle
from heatmap_amd import device, synth

pytestmark = pytest.mark.gpu


def _same(got, ref):
    got = got.sorted()
    assert got.zoom.size == ref["zoom"].size
    for k in ("zoom", "row", "col", "count"):
        assert np.array_equal(getattr(got, k), ref[k]), k


@pytest.mark.parametrize("kind,n,zmin,zmax", [("hotspots", 2_000_000, 0, 18), ("hotspots", 1_000_000, 9, 18),
                                              ("hotspots", 1_000_000, 17, 18), ("skew", 1_000_000, 0, 18),
                                              ("hotspots", 1_000_000, 0, 16), ("hotspots", 600_000, 0, 13)])
def test_hot_latlon(gpu, kind, n, zmin, zmax):
    lat, lon = synth.generate(kind, n, seed=31)
    keep = (np.arange(n) % 11 != 5).astype(np.uint8)
    with device.tuned(HM_HOT_MIN_KEYS=0, HM_SPREAD_MIN_COLD=1e12):
        got = device.count(lat, lon, keep, zmin, zmax)
    assert int(got.stage_us[6]) > 0, "no hot tiles"
    assert int(got.stage_us[7]) == 2
    _same(got, oracle.count(lat, lon, keep, zmin, zmax))


@pytest.mark.parametrize("kind,n,zmin,zmax", [("hotspots", 2_000_000, 0, 18), ("skew", 1_000_000, 0, 18),
                                              ("hotspots", 1_000_000, 12, 18), ("hotspots", 1_000_000, 0, 16),
                                              ("skew", 600_000, 0, 17)])
def test_hot_with_spread_plan(gpu, kind, n, zmin, zmax):
    """Hot tiles with the cold rest on 3-zoom levels (z5 -> z(Z-10) -> z(Z-7)):
    the tiles join the last level as children of their level-2 ancestor, which
    stays a bucket even without cold keys (forced)."""
    lat, lon = synth.generate(kind, n, seed=37)
    keep = (np.arange(n) % 13 != 4).astype(np.uint8)
    with device.tuned(HM_HOT_MIN_KEYS=0, HM_SPREAD_MIN_COLD=0):
        got = device.count(lat, lon, keep, zmin, zmax)
    assert int(got.stage_us[6]) > 0, "no hot tiles"
    assert int(got.stage_us[7]) == 3
    _same(got, oracle.count(lat, lon, keep, zmin, zmax))


def test_hot_default_knobs_skew(gpu):
    """Default thresholds: the skew cloud's one hot zoom-11 tile (90% of the
    points) is found at 1M points."""
    lat, lon = synth.generate("skew", 1_000_000, seed=5)
    got = device.count(lat, lon, None, 0, 18)
    assert int(got.stage_us[6]) == 1
    _same(got, oracle.count(lat, lon, None, 0, 18))


def test_hot_many_tiles_cap(gpu):
    """More candidate tiles than the 512 hot digits: the first 512 found are
    hot, the rest stay cold (both paths in one call)."""
    lat, lon = synth.generate("hotspots", 3_000_000, seed=8)
    with device.tuned(HM_HOT_MIN_KEYS=0, HM_HOT_INV_SHARE=1e6):
        got = device.count(lat, lon, None, 0, 18)
    assert int(got.stage_us[6]) == 512
    _same(got, oracle.count(lat, lon, None, 0, 18))


def test_hot_tiles_input_and_exotic(gpu):
    """Tile input (hm_count_tiles) with hot tiles, cells outside the square and
    a keep mask."""
    rng = np.random.default_rng(12)
    Z = 18
    n = 1_500_000
    rows = np.where(rng.random(n) < 0.6, 91558 + rng.integers(-300, 300, n), rng.integers(0, 1 << Z, n))
    cols = np.where(rng.random(n) < 0.6, 42015 + rng.integers(-300, 300, n), rng.integers(0, 1 << Z, n))
    out = rng.random(n) < 0.01
    rows = np.where(out, rows - (1 << Z), rows).astype(np.int64)
    keep = (rng.random(n) < 0.9).astype(np.uint8)
    with device.tuned(HM_HOT_MIN_KEYS=0):
        got = device.count(rows, cols.astype(np.int64), keep, 0, Z, tiles=True)
    assert int(got.stage_us[6]) > 0
    _same(got, oracle.count_tiles(rows, cols.astype(np.int64), 0, Z, keep=keep))


def test_hot_region_overflow_retry(gpu):
    """A hot tile the sample under-estimates: every 16th point (the sampled
    ones at this size) sits in tile A, one in 2048 of them in tile B; most of
    the unsampled points are in B.  B's region overflows and the level is
    re-run with exact sizes."""
    Z = 18
    n = 1 << 22
    idx = np.arange(n)
    rows = np.full(n, 5000, np.int64)
    cols = np.full(n, 9000, np.int64)          # tile A (zoom-11 tile (39, 70))
    sampled = idx % 16 == 0
    b = sampled & ((idx // 16) % 1500 == 0)       # > 1/2048 of the samples in tile B
    b |= (~sampled) & (idx % 3 != 0)              # and two thirds of the rest
    rows[b] = 200064 + (idx[b] % 60)              # one zoom-11 tile: (1563, 781)
    cols[b] = 100000 + (idx[b] % 89)
    with device.tuned(HM_HOT_MIN_KEYS=0):
        got = device.count(rows, cols, None, 0, Z, tiles=True)
    assert int(got.stage_us[6]) == 2
    _same(got, oracle.count_tiles(rows, cols, 0, Z))


def test_hot_three_tiles_48m(gpu):
    """tests/test_gpu_plan.py's skewed 48M-point cloud with hot tiles on (the
    default): three hot zoom-11 tiles take 42M points past level 2."""
    rng = np.random.default_rng(21)
    Z = 18
    hot = [(70001, 130003), (70100, 130050), (71000, 131000)]
    rows = [np.full(14_000_000, r, np.int64) for r, _ in hot]
    cols = [np.full(14_000_000, c, np.int64) for _, c in hot]
    rows.append(rng.integers(0, 1 << Z, 6_000_000))
    cols.append(rng.integers(0, 1 << Z, 6_000_000))
    rows = np.concatenate(rows)
    cols = np.concatenate(cols)
    perm = rng.permutation(rows.size)
    rows, cols = rows[perm], cols[perm]
    got = device.count(rows, cols, None, 0, Z, tiles=True)
    assert int(got.stage_us[6]) == 3
    ref = oracle.count_tiles(rows, cols, 0, Z)
    assert cells_digest(got.zoom, got.row, got.col, got.count) == \
        cells_digest(ref["zoom"], ref["row"], ref["col"], ref["count"])


def test_hot_stream_batches(gpu):
    """Streaming batches counted with hot tiles equal one count of all points."""
    from heatmap_amd.stream import StreamingHeatmap

    n = 600_000
    lat, lon = synth.generate("hotspots", 2 * n, seed=13)
    with device.tuned(HM_HOT_MIN_KEYS=0):
        s = StreamingHeatmap(0, 18, base_hour=480000, initial_cells=1 << 16)
        s.add(lat[:n], lon[:n], hour=np.full(n, 480000, np.uint32))
        s.add(lat[n:], lon[n:], hour=np.full(n, 480001, np.uint32))
        got = s.counts().sorted()
        s.close()
    _same(got, oracle.count(lat, lon, None, 0, 18))


@pytest.mark.parametrize("kind,n,zmin,zmax,contig", [("hotspots", 2_000_000, 0, 21, 1), ("hotspots", 2_000_000, 6, 21, 1),
                                                     ("hotspots", 1_000_000, 0, 19, 1), ("skew", 1_000_000, 0, 20, 1),
                                                     ("hotspots", 1_000_000, 6, 21, 0), ("hotspots", 800_000, 14, 21, 1)])
def test_hot_mid_level(gpu, kind, n, zmin, zmax, contig):
    """Mid-level hot tiles (zmax 19-21, plan z5 -> z11 -> zmax-7): zoom-11
    tiles with many points skip level 2 -- level 1 writes their keys in level
    2's u32 form into level 2's output array -- and join level 3 as level-2
    buckets, next to the cold keys (child-contiguous above every level-1
    position with HM_CONTIG, at their own positions without)."""
    lat, lon = synth.generate(kind, n, seed=41)
    keep = (np.arange(n) % 9 != 2).astype(np.uint8)
    with device.tuned(HM_HOT_MIN_KEYS=0, HM_CONTIG=contig):
        got = device.count(lat, lon, keep, zmin, zmax)
    assert int(got.stage_us[6]) > 0, "no hot tiles"
    assert int(got.stage_us[7]) == 3
    _same(got, oracle.count(lat, lon, keep, zmin, zmax))
    with device.tuned(HM_HOT_MIN_KEYS=0, HM_HOT_MID=0):
        off = device.count(lat, lon, keep, zmin, zmax)
    assert int(off.stage_us[6]) == 0
    _same(off, oracle.count(lat, lon, keep, zmin, zmax))


def test_hot_mid_level_tiles_input_and_redo(gpu):
    """Mid-level hot tiles from tile input with cells outside the square (the
    partial-tile kernel's u32 hot stores) and guard-band points (k_redo's
    tiles) at zmax 21."""
    rng = np.random.default_rng(17)
    Z = 21
    n = 1_200_007
    rows = np.where(rng.random(n) < 0.7, 732467 + rng.integers(-900, 900, n), rng.integers(0, 1 << Z, n))
    cols = np.where(rng.random(n) < 0.7, 336123 + rng.integers(-900, 900, n), rng.integers(0, 1 << Z, n))
    out = rng.random(n) < 0.01
    rows = np.where(out, rows + (1 << Z), rows).astype(np.int64)
    with device.tuned(HM_HOT_MIN_KEYS=0):
        got = device.count(rows, cols.astype(np.int64), None, 0, Z, tiles=True)
    assert int(got.stage_us[6]) > 0
    _same(got, oracle.count_tiles(rows, cols.astype(np.int64), 0, Z))
