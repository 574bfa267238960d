"""Level plans of the count pipeline (hm_api.cpp spread_replan).

Dense, evenly spread clouds switch levels 2.. from 6 to 3 zooms per level
(z5 -> z8 -> z11 at zmax 18).  At parity-test sizes the switch is forced by
lowering HM_SPREAD_MIN_KEYS (the mean level-1 bucket size it requires,
2^19 keys by default: the 1e9-point uniform bench) through hm_ctx_tune
(device.tuned).  The partition level
count is read back from hm_last_stats' slot 7.  Expected counts: the oracle
(heatmap.py:109-111's per-zoom reduceByKey).
"""
import numpy as np
import pytest

from oracle import oracle
from heatmap_amd import device, synth

pytestmark = pytest.mark.gpu


def _same(got, ref):
    got = got.sorted()
    assert got.zoom.size == ref["zoom"].size
    for k in ("zoom", "row", "col", "count"):
        assert np.array_equal(getattr(got, k), ref[k]), k


@pytest.mark.parametrize("Z,levels,n", [(18, 3, 1_500_000), (21, 4, 150_000), (16, 3, 1_500_000), (14, 2, 800_000)])
def test_spread_plan_tiles(gpu, Z, levels, n):
    """(n stays small at zoom 21: the last level's dense child space, 64 per
    non-empty zoom-11 parent, must fit HM_SCAN_LIMIT or the call takes the
    general path)"""
    rng = np.random.default_rng(Z)
    rows = rng.integers(0, 1 << Z, n).astype(np.int64)
    cols = rng.integers(0, 1 << Z, n).astype(np.int64)
    with device.tuned(HM_SPREAD_MIN_KEYS=1):
        got = device.count(rows, cols, None, 0, Z, tiles=True)
    assert int(got.stage_us[7]) == levels
    _same(got, oracle.count_tiles(rows, cols, 0, Z))


@pytest.mark.parametrize("zmin", [0, 9])
def test_spread_plan_latlon(gpu, zmin):
    lat, lon = synth.generate("uniform", 2_000_000, seed=3)
    keep = (np.arange(lat.size) % 7 != 3).astype(np.uint8)
    with device.tuned(HM_SPREAD_MIN_KEYS=1):
        got = device.count(lat, lon, keep, zmin, 18)
    assert int(got.stage_us[7]) == 3
    _same(got, oracle.count(lat, lon, keep, zmin, 18))


def test_default_plans(gpu):
    """Without the override: parity-size uniform clouds and any hotspot cloud
    keep 6 zooms per level (a hotspot histogram is never flat)."""
    lat, lon = synth.generate("uniform", 1_000_000, seed=4)
    got = device.count(lat, lon, None, 0, 18)
    assert int(got.stage_us[7]) == 2
    _same(got, oracle.count(lat, lon, None, 0, 18))
    lat, lon = synth.generate("hotspots", 1_000_000, seed=4)
    with device.tuned(HM_SPREAD_MIN_KEYS=1):
        got = device.count(lat, lon, None, 0, 18)
    assert int(got.stage_us[7]) == 2
    _same(got, oracle.count(lat, lon, None, 0, 18))


@pytest.mark.parametrize("big_min", [None, 1000000, 0])
def test_hot_children_many_runs(gpu, big_min):
    """Children with many runs -- one run per work item of their parent, the
    hot tiles of a skewed cloud -- are copied by every wave of k_rs_copy_big
    when they hold more than HM_RS_BIG_MIN runs (2048 by default: the three
    hot zoom-18 tiles here, ~5100 runs each); also with none listed (one wave
    per child) and with every child listed (the 4096-entry list overflows, the
    rest are copied in place).  A zoom-5 parent of ~5100 work items plus a
    uniform background.  Hot tiles off: with them the three tiles' keys skip
    level 2 (tests/test_gpu_hot.py runs the same cloud that way)."""
    from conftest import cells_digest
    rng = np.random.default_rng(21)
    Z = 18
    hot = [(70001, 130003), (70100, 130050), (71000, 131000)]   # one zoom-5 tile (>> 13)
    rows = [np.full(14_000_000, r, np.int64) for r, _ in hot]
    cols = [np.full(14_000_000, c, np.int64) for _, c in hot]
    rows.append(rng.integers(0, 1 << Z, 6_000_000))
    cols.append(rng.integers(0, 1 << Z, 6_000_000))
    rows = np.concatenate(rows)
    cols = np.concatenate(cols)
    perm = rng.permutation(rows.size)
    rows, cols = rows[perm], cols[perm]
    knobs = {"HM_HOT": 0} if big_min is None else {"HM_HOT": 0, "HM_RS_BIG_MIN": big_min}
    with device.tuned(**knobs):
        got = device.count(rows, cols, None, 0, Z, tiles=True)
    assert int(got.stage_us[6]) == 0
    ref = oracle.count_tiles(rows, cols, 0, Z)
    assert got.zoom.size == ref["zoom"].size
    assert cells_digest(got.zoom, got.row, got.col, got.count) == \
        cells_digest(ref["zoom"], ref["row"], ref["col"], ref["count"])
