"""Level plans of the count pipeline (hm_api.cpp spread_replan).

Dense, evenly spread clouds switch levels 2.. from 6 to 3 zooms per level
(z5 -> z8 -> z11 at zmax 18).  At parity-test sizes the switch is forced by
lowering HM_SPREAD_MIN_KEYS (the mean level-1 bucket size it requires,
2^19 keys by default: the 1e9-point uniform bench).  The partition level
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
def test_spread_plan_tiles(gpu, monkeypatch, Z, levels, n):
    """(n stays small at zoom 21: the last level's dense child space, 64 per
    non-empty zoom-11 parent, must fit HM_SCAN_LIMIT or the call takes the
    general path)"""
    monkeypatch.setenv("HM_SPREAD_MIN_KEYS", "1")
    rng = np.random.default_rng(Z)
    rows = rng.integers(0, 1 << Z, n).astype(np.int64)
    cols = rng.integers(0, 1 << Z, n).astype(np.int64)
    got = device.count(rows, cols, None, 0, Z, tiles=True)
    assert int(got.stage_us[7]) == levels
    _same(got, oracle.count_tiles(rows, cols, 0, Z))


@pytest.mark.parametrize("zmin", [0, 9])
def test_spread_plan_latlon(gpu, monkeypatch, zmin):
    monkeypatch.setenv("HM_SPREAD_MIN_KEYS", "1")
    lat, lon = synth.generate("uniform", 2_000_000, seed=3)
    keep = (np.arange(lat.size) % 7 != 3).astype(np.uint8)
    got = device.count(lat, lon, keep, zmin, 18)
    assert int(got.stage_us[7]) == 3
    _same(got, oracle.count(lat, lon, keep, zmin, 18))


def test_default_plans(gpu, monkeypatch):
    """Without the override: parity-size uniform clouds and any hotspot cloud
    keep 6 zooms per level (a hotspot histogram is never flat)."""
    monkeypatch.delenv("HM_SPREAD_MIN_KEYS", raising=False)
    lat, lon = synth.generate("uniform", 1_000_000, seed=4)
    got = device.count(lat, lon, None, 0, 18)
    assert int(got.stage_us[7]) == 2
    _same(got, oracle.count(lat, lon, None, 0, 18))
    monkeypatch.setenv("HM_SPREAD_MIN_KEYS", "1")
    lat, lon = synth.generate("hotspots", 1_000_000, seed=4)
    got = device.count(lat, lon, None, 0, 18)
    assert int(got.stage_us[7]) == 2
    _same(got, oracle.count(lat, lon, None, 0, 18))
