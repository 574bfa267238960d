"""First GPU parity: projection KATs and count pyramid vs the oracle."""
import json
import os

import numpy as np
import pytest

from oracle import oracle
from heatmap_amd import device, synth

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")
pytestmark = pytest.mark.gpu


def test_project_kat(gpu):
    """All 30k reference KATs; a column beyond int64 (KAT status 8) comes back
    exactly (HM_BIGCOL: an integer-valued double) and equals the reference's
    Python int (projection_kat_bigcols.json)."""
    from heatmap_amd import _lib

    d = np.load(os.path.join(GOLDEN, "projection_kat.npz"))
    big = {int(k): int(v) for k, v in json.load(open(os.path.join(GOLDEN, "projection_kat_bigcols.json"))).items()}
    bad = 0
    nbig = 0
    for z in np.unique(d["zoom"]):
        m = np.flatnonzero(d["zoom"] == z)
        p = device.project(d["lat"][m], d["lon"][m], int(z))
        re_, ce = d["row_err"][m], d["col_err"][m]
        exp = np.where(re_ != 0, re_, np.where(ce == 8, _lib.HM_BIGCOL, ce))
        ok = (p.status == exp) & ((exp != 0) | ((p.row == d["row"][m]) & (p.col == d["col"][m])))
        for j in np.flatnonzero(exp == _lib.HM_BIGCOL).tolist():
            i = int(m[j])
            got = int(np.array([p.col[j]], np.int64).view(np.float64)[0])
            ok[j] = ok[j] and p.row[j] == d["row"][i] and i in big and got == big[i]
            nbig += 1
        bad += int((~ok).sum())
    assert bad == 0
    assert nbig == sum(1 for i in big if d["row_err"][i] == 0)   # (a row error wins, tile.py:10-11)


def test_tile_big_column_ids(gpu):
    """Tile.tile_id_from_lat_long prints a column beyond int64 as the
    reference does (tests/golden/tile_ids.json holds such ids)."""
    from heatmap_amd.tile import Tile

    for la, lo, z, want in json.load(open(os.path.join(GOLDEN, "tile_ids.json"))):
        if "Error" in want:
            continue
        assert Tile.tile_id_from_lat_long(float(la), float(lo), z) == want, (la, lo, z)


@pytest.mark.parametrize("kind,n,zmin,zmax", [("uniform", 20000, 0, 14), ("hotspots", 200000, 0, 18),
                                               ("hotspots", 50000, 3, 21), ("skew", 100000, 0, 18),
                                               ("uniform", 1000, 0, 5), ("hotspots", 3000, 0, 0),
                                               ("uniform", 100000, 10, 14),
                                               # zmin inside the final 7-zoom pyramid of k_aggregate's
                                               # dense buckets (single- and multi-item): the register
                                               # pyramid's per-level zoom filter
                                               ("hotspots", 2_000_000, 14, 18), ("hotspots", 1_000_000, 17, 21)])
def test_count_vs_oracle(gpu, kind, n, zmin, zmax):
    lat, lon = synth.generate(kind, n, seed=3)
    keep = (np.arange(n) % 7 != 3).astype(np.uint8)
    got = device.count(lat, lon, keep, zmin, zmax).sorted()
    ref = oracle.count(lat, lon, keep, zmin, zmax)
    assert ref["status"] == 0
    assert np.array_equal(got.zoom, ref["zoom"])
    assert np.array_equal(got.row, ref["row"])
    assert np.array_equal(got.col, ref["col"])
    assert np.array_equal(got.count, ref["count"])


@pytest.mark.parametrize("kind", ["uniform", "hotspots", "skew"])
def test_synth_bit_exact(gpu, kind):
    import torch

    n = 300001
    lat = torch.empty(n, dtype=torch.float64, device="cuda")
    lon = torch.empty(n, dtype=torch.float64, device="cuda")
    device.synth(kind, lat, lon, seed=5, start=12345)
    hl, ho = synth.generate(kind, n, seed=5, start=12345)
    assert np.array_equal(lat.cpu().numpy().view(np.uint64), hl.view(np.uint64))
    assert np.array_equal(lon.cpu().numpy().view(np.uint64), ho.view(np.uint64))


def test_count_guard_band_points(gpu):
    """Boundary-adjacent latitudes take the deferred exact path (k_redo)."""
    d = np.load(os.path.join(GOLDEN, "projection_kat.npz"))
    ok = (d["row_err"] == 0) & (d["col_err"] == 0) & (np.abs(d["lat"]) < 85.05) & (np.abs(d["lon"]) < 179.9)
    lat, lon = d["lat"][ok], d["lon"][ok]
    for zmax in (14, 21):
        got = device.count(lat, lon, None, 0, zmax).sorted()
        ref = oracle.count(lat, lon, None, 0, zmax)
        assert got.slow_points > 0
        assert np.array_equal(got.count, ref["count"]) and np.array_equal(got.row, ref["row"])
        assert np.array_equal(got.col, ref["col"]) and np.array_equal(got.zoom, ref["zoom"])


@pytest.mark.parametrize("keep_polar", [False, True])
def test_count_redo_overflow_fallback(gpu, keep_polar):
    """More deferred points than the redo list holds -> fused exact fallback;
    kept, they also overflow the exotic list (rebuilt by k_collect_exotic)."""
    n = 3_000_000
    lat, lon = synth.uniform(n, seed=9)
    polar = (np.arange(n) % 5) < 2
    lat = np.where(polar, 86.0 + (lat % 3.0), lat)       # 40% beyond the fast window
    keep = np.ones(n, np.uint8) if keep_polar else (~polar).astype(np.uint8)
    got = device.count(lat, lon, keep, 0, 16).sorted()
    ref = oracle.count(lat, lon, keep, 0, 16)
    assert got.slow_points > (1 << 20)
    assert np.array_equal(got.count, ref["count"]) and np.array_equal(got.row, ref["row"])
    assert np.array_equal(got.col, ref["col"]) and np.array_equal(got.zoom, ref["zoom"])


def test_count_errors_and_exotic(gpu):
    lat, lon = synth.uniform(50000, seed=4)
    lat = lat.copy()
    lat[31337] = np.nan
    lat[40000] = 95.0
    with pytest.raises(ValueError, match="NaN"):
        device.count(lat, lon, None, 0, 14)
    lat[31337] = 10.0
    with pytest.raises(ValueError, match="domain"):
        device.count(lat, lon, None, 0, 14)
    lat[40000] = 89.0          # valid: the reference bins it at a negative row
    for keep in (None, (np.arange(50000) != 40000).astype(np.uint8)):
        got = device.count(lat, lon, keep, 0, 14).sorted()
        ref = oracle.count(lat, lon, keep, 0, 14)
        assert np.array_equal(got.count, ref["count"]) and np.array_equal(got.row, ref["row"])
        assert np.array_equal(got.col, ref["col"]) and np.array_equal(got.zoom, ref["zoom"])
    assert (device.count(lat, lon, None, 0, 14).row < 0).sum() == 15   # one negative row per zoom 0..14
