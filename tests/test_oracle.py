"""CPU: the oracle against the reference's own outputs (tests/golden/, made by
tests/golden/make_golden.py from reference tile.py / heatmap.py), and the
host-side row assembly (heatmap_amd.heatmap.assemble_rows) fed by oracle
counts against the reference's build_heatmaps rows.

This pins the oracle before any GPU result is compared with it.
"""
import collections
import gzip
import hashlib
import json
import os

import numpy as np
import pytest

from oracle import oracle
from heatmap_amd import heatmap, synth

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")
ROW_GOLDENS = sorted(f for f in os.listdir(GOLDEN) if f.startswith("heatmap_rows_"))


def _kat():
    return np.load(os.path.join(GOLDEN, "projection_kat.npz"))


def test_projection_kat():
    """tile.py:15-21 known answers (incl. bisected row boundaries, NaN/inf/domain)."""
    d = _kat()
    bad = 0
    for z in np.unique(d["zoom"]):
        m = d["zoom"] == z
        r, c, st, _ = oracle.project(d["lat"][m], d["lon"][m], int(z))
        re_, ce = d["row_err"][m], d["col_err"][m]
        exp = np.where(re_ != 0, re_, ce)          # row error wins (tile.py:10-11)
        ok = (st == exp) & ((exp != 0) | ((r == d["row"][m]) & (c == d["col"][m])))
        bad += int((~ok).sum())
    assert bad == 0
    assert len(d["lat"]) > 20000


def test_projection_kat_big_columns():
    """Columns beyond int64 (lon 1e300 at z30) are reported as out of range."""
    d = _kat()
    big = json.load(open(os.path.join(GOLDEN, "projection_kat_bigcols.json")))
    for i in map(int, big):
        _, _, st, _ = oracle.project(d["lat"][i:i + 1], d["lon"][i:i + 1], int(d["zoom"][i]))
        assert st[0] in (oracle.E_RANGE, d["row_err"][i])


def test_tile_ids_and_messages():
    """Tile.tile_id_from_lat_long strings and exception messages (tile.py:9-13)."""
    msgs = {oracle.E_NAN: "ValueError: cannot convert float NaN to integer",
            oracle.E_DOMAIN: "ValueError: math domain error",
            oracle.E_INF: "OverflowError: cannot convert float infinity to integer"}
    for la, lo, z, want in json.load(open(os.path.join(GOLDEN, "tile_ids.json"))):
        r, c, st, _ = oracle.project(np.array([float(la)]), np.array([float(lo)]), z)
        if st[0] == 0:
            got = "%d_%d_%d" % (z, r[0], c[0])
        elif st[0] == oracle.E_RANGE:
            # beyond int64: the reference prints an unbounded Python int
            got = "%d_%d_%d" % (z, oracle._row_of(float(la), z), oracle._col_of(float(lo), z))
        else:
            got = msgs.get(int(st[0]), "range")
        assert got == want, (la, lo, z)


def _digest(cells):
    h = hashlib.sha256()
    for it in cells:
        h.update((",".join(str(x) for x in it) + "\n").encode())
    return h.hexdigest()


def _check_zoom_digests(lat, lon, expect):
    zs = sorted(int(z) for z in expect)
    ref = oracle.count(lat, lon, None, min(zs), max(zs))
    assert ref["status"] == 0
    for z in zs:
        m = ref["zoom"] == z
        cells = list(zip(ref["row"][m].tolist(), ref["col"][m].tolist(), ref["count"][m].tolist()))
        e = expect[str(z)]
        assert len(cells) == e["cells"], z
        assert sum(c for _, _, c in cells) == e["total"], z
        assert _digest(cells) == e["sha256"], z


def test_zoom_digests_hotspots_and_skew():
    """Counter(Tile.tile_id_from_lat_long(...)) per zoom 0..21 (north_star zooms 0-18 and beyond)."""
    g = json.load(open(os.path.join(GOLDEN, "zoom_counts_hotspots.json")))
    lat, lon = synth.hotspots(g["n"], seed=0)
    _check_zoom_digests(lat, lon, g["zoom_counts"])
    lat, lon = synth.skew(g["skew"]["n"], seed=0)
    _check_zoom_digests(lat, lon, g["skew"]["zoom_counts"])


def test_config1_zoom_digests():
    """BASELINE config 1 (1M uniform, seed 0): per-zoom cells z0..21 digest."""
    g = json.load(open(os.path.join(GOLDEN, "config1_digest.json")))
    lat, lon = synth.uniform(g["n"], seed=0)
    _check_zoom_digests(lat, lon, g["zoom_counts"])


def _oracle_counters(lat, lon, zmin, zmax):
    """The oracle's stand-ins for hm_count / hm_count_grouped
    (heatmap.assemble_cells' counting hooks)."""

    def count_all(keep):
        r = oracle.count(lat, lon, keep.astype(np.uint8), zmin, zmax)
        assert r["status"] == 0
        return r["zoom"], r["row"], r["col"], r["count"]

    def count_grouped(keep, gid):
        parts = []
        for g in np.unique(gid[keep]).tolist():
            r = oracle.count(lat, lon, (keep & (gid == g)).astype(np.uint8), zmin, zmax)
            assert r["status"] == 0
            parts.append((np.full(r["zoom"].size, g), r["zoom"], r["row"], r["col"], r["count"]))
        return tuple(np.concatenate([p[i] for p in parts]) for i in range(5))

    return count_all, count_grouped


def _load_rows(name):
    with gzip.open(os.path.join(GOLDEN, name), "rt") as f:
        return json.load(f)


def _oracle_project(lat, lon, z):
    """ChainFix's forward projection through the oracle (CPU tests)."""
    return (np.array([oracle._row_of(a, z) for a in lat], np.int64),
            np.array([oracle._col_of(b, z) for b in lon], np.int64))


@pytest.mark.parametrize("name", ROW_GOLDENS)
def test_assemble_rows_vs_reference(name):
    """heatmap_amd's row layout + 'all' weighting on oracle counts == build_heatmaps rows."""
    g = _load_rows(name)
    rows = g["input"]
    lat = np.array([r["latitude"] for r in rows])
    lon = np.array([r["longitude"] for r in rows])
    keep = np.array([r["source"] != "background" for r in rows])
    users = [r["user_id"] for r in rows]
    mz, d = g["max_zoom_level"], g["detail_zoom_delta"]
    cells = heatmap.assemble_cells(*_oracle_counters(lat, lon, d + 1, mz + d), users, keep, mz, d,
                                   project=_oracle_project)
    assert heatmap.cells_to_rows(cells) == g["rows"]
    # the vectorised (id, JSON) table holds the same rows
    t = heatmap.cells_to_table(cells).to_pydict()
    assert {i: json.loads(h) for i, h in zip(t["id"], t["heatmap"])} == g["rows"]
    assert len(t["id"]) == len(g["rows"])


@pytest.mark.parametrize("name", ROW_GOLDENS[:3] + [n for n in ROW_GOLDENS if "chain" in n])
def test_python_row_restatement_vs_reference(name):
    """oracle.build_heatmap_rows (literal re-projection chain) == build_heatmaps rows."""
    g = _load_rows(name)
    rows = g["input"]
    got = oracle.build_heatmap_rows([r["latitude"] for r in rows], [r["longitude"] for r in rows],
                                    [r["source"] for r in rows], [r["user_id"] for r in rows],
                                    g["max_zoom_level"], g["detail_zoom_delta"])
    assert got == g["rows"]


def test_config1_heatmap_digest():
    """1M uniform points, MAX_ZOOM_LEVEL=9 (detail zooms 14..6): every row of the
    reference's build_heatmaps, by SHA-256 of the canonical (id, bin, repr(count)) list."""
    g = json.load(open(os.path.join(GOLDEN, "config1_digest.json")))
    h = g["heatmap"]
    lat, lon = synth.uniform(g["n"], seed=0)
    users = ["x"] * g["n"]
    got = heatmap.assemble_rows(*_oracle_counters(lat, lon, h["delta"] + 1, h["max_zoom_level"] + h["delta"]),
                                users, None, h["max_zoom_level"], h["delta"])
    assert len(got) == h["rows"]
    items = sorted((k, t, repr(c)) for k, dd in got.items() for t, c in dd.items())
    assert len(items) == h["bins"]
    assert _digest(items) == h["sha256"]
    for k, v in h["sample_rows"].items():
        assert got[k] == v


def test_count_tiles_matches_count():
    """oracle.count_tiles (tile input) == oracle.count on the same points' tiles."""
    from heatmap_amd import synth

    lat, lon = synth.generate("hotspots", 20000, seed=8)
    r, c, st, _ = oracle.project(lat, lon, 14)
    assert (st == 0).all()
    a = oracle.count_tiles(r, c, 0, 14)
    b = oracle.count(lat, lon, None, 0, 14)
    for k in ("zoom", "row", "col", "count"):
        assert np.array_equal(a[k], b[k]), k


@pytest.mark.parametrize("mz", ["16", "9"])
def test_weighted_locations_vs_reference(mz):
    """build_heatmaps on locations at other zooms with float counts (and one
    level's heatmap_to_locations output) -- the product's host assembly with
    the oracle's projection == the reference's rows."""
    g = json.load(gzip.open(os.path.join(GOLDEN, "weighted_locations.json.gz"), "rt"))[mz]
    locs = g["locations"]
    zs, rows, cols = zip(*[(int(a), int(b), int(c)) for a, b, c in (l["tileId"].split("_") for l in locs)])
    cells = heatmap.weighted_location_cells(zs, rows, cols, [l["userId"] for l in locs],
                                            [l["count"] for l in locs], int(mz) + 5, 5, project=_oracle_project)
    assert heatmap.cells_to_rows(cells) == g["rows"]


def test_weighted_nondyadic_vs_reference():
    """build_heatmaps on locations with non-dyadic float counts (0.1, 1/3, ...):
    the reference's sums depend on Spark's summation order (here the in-memory
    RDD's), so equality is up to rounding: the same row ids and bins, every
    value within a few ulps (measured: 85% of the bins bit-exact, worst 5.3e-16
    relative).  Integer-valued counts below 2^53 are exact in any order and
    are compared bit for bit in test_weighted_locations_vs_reference."""
    g = json.load(gzip.open(os.path.join(GOLDEN, "weighted_nondyadic.json.gz"), "rt"))
    locs = g["locations"]
    zs, rows, cols = zip(*[(int(a), int(b), int(c)) for a, b, c in (l["tileId"].split("_") for l in locs)])
    d = heatmap.DETAIL_ZOOM_DELTA
    cells = heatmap.weighted_location_cells(zs, rows, cols, [l["userId"] for l in locs], [l["count"] for l in locs],
                                            g["max_zoom_level"] + d, d, project=_oracle_project)
    got, ref = heatmap.cells_to_rows(cells), g["rows"]
    assert set(got) == set(ref)
    for k, bins in ref.items():
        assert set(got[k]) == set(bins), k
        for b, v in bins.items():
            assert abs(got[k][b] - v) <= 4e-15 * abs(v), (k, b, got[k][b], v)
