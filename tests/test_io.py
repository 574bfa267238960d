"""Columnar ingestion + (id, heatmap-JSON) sink (heatmap_amd/io.py) against the
reference's build_heatmaps rows (tests/golden/heatmap_rows_*.json.gz).  The CPU
tests count with the oracle through heatmap.assemble_rows' counter hook; the GPU
test runs the product batch_main end to end."""
import gzip
import json
import os

import numpy as np
import pyarrow as pa
import pyarrow.parquet as pq
import pytest

from heatmap_amd import heatmap, io
from test_oracle import _oracle_counters, _oracle_project

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")
NAMES = sorted(f for f in os.listdir(GOLDEN) if f.startswith("heatmap_rows_"))


def _golden(name):
    with gzip.open(os.path.join(GOLDEN, name), "rt") as f:
        return json.load(f)


def _as_rows(table):
    d = table.to_pydict()
    return {i: json.loads(h) for i, h in zip(d["id"], d["heatmap"])}


@pytest.mark.parametrize("form", ["rows", "dict", "arrow", "parquet", "pandas"])
def test_loaders_agree(tmp_path, form):
    g = _golden("heatmap_rows_world_mixed_z14.json.gz")
    rows = g["input"]
    src = rows
    cols = {c: [r[c] for r in rows] for c in ("latitude", "longitude", "source", "user_id", "timestamp")}
    if form == "dict":
        src = cols
    elif form in ("arrow", "parquet"):
        src = pa.table(cols)
        if form == "parquet":
            p = str(tmp_path / "loc.parquet")
            pq.write_table(src, p)
            src = p
    elif form == "pandas":
        import pandas as pd

        src = pd.DataFrame(cols)
    lat, lon, keep, users = io.load_locations(src)
    assert lat.dtype == np.float64 and np.array_equal(lat, np.array(cols["latitude"]))
    assert np.array_equal(lon, np.array(cols["longitude"]))
    assert keep.tolist() == [int(s != "background") for s in cols["source"]]
    # Arrow / Parquet sources keep user_id as an Arrow column (dictionary-encoded from Parquet)
    assert (users.to_pylist() if hasattr(users, "to_pylist") else list(users)) == cols["user_id"]


@pytest.mark.parametrize("name", NAMES)
def test_table_matches_reference_rows(tmp_path, name):
    g = _golden(name)
    lat, lon, keep, users = io.load_locations(g["input"])
    mz, d = g["max_zoom_level"], g["detail_zoom_delta"]
    rows = heatmap.assemble_rows(*_oracle_counters(lat, lon, d + 1, mz + d), users, keep, mz, d,
                                 project=_oracle_project)
    t = io.rows_to_table(rows)
    assert t.column_names == ["id", "heatmap"]
    p = str(tmp_path / "heatmaps.parquet")
    pq.write_table(t, p)
    assert _as_rows(pq.read_table(p)) == g["rows"]


@pytest.mark.gpu
@pytest.mark.parametrize("name", NAMES)
def test_batch_main_on_device(gpu, tmp_path, name):
    """Every reference row golden (incl. edges_z14: kept points outside
    [0, 2^z)^2; seattle_mixed_z21: the reference's own constants; chain_*:
    tiles near the poles and at |lon| > 11520, outside the shift windows),
    end to end on the device: columnar load, two device passes, vectorised
    rows."""
    g = _golden(name)
    p = str(tmp_path / "out.parquet")
    t = io.batch_main(g["input"], sink=p, max_zoom_level=g["max_zoom_level"], delta=g["detail_zoom_delta"])
    assert _as_rows(t) == g["rows"]
    assert _as_rows(pq.read_table(p)) == g["rows"]


def test_group_plan_reads_user_ids_of_kept_rows_only():
    """Background rows are dropped before their user id is read (heatmap.py:28-35):
    a null user id there is valid input; on a kept row it raises as None[:1]."""
    users = ["u1", None, "x9", "rt-4", "a|b", "all", "u1", "route"]
    keep = np.array([1, 0, 1, 1, 0, 1, 1, 1], bool)
    p = heatmap.group_plan(users, keep)
    assert p.labels == ["all", "u1", "route"]
    assert p.grouped.tolist() == [True, False, False, True, False, True, True, True]
    assert p.gid[p.grouped].tolist() == [1, 2, 0, 1, 2]
    with pytest.raises(TypeError):
        heatmap.group_plan(users, np.ones(8, bool))
    keep[1] = False
    keep[4] = True
    with pytest.raises(ValueError, match="separator"):
        heatmap.group_plan(users, keep)


def test_null_user_on_background_row(tmp_path):
    """io.batch_main input with a null user_id on a background row (CPU half:
    loading; the GPU test runs the rows)."""
    cols = {"latitude": [47.6, 47.61], "longitude": [-122.3, -122.31], "source": ["gps", "background"],
            "user_id": ["u1", None], "timestamp": [0, 1]}
    lat, lon, keep, users = io.load_locations(pa.table(cols))
    assert keep.tolist() == [1, 0] and users.to_pylist()[1] is None
    p = heatmap.group_plan(users, keep)
    assert p.labels == ["all", "u1"] and p.grouped.tolist() == [True, False]
    with pytest.raises(TypeError):   # the same null on a kept row: None[:1]
        heatmap.group_plan(users, np.ones(2, bool))


def test_chain_window_table_matches_reference_chain():
    """heatmap_amd/chain_window.py (tools/chain_window.c) against the oracle's
    literal re-projection of tile centres (tile.py:33-54, heatmap.py:60-61,89):
    agreement at the window's edges, disagreement just outside its row edges."""
    from oracle import oracle
    from heatmap_amd import chain_window as cw

    for z in (6, 14, 21):
        for j in sorted({0, 1, 5, min(z, 9)}):
            lo, hi = cw.ROWS[z][j]
            for r in (lo, lo + 1, hi - 1, 0, (1 << z) - 1):
                assert oracle._recentre(z, r, 0, z - j)[0] == r >> j, (z, j, r)
            for r in (lo - 1, hi):
                try:
                    assert oracle._recentre(z, r, 0, z - j)[0] != r >> j, (z, j, r)
                except ValueError:
                    pass   # the chain raises there (math domain error)
            clo, chi = cw.COLS[z][j]
            for c in (clo, chi - 1, -1, 1 << z):
                assert oracle._recentre(z, 0, c, z - j)[1] == c >> j, (z, j, c)


@pytest.mark.gpu
@pytest.mark.parametrize("mz", ["16", "9"])
def test_build_heatmaps_weighted_locations_on_device(gpu, mz, monkeypatch):
    """build_heatmaps(locations) with tiles at other zooms and float counts
    (the reference accepts its own heatmap_to_locations output fed back in):
    rows equal to the reference's (tests/golden/weighted_locations.json.gz)."""
    import gzip
    import json

    g = json.load(gzip.open(os.path.join(GOLDEN, "weighted_locations.json.gz"), "rt"))[mz]
    monkeypatch.setattr(heatmap, "MAX_ZOOM_LEVEL", int(mz))
    assert dict(heatmap.build_heatmaps(g["locations"])) == g["rows"]
