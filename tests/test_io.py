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
from test_oracle import _oracle_counter

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")
NAMES = ["heatmap_rows_world_mixed_z14.json.gz", "heatmap_rows_hotspots_alluser_z18.json.gz"]


def _golden(name):
    with gzip.open(os.path.join(GOLDEN, name), "rt") as f:
        return json.load(f)


def _as_rows(table):
    d = table.to_pydict()
    return {i: json.loads(h) for i, h in zip(d["id"], d["heatmap"])}


@pytest.mark.parametrize("form", ["rows", "dict", "arrow", "parquet", "pandas"])
def test_loaders_agree(tmp_path, form):
    g = _golden(NAMES[0])
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
    assert users == cols["user_id"]


@pytest.mark.parametrize("name", NAMES)
def test_table_matches_reference_rows(tmp_path, name):
    g = _golden(name)
    lat, lon, keep, users = io.load_locations(g["input"])
    mz, d = g["max_zoom_level"], g["detail_zoom_delta"]
    rows = heatmap.assemble_rows(_oracle_counter(lat, lon, d + 1, mz + d), users, keep, mz, d)
    t = io.rows_to_table(rows)
    assert t.column_names == ["id", "heatmap"]
    p = str(tmp_path / "heatmaps.parquet")
    pq.write_table(t, p)
    assert _as_rows(pq.read_table(p)) == g["rows"]


@pytest.mark.gpu
@pytest.mark.parametrize("name", NAMES)
def test_batch_main_on_device(gpu, tmp_path, name):
    g = _golden(name)
    p = str(tmp_path / "out.parquet")
    t = io.batch_main(g["input"], sink=p, max_zoom_level=g["max_zoom_level"], delta=g["detail_zoom_delta"])
    assert _as_rows(t) == g["rows"]
    assert _as_rows(pq.read_table(p)) == g["rows"]
