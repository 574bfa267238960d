"""GPU: BASELINE config 1 pinned to the reference at its stated size.

1M uniform points (synth.uniform, seed 0, bit-identical generator) through the
device, checked against tests/golden/config1_digest.json, which
make_golden.py wrote by running the reference itself: every zoom-0..21 cell
count (Counter(Tile.tile_id_from_lat_long) per zoom) and every row of
build_heatmaps at MAX_ZOOM_LEVEL = 9 (heatmap.py:107-118)."""
import hashlib
import json
import os

import numpy as np
import pytest

from heatmap_amd import device, heatmap, synth

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")
pytestmark = pytest.mark.gpu


def _digest(items):
    h = hashlib.sha256()
    for it in items:
        h.update((",".join(str(x) for x in it) + "\n").encode())
    return h.hexdigest()


@pytest.fixture(scope="module")
def config1():
    g = json.load(open(os.path.join(GOLDEN, "config1_digest.json")))
    lat, lon = synth.uniform(g["n"], seed=0)
    return g, lat, lon


def test_config1_zoom_counts_on_device(gpu, config1):
    g, lat, lon = config1
    zs = sorted(int(z) for z in g["zoom_counts"])
    got = device.count(lat, lon, None, min(zs), max(zs)).sorted()
    for z in zs:
        m = got.zoom == z
        cells = list(zip(got.row[m].tolist(), got.col[m].tolist(), got.count[m].tolist()))
        e = g["zoom_counts"][str(z)]
        assert len(cells) == e["cells"] and sum(c for _, _, c in cells) == e["total"], z
        assert _digest(cells) == e["sha256"], z


def test_config1_heatmap_rows_on_device(gpu, config1):
    g, lat, lon = config1
    h = g["heatmap"]
    users = np.full(g["n"], "x", dtype=object)
    cells = heatmap.heatmap_cells(lat, lon, users, None, h["max_zoom_level"], h["delta"])
    rows = heatmap.cells_to_rows(cells)
    assert len(rows) == h["rows"]
    items = sorted((k, t, repr(c)) for k, dd in rows.items() for t, c in dd.items())
    assert len(items) == h["bins"]
    assert _digest(items) == h["sha256"]
    for k, v in h["sample_rows"].items():
        assert rows[k] == v
    t = heatmap.cells_to_table(cells)
    assert t.num_rows == h["rows"]
