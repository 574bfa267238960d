"""CPU: the per-record Tile calls (reference tile.py:9-21) through
hm_project_scalar -- the kernels' csrc/hm_project.h compiled for the host --
against the reference's own known answers (tests/golden/, made by
tests/golden/make_golden.py from reference tile.py), and their cost per call.

The batched device form (hm_project) is checked against the same KATs on the
GPU (tests/test_gpu_smoke.py::test_project_kat); together they pin the two
forms to each other."""
import json
import math
import os
import time

import numpy as np
import pytest

from heatmap_amd import _lib
from heatmap_amd.tile import Tile, _scalar

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def test_scalar_projection_kat():
    """Every projection KAT: row, column and the row-first error kind; columns
    beyond int64 as the reference's unbounded ints."""
    d = dict(np.load(os.path.join(GOLDEN, "projection_kat.npz")))   # (an NpzFile re-reads per access)
    big = set(map(int, json.load(open(os.path.join(GOLDEN, "projection_kat_bigcols.json")))))
    bad = []
    for i in range(len(d["lat"])):
        la, lo, z = float(d["lat"][i]), float(d["lon"][i]), int(d["zoom"][i])
        st, r, c = _scalar(la, lo, z)
        exp = int(d["row_err"][i]) or int(d["col_err"][i])
        if i in big and st == _lib.HM_OK:
            # the reference's column: floor of the literal expression, an int
            ok = exp == _lib.HM_E_RANGE and r == int(d["row"][i]) and c == math.floor((lo + 180.0) / 360.0 * (2 ** z))
        else:
            ok = st == exp and (exp != 0 or (r == int(d["row"][i]) and c == int(d["col"][i])))
        if not ok:
            bad.append((i, la, lo, z, st, r, c))
    assert not bad, bad[:5]
    assert len(d["lat"]) > 30000


def test_scalar_tile_ids_and_exceptions():
    """Tile.tile_id_from_lat_long strings and exceptions (tile.py:9-13)."""
    msgs = {ValueError: "ValueError", OverflowError: "OverflowError"}
    for la, lo, z, want in json.load(open(os.path.join(GOLDEN, "tile_ids.json"))):
        try:
            got = Tile.tile_id_from_lat_long(float(la), float(lo), z)
        except (ValueError, OverflowError) as e:
            got = "%s: %s" % (msgs[type(e)], e)
        assert got == want, (la, lo, z)


def test_scalar_row_and_column_forms():
    assert Tile.row_from_latitude(47.6062, 21) == int(Tile.tile_id_from_lat_long(47.6062, -122.3321, 21).split("_")[1])
    assert Tile.column_from_longitude(-122.3321, 21) == int(Tile.tile_id_from_lat_long(47.6, -122.3321, 21).split("_")[2])
    with pytest.raises(ValueError, match="^math domain error$"):
        Tile.row_from_latitude(-90, 5)
    with pytest.raises(OverflowError):
        Tile.column_from_longitude(float("inf"), 5)
    assert Tile.column_from_longitude(1e300, 0) == math.floor((1e300 + 180.0) / 360.0)
    assert Tile.tile_id_from_lat_long(0.0, 0.0, -1) == "-1_0_0"        # parent_id of a zoom-0 tile


def test_scalar_call_cost():
    """A per-record tile_id_from_lat_long costs about a microsecond (the
    reference's CPython math: ~2.7 us with its string building)."""
    n = 20_000
    Tile.tile_id_from_lat_long(1.0, 2.0, 3)
    best = float("inf")
    for _ in range(5):          # best of 5: robust to a loaded host (pytest -n)
        t = time.perf_counter()
        for i in range(n):
            Tile.tile_id_from_lat_long(47.6 + i * 1e-7, -122.3, 21)
        best = min(best, time.perf_counter() - t)
    us = best / n * 1e6
    print("tile_id_from_lat_long: %.2f us per call" % us)
    assert us < 5.0   # ~1.3 us alone; headroom for a host shared with other jobs


def test_scalar_zoom_forms():
    """zoom as the reference's `2 ** zoom` takes it (tile.py:9-21): an integral
    float projects like the int and keeps str(zoom) in the id; numpy integers
    are accepted; a non-integral, huge or out-of-range zoom is a ValueError,
    a non-number a TypeError (as int(zoom) would raise)."""
    lat, lon = 47.6062, -122.3321
    r, c = Tile.row_from_latitude(lat, 12), Tile.column_from_longitude(lon, 12)
    assert Tile.row_from_latitude(lat, 12.0) == r and Tile.column_from_longitude(lon, 12.0) == c
    assert Tile.tile_id_from_lat_long(lat, lon, 12.0) == "12.0_%d_%d" % (r, c)
    assert Tile.tile_id_from_lat_long(lat, lon, np.int64(12)) == "12_%d_%d" % (r, c)
    for z in (12.5, 10 ** 30, -(10 ** 30), 31, float("inf"), float("nan")):
        with pytest.raises(ValueError):
            Tile.row_from_latitude(lat, z)
    with pytest.raises(TypeError):
        Tile.row_from_latitude(lat, "12")
