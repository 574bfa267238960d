"""Tile utility API (reference tile.py:23-98)
against tests/golden/tile_utils.json, which make_golden.py --only utils wrote by
running the reference's Tile."""
import json
import os

import pytest

from heatmap_amd.tile import Tile

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


@pytest.fixture(scope="module")
def fx():
    with open(os.path.join(GOLDEN, "tile_utils.json")) as f:
        return json.load(f)


def test_latitude_from_row_bit_exact(fx):
    for row, zoom, exp in fx["latitude_from_row"]:
        assert repr(Tile.latitude_from_row(row, zoom)) == exp, (row, zoom)


def test_tile_from_tile_id_fields(fx):
    for case in fx["tiles"]:
        t = Tile.tile_from_tile_id(case["id"])
        z, r, c = (int(v) for v in case["id"].split("_"))
        assert (t.tile_id, t.zoom, t.row, t.column) == (case["id"], z, r, c)
        for k, v in case["fields"].items():
            assert repr(getattr(t, k)) == v, (case["id"], k)


def test_malformed_ids(fx):
    for tid in fx["malformed"]:
        assert Tile.tile_from_tile_id(tid) is None
        assert Tile.decode_tile_id(tid) is None


@pytest.mark.gpu
def test_hierarchy_on_device(gpu, fx):
    for case in fx["tiles"]:
        t = Tile.tile_from_tile_id(case["id"])
        assert t.children() == case["children"], case["id"]
        assert Tile.tile_ids_for_all_zoom_levels(case["id"]) == case["all_zooms"], case["id"]
        if case["parent_id"] is not None:
            assert t.parent_id() == case["parent_id"], case["id"]
            assert t.parent().tile_id == case["parent_id"]
