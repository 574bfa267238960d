"""Drop-in for reference heatmap.py's hot path (dataframe_loader + build_heatmaps).

Same names, constants, key layout and output rows as reference
heatmap.py:16-129:

  row id   "<group>|alltime|<z-DELTA>_<row>_<col>"      (heatmap.py:55,85-90)
  heatmap  {"<z>_<row>_<col>": float count}             (heatmap.py:120-126)
  groups   'all' for every kept location, plus the user id unless it starts
           with 'x', 'rt-*' folded into 'route'          (heatmap.py:64-70)
  zooms    detail zooms MAX_ZOOM_LEVEL+DELTA down to DELTA+1 (heatmap.py:109)

Counting runs on the device (hm_count: projection + count pyramid, one launch
per user group).  The reference re-emits every level's 'all' bins under user
id 'all', which doubles 'all' once per level; with n = kept points, a = kept
points whose user id is literally 'all', U = kept points of every other user
group, the 'all' count of a cell k levels below the detail zoom is
    2^k (n + a) + (2^k - 1) U
(closed form verified against the reference); the
adapter below applies it to the device counts.  Counts are integers on the
device and exact as floats while below 2^53.

build_heatmaps(locations) keeps the reference's RDD-shaped interface for
locations produced by dataframe_loader (all with count 1.0 and tileId at the
detail zoom); build_heatmaps_columnar is the fast entry point.
"""
from __future__ import annotations

import json
from collections import defaultdict

import numpy as np

from . import device
from .tile import Tile

DETAIL_ZOOM_DELTA = 5
MAX_ZOOM_LEVEL = 16
KEY_SEPERATOR = "|"
KEY_FIELD = 0
VALUE_FIELD = 1


# --------------------------------------------------------------------------
# per-record functions (reference signatures)
# --------------------------------------------------------------------------

def dataframe_loader(row):
    """heatmap.py:25-36: project at the detail zoom, THEN drop background."""
    tileId = Tile.tile_id_from_lat_long(row["latitude"], row["longitude"], MAX_ZOOM_LEVEL + DETAIL_ZOOM_DELTA)
    if row["source"] == "background":
        return []
    return [{"tileId": tileId, "timestamp": row["timestamp"], "userId": row["user_id"], "count": 1.0}]


def build_timespan_label(timespanType, localDate):
    """heatmap.py:38-52 (not used by the pipeline: timespan is 'alltime')."""
    month = "%02d" % localDate.month
    day = "%02d" % localDate.day
    if timespanType == "alltime":
        return "alltime"
    if timespanType == "year":
        return str(localDate.year)
    if timespanType == "month":
        return str(localDate.year) + "-" + month
    if timespanType == "day":
        return str(localDate.year) + "-" + month + "-" + day
    return None


def build_tile_composite_key(userId, tileId, timespanLabel):
    """heatmap.py:54-55."""
    return userId + KEY_SEPERATOR + timespanLabel + KEY_SEPERATOR + tileId


def user_groups(user_id):
    """Groups a location contributes to at the detail zoom (heatmap.py:64-70)."""
    groups = ["all"]
    if not user_id[:1] == "x":
        groups.append("route" if user_id[:3] == "rt-" else user_id)
    return groups


def list_to_dict(heatmapList):
    """heatmap.py:120-126."""
    out = {}
    for entry in heatmapList:
        out[entry["tileId"]] = entry["count"]
    return out


def heatmap_to_json(heatmap):
    """heatmap.py:128-129."""
    return json.dumps(heatmap)


def heatmap_to_locations(bucket):
    """heatmap.py:92-105."""
    parts = bucket[KEY_FIELD].split(KEY_SEPERATOR)
    return [{"userId": parts[0], "count": c, "tileId": t, "timespan": parts[1]}
            for t, c in bucket[VALUE_FIELD].items()]


# --------------------------------------------------------------------------
# columnar fast path
# --------------------------------------------------------------------------

def _group_plan(user_ids, keep):
    """Per-point group masks: dict label -> uint8 keep mask, plus n/a/U masks."""
    n = len(user_ids)
    keep = np.ones(n, dtype=bool) if keep is None else np.asarray(keep).astype(bool)
    labels = np.empty(n, dtype=object)
    for i, u in enumerate(user_ids):
        if u is None:
            raise TypeError("'NoneType' object is not subscriptable")   # None[:1], heatmap.py:64
        if KEY_SEPERATOR in u:
            raise ValueError("user id %r contains the key separator %r (heatmap.py:80-84 would mis-split it)"
                             % (u, KEY_SEPERATOR))
        labels[i] = None if u[:1] == "x" else ("route" if u[:3] == "rt-" else u)
    masks = {}
    for g in sorted({l for l in labels if l is not None}):
        masks[g] = keep & (labels == g)
    lit_all = masks.pop("all", np.zeros(n, dtype=bool))
    others = np.zeros(n, dtype=bool)
    for m in masks.values():
        others |= m
    return keep, lit_all, others, masks


def _device_counter(lat, lon, zmin, zmax, tiles):
    """counter(mask) -> {zoom: {(row, col): count}} on the device (hm_count)."""

    def counter(mask):
        c = device.count(lat, lon, None if mask is None else mask.astype(np.uint8), zmin, zmax, tiles=tiles)
        out = defaultdict(dict)
        for z, r, cc, k in zip(c.zoom.tolist(), c.row.tolist(), c.col.tolist(), c.count.tolist()):
            out[z][(r, cc)] = k
        return out

    return counter


def assemble_rows(counter, user_id, keep=None, max_zoom_level=None, delta=None):
    """Heatmap rows of build_heatmaps from per-group cell counts.

    counter(mask) returns {zoom: {(row, col): count}} of the points selected by
    `mask` (None = all points) for zooms delta+1 .. max_zoom_level+delta; it is
    the only place points are touched (the device in the product, the oracle
    in the CPU tests).  Row layout: heatmap.py:55,85-90,120-126; 'all'
    weighting: heatmap.py:64-70 applied level by level (module docstring)."""
    mz = MAX_ZOOM_LEVEL if max_zoom_level is None else max_zoom_level
    d = DETAIL_ZOOM_DELTA if delta is None else delta
    zmax = mz + d
    keep, lit_all, others, groups = _group_plan(user_id, keep)
    # every point is projected (and may raise) even when not kept, as
    # dataframe_loader does (heatmap.py:27-29): the counter checks all points
    n_cells = counter(keep)
    a_cells = counter(lit_all) if lit_all.any() else {}
    u_cells = counter(others) if others.any() else {}
    rows = {}

    def put(group, z, r, c, v):
        # row tile = re-projected centre at z - d == arithmetic shift (SURVEY a-4)
        rid = "%s|alltime|%d_%d_%d" % (group, z - d, r >> d, c >> d)
        rows.setdefault(rid, {})["%d_%d_%d" % (z, r, c)] = float(v)

    for z in range(zmax, d, -1):
        k = zmax - z
        nz = n_cells.get(z, {})
        az = a_cells.get(z, {})
        uz = u_cells.get(z, {})
        for (r, c), cnt in nz.items():
            put("all", z, r, c, (cnt + az.get((r, c), 0)) * (1 << k) + ((1 << k) - 1) * uz.get((r, c), 0))
    for g, m in groups.items():
        gc = counter(m)
        for z in range(zmax, d, -1):
            for (r, c), cnt in gc.get(z, {}).items():
                put(g, z, r, c, cnt)
    return rows


def build_heatmaps_columnar(lat, lon, user_id, keep=None, max_zoom_level=None, delta=None, tiles=False):
    """Rows {row_id: {bin_id: float}} of build_heatmaps for columnar input.

    lat/lon: float64 arrays (or, with tiles=True, int64 row/col at the detail
    zoom); user_id: sequence of str; keep: mask of non-background rows."""
    mz = MAX_ZOOM_LEVEL if max_zoom_level is None else max_zoom_level
    d = DETAIL_ZOOM_DELTA if delta is None else delta
    counter = _device_counter(lat, lon, d + 1, mz + d, tiles)
    return assemble_rows(counter, user_id, keep, mz, d)


def build_heatmaps(locations):
    """heatmap.py:107-118 on an iterable (or RDD-like .collect()) of locations
    produced by dataframe_loader.  Returns [(row_id, heatmap_dict)]."""
    if hasattr(locations, "collect"):
        locations = locations.collect()
    zmax = MAX_ZOOM_LEVEL + DETAIL_ZOOM_DELTA
    rows, cols, users = [], [], []
    for loc in locations:
        if loc["count"] != 1.0:
            raise NotImplementedError("device build_heatmaps counts locations of weight 1.0 "
                                      "(dataframe_loader output); got %r" % (loc["count"],))
        z, r, c = (int(x) for x in loc["tileId"].split("_"))
        if z != zmax:
            raise NotImplementedError("locations must carry zoom-%d tile ids (dataframe_loader output)" % zmax)
        rows.append(r)
        cols.append(c)
        users.append(loc["userId"])
    out = build_heatmaps_columnar(np.array(rows, dtype=np.int64), np.array(cols, dtype=np.int64), users,
                                  tiles=True)
    return list(out.items())
