"""CPU oracle for the heatmap hot path -- TEST INFRASTRUCTURE ONLY.

Imported only by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
leg, as the checker.  The product (heatmap_amd/) never imports this module.

Two layers, both pinned against fixtures produced by running the reference
itself (tests/golden/make_golden.py):

* ``project`` / ``count``: ctypes wrappers over ``hm_oracle.c``, the literal
  glibc restatement of reference tile.py:15-21 and of the per-zoom
  reduceByKey pyramid (heatmap.py:107-111).  Pinned by
  tests/golden/projection_kat.npz, zoom_counts_hotspots.json and
  config1_digest.json.
* ``build_heatmap_rows``: a pure-Python restatement of the reference's row
  assembly (heatmap.py:25-126) -- group keying with the 'x' / 'rt-' rules
  (:64-70), the zoom-by-zoom re-projection of tile centres (:60-61, :89 via
  tile.py:23-54), the (z-delta) heatmap-row grouping (:85-90, :120-126) and the
  feedback of each level's bins as the next level's locations (:92-105, :117).
  Pinned by tests/golden/heatmap_rows_*.json.gz.
"""
from __future__ import annotations

import ctypes
import math
import os
import subprocess
from collections import defaultdict

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None

OK, E_NAN, E_DOMAIN, E_INF, E_RANGE = 0, 1, 2, 3, 8


def lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(HERE, "_build", "libhm_oracle.so")
        if not os.path.exists(path):
            subprocess.check_call(["make", "-s", "-C", HERE])
        L = ctypes.CDLL(path)
        P = ctypes.POINTER
        L.hmo_project.argtypes = [P(ctypes.c_double), P(ctypes.c_double), ctypes.c_int64, ctypes.c_int,
                                  P(ctypes.c_int64), P(ctypes.c_int64), P(ctypes.c_uint8), ctypes.c_int]
        L.hmo_project.restype = ctypes.c_int
        L.hmo_count.argtypes = [P(ctypes.c_double), P(ctypes.c_double), P(ctypes.c_uint8), ctypes.c_int64,
                                ctypes.c_int, ctypes.c_int, ctypes.c_int, P(ctypes.c_int64), P(ctypes.c_int64),
                                P(P(ctypes.c_int32)), P(P(ctypes.c_int64)), P(P(ctypes.c_int64)),
                                P(P(ctypes.c_int64)), P(ctypes.c_int)]
        L.hmo_count.restype = ctypes.c_int
        L.hmo_count_tiles.argtypes = [P(ctypes.c_int64), P(ctypes.c_int64), P(ctypes.c_uint8), ctypes.c_int64,
                                      ctypes.c_int, ctypes.c_int, P(ctypes.c_int64), P(P(ctypes.c_int32)),
                                      P(P(ctypes.c_int64)), P(P(ctypes.c_int64)), P(P(ctypes.c_int64))]
        L.hmo_count_tiles.restype = ctypes.c_int
        L.hmo_free.argtypes = [ctypes.c_void_p]
        L.hmo_row.argtypes = [ctypes.c_double, ctypes.c_int, P(ctypes.c_int64)]
        L.hmo_col.argtypes = [ctypes.c_double, ctypes.c_int, P(ctypes.c_int64)]
        _LIB = L
    return _LIB


def _p(a, t):
    return a.ctypes.data_as(ctypes.POINTER(t))


def project(lat, lon, zoom, threads=0):
    """Vectorised Tile.row_from_latitude/column_from_longitude (tile.py:15-21).
    Returns (row int64, col int64, status uint8, threads_used)."""
    lat = np.ascontiguousarray(lat, dtype=np.float64)
    lon = np.ascontiguousarray(lon, dtype=np.float64)
    n = lat.size
    row = np.zeros(n, np.int64)
    col = np.zeros(n, np.int64)
    st = np.zeros(n, np.uint8)
    used = lib().hmo_project(_p(lat, ctypes.c_double), _p(lon, ctypes.c_double), n, int(zoom),
                             _p(row, ctypes.c_int64), _p(col, ctypes.c_int64), _p(st, ctypes.c_uint8), threads)
    return row, col, st, used


def count(lat, lon, keep=None, zmin=0, zmax=18, threads=0):
    """Per-zoom cell counts, sorted by (zoom, row, col).

    Returns dict(status, err_index, zoom, row, col, count, threads)."""
    lat = np.ascontiguousarray(lat, dtype=np.float64)
    lon = np.ascontiguousarray(lon, dtype=np.float64)
    n = lat.size
    kp = None
    if keep is not None:
        keep = np.ascontiguousarray(keep, dtype=np.uint8)
        kp = _p(keep, ctypes.c_uint8)
    err = ctypes.c_int64(-1)
    nout = ctypes.c_int64(0)
    zo = ctypes.POINTER(ctypes.c_int32)()
    ro = ctypes.POINTER(ctypes.c_int64)()
    co = ctypes.POINTER(ctypes.c_int64)()
    no = ctypes.POINTER(ctypes.c_int64)()
    used = ctypes.c_int(0)
    st = lib().hmo_count(_p(lat, ctypes.c_double), _p(lon, ctypes.c_double), kp, n, zmin, zmax, threads,
                         ctypes.byref(err), ctypes.byref(nout), ctypes.byref(zo), ctypes.byref(ro),
                         ctypes.byref(co), ctypes.byref(no), ctypes.byref(used))
    out = {"status": st, "err_index": err.value, "threads": used.value}
    if st == OK:
        out.update(_collect(nout.value, zo, ro, co, no))
    return out


def _collect(m, zo, ro, co, no):
    out = {}
    out["zoom"] = np.ctypeslib.as_array(zo, (max(m, 1),))[:m].copy()
    out["row"] = np.ctypeslib.as_array(ro, (max(m, 1),))[:m].copy()
    out["col"] = np.ctypeslib.as_array(co, (max(m, 1),))[:m].copy()
    out["count"] = np.ctypeslib.as_array(no, (max(m, 1),))[:m].copy()
    for p in (zo, ro, co, no):
        lib().hmo_free(ctypes.cast(p, ctypes.c_void_p))
    z = out["zoom"]
    if m == 0:
        return out
    # zooms come from zmax down, each (row, col)-sorted by the C code: put
    # the zoom blocks in ascending order; re-sort only if a block is not sorted
    cuts = np.flatnonzero(z[1:] != z[:-1]) + 1
    blocks = np.split(np.arange(m), cuts)[::-1]
    order = np.concatenate(blocks)
    res = {k: v[order] for k, v in out.items()}
    r, c, zz = res["row"], res["col"], res["zoom"]
    same = zz[1:] == zz[:-1]
    if np.any(same & ((r[1:] < r[:-1]) | ((r[1:] == r[:-1]) & (c[1:] <= c[:-1])))):
        o = np.lexsort((c, r, zz))
        res = {k: v[o] for k, v in res.items()}
    return res


def count_tiles(rows, cols, zmin, zmax, keep=None):
    """Per-zoom cell counts of zoom-zmax tiles (the hm_count_tiles contract),
    sorted by (zoom, row, col): the per-zoom reduceByKey of heatmap.py:109-111,
    with every coarser tile the arithmetic right shift of the zoom-zmax one
    (SURVEY a-4; any int64 tile, negative or past 2^zmax)."""
    rows = np.ascontiguousarray(rows, dtype=np.int64)
    cols = np.ascontiguousarray(cols, dtype=np.int64)
    kp = None
    if keep is not None:
        keep = np.ascontiguousarray(keep, dtype=np.uint8)
        kp = _p(keep, ctypes.c_uint8)
    nout = ctypes.c_int64(0)
    zo = ctypes.POINTER(ctypes.c_int32)()
    ro = ctypes.POINTER(ctypes.c_int64)()
    co = ctypes.POINTER(ctypes.c_int64)()
    no = ctypes.POINTER(ctypes.c_int64)()
    st = lib().hmo_count_tiles(_p(rows, ctypes.c_int64), _p(cols, ctypes.c_int64), kp, rows.size, zmin, zmax,
                               ctypes.byref(nout), ctypes.byref(zo), ctypes.byref(ro), ctypes.byref(co),
                               ctypes.byref(no))
    assert st == OK
    return _collect(nout.value, zo, ro, co, no)


# --------------------------------------------------------------------------
# Pure-Python restatement of the reference row assembly (heatmap.py:25-126)
# --------------------------------------------------------------------------

def _row_of(lat, z):
    r = ctypes.c_int64(0)
    st = lib().hmo_row(float(lat), int(z), ctypes.byref(r))
    if st == E_NAN:
        raise ValueError("cannot convert float NaN to integer")
    if st == E_DOMAIN:
        raise ValueError("math domain error")
    if st == E_INF:
        raise OverflowError("cannot convert float infinity to integer")
    return r.value


def _col_of(lon, z):
    # Python ints are unbounded: restate with math.floor directly
    return math.floor((lon + 180.0) / 360.0 * (2 ** z))


def _north_lat(row, z):
    # inverse projection, tile.py:23-26
    n = math.pi - 2.0 * math.pi * row / (2 ** z)
    return 180.0 / math.pi * math.atan(0.5 * (math.exp(n) - math.exp(-n)))


def _west_lon(col, z):
    return float(col) / (2 ** z) * 360.0 - 180.0   # tile.py:28-30


def _recentre(z, row, col, z_to):
    """Tile id of the re-projected centre of tile (z,row,col) at zoom z_to
    (tile.py:33-54 then tile.py:9-13, as heatmap.py:60-61 and :89 use it)."""
    clat = (_north_lat(row, z) + _north_lat(row + 1, z)) / 2.0
    clon = (_west_lon(col + 1, z) + _west_lon(col, z)) / 2.0
    return _row_of(clat, z_to), _col_of(clon, z_to)


def group_labels(user_id):
    """User groups a location contributes to (heatmap.py:64-70)."""
    groups = ["all"]
    if not user_id[:1] == "x":
        groups.append("route" if user_id[:3] == "rt-" else user_id)
    return groups


def build_heatmap_rows(lat, lon, source, user_id, max_zoom_level=16, delta=5):
    """{row_id: {bin_tile_id: float count}} exactly as build_heatmaps emits them."""
    zmax = max_zoom_level + delta
    # dataframe_loader: project first, then drop background (heatmap.py:27-29)
    locs = []
    for la, lo, src, uid in zip(lat, lon, source, user_id):
        r, c = _row_of(la, zmax), _col_of(lo, zmax)
        if src == "background":
            continue
        locs.append((uid, zmax, r, c, 1.0))
    rows = {}
    cache = {}
    for zoom in range(zmax, delta, -1):
        # shuffle 1: (group|alltime|tile_z) -> sum (heatmap.py:110-111)
        acc = defaultdict(float)
        order = []
        for uid, z0, r, c, cnt in locs:
            key = (z0, r, c, zoom)
            if key not in cache:
                cache[key] = _recentre(z0, r, c, zoom)
            tr, tc = cache[key]
            for g in group_labels(uid):
                k = (g, tr, tc)
                if k not in acc:
                    order.append(k)
                acc[k] += cnt
        # shuffle 2: regroup bins under the (zoom - delta) tile (heatmap.py:79-90,112)
        level = {}
        for (g, tr, tc) in order:
            ck = (zoom, tr, tc, zoom - delta)
            if ck not in cache:
                cache[ck] = _recentre(zoom, tr, tc, zoom - delta)
            pr, pc = cache[ck]
            rid = "%s|alltime|%d_%d_%d" % (g, zoom - delta, pr, pc)
            level.setdefault(rid, {})["%d_%d_%d" % (zoom, tr, tc)] = acc[(g, tr, tc)]
        for rid, d in level.items():
            rows[rid] = d
        # this level's bins become the next level's locations (heatmap.py:92-105,117)
        locs = []
        for rid, d in level.items():
            g = rid.split("|")[0]
            for tid, cnt in d.items():
                z, r, c = (int(p) for p in tid.split("_"))
                locs.append((g, z, r, c, cnt))
    return rows
