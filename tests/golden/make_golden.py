#!/usr/bin/env python3
"""Generate the golden fixtures under tests/golden/ by running the REFERENCE.

Run in the build container only (it needs /root/reference, which does not
exist on the GPU box):

    python tests/golden/make_golden.py            # everything (~4 min)
    python tests/golden/make_golden.py --quick    # skip the 1M-point digest

What it calls (all read-only, no bytecode written into the reference dir):
  * tile.py          Tile.row_from_latitude / column_from_longitude /
                     tile_id_from_lat_long (tile.py:9-21) for projection
                     known-answer vectors, including boundary-adjacent
                     double pairs found by bisection;
  * heatmap.py       dataframe_loader + build_heatmaps (heatmap.py:25-126)
                     through an in-memory stand-in for the four Spark RDD
                     operations it uses.  pyspark and
                     cassandra are replaced by empty module stubs; they are only
                     referenced by the out-of-scope I/O functions.

Outputs (data only -- inputs and the reference's outputs):
  projection_kat.npz        lat, lon, zoom -> row/col or error kind
  tile_ids.json             a few hundred formatted "z_r_c" strings
  heatmap_rows_*.json.gz    build_heatmaps rows for small mixed datasets
  config1_digest.json       1M uniform points: per-zoom counts / digests
  zoom_counts_hotspots.json 100k hotspot points: per-zoom cell digests z0..21
  weighted_locations.json.gz, weighted_nondyadic.json.gz
                            build_heatmaps on location lists with float counts
"""
import argparse
import collections
import gzip
import hashlib
import json
import math
import os
import sys
import time
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"
sys.dont_write_bytecode = True
sys.path.insert(0, REPO)

from heatmap_amd import synth  # noqa: E402

# error kinds shared with include/heatmap_amd.h
OK, E_NAN, E_DOMAIN, E_INF = 0, 1, 2, 3


def load_reference():
    for name, attrs in (("pyspark", ("SparkConf", "SparkContext")),
                        ("pyspark.sql", ("SQLContext",)),
                        ("cassandra", ()),
                        ("cassandra.cluster", ("Cluster",))):
        m = types.ModuleType(name)
        for a in attrs:
            setattr(m, a, object)
        sys.modules[name] = m
    sys.path.insert(0, REF)
    import tile  # noqa
    import heatmap  # noqa
    return tile.Tile, heatmap


class RDD(list):
    """In-memory stand-in for the RDD methods heatmap.py:107-118 uses."""

    def flatMap(self, f):
        out = RDD()
        for x in self:
            out.extend(f(x))
        return out

    def map(self, f):
        return RDD(f(x) for x in self)

    def reduceByKey(self, f):
        acc = {}
        for k, v in self:
            acc[k] = f(acc[k], v) if k in acc else v
        return RDD(acc.items())

    def groupByKey(self):
        acc = collections.OrderedDict()
        for k, v in self:
            acc.setdefault(k, []).append(v)
        return RDD(acc.items())

    def mapValues(self, f):
        return RDD((k, f(v)) for k, v in self)

    def union(self, o):
        return RDD(list(self) + list(o))


def classify(fn):
    try:
        return OK, fn()
    except ValueError as e:
        if "NaN" in str(e):
            return E_NAN, 0
        if "domain" in str(e):
            return E_DOMAIN, 0
        raise
    except OverflowError as e:
        assert "infinity" in str(e), e
        return E_INF, 0


def projection_kat(Tile, rng):
    lats, lons, zooms = [], [], []

    def add(la, lo, z):
        lats.append(float(la))
        lons.append(float(lo))
        zooms.append(int(z))

    # uniform and hotspot points at every zoom 0..30
    ula, ulo = synth.uniform(6000, seed=11)
    for i in range(6000):
        add(ula[i], ulo[i], i % 31)
    hla, hlo = synth.hotspots(4000, seed=12)
    for i in range(4000):
        add(hla[i], hlo[i], (i * 7) % 31)
    # boundary-adjacent latitude pairs, found by bisection on the reference row
    for z in (4, 10, 14, 16, 18, 21, 24, 28):
        for _ in range(220):
            r = int(rng.integers(1, (1 << z) - 1)) if z > 1 else 1
            lat_b = Tile.latitude_from_row(r, z)
            lo_lat, hi_lat = lat_b - 1e-6 * (1 + abs(lat_b)), lat_b + 1e-6 * (1 + abs(lat_b))
            # row(lo_lat) >= r > row(hi_lat)?  rows decrease with latitude
            if not (Tile.row_from_latitude(lo_lat, z) >= r > Tile.row_from_latitude(hi_lat, z)):
                continue
            for _it in range(200):
                mid = (lo_lat + hi_lat) / 2
                if mid in (lo_lat, hi_lat):
                    break
                if Tile.row_from_latitude(mid, z) >= r:
                    lo_lat = mid
                else:
                    hi_lat = mid
            x = lo_lat
            for _k in range(3):
                x = math.nextafter(x, -math.inf)
            for _k in range(7):
                add(x, float(rng.uniform(-180, 180)), z)
                x = math.nextafter(x, math.inf)
    # exact column boundaries and their neighbours
    for z in (1, 5, 10, 18, 21, 26, 30):
        for _ in range(120):
            k = int(rng.integers(0, (1 << z) + 1))
            lon_b = -180.0 + k * 360.0 / (1 << z)
            x = lon_b
            for _k in range(2):
                x = math.nextafter(x, -math.inf)
            for _k in range(5):
                add(float(rng.uniform(-80, 80)), x, z)
                x = math.nextafter(x, math.inf)
    # latitude extremes, polar band, out-of-window rows, big latitudes
    specials_lat = [85.0511287798066, -85.0511287798066, 85.05112877980659, -85.05112877980659,
                    85.0511287798067, 89.9, -89.9, 89.99999, 90.0, -90.0, 95.0, -95.0, 180.0,
                    -180.0, 407.6, -312.4, 0.0, -0.0, 5e-324, -5e-324, 1e-300, 47.6, 1e6,
                    -1e6, 123456.789, 2.5e9, -2.5e9, 1e300, -1e300, 1.7976931348623157e308,
                    float("nan"), float("inf"), float("-inf")]
    specials_lon = [180.0, -180.0, 179.99999999999997, -179.99999999999997, -200.0, 540.0,
                    1e6, -1e6, 0.0, -0.0, 360.0, -540.0, 1e15, 1e300, -1e300,
                    float("nan"), float("inf"), float("-inf")]
    for la in specials_lat:
        for z in (0, 1, 6, 14, 18, 21, 30):
            add(la, 10.0, z)
    for lo in specials_lon:
        for z in (0, 1, 6, 14, 18, 21, 30):
            add(10.0, lo, z)
    for la in specials_lat[:12]:
        for lo in specials_lon:
            add(la, lo, 21)
    pol = rng.uniform(85.0, 90.0, 1500)
    for i, la in enumerate(pol):
        s = 1 if i % 2 else -1
        add(s * la, float(rng.uniform(-180, 180)), [8, 14, 18, 21][i % 4])
    big = rng.uniform(-5e5, 5e5, 1500)
    for i, la in enumerate(big):
        add(la, float(rng.uniform(-1000, 1000)), [3, 12, 21][i % 3])

    n = len(lats)
    row = np.zeros(n, np.int64)
    col = np.zeros(n, np.int64)
    row_err = np.zeros(n, np.int8)
    col_err = np.zeros(n, np.int8)
    col_big = {}
    for i in range(n):
        e, r = classify(lambda: Tile.row_from_latitude(lats[i], zooms[i]))
        row_err[i] = e
        row[i] = r if e == OK else 0
        e, c = classify(lambda: Tile.column_from_longitude(lons[i], zooms[i]))
        col_err[i] = e
        if e == OK:
            if -(1 << 63) <= c < (1 << 63):
                col[i] = c
            else:
                col_err[i] = 8            # exceeds int64 (kept as text)
                col_big[i] = str(c)
    path = os.path.join(HERE, "projection_kat.npz")
    np.savez_compressed(path, lat=np.array(lats), lon=np.array(lons), zoom=np.array(zooms, np.int8),
                        row=row, col=col, row_err=row_err, col_err=col_err)
    with open(os.path.join(HERE, "projection_kat_bigcols.json"), "w") as f:
        json.dump(col_big, f)
    # formatted ids, including negative rows and the error-free specials
    ids = []
    for i in range(0, n, max(1, n // 400)):
        try:
            ids.append([lats[i], lons[i], zooms[i], Tile.tile_id_from_lat_long(lats[i], lons[i], zooms[i])])
        except (ValueError, OverflowError) as e:
            ids.append([lats[i], lons[i], zooms[i], type(e).__name__ + ": " + str(e)])
    with open(os.path.join(HERE, "tile_ids.json"), "w") as f:
        json.dump([[repr(a), repr(b), z, s] for a, b, z, s in ids], f)
    print("projection KATs:", n, "errors(row):", int((row_err != 0).sum()), "boundary cases included")


def run_build_heatmaps(hm, rows, max_zoom_level=16, delta=5):
    hm.MAX_ZOOM_LEVEL = max_zoom_level
    hm.DETAIL_ZOOM_DELTA = delta
    try:
        locs = RDD(rows).flatMap(hm.dataframe_loader)
        out = hm.build_heatmaps(locs)
        result = {}
        for k, v in out:
            assert k not in result, k
            result[k] = v
        return result
    finally:
        hm.MAX_ZOOM_LEVEL = 16
        hm.DETAIL_ZOOM_DELTA = 5


def mixed_rows(lat, lon, rng, users, bg_frac=0.25):
    rows = []
    for i in range(len(lat)):
        rows.append({"latitude": float(lat[i]), "longitude": float(lon[i]),
                     "source": "background" if rng.random() < bg_frac else "gps",
                     "user_id": users[int(rng.integers(0, len(users)))],
                     "timestamp": 1500000000000 + i})
    return rows


def heatmap_goldens(hm, rng):
    cases = []
    users = ["x1", "x2", "u1", "u2", "rt-9", "rt-3", "route"]
    la, lo = synth.hotspots(3000, seed=21)
    # pull the cloud onto Seattle so many points share tiles
    la = 47.6 + (la - la.mean()) * 0.05
    lo = -122.3 + (lo - lo.mean()) * 0.05
    cases.append(("seattle_mixed_z21", mixed_rows(la, lo, rng, users), 16, 5))
    la, lo = synth.uniform(3000, seed=22)
    cases.append(("world_mixed_z14", mixed_rows(la, lo, rng, users), 9, 5))
    la, lo = synth.hotspots(2000, seed=23)
    cases.append(("hotspots_alluser_z18", mixed_rows(la, lo, rng, users + ["all", "all", "xall"]), 13, 5))
    la, lo = synth.hotspots(1500, seed=24)
    cases.append(("hotspots_delta3_z12", mixed_rows(la, lo, rng, ["u1", "x9", "rt-1"]), 9, 3))
    # edge coordinates that stay on the reference's shift window
    edge_lat = [85.0511287798066, -85.0511287798066, 85.05, -85.05, 0.0, -0.0, 47.6, 89.0, -89.0]
    edge_lon = [180.0, -180.0, 179.99999999999997, 0.0, -0.0, -122.3, 200.0, -200.0]
    el, eo = [], []
    for a in edge_lat:
        for b in edge_lon:
            el.append(a)
            eo.append(b)
    cases.append(("edges_z14", mixed_rows(np.array(el), np.array(eo), rng, ["u1", "x1"], 0.1), 9, 5))
    meta = []
    for name, rows, mz, d in cases:
        t0 = time.time()
        res = run_build_heatmaps(hm, rows, mz, d)
        with gzip.open(os.path.join(HERE, "heatmap_rows_%s.json.gz" % name), "wt") as f:
            json.dump({"max_zoom_level": mz, "detail_zoom_delta": d, "input": rows, "rows": res}, f)
        meta.append((name, len(rows), len(res), round(time.time() - t0, 2)))
    print("heatmap goldens:", meta)


def chain_goldens(hm, rng):
    """Rows of points whose tiles leave the shift windows (heatmap_amd/chain_window.py):
    within ~1e-6 deg of the poles and |lon| > 11520, where the reference's
    tile-centre re-projection (heatmap.py:60-61,89) is not the shift.  Points
    whose chain raises in the reference (row21 >= 7,295,112) are left out."""
    users = ["x1", "u1", "u2", "rt-9", "route"]
    cases = []
    for name, mz, d, seed in (("chain_poles_farlon_z21", 16, 5, 31), ("chain_poles_farlon_z14", 9, 5, 32)):
        r = np.random.default_rng(seed)
        la = list(47.6 + r.normal(0, 0.01, 120))
        lo = list(-122.3 + r.normal(0, 0.01, 120))
        # north pole: 90 - 10^U(-9.5, -5) (rows far below the window at zoom 21)
        for e in r.uniform(-9.5, -5.0, 40):
            la.append(90.0 - 10.0 ** e)
            lo.append(float(r.uniform(-180, 180)))
        # south pole: the chain still returns (rows up to ~7.29e6 at zoom 21)
        for e in r.uniform(-5.5, -3.5, 25):
            la.append(-90.0 + 10.0 ** e)
            lo.append(float(r.uniform(-180, 180)))
        # far longitudes: |lon| in (11520, 3e5), and a few beyond
        for v in r.uniform(11520.0, 3e5, 30):
            la.append(float(r.uniform(-60, 60)))
            lo.append(float(v) * (1 if r.random() < 0.5 else -1))
        for v in (1e6, -2.5e6, 7.77e7):
            la.append(10.0)
            lo.append(v)
        rows = mixed_rows(np.array(la), np.array(lo), rng, users, 0.15)
        # drop the points whose chain raises in the reference
        ok = []
        for row in rows:
            try:
                run_build_heatmaps(hm, [row], mz, d)
                ok.append(row)
            except (ValueError, OverflowError):
                pass
        cases.append((name, ok, mz, d))
    meta = []
    for name, rows, mz, d in cases:
        res = run_build_heatmaps(hm, rows, mz, d)
        with gzip.open(os.path.join(HERE, "heatmap_rows_%s.json.gz" % name), "wt") as f:
            json.dump({"max_zoom_level": mz, "detail_zoom_delta": d, "input": rows, "rows": res}, f)
        meta.append((name, len(rows), len(res)))
    print("chain goldens:", meta)


def weighted_locations_golden(hm, rng):
    """build_heatmaps on locations other than dataframe_loader's: tiles at other
    zooms (coarser and finer than the detail zoom), dyadic float counts (exact
    in any summation order), and one level's heatmap_to_locations output fed
    back in; with default constants and MAX_ZOOM_LEVEL = 9.  Some tiles lie
    outside the shift windows (poles, far columns)."""
    users = ["x1", "u1", "u2", "rt-9", "route", "all"]
    out = {}
    for mz in (16, 9):
        hm.MAX_ZOOM_LEVEL = mz
        try:
            zmax = mz + 5
            locs = []
            r = np.random.default_rng(40 + mz)
            for i in range(300):
                z = int(r.choice([zmax, zmax, zmax - 3, zmax + 2, 12, 7]))
                la = float(47.6 + r.normal(0, 0.05)) if i % 10 else float(r.uniform(-85, 85))
                lo = float(-122.3 + r.normal(0, 0.05)) if i % 10 else float(r.uniform(-180, 180))
                if i % 37 == 0:
                    la = 90.0 - 10.0 ** float(r.uniform(-9, -6))
                if i % 41 == 0:
                    lo = float(r.uniform(12000, 90000))
                tid = hm.Tile.tile_id_from_lat_long(la, lo, z)
                locs.append({"userId": users[int(r.integers(0, len(users)))], "tileId": tid,
                             "count": float(r.choice([1.0, 2.0, 0.5, 3.25, 7.0])), "timespan": "alltime"})
            # one level of the reference's own output, fed back in as locations
            rows = [{"latitude": float(47.6 + r.normal(0, 0.02)), "longitude": float(-122.3 + r.normal(0, 0.02)),
                     "source": "gps", "user_id": users[int(r.integers(0, len(users)))], "timestamp": 0}
                    for _ in range(200)]
            lvl = list(hm.build_heatmaps(RDD(rows).flatMap(hm.dataframe_loader)))
            lvl = [b for b in lvl if b[0].split("|")[2].startswith("%d_" % (zmax - 1 - 5))]
            for b in lvl[:40]:
                locs.extend(hm.heatmap_to_locations(b))
            res = {}
            for k, v in hm.build_heatmaps(RDD(locs)):
                assert k not in res
                res[k] = v
            out[str(mz)] = {"locations": locs, "rows": res}
        finally:
            hm.MAX_ZOOM_LEVEL = 16
    with gzip.open(os.path.join(HERE, "weighted_locations.json.gz"), "wt") as f:
        json.dump(out, f)
    print("weighted locations:", {k: (len(v["locations"]), len(v["rows"])) for k, v in out.items()})


def weighted_nondyadic_golden(hm, rng):
    """build_heatmaps on locations with NON-dyadic float counts (0.1, 0.3,
    1/3, 2.7, 0.7): their sums depend on the summation order, which in the
    reference is Spark's (here the in-memory RDD's input order), so the test
    compares with a relative tolerance, not bit for bit.  Default constants,
    MAX_ZOOM_LEVEL = 9; tiles at the detail zoom and two coarser ones."""
    users = ["x1", "u1", "u2", "rt-9", "all"]
    hm.MAX_ZOOM_LEVEL = 9
    try:
        zmax = 14
        locs = []
        for i in range(2000):
            z = int(rng.choice([zmax, zmax, zmax - 2, 11]))
            la = float(47.6 + rng.normal(0, 0.2))
            lo = float(-122.3 + rng.normal(0, 0.2))
            tid = hm.Tile.tile_id_from_lat_long(la, lo, z)
            locs.append({"userId": users[int(rng.integers(0, len(users)))], "tileId": tid,
                         "count": float(rng.choice([0.1, 0.3, 1.0 / 3.0, 2.7, 0.7])), "timespan": "alltime"})
        res = {}
        for k, v in hm.build_heatmaps(RDD(locs)):
            assert k not in res
            res[k] = v
    finally:
        hm.MAX_ZOOM_LEVEL = 16
    with gzip.open(os.path.join(HERE, "weighted_nondyadic.json.gz"), "wt") as f:
        json.dump({"max_zoom_level": 9, "locations": locs, "rows": res}, f)
    print("weighted non-dyadic:", len(locs), len(res))


def canonical_digest(items):
    h = hashlib.sha256()
    for it in items:
        h.update((",".join(str(x) for x in it) + "\n").encode())
    return h.hexdigest()


def zoom_count_digest(Tile, lat, lon, zooms):
    out = {}
    for z in zooms:
        c = collections.Counter()
        for a, b in zip(lat.tolist(), lon.tolist()):
            c[Tile.tile_id_from_lat_long(a, b, z)] += 1
        cells = sorted((int(k.split("_")[1]), int(k.split("_")[2]), v) for k, v in c.items())
        sample = [list(cells[i]) for i in range(0, len(cells), max(1, len(cells) // 200))]
        out[str(z)] = {"cells": len(cells), "total": sum(v for _, _, v in cells),
                       "sha256": canonical_digest(cells), "sample": sample}
    return out


def config1_digest(Tile, hm):
    n = 1_000_000
    lat, lon = synth.uniform(n, seed=0)
    t0 = time.time()
    zc = zoom_count_digest(Tile, lat, lon, range(0, 22))
    t_proj = time.time() - t0
    rows = [{"latitude": float(a), "longitude": float(b), "source": "gps", "user_id": "x",
             "timestamp": 0} for a, b in zip(lat.tolist(), lon.tolist())]
    t0 = time.time()
    res = run_build_heatmaps(hm, rows, 9, 5)
    t_pipe = time.time() - t0
    items = sorted((k, t, repr(c)) for k, d in res.items() for t, c in d.items())
    sample = {k: res[k] for k in sorted(res)[:: max(1, len(res) // 150)]}
    out = {"n": n, "generator": "synth.uniform(n, seed=0)", "zoom_counts": zc,
           "heatmap": {"max_zoom_level": 9, "delta": 5, "rows": len(res), "bins": len(items),
                       "sha256": canonical_digest(items), "sample_rows": sample},
           "reference_seconds": {"projection_22_zooms": round(t_proj, 1),
                                 "build_heatmaps": round(t_pipe, 1)}}
    with open(os.path.join(HERE, "config1_digest.json"), "w") as f:
        json.dump(out, f)
    print("config1 digest: rows", len(res), "bins", len(items), "t", t_pipe)


def hotspot_zoom_digest(Tile):
    lat, lon = synth.hotspots(100_000, seed=0)
    out = {"n": 100_000, "generator": "synth.hotspots(n, seed=0)",
           "zoom_counts": zoom_count_digest(Tile, lat, lon, range(0, 22))}
    lat, lon = synth.skew(50_000, seed=0)
    out["skew"] = {"n": 50_000, "generator": "synth.skew(n, seed=0)",
                   "zoom_counts": zoom_count_digest(Tile, lat, lon, [0, 5, 10, 14, 17, 18, 19, 21])}
    with open(os.path.join(HERE, "zoom_counts_hotspots.json"), "w") as f:
        json.dump(out, f)
    print("hotspot zoom digests done")


def tile_utils_golden(Tile, rng):
    """Tile utility API (tile.py:23-98): inverse projection, tile_from_tile_id,
    parent_id, children, tile_ids_for_all_zoom_levels.  Floats are stored as
    repr() strings so the fixture is bit-exact."""
    ids = ["0_0_0", "1_0_0", "1_1_1", "16_0_0", "16_65535_65535", "16_22894_10501", "12_1430_656",
           "5_12_3", "9_511_0", "14_5724_2625", "2_3_0", "16_32768_32768", "7_0_127",
           # centres whose columns pass int64 at the higher zooms (tile ids print the exact Python int)
           "16_100_10000000000000000000", "16_22894_-30000000000000000000", "10_5_123456789012345678901"]
    for _ in range(60):
        z = int(rng.integers(1, 17))
        ids.append("%d_%d_%d" % (z, int(rng.integers(0, 2 ** z)), int(rng.integers(0, 2 ** z))))
    cases = []
    for tid in ids:
        t = Tile.tile_from_tile_id(tid)
        rec = {"id": tid,
               "fields": {k: repr(getattr(t, k)) for k in
                          ("latitude_north", "latitude_south", "longitude_west", "longitude_east",
                           "center_latitude", "center_longitude")},
               "children": t.children(),
               "all_zooms": Tile.tile_ids_for_all_zoom_levels(tid)}
        rec["parent_id"] = t.parent_id()   # zoom 0: projected at zoom -1 (2 ** -1)
        cases.append(rec)
    lat_rows = []
    for _ in range(200):
        z = int(rng.integers(0, 25))
        r = int(rng.integers(-2, 2 ** z + 3))
        lat_rows.append([r, z, repr(Tile.latitude_from_row(r, z))])
    with open(os.path.join(HERE, "tile_utils.json"), "w") as f:
        json.dump({"generator": "tests/golden/make_golden.py --only utils", "tiles": cases,
                   "latitude_from_row": lat_rows, "malformed": ["1_2", "a_b_c_d", "", "3__4_5"]}, f)
    print("tile utils done: %d tiles" % len(cases))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--quick", action="store_true")
    ap.add_argument("--only", default="")
    a = ap.parse_args()
    Tile, hm = load_reference()
    rng = np.random.default_rng(20261015)
    todo = a.only.split(",") if a.only else ["kat", "rows", "hot", "c1"]
    if "kat" in todo:
        projection_kat(Tile, rng)
    if "rows" in todo:
        heatmap_goldens(hm, rng)
    if "hot" in todo:
        hotspot_zoom_digest(Tile)
    if "utils" in todo or not a.only:
        tile_utils_golden(Tile, np.random.default_rng(20261016))
    if "chain" in todo or not a.only:
        chain_goldens(hm, np.random.default_rng(20261017))
    if "weighted" in todo or not a.only:
        weighted_locations_golden(hm, np.random.default_rng(20261018))
    if "weighted_nd" in todo or not a.only:
        weighted_nondyadic_golden(hm, np.random.default_rng(20261019))
    if "c1" in todo and not a.quick:
        config1_digest(Tile, hm)


if __name__ == "__main__":
    main()
