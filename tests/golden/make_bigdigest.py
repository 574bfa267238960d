#!/usr/bin/env python3
"""Full-size cell digests for the GPU parity tests (tests/test_gpu_fullsize.py).

The bench configurations are too large to compare cell lists in a test, so the
expected result is the order-free digest of tests/conftest.py (cells, total
count, sum and xor of a 64-bit mix of every (zoom, row, col, count)), computed
here on the CPU with the C oracle (oracle/hm_oracle.c: the literal glibc
projection of tile.py:15-21 and the per-zoom sum of heatmap.py:109-111,
itself pinned to the reference's goldens by tests/test_oracle.py):

  - the points are generated chunk by chunk (heatmap_amd.synth, bit-identical
    to the device generator), each chunk counted at zoom zmax by the oracle,
    and the chunks' zoom-zmax cells summed;
  - every coarser zoom is the sum of the zoom below it over (row >> 1, col >> 1)
    (the arithmetic-shift identity of SURVEY.md a-1/a-4).

    python tests/golden/make_bigdigest.py [--only NAME]   (minutes; ~10 GB RAM)

writes tests/golden/big_digests.json.  Data only: inputs are named by their
generator and seed, outputs are digests.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.dirname(HERE))

from conftest import cells_digest  # noqa: E402
from heatmap_amd import synth  # noqa: E402
from oracle import oracle  # noqa: E402

OUT = os.path.join(HERE, "big_digests.json")
M29 = (1 << 29) - 1

# name: (kind, seed, start, n, zmin, zmax)
CASES = {
    "hotspots_1e9_z0-18": ("hotspots", 0, 0, 1_000_000_000, 0, 18),
    "skew_1e9_z0-18": ("skew", 0, 0, 1_000_000_000, 0, 18),
    "hotspots_2e8_z0-18_stream20x10M": ("hotspots", 0, 0, 200_000_000, 0, 18),
    # >= 2^19 keys per level-1 bucket: the 3-zoom spread plan at its default threshold
    "uniform_6e8_z0-18": ("uniform", 0, 0, 600_000_000, 0, 18),
    "hotspots_1e7_start0_z0-18": ("hotspots", 0, 0, 10_000_000, 0, 18),
    "hotspots_1e7_start70M_z0-18": ("hotspots", 0, 70_000_000, 10_000_000, 0, 18),
    "hotspots_1e7_start190M_z0-18": ("hotspots", 0, 190_000_000, 10_000_000, 0, 18),
    # the reference's production zooms: detail zooms 21..6 (heatmap.py:16-17,109)
    "hotspots_1e9_z6-21": ("hotspots", 0, 0, 1_000_000_000, 6, 21),
}

# grouped: name: (kind, seed, n, users, zmin, zmax); point i's group is
# ((i * 2654435761) >> 7) % users (tools/bench_grouped.py).  The digest is over
# records (zoom, (group << (zoom + 1)) | row, col, count): a group-tagged row
# that every coarser zoom's shift keeps separable (rows < 2^zoom here)
GROUPED = {
    "grouped_hotspots_1e8_u10000_z6-21": ("hotspots", 0, 100_000_000, 10_000, 6, 21),
}


def run_grouped(kind, seed, n, users, zmin, zmax):
    """The C oracle's projection of every point at zmax, the group folded into
    the row's high bits, and its tile-input count (every coarser zoom the
    shift): exactly the per-(group, zoom, row, col) counts of hm_count_grouped
    for in-square points."""
    t0 = time.time()
    lat, lon = synth.generate(kind, n, seed=seed)
    r, c, st, _ = oracle.project(lat, lon, zmax)
    del lat, lon
    assert int(st.max()) == 0
    assert r.min() >= 0 and r.max() < (1 << zmax) and c.min() >= 0 and c.max() < (1 << zmax)
    g = ((np.arange(n, dtype=np.int64) * 2654435761) >> 7) % users
    rt = (g << (zmax + 1)) | r
    del g, r
    parts = []
    for z in range(zmax, zmin - 1, -1):   # one zoom at a time (its tiles the shift of the zmax ones)
        k = zmax - z
        out = oracle.count_tiles(rt >> k, c >> k, z, z)
        parts.append(cells_digest(out["zoom"], out["row"], out["col"], out["count"]))
        print("  zoom %d: %d records (%.0f s)" % (z, parts[-1][0], time.time() - t0), flush=True)
        del out
    x = 0
    for p in parts:
        x ^= p[3]
    dg = [sum(p[0] for p in parts), sum(p[1] for p in parts), sum(p[2] for p in parts) % (1 << 64), x]
    return {"kind": kind, "seed": seed, "n": n, "users": users, "zmin": zmin, "zmax": zmax,
            "group_of_point": "((i * 2654435761) >> 7) % users", "row_tag": "(group << (zoom + 1)) | row",
            "digest": list(dg), "seconds": round(time.time() - t0, 1)}


def _merge(keys, counts, k2, c2):
    k = np.concatenate([keys, k2])
    c = np.concatenate([counts, c2])
    o = np.argsort(k, kind="stable")
    k, c = k[o], c[o]
    head = np.ones(k.size, bool)
    head[1:] = k[1:] != k[:-1]
    s = np.flatnonzero(head)
    return k[s], np.add.reduceat(c, s)


def _digest_zoom(z, keys, counts):
    return cells_digest(np.full(keys.size, z, np.int64), (keys >> np.uint64(29)).astype(np.int64),
                        (keys & np.uint64(M29)).astype(np.int64), counts)


def run_case(kind, seed, start, n, zmin, zmax, chunk=100_000_000):
    t0 = time.time()
    keys = np.zeros(0, np.uint64)
    counts = np.zeros(0, np.int64)
    for s in range(0, n, chunk):
        m = min(chunk, n - s)
        lat, lon = synth.generate(kind, m, seed=seed, start=start + s)
        r = oracle.count(lat, lon, None, zmax, zmax)
        assert r["status"] == 0
        del lat, lon
        k2 = (r["row"].astype(np.uint64) << np.uint64(29)) | r["col"].astype(np.uint64)
        keys, counts = _merge(keys, counts, k2, r["count"])
        print("  %s: %d / %d points, %d cells at zoom %d (%.0f s)" % (kind, s + m, n, keys.size, zmax,
                                                                     time.time() - t0), flush=True)
    parts = []
    for z in range(zmax, zmin - 1, -1):
        if z < zmax:
            pk = ((keys >> np.uint64(30)) << np.uint64(29)) | ((keys & np.uint64(M29)) >> np.uint64(1))
            keys, counts = _merge(np.zeros(0, np.uint64), np.zeros(0, np.int64), pk, counts)
        parts.append(_digest_zoom(z, keys, counts))
    cells = sum(p[0] for p in parts)
    total = sum(p[1] for p in parts)
    ssum = sum(p[2] for p in parts) % (1 << 64)
    x = 0
    for p in parts:
        x ^= p[3]
    return {"kind": kind, "seed": seed, "start": start, "n": n, "zmin": zmin, "zmax": zmax,
            "digest": [cells, total, ssum, x], "seconds": round(time.time() - t0, 1)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", default=None)
    a = ap.parse_args()
    d = json.load(open(OUT)) if os.path.exists(OUT) else {}
    for name, case in CASES.items():
        if a.only and name != a.only:
            continue
        print(name, flush=True)
        d[name] = run_case(*case)
        json.dump(d, open(OUT, "w"), indent=1)
        print("  ->", d[name]["digest"], flush=True)
    for name, case in GROUPED.items():
        if a.only and name != a.only:
            continue
        print(name, flush=True)
        d[name] = run_grouped(*case)
        json.dump(d, open(OUT, "w"), indent=1)
        print("  ->", d[name]["digest"], flush=True)


if __name__ == "__main__":
    main()
