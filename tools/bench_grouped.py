#!/usr/bin/env python3
"""The row-producing path (reference heatmap.py:64-75,111-112,120-129): per-user
counts in one device pass (hm_count_grouped) and heatmap_table end to end.

  device   one step = one hm_count_grouped_packed (--records int64x5:
           hm_count_grouped) over N device-resident hotspot
           points, each with one of U user groups (a hash of its index): the
           exact projection of every point, 128-bit (group, super-tile, Morton)
           keys, the LSD radix sort and the RLE zoom cascade (hm_general.hip),
           every (group, zoom, row, col, count) record written to HBM.
  table    heatmap_table on a host batch of M points with string user ids
           (factorize, two device passes, combine_cells, pyarrow rows), timed
           by phase.

    python tools/bench_grouped.py --points 1e8 --users 10000 --zmin 6 --zmax 21
Prints one JSON line per part.
"""
import argparse
import ctypes
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from heatmap_amd import _lib, device  # noqa: E402

HBM_PEAK_GBS = 8000.0


def bench_device(a):
    n = int(a.points)
    lat = torch.empty(n, dtype=torch.float64, device="cuda")
    lon = torch.empty(n, dtype=torch.float64, device="cuda")
    device.synth(a.kind, lat, lon, seed=a.seed)
    grp = ((torch.arange(n, device="cuda", dtype=torch.int64) * 2654435761) >> 7) % a.users
    grp = grp.to(torch.int32)
    ctx = device.context(0)
    w = 2 if a.packed else 5          # int64 words per record: (HM_KEY, group|count) or 5 fields
    buf = {"cap": int(a.cap_factor * n) + 1024}
    buf["cells"] = torch.empty(w * buf["cap"], dtype=torch.int64, device="cuda")
    nout = ctypes.c_int64(0)
    p = device._ptr

    def step():
        while True:
            if a.packed:
                c = buf["cells"]
                rc = ctx.L.hm_count_grouped_packed(ctx.ptr, p(lat), p(lon), ctypes.c_void_p(0), p(grp), n, a.zmin,
                                                   a.zmax, p(c), ctypes.c_void_p(c.data_ptr() + 8 * buf["cap"]),
                                                   buf["cap"], ctypes.byref(nout))
            else:
                rc = ctx.L.hm_count_grouped(ctx.ptr, p(lat), p(lon), ctypes.c_void_p(0), p(grp), n, a.zmin, a.zmax,
                                            p(buf["cells"]), buf["cap"], ctypes.byref(nout))
            if rc != _lib.HM_E_CAPACITY:
                break
            buf["cap"] = int(nout.value * 1.05) + 1024      # warm-up only: the timed steps fit
            buf["cells"] = torch.empty(w * buf["cap"], dtype=torch.int64, device="cuda")
        if rc != _lib.HM_OK:
            _lib.raise_for(rc)

    for _ in range(a.warmup):
        step()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record()
    for _ in range(a.steps):
        step()
    e1.record()
    e1.synchronize()
    dt = time.perf_counter() - t0
    ms = e0.elapsed_time(e1) / a.steps
    m = nout.value
    cells = buf["cells"]
    if a.packed:
        tot = int((cells[buf["cap"]:buf["cap"] + m] & 0xFFFFFFFF).sum().item())
    else:
        tot = int(cells[:5 * m].reshape(-1, 5)[:, 4].sum().item())
    # 16 B of lat/lon + 4 B of group id read per point, 16 B per output cell
    alg = 16 * n + 4 * n + 16 * m
    out = {"part": "hm_count_grouped_packed" if a.packed else "hm_count_grouped", "value": n / (ms * 1e-3),
           "unit": "points/s", "ms_per_step": ms,
           "host_ms_per_step": dt * 1e3 / a.steps, "points": n, "users": a.users, "kind": a.kind,
           "zooms": [a.zmin, a.zmax], "records": m,
           "check": "ok" if tot == n * (a.zmax - a.zmin + 1) else "FAIL sum %d" % tot,
           "roofline": {"bound": "hbm", "alg_bytes": alg, "achieved_GBps": alg / (ms * 1e-3) / 1e9,
                        "frac": alg / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS,
                        "alg_bytes_note": "SURVEY 8(d): 16 B lat/lon + 4 B group per point read, 16 B per "
                                          "output cell (the record layout written: %d B)" % (8 * w)}}
    print(json.dumps(out), flush=True)
    del lat, lon, grp, cells
    torch.cuda.empty_cache()


def bench_table(a):
    from heatmap_amd import heatmap as hm
    from heatmap_amd import synth

    n = int(a.table_points)
    lat, lon = synth.generate(a.kind, n, seed=a.seed)
    g = ((np.arange(n, dtype=np.int64) * 2654435761) >> 7) % a.users
    names = np.array(["u%d" % i for i in range(a.users)], dtype=object)
    user = names[g]
    user[g % 7 == 3] = "x-anon"          # 'x*' ids: counted in 'all' only (heatmap.py:64-70)
    keep = (np.arange(n) % 5 != 2)       # background rows (heatmap.py:28-29)
    if a.arrow:   # the user_id column as io.load_locations reads it from Parquet (dictionary-encoded)
        import pyarrow as pa

        user = pa.array(user, type=pa.string()).dictionary_encode()
    hm.heatmap_table(lat[:10000], lon[:10000], user[:10000], keep[:10000], a.zmax - 5, 5)   # warm-up
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    tab = hm.heatmap_table(lat, lon, user, keep, a.zmax - 5, 5)
    ph = dict(hm.LAST_TABLE_PHASES)
    tot = time.perf_counter() - t0
    print(json.dumps({"part": "heatmap_table", "arrow_user_ids": bool(a.arrow), "value": n / tot, "unit": "points/s", "seconds": tot,
                      "points": n, "users": a.users, "rows": tab.num_rows,
                      "detail_zooms": [6, a.zmax], "phases_s": ph}), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--points", type=float, default=1e8)
    ap.add_argument("--table-points", type=float, default=1e7)
    ap.add_argument("--users", type=int, default=10000)
    ap.add_argument("--kind", default="hotspots")
    ap.add_argument("--zmin", type=int, default=6)
    ap.add_argument("--zmax", type=int, default=21)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--cap-factor", type=float, default=2.0, help="first record capacity per point")
    ap.add_argument("--no-table", action="store_true")
    ap.add_argument("--arrow", action="store_true", help="table: user ids as an Arrow dictionary column")
    ap.add_argument("--records", choices=["packed", "int64x5"], default="packed",
                    help="hm_count_grouped_packed (16 B per record) or hm_count_grouped (40 B)")
    a = ap.parse_args()
    a.packed = a.records == "packed"
    bench_device(a)
    if not a.no_table:
        bench_table(a)


if __name__ == "__main__":
    main()
