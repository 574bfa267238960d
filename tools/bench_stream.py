#!/usr/bin/env python3
"""Config 5 (BASELINE.json): streaming micro-batches of 10M points with uint32
epoch-hour timestamps merged into a resident multi-zoom heatmap (hm_stream_*).

One step = one hm_stream_add of a 10M-point hotspot batch (device-resident,
synthesised outside the timed region) whose points carry `--hours` distinct
hours; the heatmap keeps growing across steps, as a stream's would.  Prints
one JSON line (points/s over the timed batches, ms per batch, resident cells).

    python tools/bench_stream.py --batches 18 --warmup 2

With the defaults (2 + 18 batches of 10M hotspot points, one hour each) the
alltime cells are checked against the C oracle's digest of the same 200M
points (tests/golden/big_digests.json, hotspots_2e8_z0-18_stream20x10M).
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import torch  # noqa: E402

from heatmap_amd import device  # noqa: E402
from heatmap_amd.stream import ALLTIME, StreamingHeatmap  # noqa: E402

BASE = 480000


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=float, default=1e7)
    ap.add_argument("--batches", type=int, default=18)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--hours", type=int, default=1, help="distinct hours per batch")
    ap.add_argument("--zmin", type=int, default=0)
    ap.add_argument("--zmax", type=int, default=18)
    ap.add_argument("--kind", default="hotspots")
    ap.add_argument("--initial-cells", type=float, default=float(1 << 26),
                    help="the resident log's first capacity (it doubles when full)")
    a = ap.parse_args()
    n = int(a.batch)
    total = a.warmup + a.batches
    lat = [torch.empty(n, dtype=torch.float64, device="cuda") for _ in range(total)]
    lon = [torch.empty(n, dtype=torch.float64, device="cuda") for _ in range(total)]
    hrs = []
    for b in range(total):
        device.synth(a.kind, lat[b], lon[b], seed=0, start=b * n)
        h = BASE + b * a.hours + (torch.arange(n, device="cuda", dtype=torch.int64) % a.hours)
        hrs.append(h.to(torch.int32))
    s = StreamingHeatmap(a.zmin, a.zmax, base_hour=BASE, initial_cells=int(a.initial_cells))
    for b in range(a.warmup):
        s.add(lat[b], lon[b], hour=hrs[b])
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for b in range(a.warmup, total):
        s.add(lat[b], lon[b], hour=hrs[b])
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    cells, cap = s.cells()
    nall, akeys, acounts = s.extract_device(ALLTIME)[:3]
    # the whole stream (warm-up batches included) against the C oracle's digest
    # of the same points, when one is committed for this configuration
    check = None
    gold = os.path.join(REPO, "tests", "golden", "big_digests.json")
    name = "%s_%.0e_z%d-%d_stream%dx10M" % (a.kind, total * n, a.zmin, a.zmax, total)
    name = name.replace("e+0", "e")
    if n == 10_000_000 and os.path.exists(gold):   # alltime: the same points whatever the hours
        g = json.load(open(gold)).get(name)
        if g is not None:
            sys.path.insert(0, os.path.join(REPO, "tests"))
            from digest import device_digest

            check = "ok" if device_digest(torch, akeys[:nall], acounts[:nall]) == g["digest"] else "FAIL"
    print(json.dumps({
        "metric": "points streamed into a resident heatmap/sec (config 5)", "value": a.batches * n / dt,
        "unit": "points/s", "ms_per_batch": dt * 1e3 / a.batches, "batch_points": n, "batches": a.batches,
        "warmup": a.warmup, "hours_per_batch": a.hours, "zooms": [a.zmin, a.zmax], "kind": a.kind,
        "resident_cells_all_buckets": cells, "alltime_cells": nall, "log_capacity": cap,
        "check": check if check is not None else "no digest for this configuration",
        "data": "synthetic (heatmap_amd.synth, generated on device, resident in HBM)"}))
    s.close()


if __name__ == "__main__":
    main()
