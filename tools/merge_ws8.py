#!/usr/bin/env python3
"""The world-size-8 exchange's device work on one GPU: count 1.25e9 hotspot
points (one rank's shard of the N = 8 bench), route the cells to 8 owners
(hm_cells_route_pieces) and merge the 8 groups as one owner's 8 received runs
(hm_cells_merge_pieces, R = 8) -- an owner's load at N = 8 (~28M cells in 8
runs), without the xGMI all-to-all.  Prints one JSON line per route-bits
setting (median of the timed repeats).

    python tools/merge_ws8.py [points] [bits ...]
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from heatmap_amd import _lib, device, multigpu  # noqa: E402


def main():
    n = int(float(sys.argv[1])) if len(sys.argv) > 1 else 1_250_000_000
    bit_list = [int(b) for b in sys.argv[2:]] or [multigpu.route_bits(8)]
    lat = torch.empty(n, dtype=torch.float64, device="cuda")
    lon = torch.empty(n, dtype=torch.float64, device="cuda")
    device.synth("hotspots", lat, lon, seed=0)
    m, bufs = device.count_device(lat, lon, None, 0, 18)
    del lat, lon
    keys, counts = bufs.keys[:m].clone(), bufs.counts[:m].clone()
    del bufs
    ops = multigpu.DeviceOps(0)
    ws = 8
    for bits in bit_list:
        S = 1 << bits
        tr, tm = [], []
        for it in range(6):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            _, parts, sizes = ops.route_pieces(keys, counts, ws, 10, bits, _lib.HM_CELLS_REC10)
            sz = sizes.cpu()
            t1 = time.perf_counter()
            offs = [0] + sz[:, 0].cumsum(0).tolist()
            runs = [(parts[0][0], None, offs[o]) for o in range(ws)]
            uk, _ = ops.merge_pieces(runs, [sz[o, 2:2 + S].tolist() for o in range(ws)], bits, _lib.HM_CELLS_REC10)
            torch.cuda.synchronize()
            t2 = time.perf_counter()
            if it:
                tr.append((t1 - t0) * 1e3)
                tm.append((t2 - t1) * 1e3)
            assert uk.numel() == int(sz[:, 0].sum())
        tr.sort()
        tm.sort()
        print(json.dumps({"bits": bits, "route_ms": tr[len(tr) // 2], "merge_ms": tm[len(tm) // 2], "cells": int(m),
                          "routed": int(sz[:, 0].sum()), "owners": ws}), flush=True)


if __name__ == "__main__":
    main()
