#!/usr/bin/env python3
"""Phase timing of the multi-GPU merge (heatmap_amd.multigpu.merge_cells) on one
GPU with a world-size-1 RCCL group: count 1.25e9 hotspot points (the N>1 bench
shard), then time the pieces exchange's route, size exchange, reduce, merge and
dense extraction separately (synchronised; at world size 1 no cell crosses
the all-to-all), and the route alone at 8 owners.  Prints one JSON line.

    python tools/merge_profile.py [points]
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29561")
os.environ.setdefault("WORLD_SIZE", "1")
os.environ.setdefault("RANK", "0")

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from heatmap_amd import _lib, device, multigpu  # noqa: E402


def main():
    n = int(float(sys.argv[1])) if len(sys.argv) > 1 else 1_250_000_000
    torch.cuda.set_device(0)
    dist.init_process_group("nccl")
    lat = torch.empty(n, dtype=torch.float64, device="cuda")
    lon = torch.empty(n, dtype=torch.float64, device="cuda")
    device.synth("hotspots", lat, lon, seed=0)
    bufs = device.CountBuffers(64 << 20)
    ops = multigpu.DeviceOps(0)
    res = {}
    bits = multigpu.route_bits(1)
    S = 1 << bits
    for it in range(3):
        t = {}

        def mark(name, t0):
            torch.cuda.synchronize()
            t[name] = (time.perf_counter() - t0) * 1e3
            return time.perf_counter()

        torch.cuda.synchronize()
        t0 = time.perf_counter()
        m, bufs = device.count_device(lat, lon, None, 0, 18, 0, buffers=bufs)
        t0 = mark("count", t0)
        keys, counts = bufs.keys[:m], bufs.counts[:m]
        grid, parts, sizes = ops.route_pieces(keys, counts, 1, 10, bits, _lib.HM_CELLS_REC10)
        t0 = mark("route", t0)
        recv = torch.empty_like(sizes)
        dist.all_to_all_single(recv, sizes)
        both = torch.stack([sizes, recv]).cpu()
        assert not bool(both[1, :, 1].any())
        t0 = mark("size_exchange", t0)
        dist.reduce(grid, dst=0)
        t0 = mark("reduce", t0)
        runs = [(parts[0][0], None, 0)]
        uk, uc = ops.merge_pieces(runs, both[1, :, 2:2 + S].tolist(), bits, _lib.HM_CELLS_REC10,
                                  out=(bufs.keys, bufs.counts))
        n = uk.numel()
        t0 = mark("merge", t0)
        dk, dc = ops.dense_cells(grid, 10, out=(bufs.keys[n:], bufs.counts[n:]))
        t0 = mark("dense_cells", t0)
        # the route at 8 owners (1024 route digits), timed alone: the sender's
        # side of a world-size-8 step
        m2, bufs = device.count_device(lat, lon, None, 0, 18, 0, buffers=bufs)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        ops.route_pieces(bufs.keys[:m2], bufs.counts[:m2], 8, 10, multigpu.route_bits(8), _lib.HM_CELLS_REC10)
        t0 = mark("route_ws8", t0)
        t["cells"] = int(m)
        t["sent"] = int(both[0, :, 0].sum())
        t["owned"] = int(n + dk.numel())
        res = t
    print(json.dumps(res), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
