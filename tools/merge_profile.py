#!/usr/bin/env python3
"""Phase timing of the multi-GPU merge (heatmap_amd.multigpu.merge_cells) on one
GPU with a world-size-1 RCCL group: count 1.25e9 hotspot points (the N>1 bench
shard), then time route, reduce, all-to-all, merge, dense extraction and the
exotic step separately (synchronised).  Prints one JSON line.

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

from heatmap_amd import device, multigpu  # noqa: E402


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
        grid, parts, sent, wide = ops.route(keys, counts, 1, 10, narrow=True)
        assert not wide
        rec = parts[0][0]
        t0 = mark("route", t0)
        dist.reduce(grid, dst=0)
        t0 = mark("reduce", t0)
        send = torch.tensor(sent, dtype=torch.int64, device="cuda")
        recv = torch.empty_like(send)
        dist.all_to_all_single(recv, send)
        rl = recv.tolist()
        nrec = torch.empty(sum(rl) * 10, dtype=torch.uint8, device="cuda")
        dist.all_to_all_single(nrec, rec, [x * 10 for x in rl], [x * 10 for x in sent])
        t0 = mark("all_to_all", t0)
        uk, uc = ops.merge(nrec, None, rl)
        t0 = mark("merge", t0)
        dk, dc = ops.dense_cells(grid, 10)
        t0 = mark("dense_cells", t0)
        k = torch.cat([uk, dk])
        c = torch.cat([uc, dc])
        bufs.keys[:k.numel()] = k
        bufs.counts[:k.numel()] = c
        t0 = mark("cat_copy", t0)
        nx_all = torch.tensor([int(bufs.nx)], dtype=torch.int64, device="cuda")
        dist.all_reduce(nx_all)
        t0 = mark("exotic_check", t0)
        t["cells"] = int(m)
        t["sent"] = int(sum(sent))
        t["owned"] = int(k.numel())
        res = t
    print(json.dumps(res), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
