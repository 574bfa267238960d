#!/usr/bin/env python3
"""Benchmark: points binned/s over zooms 0-18 on Gaussian-hotspot point clouds.

BASELINE.json metric: "points binned/sec (whole node, zooms 0-18) + % HBM
roofline".  One step = one hm_count() over the resident cloud: projection of
every point at zoom 18 (bit-exact with reference tile.py:15-21), the count
pyramid for zooms 0..18 (heatmap.py:107-111 semantics), every non-empty cell
written to HBM as (key, count).

    python bench.py                                   # 1 GPU, 1e9 points (config 2)
    python -m torch.distributed.run --nproc-per-node N bench.py --gpus N
        # N GPUs, 1.25e9 points per GPU (config 3 at N=8: 1e10), weak scaling:
        # each rank bins its shard, then the sparse cells are hash-partitioned
        # by heatmap row over RCCL all-to-all and merged

With N > 1 ranks the steps are pipelined: step k's exchange and merge run on a
second HIP stream (and host thread) while step k+1 counts, so the per-step time
is the host clock over the K steps (each step's merge ends before the final
barrier).

Rank 0 prints one JSON line.  `roofline` is for the whole step, the unit the
metric is quoted on: achieved = algorithmic bytes of one step (16 B per point
read + 16 B per non-empty output cell) / the step's average
duration from HIP events recorded on the library's stream around the timed
steps, against the 8 TB/s HBM3E peak; `traffic` is the HBM bytes of one step
from the committed rocprofv3 PMC summary (profiles/pmc_summary.json, FETCH_SIZE
doubled per the gfx950 correction + WRITE_SIZE), or null.  `kernels` breaks the
step down by stage from the library's own HIP events (hm_last_stats).
`cpu_baseline` times the C oracle (oracle/hm_oracle.c, OpenMP) on a bounded
sample of the same generator on this host's cores.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

HBM_PEAK_GBS = 8000.0      # MI355X HBM3E spec (MI355X_MICROARCH.md)
ALG_BYTES_PER_POINT = 16   # lat + lon fp64 read once
ALG_BYTES_PER_CELL = 16    # u64 key + u64 count per non-empty output cell


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--points", type=float, default=0, help="points per GPU (default 1e9, or 1.25e9 when N>1)")
    ap.add_argument("--kind", default="hotspots", choices=["hotspots", "uniform", "skew"])
    ap.add_argument("--zmin", type=int, default=0)
    ap.add_argument("--zmax", type=int, default=18)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--cpu-sample", type=float, default=2e8,
                    help="points timed on the CPU oracle, ~10-30 s of host work (0 = skip)")
    ap.add_argument("--no-check", action="store_true")
    ap.add_argument("--force-dist", action="store_true",
                    help="run the RCCL merge path even with one rank (rehearsal of the N>1 code)")
    return ap.parse_args()


def dist_init(args):
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    args.dist = ws > 1 or args.force_dist
    if args.dist:
        import torch.distributed as dist

        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("nccl")
    return ws, rank, local


def barrier(ws):
    import torch.distributed as dist

    if dist.is_available() and dist.is_initialized():
        import torch.distributed as dist

        dist.barrier()


def profile_traffic(workload_tag):
    """HBM bytes of one hm_count step from the committed PMC summary."""
    path = os.path.join(REPO, "profiles", "pmc_summary.json")
    if not os.path.exists(path):
        return None, None
    try:
        with open(path) as f:
            d = json.load(f)
        e = d.get(workload_tag)
        if not e:
            return None, None
        return e.get("hbm_bytes_per_step"), os.path.relpath(path, REPO)
    except Exception:
        return None, None


def cpu_baseline(args, lat_dev=None, lon_dev=None):
    """Time the C oracle on a bounded sample: the first `cpu_sample` points of
    the same cloud (copied from HBM when given -- hm_synth is bit-identical to
    heatmap_amd.synth -- else generated on the host)."""
    if args.cpu_sample <= 0:
        return None
    from heatmap_amd import synth
    from oracle import oracle

    n = int(args.cpu_sample)
    if lat_dev is not None and lat_dev.numel() >= n:
        lat = lat_dev[:n].cpu().numpy()
        lon = lon_dev[:n].cpu().numpy()
    else:
        lat, lon = synth.generate(args.kind, n, seed=args.seed)
    t0 = time.perf_counter()
    r = oracle.count(lat, lon, None, args.zmin, args.zmax)
    dt = time.perf_counter() - t0
    assert r["status"] == 0
    return {"value": n / dt, "unit": "points/s", "cores": int(r["threads"]), "kind": "port",
            "sample": "first %d of the %s points (seed %d), zooms %d-%d; C oracle (glibc projection, OpenMP x%d; "
                      "serial radix sort + RLE cascade), %.1f s"
                      % (n, args.kind, args.seed, args.zmin, args.zmax, int(r["threads"]), dt)}


def main():
    args = parse()
    ws, rank, local = dist_init(args)
    import torch

    from heatmap_amd import device, synth
    from heatmap_amd import multigpu

    torch.cuda.set_device(local)
    per = int(args.points) if args.points else (1_000_000_000 if ws == 1 else 1_250_000_000)
    lat = torch.empty(per, dtype=torch.float64, device="cuda")
    lon = torch.empty(per, dtype=torch.float64, device="cuda")
    device.synth(args.kind, lat, lon, seed=args.seed, start=rank * per)
    torch.cuda.synchronize()
    bufs = device.CountBuffers(64 << 20)
    ctx = device.context(local)

    def step():
        m, b = device.count_device(lat, lon, None, args.zmin, args.zmax, local, buffers=bufs)
        if args.dist:
            m = multigpu.merge_cells(b, m, ws, rank)
        return m, b

    if args.dist:
        # steps pipelined over two buffer sets: step k's exchange and merge
        # (RCCL + merge kernels, their own HIP stream and host thread) run
        # while step k+1 counts; every step's merge ends inside the timed region
        bufsets = [bufs, device.CountBuffers(64 << 20)]
        m, stages, _ = multigpu.pipelined_steps(
            lambda b: device.count_device(lat, lon, None, args.zmin, args.zmax, local, buffers=b),
            bufsets, args.warmup, ws, rank, ctx)
        torch.cuda.synchronize()
        barrier(ws)
        t0 = time.perf_counter()
        m, stages, bufs = multigpu.pipelined_steps(
            lambda b: device.count_device(lat, lon, None, args.zmin, args.zmax, local, buffers=b),
            bufsets, args.steps, ws, rank, ctx)
        torch.cuda.synchronize()
        barrier(ws)
        dt = time.perf_counter() - t0
        step_ms_ev = dt / args.steps * 1e3     # host clock: the steps overlap across two streams
    else:
        for _ in range(args.warmup):
            m, bufs = step()
        torch.cuda.synchronize()
        barrier(ws)
        stages = []
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        ev0.record()
        for _ in range(args.steps):
            m, bufs = step()
            _, us = ctx.last_stats()
            stages.append(us[:5])
        ev1.record()
        torch.cuda.synchronize()
        barrier(ws)
        dt = time.perf_counter() - t0
        step_ms_ev = ev0.elapsed_time(ev1) / args.steps
    if args.dist:
        import torch.distributed as dist

        t = torch.tensor([dt, float(m)], dtype=torch.float64, device="cuda")
        dist.all_reduce(t[:1], op=dist.ReduceOp.MAX)
        dist.all_reduce(t[1:], op=dist.ReduceOp.SUM)
        dt, cells = float(t[0]), int(t[1])
    else:
        cells = int(m)
    check = None
    if not args.no_check:
        # every zoom's counts sum to the number of points (over all ranks' owned cells)
        tot_t = bufs.counts[:m].sum().reshape(1)
        if args.dist:
            import torch.distributed as dist

            dist.all_reduce(tot_t)
        tot = int(tot_t.item())
        check = "ok" if tot == per * ws * (args.zmax - args.zmin + 1) else "FAIL sum %d" % tot
    ms = dt / args.steps * 1e3
    total_points = per * ws
    st = np.mean(np.array(stages), axis=0)
    tag = "%s_%d_z%d-%d" % (args.kind, per, args.zmin, args.zmax)
    traffic, traffic_src = profile_traffic(tag)
    alg_step = ALG_BYTES_PER_POINT * per + ALG_BYTES_PER_CELL * (cells // ws)      # one rank's step
    achieved = alg_step / (step_ms_ev * 1e-3) / 1e9
    kernels = {
        "k_project_partition": {"us": float(st[0]), "alg_bytes": ALG_BYTES_PER_POINT * per,
                                "GBps": ALG_BYTES_PER_POINT * per / (st[0] * 1e-6) / 1e9 if st[0] else None},
        "k_partition (levels >= 2)": {"us": float(st[4])},
        "level buckets, run scans, compaction, host syncs": {"us": float(st[1] - st[4])},
        "final aggregation (k_aggregate + sparse/small/merged)": {"us": float(st[2])},
        "k_pool": {"us": float(st[3])},
    }
    out = {
        "metric": "points binned/sec (whole node, zooms 0-18) + % HBM roofline at 1/2/4/8 GPU",
        "value": total_points / (dt / args.steps),
        "unit": "points/s",
        "n_gpus": ws,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (heatmap_amd.synth %s, generated on device, resident in HBM)" % args.kind,
        "config": {"workload": "%.3g %s points per GPU, zooms %d-%d, %d x MI355X" % (per, args.kind, args.zmin,
                                                                                    args.zmax, ws),
                   "points_per_gpu": per, "zmin": args.zmin, "zmax": args.zmax,
                   "partition_levels": int(ctx.last_stats()[1][7]),
                   "parallelism": "points sharded, dp%d" % ws},
        "roofline": {"bound": "hbm", "kernel": "hm_count step (all pipeline kernels, one rank)",
                     "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS,
                     "traffic": traffic, "traffic_source": traffic_src, "avg_launch_us": step_ms_ev * 1e3,
                     "alg_bytes_per_launch": alg_step, "cells_per_step": cells // ws},
        "kernels": kernels,
        "pipeline": {"slow_path_points": ctx.last_stats()[0], "check": check},
    }
    if rank == 0:
        out["cpu_baseline"] = cpu_baseline(args, lat, lon)
        print(json.dumps(out), flush=True)
    barrier(ws)


if __name__ == "__main__":
    main()
