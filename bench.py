#!/usr/bin/env python3
"""Benchmark: points binned/s over zooms 0-18 on Gaussian-hotspot point clouds.

BASELINE.json metric: "points binned/sec (whole node, zooms 0-18) + % HBM
roofline".  One step = one hm_count() over the resident cloud: projection of
every point at zoom 18 (bit-exact with reference tile.py:15-21), the count
pyramid for zooms 0..18 (heatmap.py:107-111 semantics), every non-empty cell
written to HBM as (key, count).

    python bench.py                                   # 1 GPU, 1e9 points (config 2)
    python bench.py --gpus N                          # spawns N ranks itself
    python -m torch.distributed.run --nproc-per-node N bench.py --gpus N
        # N GPUs, 1.25e9 points per GPU (config 3 at N=8: 1e10), weak scaling:
        # each rank bins its shard, then the sparse cells are hash-partitioned
        # by heatmap row over RCCL all-to-all and merged

`--gpus N` with no WORLD_SIZE in the environment starts N worker processes
(one per GPU, RANK/LOCAL_RANK/WORLD_SIZE/MASTER_* set) before anything touches
HIP, and exits with the first failing rank's status.  A launcher's WORLD_SIZE
that differs from --gpus, or fewer visible GPUs than ranks, is an error (exit
status 2): the line would otherwise claim a node it did not measure.

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


def _free_port():
    import socket

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def visible_gpus():
    """GPUs this process may use, counted without any HIP call (a HIP call
    here would initialise the runtime in the launcher before it starts the
    ranks): HIP_VISIBLE_DEVICES / ROCR_VISIBLE_DEVICES when set, else the KFD
    topology's nodes that have SIMDs (GPUs; CPU nodes report 0)."""
    for var in ("HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = os.environ.get(var)
        if v is not None:
            return len([x for x in v.split(",") if x.strip() != ""])
    root = "/sys/class/kfd/kfd/topology/nodes"
    n = 0
    try:
        for node in os.listdir(root):
            try:
                with open(os.path.join(root, node, "properties")) as f:
                    for line in f:
                        k, _, val = line.partition(" ")
                        if k == "simd_count" and int(val) > 0:
                            n += 1
            except OSError:
                pass
    except OSError:
        return None
    return n


def spawn(args):
    """--gpus N without a launcher: start N ranks of this script (no HIP call
    in this process: the GPUs are counted from the environment or the KFD
    topology), wait for all, and stop the others as soon as one fails (its
    peers would block in a collective).  Each rank also checks its own
    LOCAL_RANK against the devices it sees."""
    import subprocess

    dry = os.environ.get("HM_BENCH_DRY") == "1"     # CPU test of the spawn itself
    if not dry:
        nd = visible_gpus()
        if nd is not None and nd < args.gpus:
            print("bench.py: --gpus %d needs %d visible GPUs, found %d" % (args.gpus, args.gpus, nd),
                  file=sys.stderr, flush=True)
            return 2
    port = os.environ.get("MASTER_PORT") or str(_free_port())
    procs = []
    for r in range(args.gpus):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(args.gpus),
                   LOCAL_WORLD_SIZE=str(args.gpus), MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            c = p.poll()
            if c is None:
                continue
            live.remove(p)
            if c != 0 and rc == 0:
                rc = c
                for q in live:
                    q.kill()          # the exact child processes this call started
        if live:
            time.sleep(0.2)
    return rc


def dist_init(args):
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if ws != args.gpus:
        print("bench.py: WORLD_SIZE=%d but --gpus %d" % (ws, args.gpus), file=sys.stderr, flush=True)
        sys.exit(2)
    if os.environ.get("HM_BENCH_DRY") == "1":
        print(json.dumps({"rank": rank, "local_rank": local, "world_size": ws}), flush=True)
        sys.exit(0)
    args.dist = ws > 1 or args.force_dist
    import torch

    nd = torch.cuda.device_count()
    if local >= nd:
        print("bench.py: rank %d (local %d) has no GPU: %d visible" % (rank, local, nd), file=sys.stderr, flush=True)
        sys.exit(2)
    if args.dist:
        import torch.distributed as dist

        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    return ws, rank, local


def barrier(ws):
    import torch.distributed as dist

    if dist.is_available() and dist.is_initialized():
        import torch.distributed as dist

        dist.barrier()


def profile_traffic(workload_tag):
    """HBM bytes of one hm_count step and the executed fp64 VALU operations
    per point, from the committed PMC summary (tools/pmc_traffic.py)."""
    path = os.path.join(REPO, "profiles", "pmc_summary.json")
    if not os.path.exists(path):
        return None, None, None
    try:
        with open(path) as f:
            d = json.load(f)
        e = d.get(workload_tag)
        if not e:
            return None, None, None
        return e.get("hbm_bytes_per_step"), os.path.relpath(path, REPO), e.get("fp64")
    except Exception:
        return None, None, None


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
                      "OpenMP LSD radix sort + RLE zoom cascade), %.1f s"
                      % (n, args.kind, args.seed, args.zmin, args.zmax, int(r["threads"]), dt)}


def measured_peak(torch, lat, lon, ctx, reps=5):
    """HBM read peak on this GPU: the library's read-stream kernel
    (hm_bench_read, 16-B loads, K1's access shape) over the resident lat/lon
    (16 B per point, the bytes K1 must read), best of `reps` on the library's
    stream; plus torch's device copy of 4 GiB (read + write bytes / time) for
    comparison with the guide's 6.29 TB/s float4 copy."""
    sink = torch.zeros(4096, dtype=torch.int64, device="cuda")
    nbytes = lat.numel() * 8
    best = 0.0
    for _ in range(reps + 1):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        rc = ctx.L.hm_bench_read(ctx.ptr, lat.data_ptr(), lon.data_ptr(), nbytes, sink.data_ptr())
        e1.record()
        e1.synchronize()
        assert rc == 0, rc
        best = max(best, 2.0 * nbytes / (e0.elapsed_time(e1) * 1e-3) / 1e9)
    copy = 0.0
    a = torch.empty((4 << 30) // 8, dtype=torch.float64, device="cuda")
    b = torch.empty_like(a)
    a.fill_(1.0)
    b.copy_(a)
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        b.copy_(a)
        e1.record()
        e1.synchronize()
        copy = max(copy, 2.0 * a.numel() * 8 / (e0.elapsed_time(e1) * 1e-3) / 1e9)
    del a, b
    torch.cuda.empty_cache()
    return best, copy


def main():
    args = parse()
    if args.gpus < 1:
        print("bench.py: --gpus must be >= 1", file=sys.stderr)
        sys.exit(2)
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn(args))
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
        return device.count_device(lat, lon, None, args.zmin, args.zmax, local, buffers=bufs)

    dist_info = None
    reruns = None              # level-1 re-runs over the timed steps (single-rank path)
    if args.dist:
        import torch.distributed as dist

        # the same per-GPU workload without the exchange: what one rank alone
        # takes per step (the weak-scaling reference at this per-GPU size)
        for _ in range(args.warmup):
            m_local, bufs = step()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(args.steps):
            m_local, bufs = step()
        e1.record()
        e1.synchronize()
        local_ms = e0.elapsed_time(e1) / args.steps
        # steps pipelined over two buffer sets: step k's exchange and merge
        # (RCCL + merge kernels, their own HIP stream and host thread) run
        # while step k+1 counts; every step's merge ends inside the timed region
        bufsets = [bufs, device.CountBuffers(64 << 20)]
        merge_ms = []
        m, stages, _ = multigpu.pipelined_steps(
            lambda b: device.count_device(lat, lon, None, args.zmin, args.zmax, local, buffers=b),
            bufsets, args.warmup, ws, rank, ctx)
        torch.cuda.synchronize()
        barrier(ws)
        t0 = time.perf_counter()
        m, stages, bufs = multigpu.pipelined_steps(
            lambda b: device.count_device(lat, lon, None, args.zmin, args.zmax, local, buffers=b),
            bufsets, args.steps, ws, rank, ctx, merge_ms=merge_ms)
        torch.cuda.synchronize()
        barrier(ws)
        dt = time.perf_counter() - t0
        t = torch.tensor([dt, float(m), local_ms, float(np.mean(merge_ms)) if merge_ms else 0.0, float(m_local)],
                         dtype=torch.float64, device="cuda")
        tmax = t.clone()
        dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        dt, cells = float(tmax[0]), int(t[1])
        step_ms_ev = dt / args.steps * 1e3     # host clock, max over ranks: the steps overlap on two streams
        cells_rank = int(t[4]) // ws           # cells one rank's count emits (before the exchange)
        dist_info = {"points_per_gpu": per, "local_ms_per_step": float(tmax[2]),
                     "n1_rate_at_this_size": per / (float(tmax[2]) * 1e-3),
                     "merge_ms_per_step": float(tmax[3]), "merge_ms_mean_over_ranks": float(t[3]) / ws,
                     "efficiency_vs_local": float(tmax[2]) / step_ms_ev,
                     "note": "local = the same count on this rank's shard with no exchange (max over ranks): "
                             "n1_rate_at_this_size is the one-GPU rate at this per-GPU size (points/s); "
                             "merge = route + RCCL reduce/all-to-all + owner merge of one step, host clock on the "
                             "merge thread, overlapped with the next step's count"}
    else:
        for _ in range(args.warmup):
            m, bufs = step()
        torch.cuda.synchronize()
        stages = []
        reruns = 0
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        ev0.record()
        for _ in range(args.steps):
            m, bufs = step()
            _, us = ctx.last_stats()
            stages.append(us[:5])
            reruns += int(us[5])
        ev1.record()
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        step_ms_ev = ev0.elapsed_time(ev1) / args.steps
        cells = cells_rank = int(m)
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
    traffic, traffic_src, fp64 = profile_traffic(tag)
    peak_meas, copy_meas = measured_peak(torch, lat, lon, ctx)
    alg_step = ALG_BYTES_PER_POINT * per + ALG_BYTES_PER_CELL * cells_rank      # one rank's step
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
                     "alg_bytes_per_launch": alg_step, "cells_per_step": cells_rank,
                     "measured_peak": {"GBps": peak_meas, "frac": achieved / peak_meas,
                                       "how": "hm_bench_read: HIP read-stream kernel over the resident lat/lon "
                                              "(16-B loads, K1's access shape), best of 5",
                                       "torch_copy_GBps": copy_meas},
                     "fp64": fp64},
        "kernels": kernels,
        "pipeline": {"slow_path_points": ctx.last_stats()[0], "level1_reruns": reruns, "check": check},
    }
    if dist_info is not None:
        out["distributed"] = dist_info
    if rank == 0:
        out["cpu_baseline"] = cpu_baseline(args, lat, lon)
        print(json.dumps(out), flush=True)
    barrier(ws)


if __name__ == "__main__":
    main()
