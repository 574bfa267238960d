"""CPU, world_size 2 over gloo: the multi-GPU merge (heatmap_amd/multigpu.py).

Each rank bins its contiguous shard of the points (here with the oracle, the
device's stand-in off-GPU), exchanges cells with merge_cells, and the union of
what the ranks own must equal the single-process count of all points -- the
sum Spark's reduceByKey / groupByKey shuffles compute (heatmap.py:111-112).
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import oracle
from heatmap_amd import multigpu, synth


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


class _Bufs:
    def __init__(self, keys, counts, cap):
        self.keys = torch.zeros(cap, dtype=torch.int64)
        self.counts = torch.zeros(cap, dtype=torch.int64)
        self.keys[: len(keys)] = torch.from_numpy(keys)
        self.counts[: len(counts)] = torch.from_numpy(counts)


def _keys(z, r, c):
    return (z.astype(np.int64) << 58) | (r.astype(np.int64) << 29) | c.astype(np.int64)


def _worker(rank, ws, port, kind, n, zmin, zmax, dense_zmax, out):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=ws)
    per = n // ws
    lat, lon = synth.generate(kind, per, seed=2, start=rank * per)
    ref = oracle.count(lat, lon, None, zmin, zmax)
    k = _keys(ref["zoom"], ref["row"], ref["col"])
    b = _Bufs(k, ref["count"], 4 * len(k) + 64)
    m = multigpu.merge_cells(b, len(k), ws, rank, dense_zmax=dense_zmax)
    out[rank] = (b.keys[:m].numpy().copy(), b.counts[:m].numpy().copy())
    dist.destroy_process_group()


@pytest.mark.parametrize("kind,zmax,dense_zmax", [("hotspots", 18, 8), ("uniform", 12, -1), ("skew", 18, 10)])
def test_merge_two_ranks(kind, zmax, dense_zmax):
    ws, n, zmin = 2, 60000, 0
    mgr = mp.Manager()
    out = mgr.dict()
    mp.start_processes(_worker, args=(ws, _port(), kind, n, zmin, zmax, dense_zmax, out), nprocs=ws,
                       join=True, start_method="spawn")
    keys = np.concatenate([out[r][0] for r in range(ws)])
    counts = np.concatenate([out[r][1] for r in range(ws)])
    assert len(np.unique(keys)) == len(keys)            # every cell has exactly one owner
    o = np.argsort(keys)
    lat, lon = synth.generate(kind, n, seed=2)
    ref = oracle.count(lat, lon, None, zmin, zmax)
    rk = _keys(ref["zoom"], ref["row"], ref["col"])
    ro = np.argsort(rk)
    assert np.array_equal(keys[o], rk[ro])
    assert np.array_equal(counts[o], ref["count"][ro])
