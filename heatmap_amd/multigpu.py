"""Multi-GPU merge of per-rank cell counts (one process per GPU, RCCL over xGMI).

Points shard by contiguous ranges; each rank bins its shard with hm_count
(heatmap_amd.device.count_device).  The only exchange in the whole path is
the sum of per-cell counts -- what Spark's two shuffles compute in the
reference (reduceByKey at heatmap.py:111, groupByKey at :112):

  dense zooms 0..dense_zmax   every rank scatters its cells into one dense
                              Morton-ordered u64 grid (sum 4^z cells, 11 MB at
                              dense_zmax = 10) and the grids are summed with
                              one all_reduce;
  sparse zooms above it       cells are hash-partitioned by their heatmap row
                              (zoom, row >> 5, col >> 5) -- the groupByKey key
                              -- and exchanged with one all_to_all (counts
                              first, then keys and counts); owners merge what
                              they receive by sort + segmented sum.

Every output cell, and every heatmap row, ends with exactly one owner rank:
dense cells are kept by the rank the same row hash names.  torch.distributed
is the plumbing ("nccl" = RCCL on ROCm; "gloo" in the CPU tests).
"""
from __future__ import annotations

import torch
import torch.distributed as dist

DELTA = 5
_MASK29 = 0x1FFFFFFF


def _split(keys: torch.Tensor):
    return keys >> 58, (keys >> 29) & _MASK29, keys & _MASK29


def owner(keys: torch.Tensor, ws: int) -> torch.Tensor:
    """Rank that owns each cell: multiplicative hash of its heatmap-row key."""
    z, r, c = _split(keys)
    rk = (z << 48) ^ ((r >> DELTA) << 24) ^ (c >> DELTA)
    h = (rk * -7046029254386353131) >> 33          # wrapping int64 multiply
    return torch.remainder(h, ws)


def _spread(v: torch.Tensor) -> torch.Tensor:
    v = v & 0xFFFFFFFF
    v = (v | (v << 16)) & 0x0000FFFF0000FFFF
    v = (v | (v << 8)) & 0x00FF00FF00FF00FF
    v = (v | (v << 4)) & 0x0F0F0F0F0F0F0F0F
    v = (v | (v << 2)) & 0x3333333333333333
    v = (v | (v << 1)) & 0x5555555555555555
    return v


def _compact(v: torch.Tensor) -> torch.Tensor:
    v = v & 0x5555555555555555
    v = (v | (v >> 1)) & 0x3333333333333333
    v = (v | (v >> 2)) & 0x0F0F0F0F0F0F0F0F
    v = (v | (v >> 4)) & 0x00FF00FF00FF00FF
    v = (v | (v >> 8)) & 0x0000FFFF0000FFFF
    v = (v | (v >> 16)) & 0x00000000FFFFFFFF
    return v


def _zoom_offsets(dz: int):
    off, o = [], 0
    for z in range(dz + 1):
        off.append(o)
        o += 1 << (2 * z)
    return off, o


def _dense_merge(keys, counts, dz, ws, rank):
    off, total = _zoom_offsets(dz)
    offt = torch.tensor(off, dtype=torch.int64, device=keys.device)
    z, r, c = _split(keys)
    idx = offt[z] + ((_spread(r) << 1) | _spread(c))
    grid = torch.zeros(total, dtype=torch.int64, device=keys.device)
    grid.index_add_(0, idx, counts)
    dist.all_reduce(grid)
    nz = torch.nonzero(grid).flatten()
    zc = torch.bucketize(nz, offt, right=True) - 1
    m = nz - offt[zc]
    k = (zc << 58) | (_compact(m >> 1) << 29) | _compact(m)
    mine = owner(k, ws) == rank
    return k[mine], grid[nz][mine]


def merge_cells(buffers, m: int, ws: int, rank: int, dense_zmax: int = 10) -> int:
    """Exchange and merge the first m cells of `buffers` (int64 keys/counts,
    HM_KEY layout) in place; returns the number of cells this rank owns.
    dense_zmax < 0 sends every zoom through the all-to-all."""
    keys = buffers.keys[:m]
    counts = buffers.counts[:m]
    parts_k, parts_c = [], []
    if dense_zmax >= 0:
        zk = keys >> 58
        dm = zk <= dense_zmax
        dk, dc = _dense_merge(keys[dm], counts[dm], dense_zmax, ws, rank)
        parts_k.append(dk)
        parts_c.append(dc)
        keys, counts = keys[~dm], counts[~dm]
    own = owner(keys, ws)
    order = torch.argsort(own)
    keys = keys[order]
    counts = counts[order]
    send = torch.bincount(own, minlength=ws)
    recv = torch.empty_like(send)
    dist.all_to_all_single(recv, send)
    sl, rl = send.tolist(), recv.tolist()
    nk = torch.empty(sum(rl), dtype=torch.int64, device=keys.device)
    nc = torch.empty_like(nk)
    dist.all_to_all_single(nk, keys, rl, sl)
    dist.all_to_all_single(nc, counts, rl, sl)
    uk, inv = torch.unique(nk, sorted=True, return_inverse=True)
    tot = torch.zeros(uk.numel(), dtype=torch.int64, device=keys.device)
    tot.index_add_(0, inv, nc)
    parts_k.append(uk)
    parts_c.append(tot)
    k = torch.cat(parts_k)
    c = torch.cat(parts_c)
    n = k.numel()
    if n > buffers.keys.numel():
        raise MemoryError("merge_cells: %d owned cells exceed the buffer capacity %d" % (n, buffers.keys.numel()))
    buffers.keys[:n] = k
    buffers.counts[:n] = c
    return n
