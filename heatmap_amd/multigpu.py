"""Multi-GPU merge of per-rank cell counts (one process per GPU, RCCL).

Points shard by contiguous ranges; each rank bins its shard with hm_count.
The only exchange is the sum of cell counts: cells are hash-partitioned by
their heatmap row (zoom, row >> 5, col >> 5) -- the key Spark's groupByKey
shuffles on (reference heatmap.py:112) -- so every output row has one owner,
and sent with one RCCL all-to-all (torch.distributed "nccl" = RCCL over
xGMI).  Owners merge what they receive.
"""
from __future__ import annotations

import torch
import torch.distributed as dist

DELTA = 5


def _owner(keys: torch.Tensor, ws: int) -> torch.Tensor:
    z = keys >> 58
    r = (keys >> 29) & 0x1FFFFFFF
    c = keys & 0x1FFFFFFF
    rk = (z << 48) ^ ((r >> DELTA) << 24) ^ (c >> DELTA)
    h = (rk * -7046029254386353131) >> 33          # multiplicative hash (wrapping int64)
    return torch.remainder(h, ws)


def merge_cells(buffers, m: int, ws: int, rank: int) -> int:
    """Exchange and merge the first m cells of `buffers` in place; returns the
    number of cells this rank owns after the merge."""
    keys = buffers.keys[:m]
    counts = buffers.counts[:m]
    own = _owner(keys, ws)
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
    n = uk.numel()
    buffers.keys[:n] = uk
    buffers.counts[:n] = tot
    return n
