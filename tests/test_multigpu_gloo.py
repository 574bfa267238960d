"""CPU, world_size 2 over gloo: the multi-GPU merge (heatmap_amd/multigpu.py).

Each rank bins its contiguous shard of the points (here with the oracle, the
device's stand-in off-GPU), exchanges cells with merge_cells, and the union of
what the ranks own must equal the single-process count of all points -- the
sum Spark's reduceByKey / groupByKey shuffles compute (heatmap.py:111-112).
The three device operations (hm_cells_route / hm_cells_merge /
hm_dense_cells) are replaced by the torch stand-ins below, which follow the
same contract; the collectives and the exchange logic are the product's.
The device kernels themselves run in tests/test_gpu_multigpu.py.
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

M29 = 0x1FFFFFFF


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _spread(v):
    v = v & 0xFFFFFFFF
    for sh, m in ((16, 0x0000FFFF0000FFFF), (8, 0x00FF00FF00FF00FF), (4, 0x0F0F0F0F0F0F0F0F),
                  (2, 0x3333333333333333), (1, 0x5555555555555555)):
        v = (v | (v << sh)) & m
    return v


def _compact(v):
    v = v & 0x5555555555555555
    for sh, m in ((1, 0x3333333333333333), (2, 0x0F0F0F0F0F0F0F0F), (4, 0x00FF00FF00FF00FF),
                  (8, 0x0000FFFF0000FFFF), (16, 0x00000000FFFFFFFF)):
        v = (v | (v >> sh)) & m
    return v


class TorchOps:
    """CPU stand-ins with the contract of hm_cells_route / hm_cells_merge /
    hm_dense_cells (include/heatmap_amd.h)."""

    @staticmethod
    def route(keys, counts, ws, dz, narrow=False):
        z, r, c = keys >> 58, (keys >> 29) & M29, keys & M29
        gsz = ((1 << (2 * (dz + 1))) - 1) // 3 if dz >= 0 else 0
        grid = torch.zeros(gsz, dtype=torch.int64)
        dense = z <= dz
        if dz >= 0 and dense.any():
            zz = z[dense]
            idx = ((1 << (2 * zz)) - 1) // 3 + ((_spread(r[dense]) << 1) | _spread(c[dense]))
            grid.index_add_(0, idx, counts[dense])
        sk, sc = keys[~dense], counts[~dense]
        rec = torch.stack([sk >> 58, (sk >> 29) & M29, sk & M29], 1)
        own = multigpu.record_owner(rec, ws)
        o = torch.argsort(own, stable=True)
        # a count past 32 bits, or a key past the record's 48 (zoom > 21, row or col >= 2^21)
        zk, rk, ck = sk >> 58, (sk >> 29) & M29, sk & M29
        wide = narrow and bool((sc >> 32).any() or (zk > 21).any() or (rk >= 1 << 21).any() or (ck >= 1 << 21).any())
        parts = [(multigpu.pack_records(sk[o], sc[o]), 10)] if narrow else [(sk[o], 1), (sc[o], 1)]
        return grid, parts, torch.bincount(own, minlength=ws).tolist(), wide

    @staticmethod
    def route_grouped(keys, gcounts, ws):
        g = gcounts >> 32
        z, r, c = keys >> 58, (keys >> 29) & M29, keys & M29
        wide = bool((g >= 1 << multigpu.GKEY_GROUP_BITS).any() or (z > 21).any())
        own = multigpu.grouped_owner(keys, g, ws)
        o = torch.argsort(own, stable=True)
        mk = (g << 47) | (z << 42) | (r << 21) | c
        return [(mk[o], 1), ((gcounts & 0xFFFFFFFF)[o].to(torch.int32), 1)], torch.bincount(own, minlength=ws).tolist(), wide

    @staticmethod
    def merge(keys, counts=None, runs=None):
        if counts is None:                      # HM_CELLS_REC10 records
            keys, counts = multigpu.unpack_records(keys)
        u, inv = torch.unique(keys, return_inverse=True)
        t = torch.zeros(u.numel(), dtype=torch.int64)
        t.index_add_(0, inv, counts.to(torch.int64))
        return u, t

    @staticmethod
    def dense_cells(grid, dz, out=None):
        nz = torch.nonzero(grid).flatten()
        off = torch.tensor([((1 << (2 * z)) - 1) // 3 for z in range(dz + 1)], dtype=torch.int64)
        zc = torch.bucketize(nz, off, right=True) - 1
        m = nz - off[zc]
        return _into(out, (zc << 58) | (_compact(m >> 1) << 29) | _compact(m), grid[nz])

    @staticmethod
    def route_pieces(keys, counts, ws, dz, bits, layout, extra=1, self_rank=-1):
        """hm_cells_route_pieces: owner groups ordered by the top `bits` bits
        of fmix64(merge key), in rank order or (self_rank >= 0) with that
        owner's group last; sizes rows (sent, wide, pieces, extra zeros) by owner."""
        from heatmap_amd import _lib

        grouped = layout == _lib.HM_CELLS_G12
        if grouped:
            g = counts >> 32
            z, r, c = keys >> 58, (keys >> 29) & M29, keys & M29
            wide = bool((g >= 1 << multigpu.GKEY_GROUP_BITS).any() or (z > 21).any())
            own = multigpu.grouped_owner(keys, g, ws)
            mk, cnt = (g << 47) | (z << 42) | (r << 21) | c, (counts & 0xFFFFFFFF).to(torch.int32)
            grid = torch.zeros(0, dtype=torch.int64)
        else:
            narrow = layout == _lib.HM_CELLS_REC10
            grid, parts, _, wide = TorchOps.route(keys, counts, ws, dz, narrow)
            sp = (keys >> 58) > dz
            mk, cnt = keys[sp], counts[sp]
            own = multigpu.record_owner(torch.stack([mk >> 58, (mk >> 29) & M29, mk & M29], 1), ws)
        h = _lsr(_fmix64(mk), 64 - bits) if bits else torch.zeros_like(own)
        pos = own if self_rank < 0 else torch.where(own == self_rank, ws - 1, own - (own > self_rank).to(own.dtype))
        o = torch.argsort((pos << bits) | h, stable=True)
        S = 1 << bits
        sizes = torch.zeros((ws, 2 + S + extra), dtype=torch.int64)
        sizes[:, 0] = torch.bincount(own, minlength=ws)
        sizes[:, 1] = int(wide)
        sizes[:, 2:2 + S] = torch.bincount((own << bits) | h, minlength=ws << bits).reshape(ws, S)
        if layout == _lib.HM_CELLS_REC10:
            parts = [(multigpu.pack_records(mk[o], cnt[o]), 10)]
        else:
            parts = [(mk[o], 1), (cnt[o], 1)]
        return grid, parts, sizes

    @staticmethod
    def merge_pieces(runs, pieces, bits, layout, out=None):
        from heatmap_amd import _lib

        ks, cs = [], []
        for (kt, ct, start), row in zip(runs, pieces):
            n = int(sum(row))
            if layout == _lib.HM_CELLS_REC10:
                k, c = multigpu.unpack_records(kt[start * 10:(start + n) * 10])
            else:
                k, c = kt[start:start + n], ct[start:start + n].to(torch.int64)
            ks.append(k)
            cs.append(c)
        u, t = TorchOps.merge(torch.cat(ks), torch.cat(cs))
        return _into(out, u, t)


def _into(out, k, c):
    if out is None:
        return k, c
    n = k.numel()
    if n > out[0].numel():
        raise MemoryError("merge_cells: %d owned cells exceed the buffer capacity %d" % (n, out[0].numel()))
    out[0][:n] = k
    out[1][:n] = c
    return out[0][:n], out[1][:n]


def _lsr(v, s):
    return (v >> s) & ((1 << (64 - s)) - 1)


def _fmix64(k):
    """hms_hash (MurmurHash3's fmix64) on int64 bits, wrapping multiplies."""
    k = k ^ _lsr(k, 33)
    k = k * (0xFF51AFD7ED558CCD - (1 << 64))
    k = k ^ _lsr(k, 33)
    k = k * (0xC4CEB9FE1A85EC53 - (1 << 64))
    return k ^ _lsr(k, 33)


class _Bufs:
    def __init__(self, keys, counts, xcells, cap):
        self.keys = torch.zeros(cap, dtype=torch.int64)
        self.counts = torch.zeros(cap, dtype=torch.int64)
        self.keys[: len(keys)] = torch.from_numpy(keys)
        self.counts[: len(counts)] = torch.from_numpy(counts)
        self.xcells = torch.from_numpy(xcells.reshape(-1).copy())
        self.nx = xcells.shape[0]


def _split(ref):
    z, r, c, n = ref["zoom"].astype(np.int64), ref["row"], ref["col"], ref["count"]
    sq = (r >= 0) & (r < (1 << z)) & (c >= 0) & (c < (1 << z))
    keys = (z[sq] << 58) | (r[sq] << 29) | c[sq]
    x = np.stack([z[~sq], r[~sq], c[~sq], n[~sq]], 1)
    return keys, n[sq], x


def _cloud(kind, n, start):
    lat, lon = synth.generate(kind, n, seed=2, start=start)
    lat, lon = lat.copy(), lon.copy()
    lat[::997] = 88.0 + (np.arange(lat[::997].size) % 7) * 0.2     # kept points outside the square
    lon[5::1009] = 200.0
    return lat, lon


def _worker(rank, ws, port, kind, n, zmin, zmax, dense_zmax, out, wide_rank=1):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=ws)
    per = n // ws
    lat, lon = _cloud(kind, per, rank * per)
    k, c, x = _split(oracle.count(lat, lon, None, zmin, zmax))
    if kind == "skew" and rank == wide_rank:
        # one rank's count of one sparse cell past 2^32: every rank routes its
        # counts as int64 (the flag rides on the group-size exchange)
        j = int(np.nonzero((k >> 58) > dense_zmax)[0][0])
        c = c.copy()
        c[j] += 1 << 32
    b = _Bufs(k, c, x, 4 * len(k) + 64)
    m = multigpu.merge_cells(b, len(k), ws, rank, dense_zmax=dense_zmax, ops=TorchOps())
    out[rank] = (b.keys[:m].numpy().copy(), b.counts[:m].numpy().copy(), b.xcells[:4 * b.nx].numpy().copy())
    dist.destroy_process_group()


@pytest.mark.parametrize("ws,kind,zmax,dense_zmax", [(2, "hotspots", 18, 8), (2, "uniform", 12, -1),
                                                      (2, "skew", 18, 10), (4, "hotspots", 16, 10), (1, "hotspots", 14, 8),
                                                      (4, "skew", 18, 8)])
def test_merge_ranks(ws, kind, zmax, dense_zmax):
    """ws gloo ranks (CPU stand-ins of the device operations): the union of
    the owned cells equals one count; with ws = 4 the owner hash spreads over
    four ranks and (skew) rank ws - 1 forces every rank onto the int64 route
    (HM_E_WIDE agreement)."""
    n, zmin = 60000, 0
    wide_rank = ws - 1
    mgr = mp.Manager()
    out = mgr.dict()
    mp.start_processes(_worker, args=(ws, _port(), kind, n, zmin, zmax, dense_zmax, out, wide_rank), nprocs=ws,
                       join=True, start_method="spawn")
    keys = np.concatenate([out[r][0] for r in range(ws)])
    counts = np.concatenate([out[r][1] for r in range(ws)])
    xs = np.concatenate([out[r][2].reshape(-1, 4) for r in range(ws)])
    assert len(np.unique(keys)) == len(keys)            # every cell has exactly one owner
    if ws > 2:
        assert all(len(out[r][0]) > 0 for r in range(ws))   # the owner hash reaches every rank
    lat = np.concatenate([_cloud(kind, n // ws, r * (n // ws))[0] for r in range(ws)])
    lon = np.concatenate([_cloud(kind, n // ws, r * (n // ws))[1] for r in range(ws)])
    rk, rc, rx = _split(oracle.count(lat, lon, None, zmin, zmax))
    if kind == "skew":                                  # the count rank wide_rank raised past 2^32
        k1, _, _ = _split(oracle.count(*_cloud(kind, n // ws, wide_rank * (n // ws)), None, zmin, zmax))
        rc[np.searchsorted(rk, k1[(k1 >> 58) > dense_zmax][0])] += 1 << 32
    o, ro = np.argsort(keys), np.argsort(rk)
    assert np.array_equal(keys[o], rk[ro])
    assert np.array_equal(counts[o], rc[ro])
    assert len(rx) > 0
    xo = np.lexsort((xs[:, 2], xs[:, 1], xs[:, 0]))
    rxo = np.lexsort((rx[:, 2], rx[:, 1], rx[:, 0]))
    assert np.array_equal(xs[xo], rx[rxo])


def test_records_round_trip():
    """HM_CELLS_REC10 packing (the exchange's 10-byte cells): keys of zooms
    0..21 at their extreme rows/columns and counts up to 2^32 - 1."""
    g = torch.Generator().manual_seed(7)
    z = torch.arange(22, dtype=torch.int64).repeat(50)
    lim = (1 << z) - 1
    r = torch.where(torch.arange(z.numel()) % 2 == 0, lim, torch.randint(0, 1 << 21, z.shape, generator=g) & lim)
    c = torch.where(torch.arange(z.numel()) % 3 == 0, lim, torch.randint(0, 1 << 21, z.shape, generator=g) & lim)
    keys = (z << 58) | (r << 29) | c
    counts = torch.randint(1, 1 << 32, z.shape, generator=g, dtype=torch.int64)
    counts[:3] = torch.tensor([1, (1 << 32) - 1, 1 << 31])
    rec = multigpu.pack_records(keys, counts)
    assert rec.dtype == torch.uint8 and rec.numel() == 10 * keys.numel()
    k2, c2 = multigpu.unpack_records(rec)
    assert torch.equal(k2, keys) and torch.equal(c2, counts)


def _grouped_cells(lat, lon, grp, zmin, zmax):
    """(HM_KEY keys, groups, counts) per (group, zoom, row, col): the oracle's
    projection at zmax and every coarser zoom by the shift (the oracle's own
    pyramid is pinned in tests/test_oracle.py; this is the exchange's input)."""
    r, c, st, _ = oracle.project(lat, lon, zmax)
    assert (st == 0).all()
    ks = []
    for z in range(zmin, zmax + 1):
        ks.append((np.int64(z) << 58) | ((r >> (zmax - z)) << 29) | (c >> (zmax - z)))
    k = np.concatenate(ks)
    g = np.tile(grp.astype(np.int64), zmax - zmin + 1)
    u, cnt = np.unique(np.stack([g, k], 1), axis=0, return_counts=True)
    return u[:, 1], u[:, 0], cnt.astype(np.int64)


def _grouped_worker(rank, ws, port, n, zmin, zmax, users, out):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=ws)
    per = n // ws
    lat, lon = synth.generate("hotspots", per, seed=3, start=rank * per)
    grp = ((np.arange(rank * per, (rank + 1) * per) * 2654435761) >> 7) % users
    k, g, c = _grouped_cells(lat, lon, grp, zmin, zmax)   # stands in for hm_count_grouped_packed
    k, g, c = multigpu.merge_grouped(torch.from_numpy(k), torch.from_numpy((g << 32) | c), ws, rank, ops=TorchOps())
    out[rank] = (k.numpy().copy(), g.numpy().copy(), c.numpy().copy())
    dist.destroy_process_group()


@pytest.mark.parametrize("ws,users", [(2, 7), (2, 100_000), (2, 200_000), (3, 50)])
def test_merge_grouped_ranks(ws, users):
    """Grouped cells (hm_count_grouped_packed's records) exchanged over ws gloo
    ranks: every (group, cell) has one owner, the owner is the hash of (group,
    heatmap row), and the union equals one per-group count of all points;
    100,000 users put group ids in [2^16, 2^17) through the packed exchange (the
    merge key's top bit set: the decode must not sign-extend it); 200,000
    users pass the merge key's 2^17 groups, so every rank takes the
    int64-record exchange."""
    n, zmin, zmax = 24000, 6, 21
    mgr = mp.Manager()
    out = mgr.dict()
    mp.start_processes(_grouped_worker, args=(ws, _port(), n, zmin, zmax, users, out), nprocs=ws, join=True,
                       start_method="spawn")
    ks = np.concatenate([out[r][0] for r in range(ws)])
    gs = np.concatenate([out[r][1] for r in range(ws)])
    cs = np.concatenate([out[r][2] for r in range(ws)])
    for r in range(ws):
        own = multigpu.grouped_owner(torch.from_numpy(out[r][0]), torch.from_numpy(out[r][1]), ws)
        assert bool((own == r).all())
    per = n // ws
    lat, lon = synth.generate("hotspots", per * ws, seed=3)
    grp = ((np.arange(per * ws) * 2654435761) >> 7) % users
    ek, eg, ec = _grouped_cells(lat, lon, grp, zmin, zmax)
    o = np.lexsort((ks, gs))
    assert np.array_equal(gs[o], eg) and np.array_equal(ks[o], ek) and np.array_equal(cs[o], ec)
