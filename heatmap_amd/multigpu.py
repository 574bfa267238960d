"""Multi-GPU merge of per-rank cell counts (one process per GPU, RCCL over xGMI).

Points shard by contiguous ranges; each rank bins its shard with hm_count
(heatmap_amd.device.count_device).  The only exchange in the whole path is
the sum of per-cell counts -- what Spark's two shuffles compute in the
reference (reduceByKey at heatmap.py:111, groupByKey at :112):

  dense zooms 0..dense_zmax   hm_cells_route adds every rank's cells into one
                              dense Morton-ordered u64 grid (sum 4^z cells,
                              11 MB at dense_zmax = 10) and ONE RCCL reduce
                              sums the grids on rank 0, which owns those cells
                              (u64: at config 3's 1e10 points the zoom-0..9
                              cells pass 2^32);
  sparse zooms above it       hm_cells_route groups the cells by the rank that
                              owns their heatmap row (zoom, row >> 5, col >> 5)
                              -- the groupByKey key -- one RCCL all-to-all of
                              the group sizes, one of the keys and counts, and
                              hm_cells_merge sums equal keys on the owner;
  cells outside [0, 2^z)^2    (hm_count's records; rare) the same routing by
                              heatmap row, done with torch ops.

Every output cell, and every heatmap row, ends with exactly one owner rank.
torch.distributed is the plumbing ("nccl" = RCCL on ROCm; "gloo" in the CPU
tests, which pass torch stand-ins for the three device operations, and in the
2-process GPU test of the glue with the device operations, where gloo -- which
has no device all-to-all or reduce -- gets host copies: _all_to_all / _reduce).
"""
from __future__ import annotations

import ctypes

import torch
import torch.distributed as dist

DELTA = 5


def _host_staged(t: torch.Tensor) -> bool:
    """A device tensor under a backend without device collectives (gloo):
    the collective runs on a host copy.  RCCL ("nccl") takes the tensor as is."""
    return t.is_cuda and dist.get_backend() == "gloo"


def _all_to_all(out: torch.Tensor, inp: torch.Tensor, out_splits=None, in_splits=None):
    """dist.all_to_all_single, staged through host memory under gloo."""
    if not _host_staged(out):
        dist.all_to_all_single(out, inp, out_splits, in_splits)
        return
    o = torch.empty(out.shape, dtype=out.dtype)
    dist.all_to_all_single(o, inp.cpu(), out_splits, in_splits)
    out.copy_(o)


def _reduce(t: torch.Tensor, dst: int):
    """dist.reduce (sum into dst), staged through host memory under gloo."""
    if not _host_staged(t):
        dist.reduce(t, dst=dst)
        return
    c = t.cpu()
    dist.reduce(c, dst=dst)
    if dist.get_rank() == dst:
        t.copy_(c)


class DeviceOps:
    """hm_cells_route / hm_cells_merge / hm_dense_cells on the device."""

    def __init__(self, device: int = 0):
        from . import device as _device

        self.ctx = _device.context(device)
        self.L = self.ctx.L

    @staticmethod
    def _p(t):
        return ctypes.c_void_p(t.data_ptr()) if t is not None and t.numel() else ctypes.c_void_p(0)

    def _check(self, rc):
        from . import _lib

        if rc != _lib.HM_OK:
            _lib.raise_for(rc)

    def route(self, keys, counts, ws, dense_zmax, narrow=False):
        """-> (dense grid, parts, group sizes, wide).  parts: the cells grouped
        by owner as [(tensor, elements per cell)]: narrow -> one uint8 tensor
        of 10-byte records (HM_CELLS_REC10: 48-bit key, u32 count), else int64
        keys and int64 counts.  wide (narrow only): a count needs 64 bits and
        the parts are of no use (route again with narrow=False)."""
        from . import _lib

        n = keys.numel()
        gsz = int(self.L.hm_dense_grid_size(dense_zmax))
        grid = torch.empty(max(gsz, 1), dtype=torch.int64, device=keys.device)
        send = (ctypes.c_int64 * ws)()
        if narrow:
            rec = torch.empty(max(n, 1) * 5, dtype=torch.int16, device=keys.device)
            rc = self.L.hm_cells_route(self.ctx.ptr, self._p(keys), self._p(counts), n, ws, DELTA, dense_zmax,
                                       self._p(grid) if gsz > 0 else ctypes.c_void_p(0), self._p(rec),
                                       ctypes.c_void_p(0), _lib.HM_CELLS_REC10, send)
        else:
            ko = torch.empty(max(n, 1), dtype=torch.int64, device=keys.device)
            co = torch.empty_like(ko)
            rc = self.L.hm_cells_route(self.ctx.ptr, self._p(keys), self._p(counts), n, ws, DELTA, dense_zmax,
                                       self._p(grid) if gsz > 0 else ctypes.c_void_p(0), self._p(ko), self._p(co),
                                       _lib.HM_CELLS_U64, send)
        wide = rc == _lib.HM_E_WIDE
        if not wide:
            self._check(rc)
        sent = list(send)
        m = sum(sent)
        parts = [(rec[:5 * m].view(torch.uint8), 10)] if narrow else [(ko[:m], 1), (co[:m], 1)]
        return grid[:gsz], parts, sent, wide

    def route_grouped(self, keys, gcounts, ws):
        """hm_cells_route of grouped cells (HM_CELLS_G12): keys HM_KEY and
        gcounts group << 32 | count (hm_count_grouped_packed) -> (parts,
        group sizes, wide): parts [(u64 merge keys, 1), (u32 counts, 1)] grouped
        by owner; wide: a group id or a zoom past the merge key (exchange
        those records as int64 instead)."""
        from . import _lib

        n = keys.numel()
        ko = torch.empty(max(n, 1), dtype=torch.int64, device=keys.device)
        co = torch.empty(max(n, 1), dtype=torch.int32, device=keys.device)
        send = (ctypes.c_int64 * ws)()
        rc = self.L.hm_cells_route(self.ctx.ptr, self._p(keys), self._p(gcounts), n, ws, DELTA, -1, ctypes.c_void_p(0),
                                   self._p(ko), self._p(co), _lib.HM_CELLS_G12, send)
        wide = rc == _lib.HM_E_WIDE
        if not wide:
            self._check(rc)
        sent = list(send)
        m = sum(sent)
        return [(ko[:m], 1), (co[:m], 1)], sent, wide

    def merge(self, keys, counts=None, runs=None, out=None):
        """Sum equal keys.  keys int64 with counts int32 or int64, or (counts
        None) keys = 10-byte records (HM_CELLS_REC10, uint8); the sums are
        int64.  runs (list of sizes): consecutive runs of distinct keys (one
        sending rank's cells each), merged without count atomics.  out: (keys,
        counts) tensors to write into (their length is the capacity;
        MemoryError if the merged cells do not fit)."""
        from . import _lib

        if counts is None:
            layout, n = _lib.HM_CELLS_REC10, keys.numel() * keys.element_size() // 10
        elif counts.element_size() in (4, 8):
            layout, n = (_lib.HM_CELLS_U32 if counts.element_size() == 4 else _lib.HM_CELLS_U64), keys.numel()
        else:
            raise TypeError("merge: counts must be int32 or int64")
        if out is not None:
            ko, co = out
            cap = ko.numel()
        else:
            cap = max(n, 1)
            ko = torch.empty(cap, dtype=torch.int64, device=keys.device)
            co = torch.empty_like(ko)
        nout = ctypes.c_int64(0)
        if runs is not None:
            ra = (ctypes.c_int64 * max(len(runs), 1))(*runs)
            rc = self.L.hm_cells_merge_runs(self.ctx.ptr, self._p(keys), self._p(counts), layout, n, ra, len(runs),
                                            self._p(ko), self._p(co), cap, ctypes.byref(nout))
        else:
            rc = self.L.hm_cells_merge(self.ctx.ptr, self._p(keys), self._p(counts), layout, n, self._p(ko),
                                       self._p(co), cap, ctypes.byref(nout))
        if rc == _lib.HM_E_CAPACITY and out is not None:
            raise MemoryError("merge_cells: %d owned cells exceed the buffer capacity %d" % (nout.value, cap))
        if rc != _lib.HM_OK:
            _lib.raise_for(rc)
        return ko[:nout.value], co[:nout.value]

    def route_pieces(self, keys, counts, ws, dense_zmax, bits, layout, extra=1, self_rank=-1):
        """hm_cells_route_pieces -> (dense grid, parts, sizes): parts as route()
        (REC10: [(uint8 records, 10)]; U64: [(keys, 1), (counts, 1)]; G12:
        [(u64 merge keys, 1), (u32 counts, 1)]) with room for every cell; sizes
        a DEVICE int64 tensor [ws, 2 + 2^bits + extra]: per owner the cells
        sent, the wide flag, the 2^bits piece sizes, then `extra` zero columns
        for the caller (nothing is synchronised).  self_rank >= 0: the groups
        leave in rank order with that owner's group last."""
        from . import _lib

        self.ctx.bind_stream()
        n = keys.numel()
        gsz = int(self.L.hm_dense_grid_size(dense_zmax))
        grid = torch.empty(max(gsz, 1), dtype=torch.int64, device=keys.device)
        width = 2 + (1 << bits) + extra
        sizes = torch.zeros((ws, width), dtype=torch.int64, device=keys.device)
        if layout == _lib.HM_CELLS_REC10:
            rec = torch.empty(max(n, 1) * 5, dtype=torch.int16, device=keys.device)
            ko, co, parts = rec, None, [(rec.view(torch.uint8), 10)]
        else:
            ko = torch.empty(max(n, 1), dtype=torch.int64, device=keys.device)
            co = torch.empty(max(n, 1), dtype=torch.int32 if layout == _lib.HM_CELLS_G12 else torch.int64,
                             device=keys.device)
            parts = [(ko, 1), (co, 1)]
        rc = self.L.hm_cells_route_pieces(self.ctx.ptr, self._p(keys), self._p(counts), n, ws, DELTA, dense_zmax, bits,
                                          self_rank, self._p(grid) if gsz > 0 else ctypes.c_void_p(0), self._p(ko),
                                          self._p(co), layout, self._p(sizes), width)
        self._check(rc)
        return grid[:gsz], parts, sizes

    def merge_pieces(self, runs, pieces, bits, layout, out=None):
        """hm_cells_merge_pieces.  runs: per sender (key tensor, count tensor
        or None, first cell) -- its cells, 2^bits pieces in digit order, start
        at that cell of those tensors (REC10: uint8 records, 10 bytes a cell);
        pieces: host int64 [senders, 2^bits].  -> (keys, counts) int64, into
        `out` as merge()."""
        from . import _lib

        self.ctx.bind_stream()
        R = len(runs)
        ks = (ctypes.c_void_p * R)()
        cs = (ctypes.c_void_p * R)()
        for r, (kt, ct, start) in enumerate(runs):
            kw = 10 if layout == _lib.HM_CELLS_REC10 else 8
            ks[r] = kt.data_ptr() + start * kw if kt is not None and kt.numel() else None
            cs[r] = ct.data_ptr() + start * ct.element_size() if ct is not None and ct.numel() else None
        pa = (ctypes.c_int64 * (R << bits))(*[int(v) for row in pieces for v in row])
        n = sum(int(v) for row in pieces for v in row)
        if out is not None:
            ko, co = out
            cap = ko.numel()
        else:
            cap = max(n, 1)
            ko = torch.empty(cap, dtype=torch.int64, device=runs[0][0].device)
            co = torch.empty_like(ko)
        nout = ctypes.c_int64(0)
        rc = self.L.hm_cells_merge_pieces(self.ctx.ptr, layout, R, ks, cs, pa, bits, self._p(ko), self._p(co), cap,
                                          ctypes.byref(nout))
        if rc == _lib.HM_E_CAPACITY and out is not None:
            raise MemoryError("merge_cells: %d owned cells exceed the buffer capacity %d" % (nout.value, cap))
        if rc != _lib.HM_OK:
            _lib.raise_for(rc)
        return ko[:nout.value], co[:nout.value]

    def dense_cells(self, grid, dense_zmax, out=None):
        from . import _lib

        if out is not None:
            ko, co = out
            cap = ko.numel()
        else:
            cap = max(int((grid != 0).sum().item()), 1)
            ko = torch.empty(cap, dtype=torch.int64, device=grid.device)
            co = torch.empty_like(ko)
        nout = ctypes.c_int64(0)
        rc = self.L.hm_dense_cells(self.ctx.ptr, self._p(grid), dense_zmax, self._p(ko), self._p(co), cap,
                                   ctypes.byref(nout))
        if rc == _lib.HM_E_CAPACITY and out is not None:
            raise MemoryError("merge_cells: %d dense cells exceed the buffer capacity %d" % (nout.value, cap))
        if rc != _lib.HM_OK:
            _lib.raise_for(rc)
        return ko[:nout.value], co[:nout.value]


def pack_records(keys: torch.Tensor, counts: torch.Tensor) -> torch.Tensor:
    """HM_CELLS_REC10 records (uint8, 10 per cell: five little-endian u16) of
    HM_KEY keys (zooms <= 21) and counts < 2^32 -- the device's layout, for
    the CPU stand-ins and tests."""
    z, r, c = keys >> 58, (keys >> 29) & 0x1FFFFF, keys & 0x1FFFFF
    p = (z << 42) | (r << 21) | c
    w = torch.stack([p & 0xFFFF, (p >> 16) & 0xFFFF, (p >> 32) & 0xFFFF, counts & 0xFFFF, (counts >> 16) & 0xFFFF], 1)
    return (((w + 32768) % 65536) - 32768).to(torch.int16).reshape(-1).view(torch.uint8)


def unpack_records(rec: torch.Tensor):
    """(int64 keys, int64 counts) of HM_CELLS_REC10 records."""
    w = rec.contiguous().view(torch.int16).reshape(-1, 5).to(torch.int64) & 0xFFFF
    p = w[:, 0] | (w[:, 1] << 16) | (w[:, 2] << 32)
    keys = ((p >> 42) << 58) | (((p >> 21) & 0x1FFFFF) << 29) | (p & 0x1FFFFF)
    return keys, w[:, 3] | (w[:, 4] << 16)


def record_owner(cells: torch.Tensor, ws: int) -> torch.Tensor:
    """Owner rank of cells given as int64 records (zoom, row, col, count):
    the same heatmap-row hash as hm_cells_route, on arithmetic shifts."""
    z, r, c = cells[:, 0], cells[:, 1], cells[:, 2]
    rk = (z << 48) ^ ((r >> DELTA) << 24) ^ (c >> DELTA)
    h = (rk * -7046029254386353131) >> 33          # wrapping int64 multiply (0x9E3779B97F4A7C15)
    return torch.remainder(h, ws)


def _exchange(rows: torch.Tensor, owner: torch.Tensor, ws: int) -> torch.Tensor:
    """All-to-all of fixed-width int64 rows, grouped by owner rank."""
    order = torch.argsort(owner, stable=True)
    rows = rows[order]
    send = torch.bincount(owner, minlength=ws)
    recv = torch.empty_like(send)
    _all_to_all(recv, send)
    sl, rl = send.tolist(), recv.tolist()
    w = rows.shape[1]
    out = torch.empty(sum(rl) * w, dtype=rows.dtype, device=rows.device)
    _all_to_all(out, rows.reshape(-1).contiguous(), [x * w for x in rl], [x * w for x in sl])
    return out.reshape(-1, w)


def merge_exotic(cells: torch.Tensor, ws: int, rank: int) -> torch.Tensor:
    """Cells outside [0, 2^z)^2 as (zoom, row, col, count) records: routed to
    their heatmap row's owner and summed there."""
    got = _exchange(cells.reshape(-1, 4), record_owner(cells.reshape(-1, 4), ws), ws)
    if got.shape[0] == 0:
        return got
    u, inv = torch.unique(got[:, :3], dim=0, return_inverse=True)
    tot = torch.zeros(u.shape[0], dtype=torch.int64, device=got.device)
    tot.index_add_(0, inv, got[:, 3])
    return torch.cat([u, tot[:, None]], 1)


def pipelined_steps(count, bufsets, steps: int, ws: int, rank: int, ctx=None, dense_zmax: int = 10,
                    merge_ms=None):
    """Run `steps` count + merge steps with step k's merge overlapping step
    k+1's count: count(buffers) -> (m, buffers) runs on the calling thread
    (its hm context, the current stream); merge_cells runs on a helper thread
    with its own HIP stream and hm context, which alone issues the RCCL
    collectives (in step order, as on every rank).  bufsets: >= 2 CountBuffers
    used in turn; a set is counted into again only after its merge finished.
    Returns (cells owned after the last merge, per-step stage timings of the
    counts, the last step's buffers); merge_ms (a list): each merge's host
    time on the merge thread is appended."""
    import queue
    import threading
    import time

    todo, free = queue.Queue(), queue.Queue()
    for b in bufsets:
        free.put(b)
    owned, err, last = [], [], [None]
    # HM_MERGE_PRIORITY=1: the merge stream takes the highest priority, so its
    # kernels (and the RCCL calls' copies) are dispatched ahead of the next
    # count's, which fill the CUs
    import os

    if os.environ.get("HM_MERGE_PRIORITY", "0") == "1":
        lo, hi = torch.cuda.Stream.priority_range()
        side = torch.cuda.Stream(priority=min(lo, hi))
    else:
        side = torch.cuda.Stream()

    def merger():
        try:
            with torch.cuda.stream(side):
                while True:
                    item = todo.get()
                    if item is None:
                        return
                    m, b = item
                    t0 = time.perf_counter()
                    owned.append(merge_cells(b, m, ws, rank, dense_zmax))
                    side.synchronize()
                    if merge_ms is not None:
                        merge_ms.append((time.perf_counter() - t0) * 1e3)
                    last[0] = b
                    free.put(b)
        except BaseException as e:   # surfaced on the calling thread
            err.append(e)
            free.put(None)

    th = threading.Thread(target=merger, name="hm-merge")
    th.start()
    stages = []
    try:
        for _ in range(steps):
            b = free.get()
            if b is None:
                break
            # buffers the merge grew were allocated on its side stream: tell the
            # caching allocator the count's stream uses them too, so a later
            # growth does not hand their memory to the side stream while this
            # stream's count may still write it
            cur = torch.cuda.current_stream()
            for name in ("keys", "counts", "xcells"):
                t = getattr(b, name, None)
                if isinstance(t, torch.Tensor) and t.is_cuda:
                    t.record_stream(cur)
            m, b = count(b)
            if ctx is not None:
                stages.append(ctx.last_stats()[1][:5])
            todo.put((m, b))
    finally:
        todo.put(None)
        th.join()
    if err:
        raise err[0]
    return (owned[-1] if owned else 0), stages, last[0]


def route_bits(ws: int) -> int:
    """Merge-digit bits of the pieces route: 7 (128 pieces per owner) up to 4
    ranks, then fewer so the route keeps <= 512 digits (owner x piece): at 8
    owners 6 bits measured 1.05 ms of route + merge against 1.15 with 7
    (tools/merge_ws8.py, 28M cells)."""
    b = 7
    while (ws << b) > 512:
        b -= 1
    return b


def _exchange_pieces(parts, sent, rl, rank, device):
    """All-to-all of the routed cells (parts from route_pieces with
    self_rank = rank: the peers' groups in rank order, this rank's own group
    last) -> per sender (key tensor, count tensor or None, first cell): the
    peers' cells land in fresh receive tensors by one all_to_all_single with
    a zero own split, this rank's own group stays where the route wrote it
    (no self copy)."""
    ws = len(sent)
    others = sum(sent) - sent[rank]
    roff = [0] * (ws + 1)
    for r in range(ws):
        roff[r + 1] = roff[r] + (rl[r] if r != rank else 0)
    got = []
    for t, w in parts:
        recv = torch.empty(max(roff[ws], 1) * w, dtype=t.dtype, device=device)
        if ws > 1:
            _all_to_all(recv[:roff[ws] * w], t[:others * w],
                                   [(rl[r] if r != rank else 0) * w for r in range(ws)],
                                   [(sent[o] if o != rank else 0) * w for o in range(ws)])
        got.append(recv)
    runs = []
    for r in range(ws):
        if r == rank:
            runs.append((parts[0][0], parts[1][0] if len(parts) > 1 else None, others))
        else:
            runs.append((got[0], got[1] if len(got) > 1 else None, roff[r]))
    return runs, got


def merge_cells(buffers, m: int, ws: int, rank: int, dense_zmax: int = 10, ops=None) -> int:
    """Exchange and merge the first m cells of `buffers` (int64 keys/counts,
    HM_KEY layout; records of cells outside the square in buffers.xcells,
    buffers.nx of them) in place; returns the number of in-square cells this
    rank owns (buffers.nx becomes the owned exotic count).  dense_zmax < 0
    sends every zoom through the all-to-all.  `ops`: the device operations
    (DeviceOps), or stand-ins with the same contract (CPU tests).

    The pieces exchange: hm_cells_route_pieces groups the cells by owner and,
    inside a group, by the first merge digit (route_bits), writing the sizes
    on the device; ONE all-to-all of those rows (which also carry every
    rank's wide flag and exotic count) and ONE host sync; then the cells'
    all-to-all, and hm_cells_merge_pieces on the owner, whose own group never
    leaves the route's buffer."""
    from . import _lib

    if ops is None:
        ops = DeviceOps(buffers.keys.device.index or 0)
    keys = buffers.keys[:m]
    counts = buffers.counts[:m]
    bits = route_bits(ws)
    S = 1 << bits
    nx = int(getattr(buffers, "nx", 0))
    # cells travel as 10-byte records (48-bit key, u32 count) unless some
    # rank holds a cell count >= 2^32: every rank's flag rides on the size
    # exchange, so all ranks agree before the cells' all-to-all
    grid, parts, sizes = ops.route_pieces(keys, counts, ws, dense_zmax, bits, _lib.HM_CELLS_REC10, self_rank=rank)
    sizes[:, -1] = nx
    recv = torch.empty_like(sizes)
    _all_to_all(recv, sizes)
    both = torch.stack([sizes, recv]).cpu()
    sent = both[0, :, 0].tolist()
    rl = both[1, :, 0].tolist()
    pieces = both[1, :, 2:2 + S].tolist()
    nx_all = int(both[1, :, -1].sum())
    layout = _lib.HM_CELLS_REC10
    if bool(both[1, :, 1].any()):
        layout = _lib.HM_CELLS_U64
        grid, parts, _ = ops.route_pieces(keys, counts, ws, dense_zmax, bits, layout, self_rank=rank)
    if dense_zmax >= 0:
        _reduce(grid, 0)                            # RCCL reduce of the dense zooms over xGMI
    # the owned cells are at most the received ones plus (rank 0) the dense
    # grid's: grow this rank's buffers first (a local decision -- a rank that
    # raised here instead would leave its peers blocked in the next collective)
    need = sum(rl) + (grid.numel() if dense_zmax >= 0 and rank == 0 else 0)
    if need > buffers.keys.numel():
        buffers.keys = torch.empty(need, dtype=torch.int64, device=keys.device)
        buffers.counts = torch.empty_like(buffers.keys)
        buffers.capacity = need
    runs, got = _exchange_pieces(parts, sent, rl, rank, keys.device)
    n = 0
    if sum(rl):
        uk, _ = ops.merge_pieces(runs, pieces, bits, layout, out=(buffers.keys, buffers.counts))
        n = uk.numel()
    del got
    if dense_zmax >= 0 and rank == 0:
        dk, _ = ops.dense_cells(grid, dense_zmax, out=(buffers.keys[n:], buffers.counts[n:]))
        n += dk.numel()
    if nx_all:
        x = merge_exotic(buffers.xcells[:4 * nx], ws, rank)
        if x.numel() > buffers.xcells.numel():
            buffers.xcells = torch.empty(x.numel(), dtype=torch.int64, device=keys.device)
        buffers.xcells[:x.numel()] = x.reshape(-1)
        buffers.nx = x.shape[0]
    return n


GKEY_GROUP_BITS = 17


def grouped_owner(keys: torch.Tensor, groups: torch.Tensor, ws: int) -> torch.Tensor:
    """Owner rank of grouped in-square cells (HM_KEY keys, group ids): the
    hash hm_cells_route computes for HM_CELLS_G12 (the row key of
    heatmap.py:55 -- user, timespan, tile -- holds the group)."""
    z, r, c = keys >> 58, (keys >> 29) & 0x1FFFFFFF, keys & 0x1FFFFFFF
    gm = (groups + 1) * -2960836687051489901          # wrapping (group + 1) * 0xD6E8FEB86659FD93
    rk = ((z << 48) ^ ((r >> DELTA) << 24) ^ (c >> DELTA)) + gm
    h = (rk * -7046029254386353131) >> 33
    return torch.remainder(h, ws)


def merge_grouped(keys: torch.Tensor, gcounts: torch.Tensor, ws: int, rank: int, ops=None):
    """Exchange and merge grouped cells -- hm_count_grouped_packed's keys
    (HM_KEY) and gcounts (group << 32 | count) on every rank -- so that each
    (group, cell) ends on the rank owning its heatmap row (the reference's
    reduceByKey / groupByKey on user|alltime|tile keys, heatmap.py:54-55,
    111-112).  Returns this rank's (keys, groups, counts) int64 tensors
    (counts summed over ranks: int64).  The pieces exchange of merge_cells
    with 12-byte cells (u64 merge key of group, zoom, row, col; u32 count):
    ONE all-to-all of the size rows (wide flag included), one of keys, one of
    counts, and hm_cells_merge_pieces on the owner; if any rank holds a group
    id past 2^17 (the merge key's field) every rank exchanges (key, group,
    count) int64 records and sums them with torch ops instead."""
    from . import _lib

    if ops is None:
        ops = DeviceOps(keys.device.index or 0)
    bits = route_bits(ws)
    S = 1 << bits
    _, parts, sizes = ops.route_pieces(keys, gcounts, ws, -1, bits, _lib.HM_CELLS_G12, extra=0, self_rank=rank)
    recv = torch.empty_like(sizes)
    _all_to_all(recv, sizes)
    both = torch.stack([sizes, recv]).cpu()
    sent = both[0, :, 0].tolist()
    rl = both[1, :, 0].tolist()
    if bool(both[1, :, 1].any()):
        g = gcounts >> 32
        rows = torch.stack([keys, g, gcounts & 0xFFFFFFFF], 1)
        got = _exchange(rows, grouped_owner(keys, g, ws), ws)
        if got.shape[0] == 0:
            return got[:, 0], got[:, 1], got[:, 2]
        u, inv = torch.unique(got[:, :2], dim=0, return_inverse=True)
        tot = torch.zeros(u.shape[0], dtype=torch.int64, device=got.device).index_add_(0, inv, got[:, 2])
        return u[:, 0], u[:, 1], tot
    runs, got = _exchange_pieces(parts, sent, rl, rank, keys.device)
    if not sum(rl):
        e = torch.empty(0, dtype=torch.int64, device=keys.device)
        return e, e, e
    mk, mc = ops.merge_pieces(runs, both[1, :, 2:2 + S].tolist(), bits, _lib.HM_CELLS_G12)
    g = (mk >> 47) & 0x1FFFF   # the 17-bit group field (bits 47-63; >> on int64 is arithmetic)
    hk = (((mk >> 42) & 31) << 58) | (((mk >> 21) & 0x1FFFFF) << 29) | (mk & 0x1FFFFF)
    return hk, g, mc
