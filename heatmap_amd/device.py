"""Device-side entry points (columnar): projection and the count pyramid.

Inputs may be numpy arrays (copied to HBM first) or torch CUDA tensors
(used in place, zero copy).  PyTorch is only the memory/stream plumbing; all
arithmetic runs in the gfx950 kernels behind include/heatmap_amd.h.
"""
from __future__ import annotations

import ctypes
import threading
from dataclasses import dataclass

import numpy as np

from . import _lib

_CTX = {}
_CTX_LOCK = threading.Lock()


def gpu_available() -> bool:
    """A GPU torch can use (the host-side row assembly then sorts on it)."""
    try:
        import torch

        return torch.cuda.is_available()
    except Exception:   # pragma: no cover
        return False


def _torch():
    import torch

    if not torch.cuda.is_available():
        raise _lib.DeviceUnavailable("heatmap_amd needs a gfx950 GPU (torch.cuda.is_available() is False); "
                                     "there is no CPU fallback")
    return torch


class Context:
    """One hm_ctx per (device, host thread)."""

    def __init__(self, device: int = 0):
        torch = _torch()
        self.L = _lib.load()
        self.device = device
        p = ctypes.c_void_p()
        with torch.cuda.device(device):
            st = self.L.hm_ctx_create(ctypes.byref(p), device, ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
        if st != _lib.HM_OK:
            _lib.raise_for(st)
        self.ptr = p

    def bind_stream(self):
        torch = _torch()
        h = torch.cuda.current_stream(self.device).cuda_stream
        if h != getattr(self, "_bound", None):   # one C call per change of stream, not per call
            self.L.hm_ctx_set_stream(self.ptr, ctypes.c_void_p(h))
            self._bound = h

    def last_error(self):
        idx = ctypes.c_int64(-1)
        kind = ctypes.c_int(0)
        self.L.hm_last_error(self.ptr, ctypes.byref(idx), ctypes.byref(kind))
        return idx.value, kind.value

    def last_stats(self):
        slow = ctypes.c_int64(0)
        us = (ctypes.c_double * 8)()
        self.L.hm_last_stats(self.ptr, ctypes.byref(slow), us, 8)
        return slow.value, list(us)

    def tune(self, name: str, value: float) -> float:
        """Set one plan-tuning knob (include/heatmap_amd.h hm_ctx_tune);
        returns the previous value."""
        old = ctypes.c_double(0)
        rc = self.L.hm_ctx_tune(self.ptr, name.encode(), float(value), ctypes.byref(old))
        if rc != _lib.HM_OK:
            raise ValueError("unknown tuning knob %r" % name)
        return old.value

    def __del__(self):  # pragma: no cover
        try:
            if getattr(self, "ptr", None):
                self.L.hm_ctx_destroy(self.ptr)
        except Exception:
            pass


def context(device: int = 0) -> Context:
    key = (device, threading.get_ident())
    with _CTX_LOCK:
        c = _CTX.get(key)
        if c is None:
            c = _CTX[key] = Context(device)
    c.bind_stream()
    return c


class tuned:
    """Context manager: plan-tuning knobs of this thread's context for the
    block (tests force plans at parity sizes), restored afterwards.

        with device.tuned(HM_HOT_MIN_KEYS=0): ...
    """

    def __init__(self, device: int = 0, **knobs):
        self.device, self.knobs, self.old = device, knobs, {}

    def __enter__(self):
        ctx = context(self.device)
        for k, v in self.knobs.items():
            self.old[k] = ctx.tune(k, v)
        return ctx

    def __exit__(self, *exc):
        ctx = context(self.device)
        for k, v in self.old.items():
            ctx.tune(k, v)
        return False


def _dev(x, dtype, device):
    torch = _torch()
    if isinstance(x, torch.Tensor):
        t = x
        if t.dtype != dtype:
            t = t.to(dtype)
        if t.device.type != "cuda":
            t = t.to("cuda:%d" % device)
        return t.contiguous()
    a = np.ascontiguousarray(x)
    return torch.from_numpy(a).to(device="cuda:%d" % device, dtype=dtype)


def _ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None and t.numel() else ctypes.c_void_p(0)


@dataclass
class Projection:
    row: np.ndarray
    col: np.ndarray
    status: np.ndarray
    first_error_index: int
    first_error_kind: int
    slow_points: int


def project(lat, lon, zoom: int, device: int = 0, raise_errors: bool = False) -> Projection:
    """Tile rows/cols of every point at `zoom` (reference tile.py:15-21)."""
    torch = _torch()
    ctx = context(device)
    la = _dev(lat, torch.float64, device)
    lo = _dev(lon, torch.float64, device)
    n = la.numel()
    if lo.numel() != n:
        raise ValueError("lat and lon must have the same length")
    row = torch.empty(n, dtype=torch.int64, device=la.device)
    col = torch.empty(n, dtype=torch.int64, device=la.device)
    st = torch.empty(n, dtype=torch.uint8, device=la.device)
    rc = ctx.L.hm_project(ctx.ptr, _ptr(la), _ptr(lo), n, int(zoom), _ptr(row), _ptr(col), _ptr(st))
    idx, kind = ctx.last_error()
    slow, _ = ctx.last_stats()
    if rc not in (_lib.HM_OK, _lib.HM_E_NAN, _lib.HM_E_DOMAIN, _lib.HM_E_INF, _lib.HM_E_RANGE):
        _lib.raise_for(rc)
    if raise_errors and rc != _lib.HM_OK:
        _lib.raise_for(kind, idx)
    return Projection(row.cpu().numpy(), col.cpu().numpy(), st.cpu().numpy(), idx, kind, slow)


@dataclass
class Counts:
    zoom: np.ndarray
    row: np.ndarray
    col: np.ndarray
    count: np.ndarray
    slow_points: int
    stage_us: list

    def sorted(self) -> "Counts":
        o = np.lexsort((self.col, self.row, self.zoom))
        return Counts(self.zoom[o], self.row[o], self.col[o], self.count[o], self.slow_points, self.stage_us)

    def as_dict(self):
        """{zoom: {(row, col): count}}"""
        out = {}
        for z, r, c, n in zip(self.zoom.tolist(), self.row.tolist(), self.col.tolist(), self.count.tolist()):
            out.setdefault(z, {})[(r, c)] = n
        return out


def decode_keys(keys: np.ndarray):
    keys = keys.astype(np.uint64)
    z = (keys >> np.uint64(58)).astype(np.int32)
    r = ((keys >> np.uint64(29)) & np.uint64(0x1FFFFFFF)).astype(np.int64)
    c = (keys & np.uint64(0x1FFFFFFF)).astype(np.int64)
    return z, r, c


class CountBuffers:
    """Reusable device output buffers for count() (bench / streaming): cells
    inside [0, 2^z)^2 as (HM_KEY, count), cells outside it as 4 int64 records
    (zoom, row, col, count)."""

    def __init__(self, capacity: int, device: int = 0, xcapacity: int = 1024):
        torch = _torch()
        self.capacity = int(capacity)
        self.xcapacity = int(xcapacity)
        self.keys = torch.empty(max(self.capacity, 1), dtype=torch.int64, device="cuda:%d" % device)
        self.counts = torch.empty(max(self.capacity, 1), dtype=torch.int64, device="cuda:%d" % device)
        self.xcells = torch.empty(4 * max(self.xcapacity, 1), dtype=torch.int64, device="cuda:%d" % device)
        self.nx = 0


# points per hm_count call: the ABI takes n < 2^32 - 16 (u32 key positions);
# 2^31 keeps the level-1 regions' sampled margins inside the u32 key space
MAX_CALL_POINTS = 1 << 31


def count_device(lat, lon, keep=None, zmin: int = 0, zmax: int = 18, device: int = 0, buffers=None,
                 tiles: bool = False, chunk: int = MAX_CALL_POINTS):
    """Run the count pyramid; returns (n_cells, buffers) with results left in
    HBM (buffers.nx: cells outside the square, in buffers.xcells).

    Inputs of more than `chunk` points (one call holds < 2^32) are counted
    chunk by chunk in input order, so the first failing point is still the one
    reported, and the chunks' cells are summed on the device (hm_cells_merge;
    cells outside the square with torch ops)."""
    torch = _torch()
    ctx = context(device)
    if tiles:
        a = _dev(lat, torch.int64, device)
        b = _dev(lon, torch.int64, device)
    else:
        a = _dev(lat, torch.float64, device)
        b = _dev(lon, torch.float64, device)
    n = a.numel()
    if b.numel() != n:
        raise ValueError("coordinate arrays must have the same length")
    kp = None
    if keep is not None:
        kp = _dev(keep, torch.uint8, device)
        if kp.numel() != n:
            raise ValueError("keep must have one entry per point")
    if n > chunk:
        return _count_chunked(a, b, kp, n, zmin, zmax, device, tiles, int(chunk))
    if buffers is None:
        # cells <= 4 n + ... for small inputs; large ones start at 64M cells and
        # grow on HM_E_CAPACITY (the call is then repeated)
        buffers = CountBuffers(max(1024, min(4 * n + 64, 1 << 26)), device)
    fn = ctx.L.hm_count_tiles if tiles else ctx.L.hm_count
    while True:
        nout = ctypes.c_int64(0)
        nx = ctypes.c_int64(0)
        rc = fn(ctx.ptr, _ptr(a), _ptr(b), _ptr(kp), n, int(zmin), int(zmax), _ptr(buffers.keys),
                _ptr(buffers.counts), buffers.capacity, ctypes.byref(nout), _ptr(buffers.xcells), buffers.xcapacity,
                ctypes.byref(nx))
        if rc == _lib.HM_E_CAPACITY:
            cap = buffers.capacity if nout.value <= buffers.capacity else int(nout.value * 1.25) + 64
            xcap = buffers.xcapacity if nx.value <= buffers.xcapacity else int(nx.value * 1.25) + 64
            buffers = CountBuffers(cap, device, xcap)
            continue
        if rc != _lib.HM_OK:
            idx, kind = ctx.last_error()
            _lib.raise_for(rc, idx)
        buffers.nx = nx.value
        return nout.value, buffers


def _count_chunked(a, b, kp, n, zmin, zmax, device, tiles, chunk):
    torch = _torch()
    ctx = context(device)
    keys, counts, xcells = [], [], []
    for s in range(0, n, chunk):
        e = min(n, s + chunk)
        try:
            m, buf = count_device(a[s:e], b[s:e], None if kp is None else kp[s:e], zmin, zmax, device,
                                  tiles=tiles, chunk=chunk)
        except _lib.DevicePathUnsupported as ex:
            idx, _ = ctx.last_error()
            raise _lib.DevicePathUnsupported(str(ex).split(" (point")[0] +
                                             ("" if idx < 0 else " (point %d)" % (idx + s))) from None
        keys.append(buf.keys[:m].clone())
        counts.append(buf.counts[:m].clone())
        if buf.nx:
            xcells.append(buf.xcells[:4 * buf.nx].reshape(-1, 4).clone())
    k = torch.cat(keys)
    c = torch.cat(counts)
    cap = max(int(k.numel()), 1)
    out = CountBuffers(cap, device, 1024)
    nout = ctypes.c_int64(0)
    rc = ctx.L.hm_cells_merge(ctx.ptr, _ptr(k), _ptr(c), 8, int(k.numel()), _ptr(out.keys), _ptr(out.counts), cap,
                              ctypes.byref(nout))
    if rc != _lib.HM_OK:
        _lib.raise_for(rc)
    if xcells:
        x = torch.cat(xcells)
        u, inv = torch.unique(x[:, :3], dim=0, return_inverse=True)
        tot = torch.zeros(u.shape[0], dtype=torch.int64, device=x.device).index_add_(0, inv, x[:, 3])
        rec = torch.cat([u, tot[:, None]], dim=1)
        out.xcapacity = rec.shape[0]
        out.xcells = rec.reshape(-1).contiguous()
        out.nx = rec.shape[0]
    return nout.value, out


def count(lat, lon, keep=None, zmin: int = 0, zmax: int = 18, device: int = 0, tiles: bool = False,
          chunk: int = MAX_CALL_POINTS) -> Counts:
    """Per-(zoom, row, col) counts for zooms zmin..zmax (host arrays), cells
    inside and outside [0, 2^z)^2 together."""
    m, buf = count_device(lat, lon, keep, zmin, zmax, device, tiles=tiles, chunk=chunk)
    ctx = context(device)
    slow, us = ctx.last_stats()
    keys = buf.keys[:m].cpu().numpy().view(np.uint64)
    cnt = buf.counts[:m].cpu().numpy()
    z, r, c = decode_keys(keys)
    if buf.nx:
        x = buf.xcells[:4 * buf.nx].cpu().numpy().reshape(-1, 4)
        z = np.concatenate([z, x[:, 0].astype(np.int32)])
        r = np.concatenate([r, x[:, 1]])
        c = np.concatenate([c, x[:, 2]])
        cnt = np.concatenate([cnt, x[:, 3]])
    return Counts(z, r, c, cnt, slow, us)


@dataclass
class GroupedCounts:
    group: np.ndarray
    zoom: np.ndarray
    row: np.ndarray
    col: np.ndarray
    count: np.ndarray

    def sorted(self) -> "GroupedCounts":
        o = np.lexsort((self.col, self.row, self.zoom, self.group))
        return GroupedCounts(self.group[o], self.zoom[o], self.row[o], self.col[o], self.count[o])


def count_grouped_device(lat, lon, group, keep=None, zmin: int = 0, zmax: int = 18, device: int = 0,
                         tiles: bool = False):
    """hm_count_grouped with the records left in HBM: an int64 CUDA tensor
    [m, 5] of (group, zoom, row, col, count), in no particular order."""
    torch = _torch()
    ctx = context(device)
    dt = torch.int64 if tiles else torch.float64
    a = _dev(lat, dt, device)
    b = _dev(lon, dt, device)
    n = a.numel()
    g = _dev(np.asarray(group, dtype=np.uint32).view(np.int32) if not isinstance(group, torch.Tensor) else group,
             torch.int32, device)
    if b.numel() != n or g.numel() != n:
        raise ValueError("lat, lon and group must have the same length")
    kp = None
    if keep is not None:
        kp = _dev(keep, torch.uint8, device)
        if kp.numel() != n:
            raise ValueError("keep must have one entry per point")
    cap = _record_capacity(n, int(zmax) - int(zmin) + 1, 40, device)
    while True:
        cells = torch.empty(5 * cap, dtype=torch.int64, device=a.device)
        nout = ctypes.c_int64(0)
        fn = ctx.L.hm_count_grouped_tiles if tiles else ctx.L.hm_count_grouped
        rc = fn(ctx.ptr, _ptr(a), _ptr(b), _ptr(kp), _ptr(g), n, int(zmin), int(zmax), _ptr(cells), cap,
                ctypes.byref(nout))
        if rc == _lib.HM_E_CAPACITY:
            cap = int(nout.value * 1.25) + 64
            continue
        if rc != _lib.HM_OK:
            idx, kind = ctx.last_error()
            _lib.raise_for(rc, idx)
        break
    return _exact(cells, 5 * nout.value).view(-1, 5)


def _exact(buf, m: int):
    """buf[:m], copied out at its exact size when the first capacity guess
    (_record_capacity: up to half the free memory) left more than 256 MiB and
    a quarter of the buffer unused -- a slice would keep the whole allocation
    alive for the caller's later sorts and the library's own buffers."""
    waste = (buf.numel() - m) * buf.element_size()
    if waste > (256 << 20) and 4 * (buf.numel() - m) > buf.numel():
        out = buf[:m].clone()
        del buf
        return out
    return buf[:m]


def _record_capacity(n: int, nz: int, bytes_per: int, device: int) -> int:
    """First record capacity of a grouped count: every (point, zoom) when that
    fits half the free device memory (one pass, the usual case on a 288 GB
    part), else half the free memory's worth (more records: HM_E_CAPACITY and
    one more pass at the exact size)."""
    torch = _torch()
    free, _ = torch.cuda.mem_get_info(device)
    most = max(1024, int(free // 2) // bytes_per)
    return max(1024, min(n * nz + 64, most))


def count_grouped_packed_device(lat, lon, group, keep=None, zmin: int = 0, zmax: int = 18, device: int = 0,
                                tiles: bool = False):
    """hm_count_grouped_packed: (keys, gcounts) int64 CUDA tensors of the
    records -- keys HM_KEY(zoom, row, col), gcounts group << 32 | count, 16 B
    per record -- or None when some kept point's tile lies outside
    [0, 2^zmax)^2 (hm_count_grouped's 5-int64 records hold those)."""
    torch = _torch()
    ctx = context(device)
    dt = torch.int64 if tiles else torch.float64
    a = _dev(lat, dt, device)
    b = _dev(lon, dt, device)
    n = a.numel()
    g = _dev(np.asarray(group, dtype=np.uint32).view(np.int32) if not isinstance(group, torch.Tensor) else group,
             torch.int32, device)
    if b.numel() != n or g.numel() != n:
        raise ValueError("lat, lon and group must have the same length")
    kp = None
    if keep is not None:
        kp = _dev(keep, torch.uint8, device)
        if kp.numel() != n:
            raise ValueError("keep must have one entry per point")
    cap = _record_capacity(n, int(zmax) - int(zmin) + 1, 16, device)
    fn = ctx.L.hm_count_grouped_packed_tiles if tiles else ctx.L.hm_count_grouped_packed
    while True:
        keys = torch.empty(cap, dtype=torch.int64, device=a.device)
        gc = torch.empty(cap, dtype=torch.int64, device=a.device)
        nout = ctypes.c_int64(0)
        rc = fn(ctx.ptr, _ptr(a), _ptr(b), _ptr(kp), _ptr(g), n, int(zmin), int(zmax), _ptr(keys), _ptr(gc), cap,
                ctypes.byref(nout))
        if rc == _lib.HM_E_CAPACITY:
            del keys, gc
            cap = int(nout.value) + 64
            continue
        if rc == _lib.HM_E_EXOTIC:
            return None
        if rc != _lib.HM_OK:
            idx, kind = ctx.last_error()
            _lib.raise_for(rc, idx)
        m = nout.value
        return _exact(keys, m), _exact(gc, m)


def count_grouped(lat, lon, group, keep=None, zmin: int = 0, zmax: int = 18, device: int = 0,
                  tiles: bool = False) -> GroupedCounts:
    """Per-(group, zoom, row, col) counts in one device pass (hm_count_grouped;
    tiles=True: lat/lon are int64 zoom-zmax rows/cols, hm_count_grouped_tiles).
    group: uint32 per point; keep: points to count (all are projected)."""
    x = count_grouped_device(lat, lon, group, keep, zmin, zmax, device, tiles).cpu().numpy()
    return GroupedCounts(x[:, 0].astype(np.uint32), x[:, 1].astype(np.int32), x[:, 2].copy(), x[:, 3].copy(),
                         x[:, 4].copy())


_SYNTH_KIND = {"uniform": 0, "hotspots": 1, "skew": 2}


def synth(kind: str, lat, lon, seed: int = 0, start: int = 0, device: int = 0):
    """Fill torch CUDA tensors lat/lon with points start.. of heatmap_amd.synth's
    `kind` cloud (bit-identical to the numpy generator)."""
    torch = _torch()
    from . import synth as _synth

    ctx = context(device)
    n = lat.numel()
    tab = None
    k = 0
    if kind == "hotspots":
        clat, clon, sig, cdf = _synth.hotspot_centres(seed)
        k = len(cdf)
        tab = torch.from_numpy(np.concatenate([clat, clon, sig, cdf]).astype(np.float64)).to(lat.device)
    rc = ctx.L.hm_synth(ctx.ptr, _SYNTH_KIND[kind], int(seed) & ((1 << 64) - 1), int(start), n, _ptr(lat), _ptr(lon),
                        _ptr(tab), k)
    if rc != _lib.HM_OK:
        _lib.raise_for(rc)
    torch.cuda.current_stream(device).synchronize()
