"""Streaming micro-batches merged into a heatmap resident in HBM (BASELINE
config 5) -- host side of hm_stream_* (include/heatmap_amd.h).

The reference recomputes its pyramid per Spark job (heatmap.py:152-158) under
the one live timespan label 'alltime' (heatmap.py:62-63).  StreamingHeatmap
keeps that alltime heatmap plus one bucket per epoch hour in a device hash
table; each add() runs the count pyramid on the batch and folds its cells in,
so a caller sees the same counts as one hm_count over every point so far.
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _lib, device

ALLTIME = -1
EACH_HOUR = -2
MAX_HOURS = 131071


class StreamingHeatmap:
    def __init__(self, zmin: int = 0, zmax: int = 18, base_hour: int = 0, initial_cells: int = 1 << 20,
                 device_index: int = 0):
        self._torch = device._torch()
        self.ctx = device.context(device_index)
        self.device_index = device_index
        self.zmin, self.zmax, self.base_hour = int(zmin), int(zmax), int(base_hour)
        p = ctypes.c_void_p()
        rc = self.ctx.L.hm_stream_create(self.ctx.ptr, self.zmin, self.zmax, self.base_hour, int(initial_cells),
                                         ctypes.byref(p))
        if rc != _lib.HM_OK:
            _lib.raise_for(rc)
        self.ptr = p

    def add(self, lat, lon, keep=None, hour=None):
        """Fold one micro-batch in.  hour: uint32 epoch hours (one per point) or
        None (alltime only).  Projection errors raise as hm_count's do."""
        torch = self._torch
        self.ctx.bind_stream()
        la = device._dev(lat, torch.float64, self.device_index)
        lo = device._dev(lon, torch.float64, self.device_index)
        n = la.numel()
        if lo.numel() != n:
            raise ValueError("lat and lon must have the same length")
        kp = device._dev(keep, torch.uint8, self.device_index) if keep is not None else None
        hr = None
        if hour is not None:
            h = hour
            if not isinstance(h, torch.Tensor):
                h = torch.from_numpy(np.ascontiguousarray(np.asarray(h, dtype=np.uint32)).view(np.int32))
            hr = device._dev(h, torch.int32, self.device_index)  # uint32 bits
            if hr.numel() != n:
                raise ValueError("hour must have one entry per point")
        if kp is not None and kp.numel() != n:
            raise ValueError("keep must have one entry per point")
        rc = self.ctx.L.hm_stream_add(self.ptr, device._ptr(la), device._ptr(lo), device._ptr(kp), device._ptr(hr), n)
        if rc != _lib.HM_OK:
            idx, kind = self.ctx.last_error()
            _lib.raise_for(rc, idx)

    def cells(self):
        """(occupied table slots over every bucket, table capacity)"""
        a, b = ctypes.c_int64(0), ctypes.c_int64(0)
        self.ctx.L.hm_stream_cells(self.ptr, ctypes.byref(a), ctypes.byref(b))
        return a.value, b.value

    def extract_device(self, hour: int = ALLTIME):
        """(n, keys, counts, hours) as torch CUDA tensors (hm_count key layout)."""
        torch = self._torch
        self.ctx.bind_stream()
        cap = max(1024, self.cells()[0])
        dev = "cuda:%d" % self.device_index
        while True:
            keys = torch.empty(cap, dtype=torch.int64, device=dev)
            counts = torch.empty(cap, dtype=torch.int64, device=dev)
            hours = torch.empty(cap, dtype=torch.int32, device=dev) if hour == EACH_HOUR else None
            n = ctypes.c_int64(0)
            rc = self.ctx.L.hm_stream_extract(self.ptr, int(hour), device._ptr(keys), device._ptr(counts),
                                              device._ptr(hours), cap, ctypes.byref(n))
            if rc == _lib.HM_E_CAPACITY:
                cap = n.value + 1024
                continue
            if rc != _lib.HM_OK:
                _lib.raise_for(rc)
            return n.value, keys, counts, hours

    def counts(self, hour: int = ALLTIME) -> device.Counts:
        """Cells of one bucket (ALLTIME or an epoch hour) as host arrays."""
        n, keys, counts, _ = self.extract_device(hour)
        k = keys[:n].cpu().numpy().view(np.uint64)
        z, r, c = device.decode_keys(k)
        return device.Counts(z, r, c, counts[:n].cpu().numpy(), 0, [])

    def hourly(self):
        """{epoch hour: Counts} for every non-empty hour bucket."""
        n, keys, counts, hours = self.extract_device(EACH_HOUR)
        k = keys[:n].cpu().numpy().view(np.uint64)
        cnt = counts[:n].cpu().numpy()
        hr = hours[:n].cpu().numpy().view(np.uint32)
        out = {}
        for h in np.unique(hr).tolist():
            m = hr == h
            z, r, c = device.decode_keys(k[m])
            out[int(h)] = device.Counts(z, r, c, cnt[m], 0, [])
        return out

    def close(self):
        if getattr(self, "ptr", None):
            self.ctx.L.hm_stream_destroy(self.ptr)
            self.ptr = None

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass
