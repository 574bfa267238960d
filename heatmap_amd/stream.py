"""Streaming micro-batches merged into a heatmap resident in HBM (BASELINE
config 5) -- host side of hm_stream_* (include/heatmap_amd.h).

The reference recomputes its pyramid per Spark job (heatmap.py:152-158) and
keys every bin by user group and timespan label (heatmap.py:54-55,62-75; only
'alltime' is live there, the year/month/day labels of build_timespan_label,
heatmap.py:38-52, are commented out).  StreamingHeatmap keeps one device
bucket per (user group, epoch hour); each add() runs ONE count pass over the
batch (however many hours and groups it holds) and folds its cells in.  Every
label is a device rollup of the hour buckets:

  counts(ALLTIME) / hourly()   per-cell counts of every kept point so far
  rows(timespan)               build_heatmaps' rows, {id: {bin: count}}, for
                               'alltime', 'year', 'month' or 'day' (UTC dates
                               of the epoch hours), with the reference's user
                               groups and level-by-level 'all' weighting
                               (heatmap.heatmap.combine_cells)

so a caller sees the same rows as heatmap.assemble_rows over every point so
far, restricted to the label's period.

Kept points whose zoom-zmax tile lies outside [0, 2^zmax)^2 (|lat| > 85.0511,
lon outside [-180, 180): the reference bins them, tile.py:17,21 never clamp)
do not fit the resident table's keys.  A batch holding any (hm_stream_add
answers HM_E_EXOTIC before inserting anything) is split on the device: the
in-square points go to the table, the out-of-square ones are counted per
(group, hour) by hm_count_grouped and their (rare, pre-aggregated) cell
records are kept beside the table and joined into every rollup.
"""
from __future__ import annotations

import ctypes
import datetime

import numpy as np

from . import _lib, device
from . import heatmap as _hm

ALLTIME = -1
EACH_HOUR = -2
MAX_HOURS = 1 << 28
SPANS = {"hour": _lib.HM_SPAN_HOUR, "day": _lib.HM_SPAN_DAY, "month": _lib.HM_SPAN_MONTH,
         "year": _lib.HM_SPAN_YEAR, "alltime": _lib.HM_SPAN_ALLTIME}
NOGROUP = 0xFFFFFFFE      # kept points whose user id makes no group ('x*', or no user ids)
ALLGROUPS = 0xFFFFFFFF    # merged rollups


UNDATED_HOUR = -1         # hour of points added without one (alltime only)


def _sum_records(rec: np.ndarray, w: int) -> np.ndarray:
    """Sum column w of int64 records over equal leading columns [0, w)."""
    if not len(rec):
        return rec
    u, inv = np.unique(rec[:, :w], axis=0, return_inverse=True)
    tot = np.zeros(len(u), dtype=np.int64)
    np.add.at(tot, inv.reshape(-1), rec[:, w])
    return np.concatenate([u, tot[:, None]], axis=1)


def _period(timespan: str, hour: np.ndarray) -> np.ndarray:
    """hm_stream_rollup's period of each epoch hour: the hour, days since
    1970-01-01, year * 12 + month - 1, or the year (UTC civil calendar)."""
    if timespan == "hour":
        return hour
    days = hour // 24
    if timespan == "day":
        return days
    z = days + 719468                    # civil_from_days (H. Hinnant), as k_stream_rollup
    era = np.floor_divide(z, 146097)
    doe = z - era * 146097
    yoe = (doe - doe // 1460 + doe // 36524 - doe // 146096) // 365
    doy = doe - (365 * yoe + yoe // 4 - yoe // 100)
    mp = (5 * doy + 2) // 153
    m = np.where(mp < 10, mp + 3, mp - 9)
    y = yoe + era * 400 + (m <= 2)
    return y * 12 + m - 1 if timespan == "month" else y


def span_label(timespan: str, period: int) -> str:
    """build_timespan_label (heatmap.py:38-52) of a rollup period: days since
    1970-01-01, year*12 + month - 1, or the year."""
    if timespan == "alltime":
        return "alltime"
    if timespan == "day":
        d = datetime.date(1970, 1, 1) + datetime.timedelta(days=int(period))
    elif timespan == "month":
        d = datetime.date(int(period) // 12, int(period) % 12 + 1, 1)
    elif timespan == "year":
        d = datetime.date(int(period), 1, 1)
    else:
        raise ValueError("no reference timespan label for %r" % (timespan,))
    return _hm.build_timespan_label(timespan, d)


class StreamingHeatmap:
    def __init__(self, zmin: int = 0, zmax: int = 18, base_hour: int = 0, initial_cells: int = 1 << 20,
                 device_index: int = 0, max_buckets: int = 0):
        self._torch = device._torch()
        self.ctx = device.context(device_index)
        self.device_index = device_index
        self.zmin, self.zmax, self.base_hour = int(zmin), int(zmax), int(base_hour)
        self.labels = ["all"]          # group id -> row-key group (0: the literal user id 'all')
        self._explicit_max = -1        # largest group id passed as group= (those have no label)
        self._index = {"all": 0}
        # cells outside [0, 2^zmax)^2: (group, hour or UNDATED_HOUR, zoom, row, col, count)
        self._x = np.zeros((0, 6), dtype=np.int64)
        p = ctypes.c_void_p()
        rc = self.ctx.L.hm_stream_create(self.ctx.ptr, self.zmin, self.zmax, self.base_hour, int(initial_cells),
                                         int(max_buckets), ctypes.byref(p))
        if rc != _lib.HM_OK:
            _lib.raise_for(rc)
        self.ptr = p

    # ------------------------------------------------------------------ input

    def _groups(self, user_id, keep, n):
        """Persistent group ids of a batch's user ids (heatmap.py:64-70): kept
        points only are validated, as heatmap.group_plan does."""
        if len(user_id) != n:
            raise ValueError("user_id must have one entry per point")
        if keep is None:
            kb = np.ones(n, dtype=bool)
        else:
            kb = (keep.cpu().numpy() if hasattr(keep, "cpu") else np.asarray(keep)).astype(bool)
        codes, uniques = _hm._factorize(user_id)
        kept_codes = np.unique(codes[kb])
        if kept_codes.size and kept_codes[0] < 0:
            raise TypeError("'NoneType' object is not subscriptable")
        lut = np.full(len(uniques) + 1, NOGROUP, dtype=np.uint32)   # code -1 -> last entry
        for c in kept_codes.tolist():
            u = uniques[c]
            if not isinstance(u, str):
                raise TypeError("user id %r is not a string" % (u,))
            if _hm.KEY_SEPERATOR in u:
                raise ValueError("user id %r contains the key separator %r" % (u, _hm.KEY_SEPERATOR))
            if u[:1] == "x":
                continue
            label = "route" if u[:3] == "rt-" else u
            if label not in self._index:
                self._index[label] = len(self.labels)
                self.labels.append(label)
            lut[c] = self._index[label]
        return lut[codes]

    def add(self, lat, lon, keep=None, hour=None, user_id=None, group=None):
        """Fold one micro-batch in.  hour: uint32 epoch hours (one per point)
        or None (undated: alltime only).  user_id: the reference's user id per
        point (host strings), or group: explicit uint32 group ids.  Projection
        errors raise as hm_count's do; a failing batch changes no counts."""
        torch = self._torch
        self.ctx.bind_stream()
        la = device._dev(lat, torch.float64, self.device_index)
        lo = device._dev(lon, torch.float64, self.device_index)
        n = la.numel()
        if lo.numel() != n:
            raise ValueError("lat and lon must have the same length")
        if user_id is not None and group is not None:
            raise ValueError("pass user_id or group, not both")
        if user_id is not None:
            group = self._groups(user_id, keep, n)
        elif group is not None:
            # explicit ids: NOGROUP / ALLGROUPS are the table's own markers
            gmax = int((group.to(torch.int64) & 0xFFFFFFFF).max().item()) if isinstance(group, torch.Tensor) and \
                group.numel() else (int(np.asarray(group, dtype=np.uint32).max()) if np.size(group) else 0)
            if gmax >= NOGROUP:
                raise ValueError("group ids must be < 0x%X (0xFFFFFFFE/0xFFFFFFFF are reserved)" % NOGROUP)
            self._explicit_max = max(self._explicit_max, gmax)

        def u32(x, what):
            if x is None:
                return None
            if not isinstance(x, torch.Tensor):
                x = torch.from_numpy(np.ascontiguousarray(np.asarray(x, dtype=np.uint32)).view(np.int32))
            t = device._dev(x, torch.int32, self.device_index)  # uint32 bits
            if t.numel() != n:
                raise ValueError("%s must have one entry per point" % what)
            return t

        hr = u32(hour, "hour")
        gr = u32(group, "group")
        kp = device._dev(keep, torch.uint8, self.device_index) if keep is not None else None
        if kp is not None and kp.numel() != n:
            raise ValueError("keep must have one entry per point")
        rc = self.ctx.L.hm_stream_add(self.ptr, device._ptr(la), device._ptr(lo), device._ptr(kp), device._ptr(hr),
                                      device._ptr(gr), n)
        if rc == _lib.HM_E_EXOTIC:
            self._add_split(la, lo, kp, hr, gr, n)
            return
        if rc != _lib.HM_OK:
            idx, kind = self.ctx.last_error()
            _lib.raise_for(rc, idx)

    def _add_split(self, la, lo, kp, hr, gr, n):
        """The batch holds kept points outside the square: project once on the
        device (zoom zmax), insert the in-square ones, count the others per
        (group, hour) with hm_count_grouped.  A projection error raises before
        anything is inserted (hm_stream_add checks the whole batch)."""
        torch = self._torch
        row = torch.empty(n, dtype=torch.int64, device=la.device)
        col = torch.empty(n, dtype=torch.int64, device=la.device)
        st = torch.empty(n, dtype=torch.uint8, device=la.device)
        rc = self.ctx.L.hm_project(self.ctx.ptr, device._ptr(la), device._ptr(lo), n, self.zmax, device._ptr(row),
                                   device._ptr(col), device._ptr(st))
        if rc != _lib.HM_OK:      # before anything is inserted: the batch stays atomic
            idx, kind = self.ctx.last_error()
            _lib.raise_for(rc, idx)
        lim = 1 << self.zmax
        out = (st == 0) & ((row < 0) | (row >= lim) | (col < 0) | (col >= lim))
        if kp is not None:
            out &= kp != 0
        keep_in = (~out).to(torch.uint8) if kp is None else (kp * (~out).to(torch.uint8))
        rc = self.ctx.L.hm_stream_add(self.ptr, device._ptr(la), device._ptr(lo), device._ptr(keep_in),
                                      device._ptr(hr), device._ptr(gr), n)
        if rc != _lib.HM_OK:
            idx, kind = self.ctx.last_error()
            _lib.raise_for(rc, idx)
        sel = out.nonzero().flatten()
        g = (gr[sel].to(torch.int64) & 0xFFFFFFFF) if gr is not None else torch.full_like(sel, NOGROUP)
        h = (hr[sel].to(torch.int64) & 0xFFFFFFFF) if hr is not None else torch.full_like(sel, UNDATED_HOUR)
        pair, inv = torch.unique(torch.stack([g, h], 1), dim=0, return_inverse=True)
        gc = device.count_grouped(la[sel], lo[sel], inv.to(torch.int32), None, self.zmin, self.zmax,
                                  device=self.device_index)
        pg = pair.cpu().numpy()[gc.group.astype(np.int64)]
        rec = np.stack([pg[:, 0], pg[:, 1], gc.zoom.astype(np.int64), gc.row, gc.col, gc.count.astype(np.int64)],
                       axis=1)
        self._x = _sum_records(np.concatenate([self._x, rec]), 5)

    # ---------------------------------------------------------------- queries

    def cells(self):
        """(distinct (bucket, cell) pairs held, cell-log capacity); compacts
        the log (one bucketed merge) when it holds repeated keys"""
        a, b = ctypes.c_int64(0), ctypes.c_int64(0)
        rc = self.ctx.L.hm_stream_cells(self.ptr, ctypes.byref(a), ctypes.byref(b), None)
        if rc != _lib.HM_OK:
            _lib.raise_for(rc)
        return a.value, b.value

    def _log_capacity(self) -> int:
        b = ctypes.c_int64(0)
        self.ctx.L.hm_stream_cells(self.ptr, None, ctypes.byref(b), None)
        return b.value

    def buckets(self) -> int:
        """(group, period) buckets in use, rollup labels included"""
        c = ctypes.c_int64(0)
        self.ctx.L.hm_stream_cells(self.ptr, None, None, ctypes.byref(c))
        return c.value

    def rollup_device(self, timespan: str = "alltime", merge_groups: bool = True, select: int = -1):
        """(n, keys, counts, groups, periods) as torch CUDA tensors: the cells
        of `timespan` summed per (group, period), or over every group."""
        torch = self._torch
        self.ctx.bind_stream()
        span = SPANS[timespan]
        # start from the last rollup of this kind (the log's capacity doubles as
        # batches arrive and can far exceed the distinct cells): a short
        # estimate costs one HM_E_CAPACITY retry with the exact size
        memo = self.__dict__.setdefault("_rollup_n", {})
        mk = (span, bool(merge_groups), int(select))
        cap = min(max(1024, self._log_capacity()), max(1024, int(memo.get(mk, 1 << 20) * 1.25) + 1024))
        dev = "cuda:%d" % self.device_index
        while True:
            keys = torch.empty(cap, dtype=torch.int64, device=dev)
            counts = torch.empty(cap, dtype=torch.int64, device=dev)
            groups = torch.empty(cap, dtype=torch.int32, device=dev)
            periods = torch.empty(cap, dtype=torch.int32, device=dev)
            n = ctypes.c_int64(0)
            rc = self.ctx.L.hm_stream_rollup(self.ptr, span, int(bool(merge_groups)), int(select), device._ptr(keys),
                                             device._ptr(counts), device._ptr(groups), device._ptr(periods), cap,
                                             ctypes.byref(n))
            if rc == _lib.HM_E_CAPACITY and n.value > cap:
                cap = n.value + 1024
                continue
            if rc != _lib.HM_OK:
                _lib.raise_for(rc)
            memo[mk] = n.value
            return n.value, keys, counts, groups, periods

    def rollup(self, timespan: str = "alltime", merge_groups: bool = True, select: int = -1):
        """Host arrays (group u32, period u32, zoom, row, col, count), cells
        outside the square included."""
        n, keys, counts, groups, periods = self.rollup_device(timespan, merge_groups, select)
        z, r, c = device.decode_keys(keys[:n].cpu().numpy().view(np.uint64))
        out = (groups[:n].cpu().numpy().view(np.uint32), periods[:n].cpu().numpy().view(np.uint32), z, r, c,
               counts[:n].cpu().numpy())
        if not len(self._x):
            return out
        x = self._exotic_rollup(timespan, merge_groups, select)
        return tuple(np.concatenate([a, b.astype(a.dtype)]) for a, b in zip(out, x))

    def _exotic_rollup(self, timespan, merge_groups, select):
        """The out-of-square records summed per (group, period) of `timespan`
        (the periods hm_stream_rollup uses)."""
        g, h, z, r, c, n = self._x.T
        dated = h != UNDATED_HOUR
        if timespan == "alltime":
            period = np.zeros_like(h)
        else:
            g, h, z, r, c, n = g[dated], h[dated], z[dated], r[dated], c[dated], n[dated]
            period = _period(timespan, h)
        if select >= 0:
            m = period == select
            g, period, z, r, c, n = g[m], period[m], z[m], r[m], c[m], n[m]
        if merge_groups:
            g = np.full_like(g, ALLGROUPS)
        rec = _sum_records(np.stack([g, period, z, r, c, n], axis=1), 5) if len(g) else np.zeros((0, 6), np.int64)
        return (rec[:, 0].astype(np.uint32), rec[:, 1].astype(np.uint32), rec[:, 2].astype(np.int32), rec[:, 3],
                rec[:, 4], rec[:, 5])

    def extract_device(self, hour: int = ALLTIME):
        """(n, keys, counts, hours) as torch CUDA tensors (hm_count key
        layout), summed over groups: hour = ALLTIME, EACH_HOUR or one hour."""
        if hour == ALLTIME:
            n, k, c, _, _ = self.rollup_device("alltime")
            return n, k, c, None
        n, k, c, _, p = self.rollup_device("hour", True, -1 if hour == EACH_HOUR else int(hour))
        return n, k, c, (p if hour == EACH_HOUR else None)

    def counts(self, hour: int = ALLTIME) -> device.Counts:
        """Cells of every kept point (ALLTIME) or of one epoch hour (cells
        outside the square included)."""
        n, keys, counts, _ = self.extract_device(hour)
        z, r, c = device.decode_keys(keys[:n].cpu().numpy().view(np.uint64))
        cnt = counts[:n].cpu().numpy()
        if len(self._x):
            _, _, xz, xr, xc, xn = self._exotic_rollup("alltime" if hour == ALLTIME else "hour", True,
                                                       -1 if hour == ALLTIME else int(hour))
            z, r, c, cnt = (np.concatenate([z, xz.astype(z.dtype)]), np.concatenate([r, xr]),
                            np.concatenate([c, xc]), np.concatenate([cnt, xn]))
        return device.Counts(z, r, c, cnt, 0, [])

    def hourly(self):
        """{epoch hour: Counts} for every non-empty hour."""
        _, hr, z, r, c, cnt = self.rollup("hour")
        out = {}
        for h in np.unique(hr).tolist():
            m = hr == h
            out[int(h)] = device.Counts(z[m], r[m], c[m], cnt[m], 0, [])
        return out

    def heatmap_cells(self, timespan: str = "alltime", max_zoom_level=None, delta=None) -> "_hm.Cells":
        """The bins of build_heatmaps' rows for `timespan` ('alltime', 'year',
        'month', 'day'): every period of the span, each with its label."""
        d = _hm.DETAIL_ZOOM_DELTA if delta is None else int(delta)
        mz = self.zmax - d if max_zoom_level is None else int(max_zoom_level)
        if mz + d != self.zmax or self.zmin > d + 1:
            raise ValueError("rows need zooms %d..%d; the stream holds %d..%d" % (d + 1, mz + d, self.zmin, self.zmax))
        if timespan not in ("alltime", "year", "month", "day"):
            raise ValueError("timespan must be 'alltime', 'year', 'month' or 'day'")
        if self._explicit_max >= len(self.labels):
            raise ValueError("rows need a label per group: group id %d was passed as group= and has none "
                             "(feed the stream with user_id= to build rows)" % self._explicit_max)
        _, ap, az, ar, ac, an = self.rollup(timespan, merge_groups=True)
        gg, gp, gz, gr, gc, gn = self.rollup(timespan, merge_groups=False)
        grouped = gg != NOGROUP
        gg, gp, gz, gr, gc, gn = gg[grouped], gp[grouped], gz[grouped], gr[grouped], gc[grouped], gn[grouped]
        parts = []
        for p in np.unique(ap).tolist():
            m, q = ap == p, gp == p
            parts.append(_hm.combine_cells(self.labels, (az[m], ar[m], ac[m], an[m]),
                                           (gg[q].astype(np.int64), gz[q], gr[q], gc[q], gn[q]), mz + d, d,
                                           span_label(timespan, p)))
        return _hm.concat_cells(parts, self.labels, d)

    def rows(self, timespan: str = "alltime", max_zoom_level=None, delta=None) -> dict:
        """{row_id: {bin_id: float}} as build_heatmaps would give over every
        point so far, row ids '<group>|<timespan label>|<tile>'."""
        return _hm.cells_to_rows(self.heatmap_cells(timespan, max_zoom_level, delta))

    def table(self, timespan: str = "alltime", max_zoom_level=None, delta=None):
        """The same rows as a pyarrow Table(id, heatmap JSON)."""
        return _hm.cells_to_table(self.heatmap_cells(timespan, max_zoom_level, delta))

    def close(self):
        if getattr(self, "ptr", None):
            self.ctx.L.hm_stream_destroy(self.ptr)
            self.ptr = None

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass
