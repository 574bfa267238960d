"""ctypes binding of the C-ABI in include/heatmap_amd.h.

This module is the reference-side binding INTEGRATION.md describes: it is
exactly what a maintainer of timfpark/heatmap would add to call the library.
There is no CPU fallback: without the built library or a GPU every entry
point raises.
"""
from __future__ import annotations

import ctypes
import os
import threading

from . import build as _build

HM_OK = 0
HM_E_NAN = 1
HM_E_DOMAIN = 2
HM_E_INF = 3
HM_E_RANGE = 8
HM_BIGCOL = 10        # hm_project: column beyond int64, returned as an integer-valued double's bits
HM_E_EXOTIC = 9
HM_E_ARG = 16
HM_E_CAPACITY = 17
HM_E_HIP = 18
HM_E_NOMEM = 19
HM_E_WIDE = 20        # hm_cells_route with u32 counts: a count needs 64 bits
HM_CELLS_U64, HM_CELLS_U32, HM_CELLS_REC10, HM_CELLS_G12 = 8, 4, 10, 12   # exchanged cell layouts
HM_COUNT_MAX_ZOOM = 21
HM_ABI_VERSION = 7
HM_SPAN_HOUR, HM_SPAN_DAY, HM_SPAN_MONTH, HM_SPAN_YEAR, HM_SPAN_ALLTIME = 0, 1, 2, 3, 4

EXPORTS = ["hm_abi_version", "hm_status_string", "hm_ctx_create", "hm_ctx_set_stream", "hm_ctx_destroy", "hm_ctx_tune",
           "hm_project", "hm_project_scalar", "hm_count", "hm_count_tiles", "hm_count_grouped", "hm_count_grouped_tiles",
           "hm_count_grouped_packed", "hm_count_grouped_packed_tiles", "hm_last_error", "hm_last_stats", "hm_synth",
           "hm_stream_create", "hm_stream_add", "hm_stream_cells", "hm_stream_rollup", "hm_stream_extract",
           "hm_stream_destroy",
           "hm_dense_grid_size", "hm_cells_route", "hm_cells_merge", "hm_cells_merge_runs",
           "hm_cells_route_pieces", "hm_cells_merge_pieces", "hm_dense_cells", "hm_format_bins", "hm_format_ids", "hm_bench_read"]

_LIB = None
_LOCK = threading.Lock()


class DeviceUnavailable(RuntimeError):
    pass


class DevicePathUnsupported(NotImplementedError):
    """Input the reference accepts but this device path does not bin yet."""


def lib_path() -> str:
    return _build.LIB


def load() -> ctypes.CDLL:
    """Load the native library (building it first if sources are newer)."""
    global _LIB
    with _LOCK:
        if _LIB is not None:
            return _LIB
        path = os.environ.get("HM_LIB_PATH") or _build.LIB
        if path == _build.LIB and (not os.path.exists(path) or _build._stale()):
            try:
                _build.build(verbose=False)
            except Exception as e:  # pragma: no cover - surfaced to the caller
                raise DeviceUnavailable("heatmap_amd: cannot build %s: %s" % (path, e)) from e
        # torch first: the library then binds the HIP runtime torch loaded
        # (one runtime per process; loading ours first left torch's without
        # devices on the GPU box)
        try:
            import torch  # noqa: F401
        except ImportError:  # pragma: no cover - torch is part of the image
            pass
        L = ctypes.CDLL(path)
        if L.hm_abi_version() != HM_ABI_VERSION:
            raise DeviceUnavailable("heatmap_amd: %s has ABI %d, this binding needs %d"
                                    % (path, L.hm_abi_version(), HM_ABI_VERSION))
        c = ctypes
        P = c.POINTER
        vp = c.c_void_p
        L.hm_abi_version.restype = c.c_int
        L.hm_status_string.argtypes = [c.c_int]
        L.hm_status_string.restype = c.c_char_p
        L.hm_ctx_create.argtypes = [P(vp), c.c_int, vp]
        L.hm_ctx_set_stream.argtypes = [vp, vp]
        L.hm_ctx_destroy.argtypes = [vp]
        L.hm_ctx_tune.argtypes = [vp, c.c_char_p, c.c_double, P(c.c_double)]
        L.hm_project.argtypes = [vp, vp, vp, c.c_int64, c.c_int, vp, vp, vp]
        L.hm_project_scalar.argtypes = [c.c_double, c.c_double, c.c_int, vp]
        L.hm_project_scalar.restype = c.c_int
        L.hm_count.argtypes = [vp, vp, vp, vp, c.c_int64, c.c_int, c.c_int, vp, vp, c.c_int64, P(c.c_int64),
                               vp, c.c_int64, P(c.c_int64)]
        L.hm_count_tiles.argtypes = [vp, vp, vp, vp, c.c_int64, c.c_int, c.c_int, vp, vp, c.c_int64, P(c.c_int64),
                                     vp, c.c_int64, P(c.c_int64)]
        L.hm_count_grouped.argtypes = [vp, vp, vp, vp, vp, c.c_int64, c.c_int, c.c_int, vp, c.c_int64,
                                       P(c.c_int64)]
        L.hm_count_grouped_tiles.argtypes = L.hm_count_grouped.argtypes
        L.hm_count_grouped_packed.argtypes = [vp, vp, vp, vp, vp, c.c_int64, c.c_int, c.c_int, vp, vp, c.c_int64,
                                              P(c.c_int64)]
        L.hm_count_grouped_packed_tiles.argtypes = L.hm_count_grouped_packed.argtypes
        L.hm_last_error.argtypes = [vp, P(c.c_int64), P(c.c_int)]
        L.hm_last_stats.argtypes = [vp, P(c.c_int64), P(c.c_double), c.c_int]
        L.hm_synth.argtypes = [vp, c.c_int, c.c_uint64, c.c_int64, c.c_int64, vp, vp, vp, c.c_int]
        L.hm_bench_read.argtypes = [vp, vp, vp, c.c_int64, vp]
        L.hm_stream_create.argtypes = [vp, c.c_int, c.c_int, c.c_uint32, c.c_int64, c.c_int64, P(vp)]
        L.hm_stream_add.argtypes = [vp, vp, vp, vp, vp, vp, c.c_int64]
        L.hm_stream_cells.argtypes = [vp, P(c.c_int64), P(c.c_int64), P(c.c_int64)]
        L.hm_stream_rollup.argtypes = [vp, c.c_int, c.c_int, c.c_int64, vp, vp, vp, vp, c.c_int64, P(c.c_int64)]
        L.hm_stream_extract.argtypes = [vp, c.c_int64, vp, vp, vp, c.c_int64, P(c.c_int64)]
        L.hm_stream_destroy.argtypes = [vp]
        L.hm_dense_grid_size.argtypes = [c.c_int]
        L.hm_dense_grid_size.restype = c.c_int64
        L.hm_cells_route.argtypes = [vp, vp, vp, c.c_int64, c.c_int, c.c_int, c.c_int, vp, vp, vp, c.c_int,
                                     P(c.c_int64)]
        L.hm_cells_merge.argtypes = [vp, vp, vp, c.c_int, c.c_int64, vp, vp, c.c_int64, P(c.c_int64)]
        L.hm_cells_merge_runs.argtypes = [vp, vp, vp, c.c_int, c.c_int64, P(c.c_int64), c.c_int, vp, vp, c.c_int64,
                                          P(c.c_int64)]
        L.hm_cells_route_pieces.argtypes = [vp, vp, vp, c.c_int64, c.c_int, c.c_int, c.c_int, c.c_int, c.c_int, vp,
                                            vp, vp, c.c_int, vp, c.c_int]
        L.hm_cells_merge_pieces.argtypes = [vp, c.c_int, c.c_int, P(vp), P(vp), P(c.c_int64), c.c_int, vp, vp,
                                            c.c_int64, P(c.c_int64)]
        L.hm_dense_cells.argtypes = [vp, vp, c.c_int, vp, vp, c.c_int64, P(c.c_int64)]
        L.hm_format_bins.argtypes = [vp, vp, vp, vp, vp, vp, vp, vp, c.c_int64, vp]
        L.hm_format_ids.argtypes = [vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, c.c_int64, vp]
        for name in EXPORTS:
            getattr(L, name).restype = getattr(L, name).restype or c.c_int
        L.hm_status_string.restype = c.c_char_p
        _LIB = L
        return L


def status_string(st: int) -> str:
    return load().hm_status_string(int(st)).decode()


def raise_for(st: int, index: int = -1):
    """Raise the reference's exception for a per-point error kind."""
    if st == HM_OK:
        return
    per_point = st in (HM_E_NAN, HM_E_DOMAIN, HM_E_INF, HM_E_RANGE, HM_E_EXOTIC)
    where = "" if index < 0 or not per_point else " (point %d)" % index
    if st == HM_E_NAN:
        raise ValueError("cannot convert float NaN to integer")
    if st == HM_E_DOMAIN:
        raise ValueError("math domain error")
    if st == HM_E_INF:
        raise OverflowError("cannot convert float infinity to integer")
    if st in (HM_E_RANGE, HM_E_EXOTIC):
        raise DevicePathUnsupported(status_string(st) + where)
    if st == HM_E_HIP:
        raise DeviceUnavailable(status_string(st))
    if st == HM_E_NOMEM:
        raise MemoryError(status_string(st))
    raise RuntimeError("heatmap_amd: %s%s" % (status_string(st), where))
