"""Drop-in for reference tile.py's Tile (projection on the gfx950 device).

Same class and classmethod names, argument meaning and exceptions as
reference tile.py:3-98.  The vectorised projections (rows_from_latitudes,
columns_from_longitudes, tile_ids_from_lat_longs) run in the HIP kernel behind
hm_project; the scalar ones (row_from_latitude, column_from_longitude,
tile_id_from_lat_long), which the reference calls once per record, run the
same arithmetic (csrc/hm_project.h) compiled for the host behind
hm_project_scalar, ~1 us a call instead of a launch and a synchronisation.
Both are bit-exact with the reference's glibc arithmetic.  Pure string
helpers (ids) are plain Python, as in the reference.

Tile utility API: tile_from_tile_id, parent_id,
parent, children and tile_ids_for_all_zoom_levels (tile.py:33-98).  Their
forward projections (the centre / quarter points re-projected one zoom up or
down) go through the same device hm_project call, batched per zoom.  The inverse
projection latitude_from_row (tile.py:23-26) is a per-tile scalar with exp/atan
that the device does not restate; it is evaluated on the host in the
reference's own operation order with the same libm, so it is bit-identical
(tests/golden/tile_utils.json).  The count pyramid never needs it: the
reference's re-projection of tile centres equals a right shift on the tile
domain, which is what the device uses.
"""
from __future__ import annotations

import math
import struct

import numpy as np

from . import _lib, device


_S = None


def _scalar_mod():
    global _S
    if _S is None:
        _lib.load()   # the library (ABI check) that the binding calls into
        try:
            from . import _hm_scalar
        except ImportError as e:   # built by heatmap_amd/build.py with the library
            raise _lib.DeviceUnavailable("heatmap_amd: the per-record binding _hm_scalar is not built "
                                         "(python -m heatmap_amd.build): %s" % e) from None
        _S = _hm_scalar
    return _S


def _bigcol(c):
    """HM_BIGCOL: the column as an integer-valued double's bits -> the
    reference's unbounded Python int (tile.py:21)."""
    return int(struct.unpack("<d", struct.pack("<q", c))[0])


def _scalar(lat, lon, zoom):
    """(status, row, col) of one point by hm_project_scalar: the kernels'
    arithmetic (csrc/hm_project.h) compiled for the host, so per-record
    callers pay well under a microsecond, not a launch and a synchronisation."""
    st, r, c = (_S or _scalar_mod()).project(lat, lon, zoom)
    if st == _lib.HM_BIGCOL:
        return _lib.HM_OK, r, _bigcol(c)
    if st == _lib.HM_E_ARG:
        raise ValueError("zoom %r outside -30..30 or not integral" % (zoom,))
    return st, r, c


def _cols(p):
    """Columns of a projection as Python ints: those beyond int64 (status
    HM_BIGCOL) come back as integer-valued doubles, exact (tile.py:21 prints
    them as unbounded ints)."""
    big = p.status == _lib.HM_BIGCOL
    if not big.any():
        return p.col
    out = p.col.astype(object)
    for i in np.flatnonzero(big).tolist():
        out[i] = int(np.array([p.col[i]], np.int64).view(np.float64)[0])
    return out


def _status(p, i=0):
    st = int(p.status[i])
    return _lib.HM_OK if st == _lib.HM_BIGCOL else st


class Tile:
    MAX_ZOOM = 16
    MIN_ZOOM = 0

    # --- projection (device) -------------------------------------------------
    @classmethod
    def tile_id_from_lat_long(cls, latitude, longitude, zoom):
        """tile.py:9-13: "z_row_col"; row is evaluated (and raises) first."""
        st, tid = (_S or _scalar_mod()).tile_id(latitude, longitude, zoom)
        if st == _lib.HM_OK and type(zoom) is int:
            return tid
        if st == _lib.HM_BIGCOL or st == _lib.HM_OK:   # (an integral float zoom keeps str(zoom): "10.0_r_c")
            st, r, c = _scalar(latitude, longitude, zoom)
            return str(zoom) + "_" + str(r) + "_" + str(c)
        if st == _lib.HM_E_ARG:
            raise ValueError("zoom %r outside -30..30 or not integral" % (zoom,))
        _lib.raise_for(st)

    @classmethod
    def row_from_latitude(cls, latitude, zoom):
        """tile.py:15-17."""
        st, r, _ = _scalar(latitude, 0.0, zoom)
        if st:
            _lib.raise_for(st)
        return r

    @classmethod
    def column_from_longitude(cls, longitude, zoom):
        """tile.py:19-21."""
        st, _, c = _scalar(0.0, longitude, zoom)
        if st:
            _lib.raise_for(st)
        return c

    # vectorised forms: one device call for many points
    @classmethod
    def rows_from_latitudes(cls, latitudes, zoom):
        lat = np.asarray(latitudes, dtype=np.float64)
        p = device.project(lat, np.zeros_like(lat), zoom, raise_errors=True)
        return p.row

    @classmethod
    def columns_from_longitudes(cls, longitudes, zoom):
        lon = np.asarray(longitudes, dtype=np.float64)
        p = device.project(np.zeros_like(lon), lon, zoom, raise_errors=True)
        return _cols(p)      # int64, or Python ints when a column passes int64

    @classmethod
    def tile_ids_from_lat_longs(cls, latitudes, longitudes, zoom):
        p = device.project(np.asarray(latitudes, np.float64), np.asarray(longitudes, np.float64), zoom,
                           raise_errors=True)
        return ["%d_%d_%d" % (zoom, r, c) for r, c in zip(p.row.tolist(), list(_cols(p)))]

    # --- ids ------------------------------------------------------------------
    @classmethod
    def tile_id_from_row_column(cls, row, column, zoom):
        """tile.py:56-58."""
        return str(zoom) + "_" + str(row) + "_" + str(column)

    @classmethod
    def decode_tile_id(cls, tileId):
        """tile.py:66-77 (None for a malformed id)."""
        parts = tileId.split("_")
        if len(parts) != 3:
            return None
        return {"id": tileId, "zoom": int(parts[0]), "row": int(parts[1]), "column": int(parts[2])}

    @classmethod
    def longitude_from_column(cls, column, zoom):
        """tile.py:28-30 (three IEEE operations)."""
        return float(column) / (2 ** zoom) * 360.0 - 180.0

    @classmethod
    def latitude_from_row(cls, row, zoom):
        """tile.py:23-26, same operation order: n = pi - 2*pi*row / 2^z, then
        180/pi * atan(sinh(n)) written as 0.5*(e^n - e^-n)."""
        n = math.pi - 2.0 * math.pi * row / (2 ** zoom)
        return 180.0 / math.pi * math.atan(0.5 * (math.exp(n) - math.exp(-n)))

    @classmethod
    def tile_from_tile_id(cls, tile_id):
        """tile.py:33-54: a Tile with its bounds and centre, or None for an id
        that does not split into three parts."""
        d = cls.decode_tile_id(tile_id)
        if d is None:
            return None
        t = Tile()
        t.tile_id = tile_id
        t.zoom, t.row, t.column = d["zoom"], d["row"], d["column"]
        t.latitude_north = Tile.latitude_from_row(t.row, t.zoom)
        t.latitude_south = Tile.latitude_from_row(t.row + 1, t.zoom)
        t.longitude_west = Tile.longitude_from_column(t.column, t.zoom)
        t.longitude_east = Tile.longitude_from_column(t.column + 1, t.zoom)
        t.center_latitude = (t.latitude_north + t.latitude_south) / 2.0
        t.center_longitude = (t.longitude_east + t.longitude_west) / 2.0
        return t

    # --- hierarchy (forward projections on the device) -------------------------
    def parent_id(self):
        """tile.py:60-61: the tile holding this tile's centre one zoom up; a
        zoom-0 tile projects at zoom -1 (2 ** -1 = 0.5), as the reference does."""
        return Tile.tile_id_from_lat_long(self.center_latitude, self.center_longitude, self.zoom - 1)

    def parent(self):
        """tile.py:63-64."""
        return Tile.tile_from_tile_id(self.parent_id())

    def children(self):
        """tile.py:88-98: ids of the tiles holding the four quarter centres one
        zoom down, in the reference's order NE, NW, SE, SW (one device call)."""
        north = (self.center_latitude + self.latitude_north) / 2
        south = (self.center_latitude + self.latitude_south) / 2
        east = (self.center_longitude + self.longitude_east) / 2
        west = (self.center_longitude + self.longitude_west) / 2
        return Tile.tile_ids_from_lat_longs([north, north, south, south], [east, west, east, west], self.zoom + 1)

    @classmethod
    def tile_ids_for_all_zoom_levels(cls, tileId):
        """tile.py:79-86: the tiles holding this tile's centre at zooms
        MAX_ZOOM down to MIN_ZOOM + 1 (range(16, 0, -1) leaves out zoom 0)."""
        t = Tile.tile_from_tile_id(tileId)
        lat, lon = np.array([t.center_latitude]), np.array([t.center_longitude])
        out = []
        for z in range(Tile.MAX_ZOOM, Tile.MIN_ZOOM, -1):
            p = device.project(lat, lon, z, raise_errors=True)
            out.append(Tile.tile_id_from_row_column(int(p.row[0]), int(_cols(p)[0]), z))
        return out
