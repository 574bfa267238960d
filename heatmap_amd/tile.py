"""Drop-in for reference tile.py's Tile (projection on the gfx950 device).

Same class and classmethod names, argument meaning and exceptions as
reference tile.py:3-98.  Projection (row_from_latitude, column_from_longitude,
tile_id_from_lat_long) runs in the HIP kernel behind hm_project -- bit-exact
with the reference's glibc arithmetic -- so every call needs the GPU; the
vectorised forms (rows_from_latitudes, ...) are what callers should use in
bulk.  Pure string helpers (ids) are plain Python, as in the reference.

Not provided on the device path yet ("next"):
latitude_from_row / tile_from_tile_id / parent / children /
tile_ids_for_all_zoom_levels, which need the reference's exp/atan inverse
projection.  The count pyramid does not need them: the reference's re-projection
of tile centres equals a right shift on the tile domain, which
is what the device uses.
"""
from __future__ import annotations

import numpy as np

from . import _lib, device


def _scalar_project(lat, lon, zoom):
    p = device.project(np.array([float(lat)]), np.array([float(lon)]), int(zoom))
    return p


class Tile:
    MAX_ZOOM = 16
    MIN_ZOOM = 0

    # --- projection (device) -------------------------------------------------
    @classmethod
    def tile_id_from_lat_long(cls, latitude, longitude, zoom):
        """tile.py:9-13: "z_row_col"; row is evaluated (and raises) first."""
        p = _scalar_project(latitude, longitude, zoom)
        st = int(p.status[0])
        if st != _lib.HM_OK:
            _lib.raise_for(st)
        return Tile.tile_id_from_row_column(int(p.row[0]), int(p.col[0]), zoom)

    @classmethod
    def row_from_latitude(cls, latitude, zoom):
        """tile.py:15-17."""
        p = _scalar_project(latitude, 0.0, zoom)
        st = int(p.status[0])
        if st != _lib.HM_OK:
            _lib.raise_for(st)
        return int(p.row[0])

    @classmethod
    def column_from_longitude(cls, longitude, zoom):
        """tile.py:19-21."""
        p = _scalar_project(0.0, longitude, zoom)
        st = int(p.status[0])
        if st != _lib.HM_OK:
            _lib.raise_for(st)
        return int(p.col[0])

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
        return p.col

    @classmethod
    def tile_ids_from_lat_longs(cls, latitudes, longitudes, zoom):
        p = device.project(np.asarray(latitudes, np.float64), np.asarray(longitudes, np.float64), zoom,
                           raise_errors=True)
        return ["%d_%d_%d" % (zoom, r, c) for r, c in zip(p.row.tolist(), p.col.tolist())]

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
        raise NotImplementedError("inverse projection (tile.py:23-26) is not on the device path yet; "
                                  "see DESIGN.md 'Next'")

    @classmethod
    def tile_from_tile_id(cls, tile_id):
        raise NotImplementedError("tile_from_tile_id needs the inverse projection (tile.py:33-54); "
                                  "see DESIGN.md 'Next'")
