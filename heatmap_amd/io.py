"""Columnar ingestion and the row sink around the device path (SURVEY.md 8f
items 1 and 3).

The reference reads `locations` from Cassandra/CosmosDB into a Spark DataFrame
(get_rows, heatmap.py:131-147), runs dataframe_loader per Row, and writes
(id, heatmap-JSON) rows back (heatmap.py:149-158).  Here:

  load_locations  columns latitude, longitude, source, user_id (timestamp
                  optional) from a pyarrow Table, a Parquet path, a pandas
                  DataFrame, a dict of arrays or a list of Row-like dicts ->
                  fp64 lat/lon, the non-background keep mask
                  (heatmap.py:27-29) and the user ids (mapped to groups by
                  heatmap.group_plan: 'x*' none, 'rt-*' route, heatmap.py:64-70)
  rows_to_table   {row_id: heatmap} -> pyarrow Table ['id', 'heatmap'] with
                  the heatmap JSON-encoded (heatmap_to_json, heatmap.py:128-129,
                  156-157), the DataFrame batchMain writes
  batch_main      load -> device count pyramid -> rows -> table, optionally
                  written as Parquet in place of the Cassandra sink

Only the I/O and the string formatting live on the host (vectorised:
numpy group coding, pyarrow string kernels); counting is hm_count +
hm_count_grouped on the GPU.
"""
from __future__ import annotations

import numpy as np

from . import heatmap

COLUMNS = ("latitude", "longitude", "source", "user_id")


def _columns(source):
    """The four columns; from Arrow / Parquet the string columns stay Arrow
    arrays (Parquet's user_id read as a dictionary: the group coding then
    needs no Python string per row, heatmap._factorize)."""
    import pyarrow as pa
    import pyarrow.parquet as pq

    if isinstance(source, str):
        source = pq.read_table(source, columns=[c for c in COLUMNS], read_dictionary=["user_id"])
    if isinstance(source, pa.Table):
        return {c: source.column(c) if c in ("source", "user_id") else source.column(c).to_numpy(zero_copy_only=False)
                for c in COLUMNS}
    if hasattr(source, "to_dict") and hasattr(source, "columns"):  # pandas DataFrame
        return {c: source[c].to_numpy() for c in COLUMNS}
    if isinstance(source, dict):
        return {c: source[c] for c in COLUMNS}
    rows = list(source)  # Row-like dicts, as Spark hands them to dataframe_loader
    return {c: [r[c] for r in rows] for c in COLUMNS}


def load_locations(source):
    """-> (lat f64[n], lon f64[n], keep u8[n], user_ids): user_ids an object
    array, or the Arrow column itself for Arrow / Parquet sources."""
    import pyarrow as pa

    cols = _columns(source)
    lat = np.ascontiguousarray(np.asarray(cols["latitude"], dtype=np.float64))
    lon = np.ascontiguousarray(np.asarray(cols["longitude"], dtype=np.float64))
    src = cols["source"]
    if isinstance(src, (pa.Array, pa.ChunkedArray)):
        import pyarrow.compute as pc

        # heatmap.py:28: row['source'] == 'background' (a null source is kept)
        keep = pc.fill_null(pc.not_equal(src, "background"), True).to_numpy(zero_copy_only=False).astype(np.uint8)
    else:
        keep = (np.asarray(src, dtype=object) != "background").astype(np.uint8)
    users = cols["user_id"]
    if not isinstance(users, (pa.Array, pa.ChunkedArray)):
        users = np.asarray(users, dtype=object)
    if not (lat.size == lon.size == keep.size == len(users)):
        raise ValueError("location columns differ in length")
    return lat, lon, keep, users


def rows_to_table(rows):
    """{row_id: {bin_id: float}} -> pyarrow Table(id: string, heatmap: string)."""
    import pyarrow as pa

    ids = list(rows)
    return pa.table({"id": pa.array(ids, pa.string()),
                     "heatmap": pa.array([heatmap.heatmap_to_json(rows[i]) for i in ids], pa.string())})


def batch_main(source, sink: str = None, max_zoom_level: int = None, delta: int = None):
    """batchMain (heatmap.py:152-158) with columnar I/O: returns the rows table
    and writes it to `sink` (Parquet) when given."""
    lat, lon, keep, users = load_locations(source)
    table = heatmap.heatmap_table(lat, lon, users, keep, max_zoom_level, delta)
    if sink:
        import pyarrow.parquet as pq

        pq.write_table(table, sink)
    return table
