"""Drop-in for reference heatmap.py's hot path (dataframe_loader + build_heatmaps).

Same names, constants, key layout and output rows as reference
heatmap.py:16-129:

  row id   "<group>|alltime|<z-DELTA>_<row>_<col>"      (heatmap.py:55,85-90)
  heatmap  {"<z>_<row>_<col>": float count}             (heatmap.py:120-126)
  groups   'all' for every kept location, plus the user id unless it starts
           with 'x', 'rt-*' folded into 'route'          (heatmap.py:64-70)
  zooms    detail zooms MAX_ZOOM_LEVEL+DELTA down to DELTA+1 (heatmap.py:109)

Counting runs on the device in two passes over the points, whatever the
number of users:
  hm_count          every kept point, per (zoom, row, col)  -> n
  hm_count_grouped  kept points with a group, per (group, zoom, row, col)
User ids are dictionary-encoded on the host (vectorised) into u32 group ids;
group 0 is the literal user id 'all'.  The reference re-emits every level's
'all' bins under user id 'all', which doubles 'all' once per level; with
a = kept points whose user id is literally 'all' and U = kept points of every
other group, the 'all' count of a cell k levels below the detail zoom is
    2^k (n + a) + (2^k - 1) U
(closed form verified against the reference).
Counts are integers on the device and exact as floats while below 2^53.

Every coarser tile is the arithmetic shift of the detail-zoom tile.  The
reference re-projects tile centres instead (heatmap.py:60-61,89); the two
agree on the windows heatmap_amd/chain_window.py lists (generated and checked
tile by tile by tools/chain_window.c; they contain [0, 2^z)^2 at every zoom).
Detail tiles outside them (within ~1e-6 deg of a pole, or |lon| > 11520) take
the reference's literal chain instead (ChainFix: centres by the reference's
inverse projection, re-projected on the device), and their counts move from
the shift's cells to the tiles that chain reaches.

build_heatmaps(locations) keeps the reference's RDD-shaped interface for
locations produced by dataframe_loader (all with count 1.0 and tileId at the
detail zoom); build_heatmaps_columnar returns the same {row_id: heatmap} dict
from columns, and heatmap_table the (id, heatmap-JSON) rows as a pyarrow
Table built without per-cell Python objects.
"""
from __future__ import annotations

import json

import numpy as np

from . import _lib, chain_window, device
from .tile import Tile

DETAIL_ZOOM_DELTA = 5
MAX_ZOOM_LEVEL = 16
KEY_SEPERATOR = "|"
KEY_FIELD = 0
VALUE_FIELD = 1


# --------------------------------------------------------------------------
# per-record functions (reference signatures)
# --------------------------------------------------------------------------

def dataframe_loader(row):
    """heatmap.py:25-36: project at the detail zoom, THEN drop background."""
    tileId = Tile.tile_id_from_lat_long(row["latitude"], row["longitude"], MAX_ZOOM_LEVEL + DETAIL_ZOOM_DELTA)
    if row["source"] == "background":
        return []
    return [{"tileId": tileId, "timestamp": row["timestamp"], "userId": row["user_id"], "count": 1.0}]


def build_timespan_label(timespanType, localDate):
    """heatmap.py:38-52 (the batch pipeline's only label is 'alltime',
    heatmap.py:62-63; the streaming heatmap serves the others)."""
    month = "%02d" % localDate.month
    day = "%02d" % localDate.day
    if timespanType == "alltime":
        return "alltime"
    if timespanType == "year":
        return str(localDate.year)
    if timespanType == "month":
        return str(localDate.year) + "-" + month
    if timespanType == "day":
        return str(localDate.year) + "-" + month + "-" + day
    return None


def build_tile_composite_key(userId, tileId, timespanLabel):
    """heatmap.py:54-55."""
    return userId + KEY_SEPERATOR + timespanLabel + KEY_SEPERATOR + tileId


def user_groups(user_id):
    """Groups a location contributes to at the detail zoom (heatmap.py:64-70)."""
    groups = ["all"]
    if not user_id[:1] == "x":
        groups.append("route" if user_id[:3] == "rt-" else user_id)
    return groups


def list_to_dict(heatmapList):
    """heatmap.py:120-126."""
    out = {}
    for entry in heatmapList:
        out[entry["tileId"]] = entry["count"]
    return out


def heatmap_to_json(heatmap):
    """heatmap.py:128-129."""
    return json.dumps(heatmap)


def heatmap_to_locations(bucket):
    """heatmap.py:92-105."""
    parts = bucket[KEY_FIELD].split(KEY_SEPERATOR)
    return [{"userId": parts[0], "count": c, "tileId": t, "timespan": parts[1]}
            for t, c in bucket[VALUE_FIELD].items()]


# --------------------------------------------------------------------------
# group coding (host, vectorised over distinct user ids)
# --------------------------------------------------------------------------

class GroupPlan:
    """labels[g] is the row-key group of group id g (labels[0] = 'all', the
    literal user id, merged into the 'all' rows); gid: u32 group of every
    point; grouped: points counted per group (kept, user id not 'x*')."""

    def __init__(self, labels, gid, grouped):
        self.labels = labels
        self.gid = gid
        self.grouped = grouped


def _factorize(user_id):
    """(codes int32[n], uniques): the user ids dictionary-encoded, -1 for None.

    An Arrow column (pyarrow Array / ChunkedArray of strings, or already
    dictionary-encoded -- io.load_locations reads Parquet's user_id as a
    dictionary) is encoded by Arrow's C++ kernels without building one Python
    string per row; a pandas Categorical hands over its codes; anything else
    goes through pandas.factorize."""
    try:
        import pyarrow as pa
    except ImportError:  # pragma: no cover - pyarrow is part of the image
        pa = None
    if pa is not None and isinstance(user_id, (pa.Array, pa.ChunkedArray)):
        import pyarrow.compute as pc

        arr = user_id.combine_chunks() if isinstance(user_id, pa.ChunkedArray) else user_id
        if not pa.types.is_dictionary(arr.type):
            arr = pc.dictionary_encode(arr)
        idx = arr.indices
        codes = idx.fill_null(-1).to_numpy(zero_copy_only=False).astype(np.int32, copy=False)
        return codes, arr.dictionary.to_pylist()
    if hasattr(user_id, "codes") and hasattr(user_id, "categories"):   # pandas Categorical
        return np.asarray(user_id.codes, dtype=np.int32), list(user_id.categories)
    try:
        import pandas as pd

        codes, uniques = pd.factorize(np.asarray(user_id, dtype=object), use_na_sentinel=True)
        return codes.astype(np.int32), list(uniques)
    except ImportError:  # pragma: no cover - pandas is part of the image
        uniq, inv = np.unique(np.array([str(u) if u is not None else "\0none" for u in user_id]), return_inverse=True)
        u = [None if x == "\0none" else x for x in uniq.tolist()]
        codes = inv.astype(np.int32)
        if None in u:
            codes[codes == u.index(None)] = -1
        return codes, u


def group_plan(user_id, keep=None) -> GroupPlan:
    """Dictionary-encode the user ids of the kept points into groups
    (heatmap.py:64-70).  Background rows are dropped before their user id is
    read (heatmap.py:28-35), so only kept rows raise: a None id as the
    reference's None[:1] would (TypeError), an id containing the key separator
    as ValueError (heatmap.py:80-84 would mis-split its keys).  Linear in the
    rows (a histogram of the codes, not a sort); the per-id work is over the
    distinct ids only."""
    n = len(user_id)
    keep = np.ones(n, dtype=bool) if keep is None else np.asarray(keep).astype(bool, copy=False)
    codes, uniques = _factorize(user_id)
    # which codes occur among the kept rows (slot 0: None)
    seen = np.bincount(codes[keep] + 1 if not keep.all() else codes + 1, minlength=len(uniques) + 1)
    if seen[0]:
        raise TypeError("'NoneType' object is not subscriptable")
    kept_codes = np.flatnonzero(seen[1:])
    labels = ["all"]
    index = {"all": 0}
    lut = np.full(len(uniques) + 1, -1, dtype=np.int32)      # code + 1 -> group id; -1: no group
    for c in kept_codes.tolist():
        u = uniques[c]
        if not isinstance(u, str):
            raise TypeError("user id %r is not a string" % (u,))
        if KEY_SEPERATOR in u:
            raise ValueError("user id %r contains the key separator %r (heatmap.py:80-84 would mis-split it)"
                             % (u, KEY_SEPERATOR))
        if u[:1] == "x":
            continue
        label = "route" if u[:3] == "rt-" else u
        if label not in index:
            index[label] = len(labels)
            labels.append(label)
        lut[c + 1] = index[label]
    g = lut[codes + 1]
    grouped = keep & (g >= 0)
    np.maximum(g, 0, out=g)
    return GroupPlan(labels, g.view(np.uint32), grouped)


# --------------------------------------------------------------------------
# cells: the heatmap bins as arrays
# --------------------------------------------------------------------------

class Cells:
    """Every bin of every output row: labels[label[i]] | spans[span[i]] |
    zoom[i]-delta tile of (row[i], col[i]) -> {zoom[i]_row[i]_col[i]: value[i]}.
    The batch pipeline's only timespan label is 'alltime' (heatmap.py:62-63);
    the streaming heatmap's rollups carry year / month / day labels too."""

    def __init__(self, labels, label, zoom, row, col, value, delta, spans=("alltime",), span=None, tile_override=None):
        self.labels, self.label, self.zoom, self.row, self.col, self.value = labels, label, zoom, row, col, value
        self.delta = delta
        self.spans = list(spans)
        self.span = np.zeros(np.asarray(zoom).size, np.int64) if span is None else np.asarray(span, np.int64)
        # {(zoom, row, col): row tile} for bins outside the chain windows whose
        # row tile is not the shift (ChainFix); None: every row tile is the shift
        self.tile_override = tile_override or None

    def row_tiles(self):
        """(zoom - delta, row tile row, row tile col) of every bin"""
        d = self.delta
        z, r, c = (np.asarray(x, np.int64) for x in (self.zoom, self.row, self.col))
        tz, tr, tc = z - d, r >> d, c >> d
        if self.tile_override:
            # the few overridden bins located by a search over the bins' sorted
            # (zoom, row, col) rows, not a Python pass over every bin
            tr, tc = tr.copy(), tc.copy()
            ok = np.array(list(self.tile_override.keys()), np.int64).reshape(-1, 3)
            ov = np.array(list(self.tile_override.values()), np.int64).reshape(-1, 2)
            o = np.lexsort((c, r, z))
            zs, rs, cs = z[o], r[o], c[o]
            for j in range(ok.shape[0]):
                lo = np.searchsorted(zs, ok[j, 0], "left")
                hi = np.searchsorted(zs, ok[j, 0], "right")
                a = lo + np.searchsorted(rs[lo:hi], ok[j, 1], "left")
                b = lo + np.searchsorted(rs[lo:hi], ok[j, 1], "right")
                k = a + np.searchsorted(cs[a:b], ok[j, 2], "left")
                while k < b and cs[k] == ok[j, 2]:
                    tr[o[k]], tc[o[k]] = ov[j]
                    k += 1
        return tz, tr, tc

    def __len__(self):
        return int(self.zoom.size)


def concat_cells(parts, labels, delta) -> Cells:
    """One Cells from per-timespan Cells (same labels and delta), keeping
    each part's span labels."""
    spans, span = [], []
    for c in parts:
        remap = []
        for x in c.spans:
            if x not in spans:
                spans.append(x)
            remap.append(spans.index(x))
        span.append(np.asarray(remap, np.int64)[c.span])

    def cat(name, dtype):
        return np.concatenate([np.asarray(getattr(c, name), dtype) for c in parts]) if parts else np.zeros(0, dtype)

    over = {}
    for c in parts:
        over.update(c.tile_override or {})
    return Cells(labels, cat("label", np.int64), cat("zoom", np.int64), cat("row", np.int64), cat("col", np.int64),
                 cat("value", np.float64), delta, spans or ["alltime"],
                 np.concatenate(span) if span else np.zeros(0, np.int64), tile_override=over)


# cells above which _sum_by_cell sorts on the GPU (a 3-key numpy lexsort of
# the 94M bins of 1e7 points x 10,000 users at zooms 6-21 took ~20 s)
SUM_BY_CELL_DEVICE_MIN = 1 << 20


def _sum_by_cell_device(z, r, c, v):
    """_sum_by_cell of in-square cells on the GPU: HM_KEY-packed keys (their
    order is the (zoom, row, col) order), one sort, one index_add."""
    import torch

    key = torch.from_numpy((z << 58) | (r << 29) | c).cuda()
    uk, inv = torch.unique(key, sorted=True, return_inverse=True)
    sums = torch.zeros((uk.numel(), v.shape[1]), dtype=torch.int64, device=key.device)
    sums.index_add_(0, inv, torch.from_numpy(np.ascontiguousarray(v)).cuda())
    k = uk.cpu().numpy()
    return k >> 58, (k >> 29) & 0x1FFFFFFF, k & 0x1FFFFFFF, sums.cpu().numpy()


def _sum_by_cell(parts, device_min=None):
    """parts: [(zoom, row, col, values[k x m])] -> unique (zoom, row, col) and
    the summed value columns (int64), sorted by (zoom, row, col)."""
    z = np.concatenate([p[0] for p in parts]).astype(np.int64)
    r = np.concatenate([p[1] for p in parts]).astype(np.int64)
    c = np.concatenate([p[2] for p in parts]).astype(np.int64)
    v = np.concatenate([p[3] for p in parts], axis=0)
    if z.size == 0:
        return z, r, c, v
    lim = SUM_BY_CELL_DEVICE_MIN if device_min is None else device_min
    if z.size >= lim and v.dtype.kind in "iu" and device.gpu_available() and r.min() >= 0 and c.min() >= 0 and \
            max(int(r.max()), int(c.max())) < (1 << 29) and int(z.max()) < 64:
        return _sum_by_cell_device(z, r, c, v)
    o = np.lexsort((c, r, z))
    z, r, c, v = z[o], r[o], c[o], v[o]
    head = np.ones(z.size, dtype=bool)
    head[1:] = (z[1:] != z[:-1]) | (r[1:] != r[:-1]) | (c[1:] != c[:-1])
    starts = np.flatnonzero(head)
    return z[starts], r[starts], c[starts], np.add.reduceat(v, starts, axis=0)


def _in_chain_window(row, col, zmax, d):
    """Mask of detail-zoom tiles (row, col) whose every level lies inside the
    windows on which the reference's centre re-projection (heatmap.py:60-61,
    89) equals the shift (heatmap_amd/chain_window.py)."""
    row, col = np.asarray(row, np.int64), np.asarray(col, np.int64)
    ok = np.ones(row.size, dtype=bool)
    for z in range(zmax, d, -1):
        # row tile at z - d (heatmap.py:89); level z re-projected from z+1,
        # the first level at its own zoom (heatmap.py:60-61)
        for zz, j in [(z, d), (z, 0) if z == zmax else (z + 1, 1)]:
            kk = zmax - zz
            (rlo, rhi), (clo, chi) = chain_window.ROWS[zz][j], chain_window.COLS[zz][j]
            r, c = row >> kk, col >> kk
            ok &= (r >= rlo) & (r < rhi) & (c >= clo) & (c < chi)
    return ok


def _device_project(lat, lon, z):
    p = device.project(lat, lon, z, raise_errors=True)
    return np.asarray(p.row, np.int64), np.asarray(p.col, np.int64)


def _recentre(z, rows, cols, z_to, project=None):
    """Tiles at zoom z_to holding the centres of tiles (z, rows, cols), as
    reference tile.py:33-54 then tile.py:9-21 compute them: the centre on the
    host with the reference's inverse projection and operation order
    (Tile.latitude_from_row: exp/atan, raising what the reference raises), its
    forward projection on the device (hm_project, bit-exact)."""
    if len(rows) == 0:
        return np.zeros(0, np.int64), np.zeros(0, np.int64)
    lat = np.array([(Tile.latitude_from_row(int(r), z) + Tile.latitude_from_row(int(r) + 1, z)) / 2.0
                    for r in rows], np.float64)
    lon = np.array([(Tile.longitude_from_column(int(c) + 1, z) + Tile.longitude_from_column(int(c), z)) / 2.0
                    for c in cols], np.float64)
    return (project or _device_project)(lat, lon, z_to)


class ChainFix:
    """The reference's literal re-projection chain for the detail tiles that
    leave the shift windows (within ~1e-6 deg of a pole, |lon| > 11520): per
    level z, the tile each such detail tile's points reach (t_z) and the row
    tile of that level's bins (heatmap.py:89).  first_applied: the detail tiles
    are already the first level's (t_zmax given).  project(lat, lon, z) ->
    (rows, cols): the forward projection (the device's hm_project; the CPU
    tests pass the oracle's)."""

    def __init__(self, rows, cols, zmax, d, first_applied=False, project=None):
        self.rows, self.cols, self.zmax, self.d = np.asarray(rows, np.int64), np.asarray(cols, np.int64), zmax, d
        self.level, self.rowtile = {}, {}
        r, c = (self.rows, self.cols) if first_applied else _recentre(zmax, self.rows, self.cols, zmax, project)
        for z in range(zmax, d, -1):
            if z < zmax:
                r, c = _recentre(z + 1, r, c, z, project)
            self.level[z] = (r, c)
            self.rowtile[z] = _recentre(z, r, c, z - d, project)

    def shift_and_chain(self, z):
        """(shift rows, shift cols, chain rows, chain cols) of the detail tiles at zoom z"""
        k = self.zmax - z
        r, c = self.level[z]
        return self.rows >> k, self.cols >> k, r, c

    def overrides(self):
        """{(z, row, col): (row tile row, row tile col)} where the row tile is
        not the shift (heatmap.py:89 re-projects the bin's centre)"""
        out = {}
        for z, (tr, tc) in self.rowtile.items():
            r, c = self.level[z]
            for i in np.flatnonzero((tr != (r >> self.d)) | (tc != (c >> self.d))).tolist():
                out[(z, int(r[i]), int(c[i]))] = (int(tr[i]), int(tc[i]))
        return out


def _apply_chain(all_cells, grouped_cells, zmax, d, first_applied=False, project=None):
    """Device cells (the shift pyramid) corrected for detail tiles outside the
    chain windows: each such tile's counts move, level by level, from the
    shift's cell to the reference's re-projected tile.  Returns (all_cells,
    grouped_cells, row-tile overrides or None)."""
    nz, nr, nc = (np.asarray(x, np.int64) for x in all_cells[:3])
    gg, gz, gr, gc = (np.asarray(x, np.int64) for x in grouped_cells[:4])
    nn, gn = np.asarray(all_cells[3]), np.asarray(grouped_cells[4])
    det = nz == zmax
    bad = det & ~_in_chain_window(nr, nc, zmax, d)
    if not bad.any():
        return all_cells, grouped_cells, None
    fix = ChainFix(nr[bad], nc[bad], zmax, d, first_applied, project)
    index = {(int(r), int(c)): i for i, (r, c) in enumerate(zip(fix.rows.tolist(), fix.cols.tolist()))}
    # all points: n per detail tile, moved at every level
    nb = nn[bad]
    parts = [(nz, nr, nc, nn[:, None])]
    for z in range(zmax, d, -1):
        sr, sc, cr, cc = fix.shift_and_chain(z)
        zz = np.full(sr.size, z, np.int64)
        parts += [(zz, sr, sc, -nb[:, None]), (zz, cr, cc, nb[:, None])]
    az, ar, ac, av = _sum_by_cell(parts, device_min=1 << 62)
    keepc = av[:, 0] != 0
    all_out = (az[keepc], ar[keepc], ac[keepc], av[keepc, 0])
    # grouped points: the same move per (group, detail tile); the group rides
    # in the zoom field (zoom < 64) of the cell key
    gdet = (gz == zmax) & ~_in_chain_window(gr, gc, zmax, d)
    if gdet.any():
        ti = np.array([index[(int(r), int(c))] for r, c in zip(gr[gdet].tolist(), gc[gdet].tolist())], np.int64)
        gb, gnb = gg[gdet], gn[gdet]
        parts = [(gg * 64 + gz, gr, gc, gn[:, None])]
        for z in range(zmax, d, -1):
            sr, sc, cr, cc = fix.shift_and_chain(z)
            zz = gb * 64 + z
            parts += [(zz, sr[ti], sc[ti], -gnb[:, None]), (zz, cr[ti], cc[ti], gnb[:, None])]
        kz, kr, kc, kv = _sum_by_cell(parts, device_min=1 << 62)
        keepg = kv[:, 0] != 0
        grouped_cells = (kz[keepg] // 64, kz[keepg] % 64, kr[keepg], kc[keepg], kv[keepg, 0])
    return all_out, grouped_cells, fix.overrides()


def combine_cells(labels, all_cells, grouped_cells, zmax, d, span_label="alltime", first_applied=False,
                  project=None, exact_levels=None) -> Cells:
    """The bins of one timespan's rows from its per-cell counts.

    all_cells = (zoom, row, col, n): every kept point; grouped_cells =
    (group, zoom, row, col, count) per group id (group 0: the literal user id
    'all', merged into the 'all' rows).  Row layout: heatmap.py:55,85-90,
    120-126; 'all' weighting: heatmap.py:64-70 applied level by level (module
    docstring)."""
    if exact_levels is None:
        all_cells, grouped_cells, over = _apply_chain(all_cells, grouped_cells, zmax, d, first_applied, project)
    else:   # the cells already follow the reference's chain; exact_levels: its row-tile overrides
        over = exact_levels
    nz, nr, nc = (np.asarray(x, np.int64) for x in all_cells[:3])
    gg, gz, gr, gc = (np.asarray(x, np.int64) for x in grouped_cells[:4])
    # counts (int64), or float weights (build_heatmaps of weighted locations)
    vt = np.float64 if (np.asarray(all_cells[3]).dtype.kind == "f" or
                        np.asarray(grouped_cells[4]).dtype.kind == "f") else np.int64
    nn, gn = np.asarray(all_cells[3], vt), np.asarray(grouped_cells[4], vt)
    # 'all' rows: per cell n, a (literal 'all'), U (other groups)
    nv = np.stack([nn, np.zeros(nz.size, vt), np.zeros(nz.size, vt)], 1)
    lit = gg == 0
    gv = np.stack([np.zeros(gz.size, vt), np.where(lit, gn, 0), np.where(lit, 0, gn)], 1)
    az, ar, ac, av = _sum_by_cell([(nz, nr, nc, nv), (gz, gr, gc, gv)])
    sel = az > d
    az, ar, ac, av = az[sel], ar[sel], ac[sel], av[sel]
    k = zmax - az
    w = np.left_shift(np.int64(1), k).astype(vt)
    value_all = ((av[:, 0] + av[:, 1]) * w + (w - 1) * av[:, 2]).astype(np.float64)
    # user-group rows (the literal 'all' group is not a row of its own)
    us = (~lit) & (gz > d)
    label = np.concatenate([np.zeros(az.size, np.int64), gg[us]])
    return Cells(labels, label, np.concatenate([az, gz[us]]), np.concatenate([ar, gr[us]]),
                 np.concatenate([ac, gc[us]]), np.concatenate([value_all, gn[us].astype(np.float64)]), d,
                 [span_label], tile_override=over)


def assemble_cells(count_all, count_grouped, user_id, keep=None, max_zoom_level=None, delta=None,
                   project=None) -> Cells:
    """The bins of build_heatmaps' rows from per-cell counts.

    count_all(keep) -> (zoom, row, col, count) arrays of the kept points;
    count_grouped(keep, gid) -> (group, zoom, row, col, count) per group id.
    Both cover zooms delta+1 .. max_zoom_level+delta and are the only places
    points are touched (the device in the product, the oracle in the CPU
    tests); project: the forward projection of re-projected tile centres
    (ChainFix; the device by default)."""
    mz = MAX_ZOOM_LEVEL if max_zoom_level is None else max_zoom_level
    d = DETAIL_ZOOM_DELTA if delta is None else delta
    zmax = mz + d
    n = len(user_id)
    keep = np.ones(n, dtype=bool) if keep is None else np.asarray(keep).astype(bool)
    plan = group_plan(user_id, keep)
    # every point is projected (and may raise) even when not kept, as
    # dataframe_loader does (heatmap.py:27-29): count_all sees all points
    allc = count_all(keep)
    if plan.grouped.any():
        grp = count_grouped(plan.grouped, plan.gid)
    else:
        grp = tuple(np.zeros(0, np.int64) for _ in range(5))
    return combine_cells(plan.labels, allc, grp, zmax, d, project=project)


def cells_to_rows(cells: Cells) -> dict:
    """{row_id: {bin_id: float}} (heatmap.py:85-90,120-126)."""
    rows = {}
    labels, spans = cells.labels, cells.spans
    tz, tr, tc = cells.row_tiles()
    for g, t, z, r, c, v, a, b, e in zip(cells.label.tolist(), cells.span.tolist(), cells.zoom.tolist(),
                                         cells.row.tolist(), cells.col.tolist(), cells.value.tolist(), tz.tolist(),
                                         tr.tolist(), tc.tolist()):
        rid = "%s|%s|%d_%d_%d" % (labels[g], spans[t], a, b, e)
        rows.setdefault(rid, {})["%d_%d_%d" % (z, r, c)] = v
    return rows


def _row_order(label, span, tz, tr, tc, zoom, row, col, device_min=None):
    """The permutation sorting bins by (label, span, row tile, zoom, row,
    col): np.lexsort, or three stable GPU sorts of packed keys for large sets
    (a 94M-bin 8-key lexsort took ~15 s on the host).  Bins are distinct, so
    every sort gives the same order."""
    lim = SUM_BY_CELL_DEVICE_MIN if device_min is None else device_min
    n = np.asarray(label).size
    if n >= lim and device.gpu_available():
        z, r, c = (np.asarray(x, np.int64) for x in (zoom, row, col))
        a, b, t = (np.asarray(x, np.int64) for x in (label, span, tz))
        if (r.min() >= 0 and c.min() >= 0 and max(int(r.max()), int(c.max())) < (1 << 29) and int(z.max()) < 64
                and int(t.min()) >= 0 and int(t.max()) < 64 and int(a.min()) >= 0 and int(a.max()) < (1 << 40)
                and int(b.min()) >= 0 and int(b.max()) < (1 << 20)):
            import torch

            def stable(keys, perm):
                k = torch.from_numpy(keys).cuda()[perm]
                return perm[torch.sort(k, stable=True).indices]

            perm = torch.arange(n, device="cuda")
            perm = stable((z << 58) | (r << 29) | c, perm)
            perm = stable((t << 58) | (np.asarray(tr, np.int64) << 29) | np.asarray(tc, np.int64), perm)
            perm = stable((a << 20) | b, perm)
            return perm.cpu().numpy()
    return np.lexsort((col, row, zoom, tc, tr, tz, span, label))


def _heat_text_gpu(dz, dr, dc, dv, st):
    """The rows' heatmap JSON from bins in row order (int64 CUDA tensors;
    non-negative, counts below 1e16) and the rows' first bins st: written by
    hm_format_bins, one thread per bin at an exclusive scan of the bins' text
    lengths.  A pyarrow LargeStringArray."""
    import ctypes
    import time

    import pyarrow as pa
    import torch

    _T_JSON[0] = time.perf_counter()
    n = dz.numel()
    head = torch.zeros(n, dtype=torch.uint8, device=dz.device)
    head[st] = 1
    last = torch.zeros(n, dtype=torch.uint8, device=dz.device)
    last[st[1:] - 1] = 1
    last[n - 1] = 1

    ln = _digits(dz) + _digits(dr) + _digits(dc) + _digits(dv) + 8 + head.to(torch.int64) + 2 - last.to(torch.int64)
    off = torch.cumsum(ln, 0) - ln
    total = int((off[-1] + ln[-1]).item())
    text = torch.empty(max(total, 1), dtype=torch.uint8, device=dz.device)
    ctx = device.context(dz.device.index or 0)
    p = lambda x: ctypes.c_void_p(x.data_ptr())  # noqa: E731
    dz, dr, dc, dv = (x.contiguous() for x in (dz, dr, dc, dv))
    rc = ctx.L.hm_format_bins(ctx.ptr, p(dz), p(dr), p(dc), p(dv), p(head), p(last), p(off), n, p(text))
    if rc != _lib.HM_OK:
        _lib.raise_for(rc)
    import time

    t0 = time.perf_counter()
    torch.cuda.current_stream(dz.device).synchronize()
    LAST_TABLE_PHASES["JSON: text written (device, of which)"] = time.perf_counter() - _T_JSON[0]
    offsets = _offsets_to_host(off[st], total)
    data = _to_host(text[:total])
    return pa.LargeStringArray.from_buffers(int(st.numel()), pa.py_buffer(offsets), pa.py_buffer(data))


def _heat_text_device(z, r, c, v, starts, device_min=None):
    """_heat_text_gpu of host arrays, or None (small sets, no GPU, negative
    values: the host path)."""
    lim = SUM_BY_CELL_DEVICE_MIN if device_min is None else device_min
    n = int(np.asarray(z).size)
    if n < lim or not device.gpu_available() or min(int(np.min(z)), int(np.min(r)), int(np.min(c))) < 0:
        return None
    import torch

    dz, dr, dc, dv = (torch.from_numpy(np.ascontiguousarray(x, np.int64)).cuda() for x in (z, r, c, v))
    return _heat_text_gpu(dz, dr, dc, dv, torch.from_numpy(np.asarray(starts, np.int64)).cuda())


def _cells_to_table_device(cells: Cells):
    """cells_to_table with the bins kept on the GPU from the row sort to the
    JSON text: one upload, the order and every per-bin gather on the device;
    only per-row fields come back for the ids.  None when a value is not a
    non-negative integer below 1e16 or a coordinate is out of packing range
    (the host path then)."""
    import pyarrow as pa
    import torch

    d = cells.delta
    v = np.asarray(cells.value, np.float64)
    vi = v.astype(np.int64)
    if not (np.array_equal(v, vi) and vi.min() >= 0 and vi.max() < 10 ** 16):
        return None
    cu = lambda x: torch.from_numpy(np.ascontiguousarray(x, np.int64)).cuda()  # noqa: E731
    lab, sp, z, r, c = (cu(x) for x in (cells.label, cells.span, cells.zoom, cells.row, cells.col))
    if (min(int(r.min()), int(c.min()), int(lab.min()), int(sp.min()), int(z.min()) - d) < 0 or
            max(int(r.max()), int(c.max())) >= (1 << 29) or int(z.max()) >= 64 or int(lab.max()) >= (1 << 40) or
            int(sp.max()) >= (1 << 20)):
        return None
    dv = cu(vi)
    if cells.tile_override:   # ChainFix: some bins' row tiles are not the shift
        htz, htr, htc = cells.row_tiles()
        if min(int(htr.min()), int(htc.min())) < 0 or max(int(htr.max()), int(htc.max())) >= (1 << 29):
            return None
        tz, tr, tc = cu(htz), cu(htr), cu(htc)
    else:
        tz, tr, tc = z - d, r >> d, c >> d
    perm = torch.arange(z.numel(), device=z.device)
    for key in ((z << 58) | (r << 29) | c, (tz << 58) | (tr << 29) | tc, (lab << 20) | sp):
        perm = perm[torch.sort(key[perm], stable=True).indices]
    lab, sp, z, r, c, dv, tz, tr, tc = (x[perm] for x in (lab, sp, z, r, c, dv, tz, tr, tc))
    hi, lo = (lab << 20) | sp, (tz << 58) | (tr << 29) | tc
    head = torch.ones_like(hi, dtype=torch.bool)
    head[1:] = (hi[1:] != hi[:-1]) | (lo[1:] != lo[:-1])
    st = torch.nonzero(head).flatten()
    heat = _heat_text_gpu(z, r, c, dv, st)
    ids = _ids_gpu(cells.labels, cells.spans, lab[st], sp[st], tz[st], tr[st], tc[st])
    return pa.table({"id": ids, "heatmap": heat})


def cells_to_table(cells: Cells):
    """pyarrow Table(id: string, heatmap: string) of the rows, the heatmap
    JSON-encoded as heatmap_to_json would (json.dumps of the bin dict, floats
    as repr: 163838.0), built with vectorised string kernels."""
    import pyarrow as pa
    import pyarrow.compute as pc

    d = cells.delta
    if len(cells) == 0:
        return pa.table({"id": pa.array([], pa.large_string()), "heatmap": pa.array([], pa.large_string())})
    if len(cells) >= SUM_BY_CELL_DEVICE_MIN and device.gpu_available():
        tab = _cells_to_table_device(cells)
        if tab is not None:
            return tab
    tz, tr, tc = cells.row_tiles()
    o = _row_order(cells.label, cells.span, tz, tr, tc, cells.zoom, cells.row, cells.col)
    lab, sp, z, r, c, v = cells.label[o], cells.span[o], cells.zoom[o], cells.row[o], cells.col[o], cells.value[o]
    tz, tr, tc = tz[o], tr[o], tc[o]
    head = np.ones(lab.size, dtype=bool)
    head[1:] = ((lab[1:] != lab[:-1]) | (sp[1:] != sp[:-1]) | (tz[1:] != tz[:-1]) | (tr[1:] != tr[:-1]) |
                (tc[1:] != tc[:-1]))
    starts = np.flatnonzero(head)
    s = lambda a: pc.cast(pa.array(a), pa.large_string())  # noqa: E731
    t = lambda x: pa.scalar(x, pa.large_string())  # noqa: E731
    # float repr of integer-valued counts below 1e16 is "<int>.0"; others via repr
    vi = v.astype(np.int64)
    small = (v == vi) & (np.abs(v) < 1e16)
    heat = _heat_text_device(z, r, c, vi, starts) if small.all() and vi.min() >= 0 else None
    if heat is None:
        vs = pc.binary_join_element_wise(s(vi), t(".0"), t(""))
        if not small.all():
            vs = vs.to_pylist()
            for i in np.flatnonzero(~small).tolist():
                vs[i] = repr(float(v[i]))
            vs = pa.array(vs, pa.large_string())
        bins = pc.binary_join_element_wise(s(z), s(r), s(c), t("_"))
        pieces = pc.binary_join_element_wise(t('"'), bins, t('": '), vs, t(""))
        # 64-bit offsets throughout: a batch can hold more than 2^31 bins or 2 GiB
        # of JSON text (int32 offsets would wrap silently)
        offsets = np.append(starts, lab.size).astype(np.int64)
        joined = pc.binary_join(pa.LargeListArray.from_arrays(pa.array(offsets, pa.int64()), pieces), t(", "))
        heat = pc.binary_join_element_wise(t("{"), joined, t("}"), t(""))
    names = pa.array(cells.labels, pa.large_string()).take(pa.array(lab[starts]))
    spans = pa.array(cells.spans, pa.large_string()).take(pa.array(sp[starts]))
    ids = pc.binary_join_element_wise(names, spans,
                                      pc.binary_join_element_wise(s(tz[starts]), s(tr[starts]), s(tc[starts]), t("_")),
                                      t(KEY_SEPERATOR))
    return pa.table({"id": ids, "heatmap": heat})


def assemble_rows(count_all, count_grouped, user_id, keep=None, max_zoom_level=None, delta=None,
                  project=None) -> dict:
    """assemble_cells -> {row_id: heatmap dict}."""
    return cells_to_rows(assemble_cells(count_all, count_grouped, user_id, keep, max_zoom_level, delta, project))


# --------------------------------------------------------------------------
# device entry points
# --------------------------------------------------------------------------

def _device_counters(lat, lon, zmin, zmax, tiles):
    def count_all(keep):
        c = device.count(lat, lon, keep.astype(np.uint8), zmin, zmax, tiles=tiles)
        return c.zoom, c.row, c.col, c.count

    def count_grouped(keep, gid):
        g = device.count_grouped(lat, lon, gid, keep.astype(np.uint8), zmin, zmax, tiles=tiles)
        return g.group, g.zoom, g.row, g.col, g.count

    return count_all, count_grouped


def heatmap_cells(lat, lon, user_id, keep=None, max_zoom_level=None, delta=None, tiles=False) -> Cells:
    """Bins of every build_heatmaps row for columnar input (two device passes)."""
    mz = MAX_ZOOM_LEVEL if max_zoom_level is None else max_zoom_level
    d = DETAIL_ZOOM_DELTA if delta is None else delta
    ca, cg = _device_counters(lat, lon, d + 1, mz + d, tiles)
    return assemble_cells(ca, cg, user_id, keep, mz, d)


def build_heatmaps_columnar(lat, lon, user_id, keep=None, max_zoom_level=None, delta=None, tiles=False):
    """Rows {row_id: {bin_id: float}} of build_heatmaps for columnar input.

    lat/lon: float64 arrays (or, with tiles=True, int64 row/col at the detail
    zoom); user_id: sequence of str; keep: mask of non-background rows."""
    return cells_to_rows(heatmap_cells(lat, lon, user_id, keep, max_zoom_level, delta, tiles))


# seconds per phase of the last heatmap_table call (device path)
LAST_TABLE_PHASES = {}


_POW10 = {}


def _digits(x):
    """decimal digits of non-negative int64 CUDA tensors: 1 + the number of
    powers 10^1 .. 10^18 at or below x, one searchsorted pass (18 compare-adds
    over the whole array before)"""
    import torch

    p = _POW10.get(x.device)
    if p is None:
        p = _POW10[x.device] = torch.tensor([10 ** k for k in range(1, 19)], dtype=torch.int64, device=x.device)
    return torch.searchsorted(p, x, right=True) + 1


def _offsets_to_host(off, total: int):
    """int64 string offsets (a CUDA tensor of the starts, then total) as one
    host array: appended on the device and copied once (np.append on the
    host copied the 300 MB of a 1e7-point table's ids twice more)"""
    import torch

    o = torch.cat([off.to(torch.int64), off.new_full((1,), int(total), dtype=torch.int64)])
    return _to_host(o.view(torch.uint8)).view(np.int64)


_COPY_POOL = None
_T_JSON = [0.0]
THREADED_COPY_MIN = 128 << 20   # bytes; smaller texts take one copy


def _to_host(t):
    """A CUDA uint8 tensor (the table's text columns: GBs) as a host numpy
    array.  A single pageable copy runs at ~8 GB/s and a fresh pinned buffer
    costs its page locking (~10 GB/s together); 64 MB chunks copied from 8
    host threads into one pageable array reach ~55 GB/s
    (tools/copy_probe.py, profiles/r6/copy_probe.json)."""
    import os
    from concurrent.futures import ThreadPoolExecutor

    import torch

    global _COPY_POOL
    n = t.numel()
    if n < THREADED_COPY_MIN or os.environ.get("HM_TABLE_THREADED_COPY", "1") == "0":
        return t.cpu().numpy()
    dst = np.empty(n, np.uint8)
    step = max(1 << 20, min(64 << 20, THREADED_COPY_MIN // 2))
    if _COPY_POOL is None:
        _COPY_POOL = ThreadPoolExecutor(8, thread_name_prefix="hm-d2h")
    dev = t.device
    torch.cuda.current_stream(dev).synchronize()   # the text is written

    def part(a):
        with torch.cuda.device(dev):
            torch.from_numpy(dst[a:a + step]).copy_(t[a:a + step])

    list(_COPY_POOL.map(part, range(0, n, step)))
    return dst


def _ids_gpu(labels, spans, rl, rs, rz, rr, rc):
    """Row ids "<label>|<span>|<z>_<row>_<col>" of per-row int64 CUDA tensors,
    written on the GPU (hm_format_ids) at an exclusive scan of their lengths.
    A pyarrow LargeStringArray."""
    import ctypes

    import pyarrow as pa
    import torch

    dev = rl.device

    def blob(texts):
        b = [t.encode() for t in texts]
        off = np.zeros(len(b) + 1, np.int64)
        off[1:] = np.cumsum([len(x) for x in b])
        data = np.frombuffer(b"".join(b) or b"\0", np.uint8)
        return torch.from_numpy(data.copy()).to(dev), torch.from_numpy(off).to(dev)

    names, noff = blob(labels)
    sp, soff = blob(spans)
    n = rl.numel()
    ln = (noff[rl + 1] - noff[rl]) + (soff[rs + 1] - soff[rs]) + _digits(rz) + _digits(rr) + _digits(rc) + 4
    off = torch.cumsum(ln, 0) - ln
    total = int((off[-1] + ln[-1]).item()) if n else 0
    text = torch.empty(max(total, 1), dtype=torch.uint8, device=dev)
    ctx = device.context(dev.index or 0)
    p = lambda x: ctypes.c_void_p(x.data_ptr())  # noqa: E731
    rl, rs, rz, rr, rc = (x.contiguous() for x in (rl, rs, rz, rr, rc))
    if n:
        rc_ = ctx.L.hm_format_ids(ctx.ptr, p(names), p(noff), p(rl), p(sp), p(soff), p(rs), p(rz), p(rr), p(rc),
                                  p(off), n, p(text))
        if rc_ != _lib.HM_OK:
            _lib.raise_for(rc_)
    offsets = _offsets_to_host(off, total)
    data = _to_host(text[:total])
    return pa.LargeStringArray.from_buffers(int(n), pa.py_buffer(offsets), pa.py_buffer(data))


def _device_table(labels, keys, counts, grouped, zmax, d, phases):
    """heatmap_table's rows from device-resident counts, end to end on the
    GPU: keys/counts = hm_count's in-square cells (HM_KEY, n) of the kept
    points; grouped = hm_count_grouped_packed's (keys, group << 32 | count)
    or hm_count_grouped's [m, 5] records.  The 'all' closed
    form (combine_cells) by a sort of the cell keys and index_adds, the row
    order by one sort of packed (label, row tile, row, col) keys, the JSON by
    hm_format_bins; only the per-row id fields come back.  None when the keys
    do not pack into one int64 (combine_cells + cells_to_table then)."""
    import time

    import pyarrow as pa
    import torch

    t0 = time.perf_counter()
    ks, o = torch.sort(keys)
    n = counts[o]
    z = ks >> 58
    w = torch.ones_like(ks) << (zmax - z)
    a = torch.zeros_like(n)
    u = torch.zeros_like(n)
    if isinstance(grouped, tuple):   # hm_count_grouped_packed: (HM_KEY, group << 32 | count)
        gk, gcn = grouped
        gg, gn = gcn >> 32, gcn & 0xFFFFFFFF
    elif grouped.numel():
        gg, gz, gr, gc, gn = grouped.unbind(1)
        gk = (gz << 58) | (gr << 29) | gc
    else:
        gk = None
    if gk is not None and gk.numel():
        pos = torch.searchsorted(ks, gk)
        lit = gg == 0
        a.index_add_(0, pos[lit], gn[lit])
        u.index_add_(0, pos[~lit], gn[~lit])
        us = ~lit
        ug, uk, un = gg[us], gk[us], gn[us]
    else:
        ug = uk = un = torch.zeros(0, dtype=torch.int64, device=keys.device)
    value_all = (n + a) * w + (w - 1) * u
    label = torch.cat([torch.zeros_like(ks), ug])
    key = torch.cat([ks, uk])
    val = torch.cat([value_all, un])
    torch.cuda.synchronize()
    phases["combine (device)"] = time.perf_counter() - t0
    t0 = time.perf_counter()
    if val.numel() and int(val.max()) >= 10 ** 16:
        return None
    lb = max(int(label.max()).bit_length(), 1) if label.numel() else 1
    if lb + 6 + 2 * zmax > 63:
        return None
    z = key >> 58
    r = (key >> 29) & 0x1FFFFFFF
    c = key & 0x1FFFFFFF
    m = (1 << d) - 1
    tb = zmax - d
    # (label, row-tile zoom, row-tile row, row-tile col, row, col): within a
    # row tile (fixed zoom) the bins' (row, col) order is their low bits' order
    sk = ((label << (6 + 2 * zmax)) | ((z - d) << (2 * zmax)) | ((r >> d) << (tb + 2 * d)) |
          ((c >> d) << (2 * d)) | ((r & m) << d) | (c & m))
    sk, o = torch.sort(sk)
    z, r, c, val = z[o], r[o], c[o], val[o]
    rk = sk >> (2 * d)
    head = torch.ones_like(rk, dtype=torch.bool)
    head[1:] = rk[1:] != rk[:-1]
    st = torch.nonzero(head).flatten()
    torch.cuda.synchronize()
    phases["order (device)"] = time.perf_counter() - t0
    t0 = time.perf_counter()
    heat = _heat_text_gpu(z, r, c, val, st)
    phases["JSON (device text + copy to host)"] = time.perf_counter() - t0
    t0 = time.perf_counter()
    rt = rk[st]
    ids = _ids_gpu(labels, ["alltime"], rt >> (6 + 2 * tb), torch.zeros_like(rt), (rt >> (2 * tb)) & 63,
                   (rt >> tb) & ((1 << tb) - 1), rt & ((1 << tb) - 1))
    phases["ids (device)"] = time.perf_counter() - t0
    return pa.table({"id": ids, "heatmap": heat})


def heatmap_table(lat, lon, user_id, keep=None, max_zoom_level=None, delta=None, tiles=False):
    """The same rows as a pyarrow Table(id, heatmap JSON): batchMain's
    DataFrame (heatmap.py:156-157) without per-cell Python objects.  Cells
    stay on the device from the two counting passes to the JSON text
    (_device_table); cells outside [0, 2^z)^2 -- the only ones that can leave
    the chain windows -- take combine_cells + cells_to_table."""
    import time

    mz = MAX_ZOOM_LEVEL if max_zoom_level is None else max_zoom_level
    d = DETAIL_ZOOM_DELTA if delta is None else delta
    zmax = mz + d
    n = len(user_id)
    keep = np.ones(n, dtype=bool) if keep is None else np.asarray(keep).astype(bool)
    ph = LAST_TABLE_PHASES
    ph.clear()
    t0 = time.perf_counter()
    plan = group_plan(user_id, keep)
    ph["group_plan (host)"] = time.perf_counter() - t0
    t0 = time.perf_counter()
    m, buf = device.count_device(lat, lon, keep.astype(np.uint8), d + 1, zmax, tiles=tiles)
    keys, counts = buf.keys[:m], buf.counts[:m]
    packed = None
    if buf.nx == 0 and plan.grouped.any():
        # 16-B records (HM_KEY, group | count); None if a kept tile leaves the square
        packed = device.count_grouped_packed_device(lat, lon, plan.gid, plan.grouped.astype(np.uint8), d + 1, zmax,
                                                    tiles=tiles)
    ph["counts (device)"] = time.perf_counter() - t0
    tab = None
    if buf.nx == 0 and (packed is not None or not plan.grouped.any()):
        grouped = packed if packed is not None else keys.new_zeros((0, 5))
        tab = _device_table(plan.labels, keys, counts, grouped, zmax, d, ph)
    if tab is not None:
        return tab
    packed = grouped = None   # free the packed records before the 5-int64 pass sizes itself
    t0 = time.perf_counter()
    if plan.grouped.any():
        grouped = device.count_grouped_device(lat, lon, plan.gid, plan.grouped.astype(np.uint8), d + 1, zmax,
                                              tiles=tiles)
    else:
        grouped = keys.new_zeros((0, 5))
    ph["counts (device, 5-int64 records)"] = time.perf_counter() - t0
    # host assembly from the same counts
    zk, rk, ck = device.decode_keys(keys.cpu().numpy().view(np.uint64))
    cnt = counts.cpu().numpy()
    if buf.nx:
        x = buf.xcells[:4 * buf.nx].cpu().numpy().reshape(-1, 4)
        zk, rk, ck, cnt = (np.concatenate([p, q]) for p, q in ((zk, x[:, 0]), (rk, x[:, 1]), (ck, x[:, 2]),
                                                               (cnt, x[:, 3])))
    g = grouped.cpu().numpy()
    cells = combine_cells(plan.labels, (zk, rk, ck, cnt), tuple(g[:, i] for i in range(5)), zmax, d)
    return cells_to_table(cells)


def build_heatmaps(locations):
    """heatmap.py:107-118 on an iterable (or RDD-like .collect()) of locations
    {"userId", "tileId", "count"}: dataframe_loader output (zoom-21 tiles,
    count 1.0: the device counts the tiles), or any zoom and any float count
    -- heatmap_to_locations output fed back in, say.  Returns [(row_id,
    heatmap_dict)]."""
    if hasattr(locations, "collect"):
        locations = locations.collect()
    d = DETAIL_ZOOM_DELTA
    zmax = MAX_ZOOM_LEVEL + d
    zs, rows, cols, users, w = [], [], [], [], []
    for loc in locations:
        z, r, c = (int(x) for x in loc["tileId"].split("_"))
        zs.append(z)
        rows.append(r)
        cols.append(c)
        users.append(loc["userId"])
        w.append(float(loc["count"]))
    if all(z == zmax for z in zs) and all(x == 1.0 for x in w):
        out = build_heatmaps_columnar(np.array(rows, dtype=np.int64), np.array(cols, dtype=np.int64), users,
                                      tiles=True)
        return list(out.items())
    return list(cells_to_rows(weighted_location_cells(zs, rows, cols, users, w, zmax, d)).items())


def weighted_location_cells(zs, rows, cols, users, weights, zmax, d, project=None) -> Cells:
    """Bins of build_heatmaps' rows for locations at any zoom with any float
    count.  The first level takes the tile holding each location tile's centre
    at the detail zoom (heatmap.py:60-61: tile_from_tile_id, then
    tile_id_from_lat_long); the levels below follow the shift, or the literal
    chain outside its windows (ChainFix); weights are summed per (group, cell)
    in float64 (the reference's reduceByKey sums; exact for integer-valued
    counts below 2^53)."""
    zs = np.asarray(zs, np.int64)
    n = zs.size
    T_r = np.zeros(n, np.int64)
    T_c = np.zeros(n, np.int64)
    for z0 in np.unique(zs).tolist():
        m = np.flatnonzero(zs == z0)
        keys = sorted({(rows[i], cols[i]) for i in m.tolist()})
        tr, tc = _recentre(z0, [k[0] for k in keys], [k[1] for k in keys], zmax, project)
        at = {k: j for j, k in enumerate(keys)}
        for i in m.tolist():
            j = at[(rows[i], cols[i])]
            T_r[i], T_c[i] = tr[j], tc[j]
    wv = np.asarray(weights, np.float64)
    # integer-valued counts (dataframe_loader's 1.0s, heatmap_to_locations of
    # such rows) are summed as int64 -- exact in any order, so on the GPU for
    # large lists (_sum_by_cell); other floats in float64 on the host, in input
    # order within a cell as the reference's reduceByKey folds them
    if np.all(wv == np.trunc(wv)) and float(np.abs(wv).sum()) < 2.0 ** 53:
        wv = wv.astype(np.int64)
    plan = group_plan(users)
    # every level's tile of each distinct first-level tile: the shift inside
    # the windows, the literal chain outside (ChainFix)
    U, inv = np.unique(np.stack([T_r, T_c], 1), axis=0, return_inverse=True)
    inv = inv.reshape(-1)
    ur, uc = U[:, 0].copy(), U[:, 1].copy()
    lev = {z: (ur >> (zmax - z), uc >> (zmax - z)) for z in range(zmax, d, -1)}
    bad = ~_in_chain_window(ur, uc, zmax, d)
    over = {}
    if bad.any():
        fix = ChainFix(ur[bad], uc[bad], zmax, d, first_applied=True, project=project)
        for z in range(zmax, d, -1):
            r, c = lev[z][0].copy(), lev[z][1].copy()
            r[bad], c[bad] = fix.level[z]
            lev[z] = (r, c)
        over = fix.overrides()
    gsel = plan.grouped
    az, ar, ac, av, gg, gz, gr, gc, gv = [], [], [], [], [], [], [], [], []
    for z in range(zmax, d, -1):
        lr, lc = lev[z][0][inv], lev[z][1][inv]
        az.append(np.full(n, z, np.int64))
        ar.append(lr)
        ac.append(lc)
        av.append(wv)
        gg.append(plan.gid[gsel].astype(np.int64))
        gz.append(np.full(int(gsel.sum()), z, np.int64))
        gr.append(lr[gsel])
        gc.append(lc[gsel])
        gv.append(wv[gsel])
    cz, cr, cc, cv = _sum_by_cell([(np.concatenate(az), np.concatenate(ar), np.concatenate(ac),
                                    np.concatenate(av)[:, None])])
    allc = (cz, cr, cc, cv[:, 0])
    if gsel.any():
        kz, kr, kc, kv = _sum_by_cell([(np.concatenate(gg) * 64 + np.concatenate(gz), np.concatenate(gr),
                                        np.concatenate(gc), np.concatenate(gv)[:, None])])
        grp = (kz // 64, kz % 64, kr, kc, kv[:, 0])
    else:
        grp = (np.zeros(0, np.int64),) * 4 + (np.zeros(0, wv.dtype),)
    if wv.dtype.kind == "i":   # the reference's counts are floats
        allc = allc[:3] + (allc[3].astype(np.float64),)
        grp = grp[:4] + (grp[4].astype(np.float64),)
    return combine_cells(plan.labels, allc, grp, zmax, d, exact_levels=over)
