"""GPU: the general count path (hm_general.hip) against the oracle.

Kept points outside [0, 2^z)^2 -- polar latitudes (negative rows, rows past
2^z), longitudes at or beyond +-180 (columns >= 2^z or < 0) -- are binned by the
reference like any other (tile.py:17,21 never clamp; heatmap.py:27-36 keeps
them).  Grouped counts (hm_count_grouped) are the per-user keys of
heatmap.py:64-75 in one pass."""
import numpy as np
import pytest

from oracle import oracle
from heatmap_amd import device, synth

pytestmark = pytest.mark.gpu


def _exotic_cloud(n, seed, frac=0.05):
    rng = np.random.default_rng(seed)
    lat, lon = synth.generate("hotspots", n, seed=seed)
    lat, lon = lat.copy(), lon.copy()
    m = rng.random(n) < frac
    k = int(m.sum())
    lat[m] = rng.choice([-1.0, 1.0], k) * rng.uniform(85.06, 89.9, k)
    lon[m] = rng.choice([180.0, 200.0, -200.0, 540.0, -180.0, 179.99999999999997], k)
    return lat, lon


def _same(got, ref):
    assert ref["status"] == 0
    for k in ("zoom", "row", "col", "count"):
        assert np.array_equal(getattr(got, k), ref[k]), k


@pytest.mark.parametrize("zmax", [14, 18, 21])
def test_exotic_vs_oracle(gpu, zmax):
    lat, lon = _exotic_cloud(200_000, seed=zmax)
    keep = (np.arange(lat.size) % 9 != 4).astype(np.uint8)
    got = device.count(lat, lon, keep, 0, zmax).sorted()
    _same(got, oracle.count(lat, lon, keep, 0, zmax))
    assert (got.row < 0).any() and (got.col >= (1 << got.zoom)).any()


def test_exotic_only_and_single(gpu):
    for lat, lon in ((np.array([89.0]), np.array([200.0])),
                     (np.array([-86.5, 86.5, 89.99999998]), np.array([-540.0, 1e6, 180.0]))):
        for zmin, zmax in ((0, 21), (6, 14), (0, 0)):
            _same(device.count(lat, lon, None, zmin, zmax).sorted(), oracle.count(lat, lon, None, zmin, zmax))


def test_exotic_tiles(gpu):
    """hm_count_tiles with tiles outside the square (negative, >= 2^z, huge)."""
    rng = np.random.default_rng(5)
    n = 100_000
    z = 16
    rows = rng.integers(-(8 << z), 8 << z, n)
    cols = rng.integers(-(1 << 40), 1 << 40, n)
    cols[::3] = rng.integers(0, 1 << z, (n + 2) // 3)
    got = device.count(rows, cols, None, 0, z, tiles=True).sorted()
    ref = oracle.count_tiles(rows, cols, 0, z)
    o = np.lexsort((ref["col"], ref["row"], ref["zoom"]))
    for k in ("zoom", "row", "col", "count"):
        assert np.array_equal(getattr(got, k), ref[k][o]), k


@pytest.mark.parametrize("zmin,zmax,groups", [(0, 14, 7), (6, 21, 1000), (3, 18, 1)])
def test_grouped_vs_oracle(gpu, zmin, zmax, groups):
    lat, lon = _exotic_cloud(120_000, seed=groups, frac=0.02)
    rng = np.random.default_rng(groups)
    g = rng.integers(0, groups, lat.size).astype(np.uint32) * 7919   # sparse ids
    keep = (rng.random(lat.size) < 0.8).astype(np.uint8)
    got = device.count_grouped(lat, lon, g, keep, zmin, zmax).sorted()
    exp = {k: [] for k in ("group", "zoom", "row", "col", "count")}
    for gid in np.unique(g[keep.astype(bool)]):
        ref = oracle.count(lat, lon, keep & (g == gid), zmin, zmax)
        assert ref["status"] == 0
        exp["group"].append(np.full(ref["zoom"].size, gid, np.uint32))
        for k in ("zoom", "row", "col", "count"):
            exp[k].append(ref[k])
    for k in exp:
        assert np.array_equal(getattr(got, k), np.concatenate(exp[k])), k


@pytest.mark.parametrize("zmin,zmax,groups", [(0, 14, 7), (6, 21, 1000), (3, 18, 1), (6, 21, 5_000_000)])
def test_grouped_packed_vs_oracle(gpu, zmin, zmax, groups):
    """hm_count_grouped_packed (16-B records: HM_KEY, group << 32 | count) on
    in-square points == the oracle per group, and records of one zoom are
    contiguous, zoom zmax first; groups past 2^22 make the sort's keys 128-bit
    at zoom 21.  A kept point outside the square: None (HM_E_EXOTIC); an
    unkept one does not matter."""
    lat, lon = synth.generate("hotspots", 80_000, seed=groups)
    rng = np.random.default_rng(groups)
    g = rng.integers(0, groups, lat.size).astype(np.uint32) * (7919 if groups < 1000 else 1)
    keep = (rng.random(lat.size) < 0.8).astype(np.uint8)
    keys, gc = device.count_grouped_packed_device(lat, lon, g, keep, zmin, zmax)
    k = keys.cpu().numpy().view(np.uint64)
    z = (k >> np.uint64(58)).astype(np.int32)
    assert np.all(np.diff(z) <= 0) and z[0] == zmax
    gcn = gc.cpu().numpy().view(np.uint64)
    got = device.GroupedCounts((gcn >> np.uint64(32)).astype(np.uint32), z,
                               ((k >> np.uint64(29)) & np.uint64(0x1FFFFFFF)).astype(np.int64),
                               (k & np.uint64(0x1FFFFFFF)).astype(np.int64),
                               (gcn & np.uint64(0xFFFFFFFF)).astype(np.int64)).sorted()
    ref = device.count_grouped(lat, lon, g, keep, zmin, zmax).sorted()
    for f in ("group", "zoom", "row", "col", "count"):
        assert np.array_equal(getattr(got, f), getattr(ref, f)), f
    if groups <= 7:   # pinned to the oracle directly as well
        for gid in np.unique(g[keep.astype(bool)])[:3]:
            o = oracle.count(lat, lon, keep & (g == gid), zmin, zmax)
            m = got.group == gid
            assert np.array_equal(got.count[m], o["count"][np.lexsort((o["col"], o["row"], o["zoom"]))])
    lat2 = lat.copy()
    lat2[5] = 88.0
    keep2 = keep.copy()
    keep2[5] = 1
    assert device.count_grouped_packed_device(lat2, lon, g, keep2, zmin, zmax) is None
    keep2[5] = 0
    assert device.count_grouped_packed_device(lat2, lon, g, keep2, zmin, zmax) is not None


def test_grouped_many_unsettled_points(gpu):
    """More points than the fast projection's list holds (2^16 here) left to
    the exact chain -- 60% polar or beyond +-180: the exact pass sweeps the
    whole input again; the counts still equal the oracle's per group."""
    lat, lon = _exotic_cloud(150_000, seed=77, frac=0.6)
    g = (np.arange(lat.size) % 3).astype(np.uint32) * 11
    got = device.count_grouped(lat, lon, g, None, 4, 18).sorted()
    for gid in (0, 11, 22):
        ref = oracle.count(lat, lon, (g == gid).astype(np.uint8), 4, 18)
        m = got.group == gid
        for k in ("zoom", "row", "col", "count"):
            assert np.array_equal(getattr(got, k)[m], ref[k]), k


def test_grouped_errors(gpu):
    lat, lon = synth.uniform(10000, seed=2)
    lat = lat.copy()
    lat[777] = np.inf
    with pytest.raises(ValueError, match="domain"):
        device.count_grouped(lat, lon, np.zeros(lat.size, np.uint32), None, 0, 10)


@pytest.mark.parametrize("n,zmin,zmax,fallback", [(1_000_000, 0, 21, True), (300_000, 12, 20, False)])
def test_sparse_fallback_vs_oracle(gpu, n, zmin, zmax, fallback):
    """Uniform 1M points at zoom 21: the pipeline's dense per-level child space
    would pass its limit, so hm_count takes the general path (in-square cells
    still come back as HM_KEYs, exotic ones as records); 300k at zoom 20 stays
    on the pipeline."""
    lat, lon = synth.uniform(n, seed=11)
    lat, lon = lat.copy(), lon.copy()
    lat[::1000] = 88.5
    lon[1::1000] = 200.0
    got = device.count(lat, lon, None, zmin, zmax)
    assert (int(got.stage_us[7]) == 0) == fallback   # slot 7: the plan's partition levels (0: general path)
    _same(got.sorted(), oracle.count(lat, lon, None, zmin, zmax))


def test_huge_latitudes(gpu):
    """|lat pi/180| >= 105414350: glibc reduces with __branred, restated on the
    device (hm_branred.h); projection statuses/rows and counts equal the
    oracle's (live libm)."""
    rng = np.random.default_rng(12)
    n = 100_000
    lat = np.exp(rng.uniform(np.log(6.1e9), np.log(1e300), n)) * rng.choice([-1.0, 1.0], n)
    lon = rng.uniform(-180.0, 180.0, n)
    for z in (0, 14, 18, 21):
        p = device.project(lat, lon, z)
        ro, co, so, _ = oracle.project(lat, lon, z)
        assert np.array_equal(p.status, so), z
        ok = so == 0
        assert np.array_equal(p.row[ok], ro[ok]) and np.array_equal(p.col[ok], co[ok]), z
    keep = (oracle.project(lat, lon, 18)[2] == 0).astype(np.uint8)
    lat2, lon2 = np.where(keep == 1, lat, 10.0), lon
    _same(device.count(lat2, lon2, None, 0, 18).sorted(), oracle.count(lat2, lon2, None, 0, 18))


def test_sum_by_cell_device_matches_host(gpu):
    """heatmap._sum_by_cell on the GPU (row assembly of large row sets) equals
    the numpy lexsort path: unique (zoom, row, col) in order, summed columns."""
    from heatmap_amd import heatmap as hm

    g = np.random.default_rng(3)
    parts = []
    for m in (700_000, 500_000):
        z = g.integers(7, 22, m)
        r = g.integers(0, 1 << 12, m) & ((1 << z) - 1)
        c = g.integers(0, 1 << 12, m) & ((1 << z) - 1)
        v = g.integers(0, 1 << 40, (m, 3))
        parts.append((z, r, c, v))
    dev = hm._sum_by_cell(parts, device_min=1)
    host = hm._sum_by_cell(parts, device_min=1 << 62)
    for a, b in zip(dev, host):
        assert np.array_equal(np.asarray(a), np.asarray(b))


def test_row_order_device_matches_host(gpu):
    """heatmap._row_order's GPU sorts give np.lexsort's permutation on
    distinct bins."""
    from heatmap_amd import heatmap as hm

    g = np.random.default_rng(4)
    m = 1_500_000
    zoom = g.integers(7, 22, m)
    row = g.integers(0, 1 << 21, m) & ((1 << zoom) - 1)
    col = g.integers(0, 1 << 21, m) & ((1 << zoom) - 1)
    label = g.integers(0, 3000, m)
    span = g.integers(0, 3, m)
    key = (label << 40) | (span << 36) | (zoom << 30) | (row << 15) | col
    keep = np.unique(key, return_index=True)[1]       # distinct bins
    zoom, row, col, label, span = zoom[keep], row[keep], col[keep], label[keep], span[keep]
    d = 5
    args = (label, span, zoom - d, row >> d, col >> d, zoom, row, col)
    assert np.array_equal(hm._row_order(*args, device_min=1), hm._row_order(*args, device_min=1 << 62))


def test_heat_text_device_matches_host(gpu):
    """Row JSON written on the GPU (hm_format_bins) is byte-identical to the
    pyarrow host assembly: rows of 1..40 bins, counts 0 .. 1e16 - 1."""
    import pyarrow as pa

    from heatmap_amd import heatmap as hm

    g = np.random.default_rng(5)
    sizes = g.integers(1, 41, 60_000)
    n = int(sizes.sum())
    starts = np.concatenate([[0], np.cumsum(sizes)[:-1]]).astype(np.int64)
    z = g.integers(0, 22, n)
    r = g.integers(0, 1 << 21, n) & ((1 << z) - 1)
    c = g.integers(0, 1 << 21, n) & ((1 << z) - 1)
    v = np.where(g.random(n) < 0.5, g.integers(0, 1000, n), g.integers(0, 10 ** 16, n))
    v[:3] = [0, 10 ** 16 - 2, 9]
    v = v.astype(np.float64).astype(np.int64)   # the product's counts are float64 values (Cells.value)
    dev = hm._heat_text_device(z, r, c, v, starts, device_min=1)
    assert dev is not None and len(dev) == starts.size
    host = []
    ends = np.append(starts[1:], n)
    for a, b in zip(starts[:2000].tolist(), ends[:2000].tolist()):
        host.append("{" + ", ".join('"%d_%d_%d": %s' % (z[i], r[i], c[i], repr(float(v[i])))
                                    for i in range(a, b)) + "}")
    assert isinstance(dev, pa.LargeStringArray)
    assert dev.slice(0, 2000).to_pylist() == host


@pytest.mark.parametrize("override", [False, True])
def test_cells_to_table_device_matches_host(gpu, override):
    """cells_to_table's device path (order, gathers and JSON on the GPU) gives
    the host path's table exactly: ids and heatmap strings, row by row; with
    ChainFix row-tile overrides on some bins too (Cells.row_tiles)."""
    from heatmap_amd import heatmap as hm

    g = np.random.default_rng(6)
    m = 400_000
    zoom = g.integers(6, 22, m)
    row = g.integers(0, 1 << 21, m) & ((1 << zoom) - 1)
    col = g.integers(0, 1 << 21, m) & ((1 << zoom) - 1)
    label = g.integers(0, 50, m)
    span = g.integers(0, 2, m)
    key = (label << 44) | (span << 43) | (zoom << 38) | (row << 19) | col
    keep = np.unique(key, return_index=True)[1]
    val = g.integers(1, 10 ** 9, keep.size).astype(np.float64)
    over = None
    if override:   # a few (zoom, row, col) bins whose row tile is a neighbour of the shift
        idx = g.choice(keep.size, 40, replace=False)
        over = {(int(zoom[keep][i]), int(row[keep][i]), int(col[keep][i])):
                ((int(row[keep][i]) >> 5) ^ 1, int(col[keep][i]) >> 5) for i in idx}
    cells = hm.Cells(["u%d" % i for i in range(50)], label[keep], zoom[keep], row[keep], col[keep], val, 5,
                     ["alltime", "2024"], span[keep], tile_override=over)
    dev = hm._cells_to_table_device(cells)
    old = hm.SUM_BY_CELL_DEVICE_MIN
    hm.SUM_BY_CELL_DEVICE_MIN = 1 << 62
    try:
        host = hm.cells_to_table(cells)
    finally:
        hm.SUM_BY_CELL_DEVICE_MIN = old
    assert dev is not None
    assert dev.column("id").to_pylist() == host.column("id").to_pylist()
    assert dev.column("heatmap").to_pylist() == host.column("heatmap").to_pylist()


@pytest.mark.parametrize("threaded_copy", [False, True])
def test_heatmap_table_device_matches_host(gpu, threaded_copy, monkeypatch):
    """heatmap_table end to end on the device (counts resident from hm_count /
    hm_count_grouped through the JSON) == combine_cells + the host
    cells_to_table on the same counts: 200K hotspot points, 300 users with
    'x*', 'rt-*' and literal 'all' ids, background rows, zooms 6-21;
    threaded_copy: the text columns leave in 1 MB chunks from the copy
    threads (heatmap._to_host) instead of one copy."""
    from heatmap_amd import heatmap as hm
    from heatmap_amd import synth

    if threaded_copy:
        monkeypatch.setattr(hm, "THREADED_COPY_MIN", 2 << 20)

    n = 200_000
    lat, lon = synth.generate("hotspots", n, seed=11)
    g = np.random.default_rng(11)
    names = np.array(["u%d" % i for i in range(300)] + ["x-anon", "rt-7", "rt-9", "all"], dtype=object)
    user = names[g.integers(0, names.size, n)]
    keep = g.random(n) > 0.2
    dev = hm.heatmap_table(lat, lon, user, keep, 16, 5)
    assert "combine (device)" in hm.LAST_TABLE_PHASES     # the device path ran
    old = hm.SUM_BY_CELL_DEVICE_MIN
    hm.SUM_BY_CELL_DEVICE_MIN = 1 << 62
    try:
        host = hm.cells_to_table(hm.heatmap_cells(lat, lon, user, keep, 16, 5))
    finally:
        hm.SUM_BY_CELL_DEVICE_MIN = old
    assert dev.num_rows == host.num_rows
    assert dev.column("id").to_pylist() == host.column("id").to_pylist()
    assert dev.column("heatmap").to_pylist() == host.column("heatmap").to_pylist()
