"""Final-level bucket paths at their size boundaries (hm_count_tiles input).

The last pipeline level bins each zoom-(Z-7) bucket (128 x 128 zoom-Z tiles)
by one of three kernels chosen by its key count: k_small_sort/k_small_emit
(<= 2048 keys, one wavefront; register sorts of 64/128/256/512/1024/2048 keys),
k_aggregate (dense, one 256K-key work item) and k_aggregate_merged (several
items).  Every boundary is hit with several key patterns, and with zoom
windows that drop some of the pyramid levels.  Expected counts: oracle.count_tiles
(the per-zoom reduceByKey of heatmap.py:109-111 over tile ids).
"""
import numpy as np
import pytest

from conftest import cells_digest
from oracle import oracle
from heatmap_amd import device

pytestmark = pytest.mark.gpu

SIZES = [1, 2, 3, 63, 64, 65, 127, 128, 129, 255, 256, 257, 511, 512, 513, 777, 1023, 1024, 1025, 2047, 2048, 2049,
         4096, 70000, 300000]
PATTERNS = ["spread", "same", "row", "pairs", "corner"]


def _bucket_tiles(rng, Z, sizes, patterns):
    """Tiles at zoom Z, bucket by bucket (each bucket a distinct 128x128 block)."""
    side = 1 << (Z - 7)
    nb = len(sizes) * len(patterns)
    ids = rng.choice(side * side, size=nb, replace=False)
    rows, cols = [], []
    k = 0
    for s in sizes:
        for p in patterns:
            br, bc = divmod(int(ids[k]), side)
            k += 1
            if p == "spread":
                r = rng.integers(0, 128, s)
                c = rng.integers(0, 128, s)
            elif p == "same":
                r = np.full(s, 77)
                c = np.full(s, 5)
            elif p == "row":
                r = np.full(s, 127)
                c = rng.integers(0, 128, s)
            elif p == "pairs":
                r = np.where(np.arange(s) % 2 == 0, 0, 127)
                c = np.where(np.arange(s) % 2 == 0, 0, 127)
            else:   # 2x2 corner: 4 cells share one parent at every level
                r = rng.integers(0, 2, s)
                c = rng.integers(126, 128, s)
            rows.append(br * 128 + r)
            cols.append(bc * 128 + c)
    rows = np.concatenate(rows).astype(np.int64)
    cols = np.concatenate(cols).astype(np.int64)
    perm = rng.permutation(rows.size)            # scatter every bucket over the input
    return rows[perm], cols[perm]


def _check(rows, cols, zmin, zmax):
    got = device.count(rows, cols, None, zmin, zmax, tiles=True)
    ref = oracle.count_tiles(rows, cols, zmin, zmax)
    assert got.zoom.size == ref["zoom"].size
    if got.zoom.size > 4_000_000:   # order-free comparison of large outputs
        assert cells_digest(got.zoom, got.row, got.col, got.count) == \
            cells_digest(ref["zoom"], ref["row"], ref["col"], ref["count"])
        return
    got = got.sorted()
    for k in ("zoom", "row", "col", "count"):
        assert np.array_equal(getattr(got, k), ref[k]), k


@pytest.mark.parametrize("zmin", [0, 12, 16, 18])
def test_bucket_boundaries_z18(gpu, zmin):
    rng = np.random.default_rng(11 + zmin)
    rows, cols = _bucket_tiles(rng, 18, SIZES, PATTERNS)
    _check(rows, cols, zmin, 18)


@pytest.mark.parametrize("Z", [10, 13, 21])
def test_bucket_boundaries_other_zooms(gpu, Z):
    rng = np.random.default_rng(Z)
    rows, cols = _bucket_tiles(rng, Z, [1, 64, 65, 256, 512, 513, 2048, 2049, 9000], PATTERNS)
    _check(rows, cols, 0, Z)


def test_many_small_buckets(gpu):
    """~100k buckets of 1..600 keys: the small path's batching and one-reservation scan."""
    rng = np.random.default_rng(5)
    Z = 18
    side = 1 << (Z - 7)
    nb = 50_000
    ids = rng.choice(side * side, size=nb, replace=False)
    sz = rng.integers(1, 600, nb)
    br = np.repeat(ids // side, sz)
    bc = np.repeat(ids % side, sz)
    rows = (br * 128 + rng.integers(0, 128, br.size)).astype(np.int64)
    cols = (bc * 128 + rng.integers(0, 128, bc.size)).astype(np.int64)
    perm = rng.permutation(rows.size)
    _check(rows[perm], cols[perm], 0, Z)


@pytest.mark.parametrize("Z,n", [(3, 50), (6, 5000), (7, 300), (8, 70000)])
def test_low_zoom_single_bucket(gpu, Z, n):
    """Z <= 8: one or a few final buckets of side 2^min(Z, 7)."""
    rng = np.random.default_rng(Z)
    rows = rng.integers(0, 1 << Z, n).astype(np.int64)
    cols = rng.integers(0, 1 << Z, n).astype(np.int64)
    _check(rows, cols, 0, Z)
