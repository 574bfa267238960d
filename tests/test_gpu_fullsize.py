"""Parity at the bench sizes: 1e9-point clouds (BASELINE configs 2 and 4) and
a 20-batch x 10M-point stream (config 5), cell for cell through the
order-free digest of tests/conftest.py, computed on the device and compared
with tests/golden/big_digests.json (the C oracle, tests/golden/make_bigdigest.py).

These are the sizes at which paths switch on that smaller tests reach only
with tuned thresholds: hot tiles at their default share, the region-sized
level 1 with its sampled margins, many-run children copied by k_rs_copy_big
(skew with hot tiles off: ~110k runs in one child), multi-item buckets merged
through global slots.
"""
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN
from heatmap_amd import device

pytestmark = pytest.mark.gpu

from digest import device_cells_digest, device_digest  # noqa: E402


@pytest.fixture(autouse=True)
def _release_device_memory():
    """Each full-size case starts on an emptied device: the library's cached
    contexts (their count buffers sized by the last 1e9-point call) and
    torch's cached blocks are released after every case.  The concurrent
    per-bucket stream allocates one context per bucket, and after the grouped
    cases it ran out of device memory when this file ran first."""
    yield
    import gc

    import torch

    device._CTX.clear()
    gc.collect()
    torch.cuda.empty_cache()


def _golden(name):
    path = os.path.join(GOLDEN, "big_digests.json")
    d = json.load(open(path))
    if name not in d:
        pytest.skip("%s not in big_digests.json" % name)
    return d[name]


@pytest.mark.parametrize("name,hot", [("hotspots_1e9_z0-18", 1), ("hotspots_1e9_z0-18", 0),
                                      ("skew_1e9_z0-18", 1), ("skew_1e9_z0-18", 0), ("uniform_6e8_z0-18", 1),
                                      ("hotspots_1e9_z6-21", 1)])
def test_fullsize_cloud(gpu, name, hot):
    torch = gpu
    g = _golden(name)
    n = g["n"]
    lat = torch.empty(n, dtype=torch.float64, device="cuda")
    lon = torch.empty(n, dtype=torch.float64, device="cuda")
    device.synth(g["kind"], lat, lon, seed=g["seed"], start=g["start"])
    with device.tuned(HM_HOT=hot):
        m, buf = device.count_device(lat, lon, None, g["zmin"], g["zmax"])
        st = device.context(0).last_stats()[1]
    del lat, lon
    assert buf.nx == 0
    if hot and name.startswith("skew"):
        assert int(st[6]) == 1
    if not hot:
        assert int(st[6]) == 0
    if name.startswith("uniform"):
        assert int(st[7]) == 3       # the spread plan, by default at this size
    assert device_digest(torch, buf.keys[:m], buf.counts[:m]) == g["digest"]


def test_fullsize_stream(gpu):
    """20 batches of 10M points, one epoch hour each, folded into a resident
    heatmap: the alltime cells equal the oracle's count of all 200M points,
    and three hours' cells equal their batches' counts."""
    torch = gpu
    from heatmap_amd.stream import ALLTIME, StreamingHeatmap

    base = 480000
    g = _golden("hotspots_2e8_z0-18_stream20x10M")
    b = 10_000_000
    s = StreamingHeatmap(0, 18, base_hour=base, initial_cells=1 << 26)
    lat = torch.empty(b, dtype=torch.float64, device="cuda")
    lon = torch.empty(b, dtype=torch.float64, device="cuda")
    for k in range(20):
        device.synth("hotspots", lat, lon, seed=0, start=k * b)
        s.add(lat, lon, hour=torch.full((b,), base + k, dtype=torch.int32, device="cuda"))
    n, keys, counts = s.extract_device(ALLTIME)[:3]
    assert device_digest(torch, keys[:n], counts[:n]) == g["digest"]
    for k, name in ((0, "hotspots_1e7_start0_z0-18"), (7, "hotspots_1e7_start70M_z0-18"),
                    (19, "hotspots_1e7_start190M_z0-18")):
        n, keys, counts = s.extract_device(base + k)[:3]
        assert device_digest(torch, keys[:n], counts[:n]) == _golden(name)["digest"], name
    s.close()


def test_fullsize_grouped(gpu):
    """hm_count_grouped at the reference's production zooms (detail zooms 21..6,
    heatmap.py:16-17,109): 1e8 hotspot points x 10,000 user groups, every
    (group, zoom, row, col, count) record against the C oracle's digest
    (tests/golden/make_bigdigest.py: group-tagged rows, every zoom the shift)."""
    torch = gpu
    import ctypes

    from heatmap_amd import _lib

    g = _golden("grouped_hotspots_1e8_u10000_z6-21")
    n, users, zmin, zmax = g["n"], g["users"], g["zmin"], g["zmax"]
    lat = torch.empty(n, dtype=torch.float64, device="cuda")
    lon = torch.empty(n, dtype=torch.float64, device="cuda")
    device.synth(g["kind"], lat, lon, seed=g["seed"])
    grp = (((torch.arange(n, device="cuda", dtype=torch.int64) * 2654435761) >> 7) % users).to(torch.int32)
    ctx = device.context(0)
    cap = 10 * n
    cells = torch.empty(5 * cap, dtype=torch.int64, device="cuda")
    nout = ctypes.c_int64(0)
    p = device._ptr
    rc = ctx.L.hm_count_grouped(ctx.ptr, p(lat), p(lon), ctypes.c_void_p(0), p(grp), n, zmin, zmax, p(cells), cap,
                                ctypes.byref(nout))
    assert rc == _lib.HM_OK, rc
    del lat, lon, grp
    rec = cells[:5 * nout.value].reshape(-1, 5)
    gr, z, r, c, cnt = (rec[:, i] for i in range(5))
    assert device_cells_digest(torch, z, (gr << (z + 1)) | r, c, cnt) == g["digest"]


def test_fullsize_grouped_packed(gpu):
    """The same production-zoom grouped count through the 16-B packed records
    (hm_count_grouped_packed), against the same oracle digest."""
    torch = gpu
    g = _golden("grouped_hotspots_1e8_u10000_z6-21")
    n, users, zmin, zmax = g["n"], g["users"], g["zmin"], g["zmax"]
    lat = torch.empty(n, dtype=torch.float64, device="cuda")
    lon = torch.empty(n, dtype=torch.float64, device="cuda")
    device.synth(g["kind"], lat, lon, seed=g["seed"])
    grp = (((torch.arange(n, device="cuda", dtype=torch.int64) * 2654435761) >> 7) % users).to(torch.int32)
    keys, gc = device.count_grouped_packed_device(lat, lon, grp, None, zmin, zmax)
    del lat, lon, grp
    z, r, c = keys >> 58, (keys >> 29) & 0x1FFFFFFF, keys & 0x1FFFFFFF
    gr, cnt = gc >> 32, gc & 0xFFFFFFFF
    assert device_cells_digest(torch, z, (gr << (z + 1)) | r, c, cnt) == g["digest"]


def test_fullsize_stream_multi_hour_batches(gpu):
    """The same 20 x 10M-point stream with 2 or 3 hours per batch (alternating),
    the concurrent per-bucket path (stream_fold_parts_par: one context, HIP
    stream and host thread per bucket run): the alltime cells equal the
    oracle's digest of all 200M points, and the hours of batches 0 and 19,
    summed (hm_cells_merge), equal their batches' digests."""
    torch = gpu
    from heatmap_amd import multigpu
    from heatmap_amd.stream import ALLTIME, StreamingHeatmap

    base = 480000
    g = _golden("hotspots_2e8_z0-18_stream20x10M")
    b = 10_000_000
    s = StreamingHeatmap(0, 18, base_hour=base, initial_cells=1 << 26)
    lat = torch.empty(b, dtype=torch.float64, device="cuda")
    lon = torch.empty(b, dtype=torch.float64, device="cuda")
    first = {}
    h0 = base
    for k in range(20):
        nh = 2 + (k & 1)
        first[k] = (h0, nh)
        device.synth("hotspots", lat, lon, seed=0, start=k * b)
        hour = (h0 + torch.arange(b, device="cuda", dtype=torch.int64) % nh).to(torch.int32)
        s.add(lat, lon, hour=hour)
        h0 += nh
    n, keys, counts = s.extract_device(ALLTIME)[:3]
    assert device_digest(torch, keys[:n], counts[:n]) == g["digest"]
    ops = multigpu.DeviceOps(0)
    for k, name in ((0, "hotspots_1e7_start0_z0-18"), (19, "hotspots_1e7_start190M_z0-18")):
        h, nh = first[k]
        parts = []
        for j in range(nh):   # (copies: a rollup's outputs may live in the stream's scratch)
            m, kk, cc = s.extract_device(h + j)[:3]
            parts.append((kk[:m].clone(), cc[:m].clone()))
        mk = torch.cat([p[0] for p in parts])
        mc = torch.cat([p[1] for p in parts])
        uk, uc = ops.merge(mk, mc)
        assert device_digest(torch, uk, uc) == _golden(name)["digest"], name
    s.close()
