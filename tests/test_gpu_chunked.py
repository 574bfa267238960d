"""GPU: inputs larger than one hm_count call (device.MAX_CALL_POINTS = 2^31)
are counted chunk by chunk and the chunks' cells summed on the device
(device.count_device, hm_cells_merge).  Small forced chunks against the
oracle (cells inside and outside the square, keep masks); the first failing
point keeps its global index; and a 2^32 + 2^20-point cloud on one GPU (3 and
4 chunks), whose per-zoom totals must be n and whose cells must not depend on
the chunking."""
import numpy as np
import pytest

from oracle import oracle
from heatmap_amd import _lib, device
from test_gpu_general import _exotic_cloud, _same

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("zmax,chunk", [(14, 70_001), (18, 65_536), (21, 150_000)])
def test_chunked_vs_oracle(gpu, zmax, chunk):
    lat, lon = _exotic_cloud(300_000, seed=40 + zmax, frac=0.01)
    keep = (np.arange(lat.size) % 7 != 3).astype(np.uint8)
    got = device.count(lat, lon, keep, 0, zmax, chunk=chunk).sorted()
    _same(got, oracle.count(lat, lon, keep, 0, zmax))


def test_chunked_error_index(gpu):
    lat, lon = _exotic_cloud(200_000, seed=3, frac=0.0)
    lon = lon.copy()
    lon[150_123] = 1e300         # column beyond int64: HM_E_RANGE
    lon[190_000] = -1e300
    with pytest.raises(_lib.DevicePathUnsupported, match=r"\(point 150123\)"):
        device.count(lat, lon, None, 0, 14, chunk=70_000)


def test_over_one_call(gpu):
    import torch

    n = (1 << 32) + (1 << 20)
    lat = torch.empty(n, dtype=torch.float64, device="cuda")
    lon = torch.empty(n, dtype=torch.float64, device="cuda")
    device.synth("hotspots", lat, lon, seed=7)
    res = {}
    for chunk in (device.MAX_CALL_POINTS, 3 << 29):
        m, buf = device.count_device(lat, lon, None, 0, 16, chunk=chunk)
        assert buf.nx == 0
        k, order = torch.sort(buf.keys[:m])
        c = buf.counts[:m][order]
        zoom = (k.view(torch.int64) >> 58) & 63
        per_zoom = torch.zeros(17, dtype=torch.int64, device="cuda").index_add_(0, zoom, c)
        assert bool((per_zoom == n).all()), per_zoom.tolist()
        res[chunk] = (k.cpu(), c.cpu())
        del buf
        torch.cuda.empty_cache()
    (k1, c1), (k2, c2) = res.values()
    assert torch.equal(k1, k2) and torch.equal(c1, c2)
