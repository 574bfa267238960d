"""Config 3's exchange (10B points over 8 GPUs, BASELINE.json configs[2]) on ONE
GPU, cell for cell: eight emulated ranks.

The 1e9-point hotspot cloud of tests/golden/big_digests.json
("hotspots_1e9_z0-18") is cut into 8 contiguous shards of 1.25e8 points --
exactly the points rank r of an 8-GPU run would hold.  Each shard is counted
by hm_count and routed by hm_cells_route_pieces(nranks=8, dense_zmax=10), the
kernels multigpu.merge_cells runs on every rank; then what the collectives
would do is done with tensor ops on the one device:

  RCCL reduce       the 8 dense zoom-0..10 grids are summed, hm_dense_cells
                    lists the result (rank 0's cells);
  all-to-all        owner o takes shard r's group o (r = 0..7) -- read in
                    place, as merge_cells reads its own group -- and
                    hm_cells_merge_pieces sums equal keys.

The union of the 8 owners' cells plus the dense cells must equal the C
oracle's digest of the whole cloud, and every merged cell must hash to the
owner that holds it (multigpu.record_owner, the heatmap-row key of
/root/reference/heatmap.py:111-112), so every cell has exactly one owner.

The wide variant adds 2^32 to one sparse cell of shard 3 before routing: its
narrow route flags wide in every size row, so (as in merge_cells) every shard
is routed again with int64 keys and counts; the 2^32 is taken off the merged cell
before the digest.
"""
import json
import os

import pytest

from conftest import GOLDEN
from digest import device_cells_digest
from heatmap_amd import _lib, device, multigpu

pytestmark = pytest.mark.gpu

WS = 8
DZ = 10
M29 = (1 << 29) - 1
U64 = (1 << 64) - 1


def _combine(a, b):
    return [a[0] + b[0], a[1] + b[1], (a[2] + b[2]) & U64, a[3] ^ b[3]]


@pytest.mark.parametrize("wide", [False, True])
def test_config3_exchange_on_one_gpu(gpu, wide):
    torch = gpu
    g = json.load(open(os.path.join(GOLDEN, "big_digests.json")))["hotspots_1e9_z0-18"]
    n, per = g["n"], g["n"] // WS
    ops = multigpu.DeviceOps(0)
    bits = multigpu.route_bits(WS)
    S = 1 << bits
    lat = torch.empty(per, dtype=torch.float64, device="cuda")
    lon = torch.empty(per, dtype=torch.float64, device="cuda")
    shards = []
    bump = None
    for r in range(WS):
        device.synth(g["kind"], lat, lon, seed=g["seed"], start=g["start"] + r * per)
        m, buf = device.count_device(lat, lon, None, g["zmin"], g["zmax"])
        assert buf.nx == 0
        keys, counts = buf.keys[:m].clone(), buf.counts[:m].clone()
        del buf
        if wide and r == 3:
            j = int(torch.nonzero((keys >> 58) > DZ)[0])
            counts[j] += 1 << 32
            bump = int(keys[j])
        grid, parts, sizes = ops.route_pieces(keys, counts, WS, DZ, bits, _lib.HM_CELLS_REC10)
        sz = sizes.cpu()
        assert bool(sz[:, 1].all()) == (wide and r == 3) and bool(sz[:, 1].any()) == (wide and r == 3)
        assert int(sz[:, 0].sum()) == int(((keys >> 58) > DZ).sum())
        assert torch.equal(sz[:, 2:2 + S].sum(1), sz[:, 0])
        shards.append([keys, counts, grid.clone(), parts, sz])
    del lat, lon
    layout = _lib.HM_CELLS_REC10
    if wide:
        # every rank learns of the flag from the size exchange and routes again
        layout = _lib.HM_CELLS_U64
        for s in shards:
            grid, parts, sizes = ops.route_pieces(s[0], s[1], WS, DZ, bits, layout)
            assert torch.equal(sizes.cpu(), s[4] * torch.tensor([1, 0] + [1] * (S + 1)))
            s[2], s[3] = grid.clone(), parts
    # RCCL reduce of the dense grids -> rank 0's dense cells
    dense = torch.stack([s[2] for s in shards]).sum(0)
    dk, dc = ops.dense_cells(dense, DZ)
    assert bool(((dk >> 58) <= DZ).all())
    total = device_cells_digest(torch, dk >> 58, (dk >> 29) & M29, dk & M29, dc)
    # all-to-all: owner o gets group o of every shard; the pieces merge reads
    # each shard's group where it lies (no copy)
    offs = [[0] + s[4][:, 0].cumsum(0).tolist() for s in shards]
    seen_bump = 0
    for o in range(WS):
        runs = [(s[3][0][0], s[3][1][0] if len(s[3]) > 1 else None, offs[i][o]) for i, s in enumerate(shards)]
        uk, uc = ops.merge_pieces(runs, [s[4][o, 2:2 + S].tolist() for s in shards], bits, layout)
        z, row, col = uk >> 58, (uk >> 29) & M29, uk & M29
        assert bool((z > DZ).all())
        own = multigpu.record_owner(torch.stack([z, row, col], 1), WS)
        assert bool((own == o).all()), "a merged cell is held by a rank that does not own it"
        if wide and bump is not None:
            hit = uk == bump
            seen_bump += int(hit.sum())
            uc = torch.where(hit, uc - (1 << 32), uc)
        total = _combine(total, device_cells_digest(torch, z, row, col, uc))
        del uk, uc
    if wide:
        assert seen_bump == 1
    assert total == g["digest"]
