"""GPU: the multi-GPU exchange on the device (hm_merge.hip) and the RCCL path.

- hm_cells_route / hm_cells_merge / hm_dense_cells against the CPU stand-ins of
  tests/test_multigpu_gloo.py (the same contract: dense zooms summed into the
  Morton grid, sparse cells grouped by heatmap-row owner, equal keys summed);
- merge_cells over a real RCCL ("nccl") process group of world size 1: the
  reduce and the all-to-alls run on the GPU, and the merged cells equal one
  hm_count over the same points.  (8-GPU runs are the driver's; ranks cannot
  share one GPU under RCCL.)"""
import numpy as np
import pytest
import torch
import torch.distributed as dist

from heatmap_amd import device, multigpu, synth
from test_multigpu_gloo import TorchOps

pytestmark = pytest.mark.gpu


def _cells(n, seed):
    lat, lon = synth.generate("hotspots", n, seed=seed)
    c = device.count(lat, lon, None, 0, 18)
    keys = (c.zoom.astype(np.int64) << 58) | (c.row << 29) | c.col
    return torch.from_numpy(keys), torch.from_numpy(c.count)


@pytest.mark.parametrize("ws,dz,narrow", [(1, 10, False), (5, 8, True), (8, -1, True), (64, 4, False)])
def test_route_kernel_contract(gpu, ws, dz, narrow):
    keys, counts = _cells(300_000, ws)
    ops = multigpu.DeviceOps(0)
    g, parts, sent, wide = ops.route(keys.cuda(), counts.cuda(), ws, dz, narrow=narrow)
    rg, rparts, rsent, rwide = TorchOps.route(keys, counts, ws, dz, narrow=narrow)
    assert sent == rsent and not wide and not rwide
    assert [w for _, w in parts] == ([10] if narrow else [1, 1])
    assert torch.equal(g.cpu(), rg)
    if narrow:   # 10-byte records: the same bytes as the CPU packing, cell by cell
        sk, sc = multigpu.unpack_records(parts[0][0].cpu())
        rk, rc = multigpu.unpack_records(rparts[0][0])
    else:
        sk, sc = parts[0][0].cpu(), parts[1][0].cpu()
        rk, rc = rparts[0][0], rparts[1][0]
    at = 0
    for n in sent:                         # same cells per owner (order inside a group is free)
        a = torch.argsort(sk[at:at + n])
        b = torch.argsort(rk[at:at + n])
        assert torch.equal(sk[at:at + n][a], rk[at:at + n][b])
        assert torch.equal(sc[at:at + n][a], rc[at:at + n][b])
        at += n
    if dz >= 0:
        dk, dc = ops.dense_cells(g, dz)
        ek, ec = TorchOps.dense_cells(rg, dz)
        o, eo = torch.argsort(dk.cpu()), torch.argsort(ek)
        assert torch.equal(dk.cpu()[o], ek[eo]) and torch.equal(dc.cpu()[o], ec[eo])


def test_route_narrow_flags_wide_counts(gpu):
    """narrow routing of a count >= 2^32 (a sparse zoom's cell): HM_E_WIDE
    -> wide, with the group sizes still filled; routing again wide sends it."""
    keys, counts = _cells(100_000, 9)
    counts = counts.clone()
    z = keys >> 58
    i = int(torch.nonzero(z == 15)[0])
    counts[i] = (1 << 33) + 7
    ops = multigpu.DeviceOps(0)
    _, _, sent, wide = ops.route(keys.cuda(), counts.cuda(), 4, 10, narrow=True)
    assert wide and sum(sent) == int((z > 10).sum())
    _, parts, sent2, wide2 = ops.route(keys.cuda(), counts.cuda(), 4, 10, narrow=False)
    sk, sc = parts[0][0].cpu(), parts[1][0].cpu()
    assert not wide2 and sent2 == sent
    assert int(sc[sk == keys[i]].item()) == (1 << 33) + 7


def test_route_narrow_flags_wide_keys(gpu):
    """narrow routing of sparse keys beyond the 10-byte record's 48 bits (a
    zoom-22 cell; a row of 2^21): HM_E_WIDE, as the CPU stand-in flags; routed
    again wide, the keys arrive intact."""
    keys, counts = _cells(50_000, 4)
    for bad in ((22 << 58) | (5 << 29) | 7, (20 << 58) | ((1 << 21) << 29) | 3):
        k2 = torch.cat([keys, torch.tensor([bad], dtype=torch.int64)])
        c2 = torch.cat([counts, torch.tensor([3], dtype=torch.int64)])
        ops = multigpu.DeviceOps(0)
        _, _, sent, wide = ops.route(k2.cuda(), c2.cuda(), 4, 10, narrow=True)
        _, _, rsent, rwide = TorchOps.route(k2, c2, 4, 10, narrow=True)
        assert wide and rwide and sent == rsent
        _, parts, _, wide2 = ops.route(k2.cuda(), c2.cuda(), 4, 10, narrow=False)
        assert not wide2 and int((parts[0][0].cpu() == bad).sum()) == 1


def test_merge_narrow_counts(gpu):
    """hm_cells_merge(_runs) of int32 counts (the exchange's width) sums into
    int64, past 2^32 where many ranks' counts of one cell add up."""
    g = torch.Generator().manual_seed(5)
    base = torch.randint(0, 1 << 62, (400_000,), generator=g, dtype=torch.int64)
    runs = [base, base[::2], base[::3], base[::2]]
    k = torch.cat(runs)
    c = torch.randint(1 << 30, (1 << 31) - 1, (k.numel(),), generator=g, dtype=torch.int64)
    ek, ec = TorchOps.merge(k, c)
    ops = multigpu.DeviceOps(0)
    for r in (None, [x.numel() for x in runs]):
        uk, uc = ops.merge(k.cuda(), c.to(torch.int32).cuda(), r)
        o = torch.argsort(uk.cpu())
        assert torch.equal(uk.cpu()[o], ek) and torch.equal(uc.cpu()[o], ec)
    assert int(ec.max()) >= 1 << 32


@pytest.mark.parametrize("n", [1, 100, 5000, 3_000_000])
def test_merge_records(gpu, n):
    """hm_cells_merge(_runs) of HM_CELLS_REC10 records (48-bit keys of
    zooms 11..21, u32 counts), sums past 2^32."""
    g = torch.Generator().manual_seed(n)
    z = torch.randint(11, 22, (n,), generator=g, dtype=torch.int64)
    r = torch.randint(0, 1 << 21, (n,), generator=g, dtype=torch.int64) & ((1 << z) - 1)
    c = torch.randint(0, 1 << 21, (n,), generator=g, dtype=torch.int64) & ((1 << z) - 1)
    base = (z << 58) | (r << 29) | c
    runs = [base, base[::2], base[::3]]
    k = torch.cat(runs)
    cnt = torch.randint(1, (1 << 32) - 1, (k.numel(),), generator=g, dtype=torch.int64)
    rec = multigpu.pack_records(k, cnt)
    kk, cc = multigpu.unpack_records(rec)
    assert torch.equal(kk, k) and torch.equal(cc, cnt)
    ek, ec = TorchOps.merge(k, cnt)
    ops = multigpu.DeviceOps(0)
    for rl in (None, [x.numel() for x in runs]):
        uk, uc = ops.merge(rec.cuda(), None, rl)
        o = torch.argsort(uk.cpu())
        assert torch.equal(uk.cpu()[o], ek) and torch.equal(uc.cpu()[o], ec)


def test_merge_kernel_sums_duplicates(gpu):
    keys, counts = _cells(200_000, 3)
    k = torch.cat([keys, keys[::3], keys[::7]])
    c = torch.cat([counts, counts[::3] * 2, counts[::7] + 5])
    p = torch.randperm(k.numel(), generator=torch.Generator().manual_seed(1))
    uk, uc = multigpu.DeviceOps(0).merge(k[p].cuda(), c[p].cuda())
    ek, ec = TorchOps.merge(k, c)
    o = torch.argsort(uk.cpu())
    assert torch.equal(uk.cpu()[o], ek) and torch.equal(uc.cpu()[o], ec)


@pytest.mark.parametrize("n", [1, 100, 1801, 300_000, 6_000_000])
def test_merge_partition_passes(gpu, n):
    """hm_cells_merge at sizes that take zero, one and two hash-partition
    passes (2^lb buckets of <= ~1800 cells), keys repeated up to 3 times."""
    g = torch.Generator().manual_seed(n)
    base = torch.randint(0, 1 << 62, (n,), generator=g, dtype=torch.int64)
    k = torch.cat([base, base[::2], base[::5]])
    c = torch.randint(1, 1 << 31, (k.numel(),), generator=g, dtype=torch.int64)
    p = torch.randperm(k.numel(), generator=g)
    uk, uc = multigpu.DeviceOps(0).merge(k[p].cuda(), c[p].cuda())
    ek, ec = TorchOps.merge(k, c)
    o = torch.argsort(uk.cpu())
    assert torch.equal(uk.cpu()[o], ek) and torch.equal(uc.cpu()[o], ec)


def test_merge_runs_of_distinct_keys(gpu):
    """hm_cells_merge_runs: three runs (one per sending rank), each of distinct
    keys, overlapping across runs; an empty run in between."""
    keys, counts = _cells(200_000, 4)
    runs = [keys, keys[::3], keys[1::7]]
    vals = [counts, counts[::3] * 2, counts[1::7] + 5]
    perm = [torch.randperm(r.numel(), generator=torch.Generator().manual_seed(i)) for i, r in enumerate(runs)]
    k = torch.cat([r[q] for r, q in zip(runs, perm)] + [keys[:0]])
    c = torch.cat([v[q] for v, q in zip(vals, perm)] + [counts[:0]])
    sizes = [r.numel() for r in runs[:2]] + [0] + [runs[2].numel()]
    uk, uc = multigpu.DeviceOps(0).merge(k.cuda(), c.cuda(), sizes)
    ek, ec = TorchOps.merge(k, c)
    o = torch.argsort(uk.cpu())
    assert torch.equal(uk.cpu()[o], ek) and torch.equal(uc.cpu()[o], ec)


@pytest.fixture(scope="module")
def nccl_world():
    store = dist.HashStore()
    dist.init_process_group("nccl", store=store, rank=0, world_size=1)
    yield
    dist.destroy_process_group()


@pytest.mark.parametrize("dz", [-1, 8, 10])
def test_merge_cells_over_rccl(gpu, nccl_world, dz):
    n = 2_000_000
    lat, lon = synth.generate("hotspots", n, seed=dz + 2)
    lat, lon = lat.copy(), lon.copy()
    lat[::9973] = 88.5                      # cells outside the square travel as records
    ref = device.count(lat, lon, None, 0, 18).sorted()
    m, bufs = device.count_device(torch.from_numpy(lat).cuda(), torch.from_numpy(lon).cuda(), None, 0, 18)
    m = multigpu.merge_cells(bufs, m, 1, 0, dense_zmax=dz)
    k = bufs.keys[:m].cpu().numpy().view(np.uint64)
    z = (k >> np.uint64(58)).astype(np.int32)
    r = ((k >> np.uint64(29)) & np.uint64(0x1FFFFFFF)).astype(np.int64)
    c = (k & np.uint64(0x1FFFFFFF)).astype(np.int64)
    x = bufs.xcells[:4 * bufs.nx].cpu().numpy().reshape(-1, 4)
    got = device.Counts(np.concatenate([z, x[:, 0].astype(np.int32)]), np.concatenate([r, x[:, 1]]),
                        np.concatenate([c, x[:, 2]]), np.concatenate([bufs.counts[:m].cpu().numpy(), x[:, 3]]),
                        0, []).sorted()
    for f in ("zoom", "row", "col", "count"):
        assert np.array_equal(getattr(got, f), getattr(ref, f)), f


def test_pipelined_steps_over_rccl(gpu, nccl_world):
    """bench.py's N>1 schedule: step k's merge (helper thread, own stream)
    overlaps step k+1's count; after 5 steps over 2 buffer sets the last
    merged cells equal one count of the cloud."""
    n = 3_000_000
    lat, lon = synth.generate("hotspots", n, seed=17)
    la, lo = torch.from_numpy(lat).cuda(), torch.from_numpy(lon).cuda()
    ref = device.count(lat, lon, None, 0, 18).sorted()
    ctx = device.context(0)
    bufsets = [device.CountBuffers(1 << 24), device.CountBuffers(1 << 24)]
    m, stages, bufs = multigpu.pipelined_steps(lambda b: device.count_device(la, lo, None, 0, 18, buffers=b),
                                               bufsets, 5, 1, 0, ctx)
    torch.cuda.synchronize()
    assert len(stages) == 5 and bufs.nx == 0
    k = bufs.keys[:m].cpu().numpy().view(np.uint64)
    got = device.Counts((k >> np.uint64(58)).astype(np.int32), ((k >> np.uint64(29)) & np.uint64(0x1FFFFFFF)).astype(np.int64),
                        (k & np.uint64(0x1FFFFFFF)).astype(np.int64), bufs.counts[:m].cpu().numpy(), 0, []).sorted()
    for f in ("zoom", "row", "col", "count"):
        assert np.array_equal(getattr(got, f), getattr(ref, f)), f


def _grouped(n, seed, users):
    lat, lon = synth.generate("hotspots", n, seed=seed)
    grp = (((np.arange(n) * 2654435761) >> 7) % users).astype(np.uint32)
    return lat, lon, grp


@pytest.mark.parametrize("ws,users", [(1, 1000), (5, 1000), (8, 30), (8, 200_000)])
def test_route_grouped_kernel_contract(gpu, ws, users):
    """hm_cells_route of grouped cells (HM_CELLS_G12) == the CPU stand-in:
    the same owner group sizes and, per owner, the same (merge key, count)
    multiset; group ids past 2^17 answer wide."""
    lat, lon, grp = _grouped(300_000, ws, users)
    keys, gc = device.count_grouped_packed_device(lat, lon, grp, None, 6, 21)
    parts, sent, wide = multigpu.DeviceOps(0).route_grouped(keys, gc, ws)
    rparts, rsent, rwide = TorchOps.route_grouped(keys.cpu(), gc.cpu(), ws)
    assert wide == rwide == (users > (1 << 17))
    assert sent == rsent
    if wide:
        return
    sk, sc = parts[0][0].cpu(), parts[1][0].cpu().to(torch.int64)
    rk, rc = rparts[0][0], rparts[1][0].to(torch.int64)
    at = 0
    for m in sent:
        a, b = torch.argsort(sk[at:at + m]), torch.argsort(rk[at:at + m])
        assert torch.equal(sk[at:at + m][a], rk[at:at + m][b]) and torch.equal(sc[at:at + m][a], rc[at:at + m][b])
        at += m


@pytest.mark.parametrize("users", [1000, 200_000])
def test_merge_grouped_over_rccl(gpu, nccl_world, users):
    """merge_grouped over a real RCCL group of world size 1: the device route,
    the all-to-alls and hm_cells_merge_runs (or, past 2^17 groups, the int64
    records) give back exactly the grouped count."""
    lat, lon, grp = _grouped(500_000, 3, users)
    keys, gc = device.count_grouped_packed_device(lat, lon, grp, None, 6, 21)
    k, g, c = multigpu.merge_grouped(keys, gc, 1, 0)
    got = np.lexsort((k.cpu().numpy(), g.cpu().numpy()))
    ref = np.lexsort((keys.cpu().numpy(), (gc >> 32).cpu().numpy()))
    assert np.array_equal(k.cpu().numpy()[got], keys.cpu().numpy()[ref])
    assert np.array_equal(g.cpu().numpy()[got], (gc >> 32).cpu().numpy()[ref])
    assert np.array_equal(c.cpu().numpy()[got], (gc & 0xFFFFFFFF).cpu().numpy()[ref])


@pytest.mark.parametrize("users", [5000, 100_000])
def test_grouped_exchange_8_emulated_ranks(gpu, users):
    """The grouped pyramid sharded over 8 emulated ranks on one GPU: each
    shard's hm_count_grouped_packed, routed by hm_cells_route(G12, nranks=8);
    owner o merges group o of every shard (hm_cells_merge_runs).  Every
    (group, cell) has one owner and the union equals one grouped count of all
    points (heatmap.py:54-55,111-112).  100,000 users: group ids in [2^16,
    2^17), the merge key's top bit set, still on the packed route."""
    ws, n = 8, 2_000_000
    lat, lon, grp = _grouped(n, 9, users)
    ops = multigpu.DeviceOps(0)
    per = n // ws
    routed = []
    for r in range(ws):
        sl = slice(r * per, (r + 1) * per)
        k, gc = device.count_grouped_packed_device(lat[sl], lon[sl], grp[sl], None, 6, 21)
        parts, sent, wide = ops.route_grouped(k, gc, ws)
        assert not wide
        routed.append((parts[0][0].clone(), parts[1][0].clone(), [0] + np.cumsum(sent).tolist(), sent))
    allk, allg, allc = [], [], []
    for o in range(ws):
        mk = torch.cat([x[0][x[2][o]:x[2][o + 1]] for x in routed])
        mc = torch.cat([x[1][x[2][o]:x[2][o + 1]] for x in routed])
        uk, uc = ops.merge(mk, mc, [x[3][o] for x in routed])
        g = (uk >> 47) & 0x1FFFF
        hk = (((uk >> 42) & 31) << 58) | (((uk >> 21) & 0x1FFFFF) << 29) | (uk & 0x1FFFFF)
        assert bool((multigpu.grouped_owner(hk, g, ws) == o).all())
        allk.append(hk.cpu().numpy())
        allg.append(g.cpu().numpy())
        allc.append(uc.cpu().numpy())
    ks, gs, cs = np.concatenate(allk), np.concatenate(allg), np.concatenate(allc)
    keys, gc = device.count_grouped_packed_device(lat, lon, grp, None, 6, 21)
    rk, rg, rc = keys.cpu().numpy(), (gc >> 32).cpu().numpy(), (gc & 0xFFFFFFFF).cpu().numpy()
    a, b = np.lexsort((ks, gs)), np.lexsort((rk, rg))
    assert np.array_equal(ks[a], rk[b]) and np.array_equal(gs[a], rg[b]) and np.array_equal(cs[a], rc[b])


# ---- the pieces exchange (hm_cells_route_pieces / hm_cells_merge_pieces) ----
from heatmap_amd import _lib  # noqa: E402


def _piece_cells(parts, layout, lo, hi):
    """(keys, counts) int64 of cells lo..hi of route parts (CPU)."""
    if layout == _lib.HM_CELLS_REC10:
        return multigpu.unpack_records(parts[0][0][lo * 10:hi * 10].cpu())
    return parts[0][0][lo:hi].cpu(), parts[1][0][lo:hi].cpu().to(torch.int64)


@pytest.mark.parametrize("ws,dz,layout,n,me", [(1, 10, 10, 300_000, -1), (5, 8, 10, 300_000, 2),
                                               (8, -1, 10, 300_000, -1), (8, 10, 8, 300_000, 0),
                                               (64, 4, 8, 300_000, 63), (8, -1, 12, 200_000, 5),
                                               (3, 8, 10, 7, 1), (2, 10, 10, 0, -1)])
def test_route_pieces_contract(gpu, ws, dz, layout, n, me):
    """hm_cells_route_pieces == its CPU stand-in: the same size rows (owner
    totals, wide flag and the 2^bits digit pieces -- the device's fmix64 and
    the stand-in's agree) and, piece by piece, the same cells."""
    bits = multigpu.route_bits(ws)
    if layout == _lib.HM_CELLS_G12:
        lat, lon, grp = _grouped(n, ws, 3000)
        keys, counts = device.count_grouped_packed_device(lat, lon, grp, None, 6, 21)
        keys, counts = keys.cpu(), counts.cpu()
    elif n:
        keys, counts = _cells(n, ws)
        keys, counts = keys[: n], counts[: n]
    else:
        keys = counts = torch.zeros(0, dtype=torch.int64)
    ops = multigpu.DeviceOps(0)
    g, parts, sizes = ops.route_pieces(keys.cuda(), counts.cuda(), ws, dz, bits, layout, self_rank=me)
    rg, rparts, rsizes = TorchOps.route_pieces(keys, counts, ws, dz, bits, layout, self_rank=me)
    sizes = sizes.cpu()
    assert torch.equal(sizes, rsizes)
    assert not bool(sizes[:, 1].any())
    if dz >= 0:
        assert torch.equal(g.cpu(), rg)
    S = 1 << bits
    order = [o for o in range(ws) if o != me] + ([me] if me >= 0 else [])   # the groups' order in the output
    flat = sizes[order, 2:2 + S].reshape(-1).tolist()
    at = 0
    for m in flat:                        # the same cells per (owner, digit) piece
        sk, sc = _piece_cells(parts, layout, at, at + m)
        rk, rc = _piece_cells(rparts, layout, at, at + m)
        a, b = torch.argsort(sk), torch.argsort(rk)
        assert torch.equal(sk[a], rk[b]) and torch.equal(sc[a], rc[b])
        at += m
    assert at == int(sizes[:, 0].sum())


@pytest.mark.parametrize("layout,n,R", [(10, 1, 1), (10, 100, 3), (10, 5000, 8), (10, 3_000_000, 8),
                                        (8, 300_000, 5), (12, 400_000, 8), (10, 6_000_000, 1)])
def test_merge_pieces(gpu, layout, n, R):
    """hm_cells_merge_pieces of R senders' cells as the exchange leaves them:
    each sender's hm_cells_route_pieces output (2 owners) in its own tensor,
    owner 1's group starting mid-tensor; equal keys summed (past 2^32 from
    u32 inputs), every key once, and only owner 1's cells."""
    gen = torch.Generator().manual_seed(n + R)
    z = torch.randint(11, 22, (n,), generator=gen, dtype=torch.int64)
    r = torch.randint(0, 1 << 21, (n,), generator=gen, dtype=torch.int64) & ((1 << z) - 1)
    c = torch.randint(0, 1 << 21, (n,), generator=gen, dtype=torch.int64) & ((1 << z) - 1)
    keys = torch.unique((z << 58) | (r << 29) | c)
    bits = multigpu.route_bits(2)
    S = 1 << bits
    ops = multigpu.DeviceOps(0)
    runs, pieces, ak, ac = [], [], [], []
    for s in range(R):
        k = keys[torch.randperm(keys.numel(), generator=gen)[: max(1, keys.numel() * (s + 2) // (R + 2))]]
        if layout == _lib.HM_CELLS_U64:
            cnt = torch.randint(1, 1 << 40, (k.numel(),), generator=gen, dtype=torch.int64)
        else:
            cnt = torch.randint(1 << 31, (1 << 32) - 1, (k.numel(),), generator=gen, dtype=torch.int64)
        if layout == _lib.HM_CELLS_G12:
            grp = (k & 7) * 1000
            own = multigpu.grouped_owner(k, grp, 2)
            mk = (grp << 47) | ((k >> 58) << 42) | (((k >> 29) & 0x1FFFFF) << 21) | (k & 0x1FFFFF)
            cin = (grp << 32) | cnt
        else:
            own = multigpu.record_owner(torch.stack([k >> 58, (k >> 29) & 0x1FFFFFFF, k & 0x1FFFFFFF], 1), 2)
            mk, cin = k, cnt
        _, parts, sizes = ops.route_pieces(k.cuda(), cin.cuda(), 2, -1, bits, layout)
        sz = sizes.cpu()
        runs.append((parts[0][0], parts[1][0] if len(parts) > 1 else None, int(sz[0, 0])))
        pieces.append(sz[1, 2:2 + S].tolist())
        ak.append(mk[own == 1])
        ac.append(cnt[own == 1])
    uk, uc = ops.merge_pieces(runs, pieces, bits, layout)
    ek, ec = TorchOps.merge(torch.cat(ak), torch.cat(ac))
    o = torch.argsort(uk.cpu())
    assert torch.equal(uk.cpu()[o], ek) and torch.equal(uc.cpu()[o], ec)
    if layout != _lib.HM_CELLS_U64 and R > 2:
        assert int(ec.max()) >= 1 << 32


@pytest.mark.parametrize("env", [{"HM_GATHER_BCAP": "64"}, {"HM_GATHER_FILL": "0"}])
def test_merge_pieces_counted_forms(gpu, env, monkeypatch):
    """hm_cells_merge_pieces' other partitions: buckets of a fixed capacity
    overflowing (HM_GATHER_BCAP, a test hook) fall back to the counted
    partition; HM_GATHER_FILL=0 always counts.  Same cells either way."""
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    test_merge_pieces(gpu, 10, 300_000, 4)
