"""Streaming micro-batches into a resident heatmap (hm_stream_*, BASELINE config 5)
vs the oracle: after any sequence of add() calls, the alltime rollup equals one
oracle count over every kept point so far, each hour equals the oracle count
over that hour's kept points, and rows() equals the oracle's literal
restatement of build_heatmaps (oracle.build_heatmap_rows, pinned to the
reference's row goldens by tests/test_oracle.py) over every point so far --
for 'alltime' and, restricted to each period with the period's
build_timespan_label (heatmap.py:38-52), for 'year', 'month' and 'day' (those
labels are dead code in the reference, heatmap.py:62-63: parity for them is
pinned only through the alltime rows and the label function)."""
import datetime
import json

import numpy as np
import pytest

from oracle import oracle
from heatmap_amd import _lib, heatmap, synth
from heatmap_amd.device import Counts
from heatmap_amd.stream import ALLTIME, NOGROUP, StreamingHeatmap

pytestmark = pytest.mark.gpu
BASE = 480000  # epoch hour (2024-10-04)


def _same(got, ref):
    got = got.sorted()
    assert ref["status"] == 0
    assert np.array_equal(got.zoom, ref["zoom"])
    assert np.array_equal(got.row, ref["row"])
    assert np.array_equal(got.col, ref["col"])
    assert np.array_equal(got.count, ref["count"])


def _batches(kind, nb, n, seed):
    out = []
    for b in range(nb):
        lat, lon = synth.generate(kind, n, seed=seed, start=b * n)
        rng = np.random.default_rng(seed * 100 + b)
        hour = (BASE + 3 * b + rng.integers(0, 3, n)).astype(np.uint32)  # batches overlap hours
        keep = (rng.random(n) > 0.1).astype(np.uint8)
        out.append((lat, lon, keep, hour))
    return out


@pytest.mark.parametrize("kind,zmin,zmax,initial", [("hotspots", 0, 18, 1 << 10), ("uniform", 3, 14, 1 << 22),
                                                    ("skew", 0, 21, 5000)])
def test_stream_matches_oracle(gpu, kind, zmin, zmax, initial):
    bs = _batches(kind, 4, 40000, seed=7)
    s = StreamingHeatmap(zmin, zmax, base_hour=BASE, initial_cells=initial)
    for lat, lon, keep, hour in bs:
        s.add(lat, lon, keep, hour)
    lat = np.concatenate([b[0] for b in bs])
    lon = np.concatenate([b[1] for b in bs])
    keep = np.concatenate([b[2] for b in bs])
    hour = np.concatenate([b[3] for b in bs])
    _same(s.counts(ALLTIME), oracle.count(lat, lon, keep, zmin, zmax))
    hourly = s.hourly()
    assert sorted(hourly) == sorted(np.unique(hour[keep == 1]).tolist())
    for h, c in hourly.items():
        _same(c, oracle.count(lat, lon, keep & (hour == h).astype(np.uint8), zmin, zmax))
    h0 = int(np.unique(hour)[0])
    _same(s.counts(h0), oracle.count(lat, lon, keep & (hour == h0).astype(np.uint8), zmin, zmax))
    cells, cap = s.cells()
    assert cells == sum(len(c.count) for c in hourly.values())   # one bucket per hour; labels are rollups
    assert cells <= cap
    s.close()


@pytest.mark.parametrize("vmm", ["1", "0"])
def test_stream_log_growth(gpu, monkeypatch, vmm):
    """The cell log grown from 1024 cells over one-hour batches, as virtual
    address reservations mapped in place (and ahead, on a host thread) or, with
    HM_STREAM_VMM=0, as plain allocations copied into twice the size: the same
    cells as the oracle either way, and a late batch of an older hour (the
    compaction target allocated and grown with the log) after that."""
    monkeypatch.setenv("HM_STREAM_VMM", vmm)
    n, nb = 30000, 8
    s = StreamingHeatmap(0, 18, base_hour=BASE, initial_cells=1024)
    lats, lons, hours = [], [], []
    for b in range(nb + 1):
        lat, lon = synth.generate("hotspots", n, seed=5, start=b * n)
        hour = np.full(n, BASE + (b if b < nb else 2), np.uint32)   # the last batch: hour 2 again
        s.add(lat, lon, None, hour)
        lats.append(lat)
        lons.append(lon)
        hours.append(hour)
        cells, cap = s.cells()
        assert cells <= cap
    lat, lon, hour = np.concatenate(lats), np.concatenate(lons), np.concatenate(hours)
    _same(s.counts(ALLTIME), oracle.count(lat, lon, None, 0, 18))
    for h in (BASE, BASE + 2, BASE + nb - 1):
        _same(s.counts(h), oracle.count(lat, lon, (hour == h).astype(np.uint8), 0, 18))
    s.close()


def test_stream_alltime_only_and_errors(gpu):
    lat, lon = synth.generate("hotspots", 30000, seed=2)
    s = StreamingHeatmap(0, 16, base_hour=BASE)
    s.add(lat[:10000], lon[:10000])
    s.add(lat[10000:], lon[10000:])
    _same(s.counts(), oracle.count(lat, lon, None, 0, 16))
    bad = lat[:100].copy()
    bad[37] = np.nan
    with pytest.raises(ValueError):
        s.add(bad, lon[:100])
    with pytest.raises(Exception):  # hour before the stream's base hour
        s.add(lat[:10], lon[:10], hour=np.full(10, BASE - 1, np.uint32))
    # a failed add leaves the resident heatmap unchanged
    _same(s.counts(), oracle.count(lat, lon, None, 0, 16))
    s.close()


def test_stream_empty_and_unkept(gpu):
    s = StreamingHeatmap(0, 12, base_hour=BASE)
    s.add(np.zeros(0), np.zeros(0))
    lat, lon = synth.generate("uniform", 1000, seed=4)
    s.add(lat, lon, keep=np.zeros(1000, np.uint8), hour=np.full(1000, BASE, np.uint32))
    assert s.counts().count.size == 0
    assert s.cells()[0] == 0
    s.close()


def test_stream_single_hour_batches(gpu):
    """Time-ordered batches, one hour each (the fast path that folds `keep` directly)."""
    lat, lon = synth.generate("hotspots", 60000, seed=9)
    rng = np.random.default_rng(9)
    keep = (rng.random(60000) > 0.2).astype(np.uint8)
    hour = (BASE + np.arange(60000) // 20000).astype(np.uint32)  # 3 batches, 1 hour each
    s = StreamingHeatmap(2, 17, base_hour=BASE, initial_cells=2000)
    for b in range(3):
        sl = slice(b * 20000, (b + 1) * 20000)
        s.add(lat[sl], lon[sl], keep[sl], hour[sl])
    s.add(lat[:5000], lon[:5000], keep[:5000], hour[:5000])  # a late batch for an older hour
    lat2, lon2 = np.concatenate([lat, lat[:5000]]), np.concatenate([lon, lon[:5000]])
    keep2, hour2 = np.concatenate([keep, keep[:5000]]), np.concatenate([hour, hour[:5000]])
    _same(s.counts(ALLTIME), oracle.count(lat2, lon2, keep2, 2, 17))
    for h, c in s.hourly().items():
        _same(c, oracle.count(lat2, lon2, keep2 & (hour2 == h).astype(np.uint8), 2, 17))
    s.close()


def _reference_rows(lat, lon, keep, users, mz, d, label="alltime"):
    src = np.where(keep.astype(bool), "mobile", "background")
    rows = oracle.build_heatmap_rows(lat, lon, src, users, mz, d)
    return {k.replace("|alltime|", "|%s|" % label, 1): v for k, v in rows.items()}


USERS = ["all", "u1", "u2", "xhidden", "rt-7", "rt-9", "u3"]


def test_stream_rows_match_reference(gpu):
    """rows() over several multi-hour, multi-user batches == build_heatmaps over
    the concatenated points (alltime), and per period for year/month/day.  The
    hours cross a day, month and year boundary (2024-12-31 21:00 .. 2025-01-01
    03:00 UTC); batches repeat hours and users, so buckets are shared."""
    mz, d = 9, 5
    h0 = int(datetime.datetime(2024, 12, 31, 21, tzinfo=datetime.timezone.utc).timestamp()) // 3600
    rng = np.random.default_rng(5)
    bs = []
    for b in range(4):
        n = 1500
        lat, lon = synth.generate("hotspots", n, seed=21, start=b * n)
        keep = (rng.random(n) > 0.15).astype(np.uint8)
        hour = (h0 + rng.integers(0, 7, n)).astype(np.uint32)
        users = [USERS[i] for i in rng.integers(0, len(USERS), n)]
        bs.append((lat, lon, keep, hour, users))
    s = StreamingHeatmap(0, mz + d, base_hour=h0 - 100)
    for lat, lon, keep, hour, users in bs:
        s.add(lat, lon, keep, hour, user_id=users)
    lat = np.concatenate([b[0] for b in bs])
    lon = np.concatenate([b[1] for b in bs])
    keep = np.concatenate([b[2] for b in bs])
    hour = np.concatenate([b[3] for b in bs])
    users = sum((b[4] for b in bs), [])
    assert s.rows("alltime") == _reference_rows(lat, lon, keep, users, mz, d)
    # the device row table (ids + heatmap JSON) carries the same rows
    t = s.table("alltime")
    got = {i: json.loads(h) for i, h in zip(t.column("id").to_pylist(), t.column("heatmap").to_pylist())}
    assert got == _reference_rows(lat, lon, keep, users, mz, d)
    day = hour // 24
    dates = [datetime.date(1970, 1, 1) + datetime.timedelta(days=int(x)) for x in day]
    for span in ("day", "month", "year"):
        key = np.array([heatmap.build_timespan_label(span, x) for x in dates])
        want = {}
        for lab in np.unique(key).tolist():
            m = key == lab
            want.update(_reference_rows(lat[m], lon[m], keep[m], [u for u, t in zip(users, m) if t], mz, d, lab))
        got = s.rows(span)
        assert got == want, span
        assert len({k.split("|")[1] for k in got}) == 2   # the hours span two days, months and years
    # group rollups: every group's alltime cells == the oracle count of its points
    g, p, z, r, c, cnt = s.rollup("alltime", merge_groups=False)
    for lab in ("u1", "route"):
        gid = s.labels.index(lab)
        pts = np.array([(u == lab or (lab == "route" and u.startswith("rt-"))) for u in users]) & (keep == 1)
        ref = oracle.count(lat, lon, pts.astype(np.uint8), 0, mz + d)
        m = g == gid
        _same(Counts(z[m], r[m], c[m], cnt[m], 0, []), ref)
    # x* users have no group of their own but are in every 'all' count
    assert (g == NOGROUP).any()
    s.close()


def test_stream_batch_is_atomic(gpu):
    """A batch whose SECOND hour holds a failing point (NaN latitude) raises
    and changes no counts (one count pass, checked before insertion), also
    when the batch holds points outside the square (the split path)."""
    lat, lon = synth.generate("hotspots", 4000, seed=3)
    hour = np.full(4000, BASE, np.uint32)
    hour[2000:] += 1
    s = StreamingHeatmap(0, 16, base_hour=BASE)
    s.add(lat, lon, None, hour, user_id=["u%d" % (i % 5) for i in range(4000)])
    before = s.counts().sorted()
    lat2 = lat.copy()
    lat2[3000] = np.nan
    with pytest.raises(ValueError):
        s.add(lat2, lon, None, hour, user_id=["u%d" % (i % 5) for i in range(4000)])
    with pytest.raises(ValueError):   # one hour: the hm_count path
        s.add(lat2, lon, None, np.full(4000, BASE + 5, np.uint32))
    lon2 = lon.copy()
    lon2[100] = 200.0                 # outside the square, with the NaN: the split path must not insert
    with pytest.raises(ValueError):
        s.add(lat2, lon2, None, hour)
    after = s.counts().sorted()
    for k in ("zoom", "row", "col", "count"):
        assert np.array_equal(getattr(before, k), getattr(after, k))
    assert sorted(s.hourly()) == [BASE, BASE + 1]
    s.close()


@pytest.mark.parametrize("nusers,nhours", [(1, 2), (3, 5), (150, 1)])
def test_stream_paths_per_bucket_count(gpu, nusers, nhours):
    """One bucket (hm_count), a few (gathered runs, one hm_count each) and more
    than HMS_MAX_PARTS (the grouped general path) give the same counts: every
    group's alltime cells and every hour's cells == the oracle's."""
    n = 30000
    lat, lon = synth.generate("skew", n, seed=nusers + nhours)
    rng = np.random.default_rng(nusers)
    keep = (rng.random(n) > 0.05).astype(np.uint8)
    hour = (BASE + rng.integers(0, nhours, n)).astype(np.uint32)
    gid = rng.integers(0, nusers, n).astype(np.uint32)
    s = StreamingHeatmap(0, 17, base_hour=BASE)
    s.add(lat, lon, keep, hour, group=gid)
    s.add(lat[:5000], lon[:5000], keep[:5000], hour[:5000], group=gid[:5000])
    lat2, lon2 = np.concatenate([lat, lat[:5000]]), np.concatenate([lon, lon[:5000]])
    keep2, hour2, gid2 = (np.concatenate([x, x[:5000]]) for x in (keep, hour, gid))
    _same(s.counts(), oracle.count(lat2, lon2, keep2, 0, 17))
    for h, c in s.hourly().items():
        _same(c, oracle.count(lat2, lon2, keep2 & (hour2 == h).astype(np.uint8), 0, 17))
    g, p, z, r, c, cnt = s.rollup("alltime", merge_groups=False)
    for u in sorted(set(range(nusers)) & {0, 1, nusers - 1}):
        m = g == u
        _same(Counts(z[m], r[m], c[m], cnt[m], 0, []),
              oracle.count(lat2, lon2, keep2 & (gid2 == u).astype(np.uint8), 0, 17))
    bad = lat.copy()
    bad[n - 7] = np.nan                      # error in the last bucket's run: reported at its input index
    with pytest.raises(ValueError):
        s.add(bad, lon, keep, hour, group=gid)
    _same(s.counts(), oracle.count(lat2, lon2, keep2, 0, 17))
    s.close()


def test_stream_exotic_points(gpu):
    """Kept points outside [0, 2^zmax)^2 (|lat| in (85.06, 89.9), lon at or
    beyond +-180) are binned like the reference's (tile.py:17,21 never clamp):
    counts, hours and rows over several batches equal the oracle's over the
    concatenated points, with users and undated batches mixed in."""
    mz, d = 9, 5
    rng = np.random.default_rng(9)
    bs = []
    for b in range(4):
        n = 3000
        lat, lon = synth.generate("hotspots", n, seed=31, start=b * n)
        lat, lon = lat.copy(), lon.copy()
        m = rng.random(n) < 0.03
        k = int(m.sum())
        lat[m] = rng.choice([-1.0, 1.0], k) * rng.uniform(85.06, 89.9, k)
        lon[m] = rng.choice([180.0, 200.0, -200.0, 540.0, -180.0, 179.99999999999997], k)
        keep = (rng.random(n) > 0.1).astype(np.uint8)
        hour = (BASE + rng.integers(0, 3, n)).astype(np.uint32)
        users = [USERS[i] for i in rng.integers(0, len(USERS), n)]
        bs.append((lat, lon, keep, hour, users))
    s = StreamingHeatmap(0, mz + d, base_hour=BASE - 10)
    for b, (lat, lon, keep, hour, users) in enumerate(bs):
        s.add(lat, lon, keep, hour if b != 2 else None, user_id=users)
    lat = np.concatenate([b[0] for b in bs])
    lon = np.concatenate([b[1] for b in bs])
    keep = np.concatenate([b[2] for b in bs])
    users = sum((b[4] for b in bs), [])
    c = s.counts(ALLTIME)
    assert (c.row < 0).any() and (c.col >= (1 << c.zoom)).any()
    _same(c, oracle.count(lat, lon, keep, 0, mz + d))
    for h in range(BASE, BASE + 3):
        sel = np.concatenate([(b[3] == h) & (b[2] == 1) if i != 2 else np.zeros(len(b[0]), bool)
                              for i, b in enumerate(bs)])
        _same(s.counts(h), oracle.count(lat, lon, sel.astype(np.uint8), 0, mz + d))
    assert s.rows("alltime") == _reference_rows(lat, lon, keep, users, mz, d)
    s.close()


@pytest.mark.parametrize("knobs", [dict(HM_HOT_MIN_KEYS=0, HM_HOT_INV_SHARE=64),
                                   dict(HM_HOT=0, HM_SPREAD_MIN_KEYS=0, HM_SAMPLE_LOG2=10)])
def test_stream_forced_plan_on_concurrent_buckets(gpu, knobs):
    """A 2-3-bucket batch is counted concurrently on helper contexts
    (stream_fold_parts_par); plan knobs set on the stream's context
    (device.tuned) reach them, and the forced plans still give the oracle's
    counts for every hour."""
    from heatmap_amd import device

    n = 200_000
    lat, lon = synth.generate("skew", n, seed=11)
    rng = np.random.default_rng(11)
    keep = (rng.random(n) > 0.05).astype(np.uint8)
    with device.tuned(**knobs):
        s = StreamingHeatmap(0, 18, base_hour=BASE)
        for nh in (2, 3):
            hour = (BASE + 4 * nh + rng.integers(0, nh, n)).astype(np.uint32)
            s.add(lat, lon, keep, hour)
            for h in range(BASE + 4 * nh, BASE + 5 * nh):
                _same(s.counts(h), oracle.count(lat, lon, keep & (hour == h).astype(np.uint8), 0, 18))
        s.close()


def test_stream_device_views_ragged(gpu):
    """A ragged batch (n = 4k + 3 points) passed as host arrays and as device
    views one element in (no array 16-B aligned) gives the oracle's counts,
    hours and groups.  (A k_stream_buckets with 16-B loads and this fallback
    measured no faster: profiles/r6/stream_bucket_vec_ab.txt.)"""
    import torch

    n = 40003
    lat, lon = synth.generate("skew", n + 1, seed=11)
    rng = np.random.default_rng(11)
    keep = (rng.random(n + 1) > 0.1).astype(np.uint8)
    hour = (BASE + rng.integers(0, 3, n + 1)).astype(np.uint32)
    gid = rng.integers(0, 5, n + 1).astype(np.uint32)
    for off in (0, 1):
        s = StreamingHeatmap(0, 16, base_hour=BASE)
        sl = slice(off, off + n)
        if off:
            dev = lambda x, dt: torch.from_numpy(np.ascontiguousarray(x)).to("cuda")[sl]   # noqa: E731
            s.add(dev(lat, None), dev(lon, None), dev(keep, None), dev(hour.view(np.int32), None),
                  group=dev(gid.view(np.int32), None))
        else:
            s.add(lat[sl], lon[sl], keep[sl], hour[sl], group=gid[sl])
        k, h, g = keep[sl], hour[sl], gid[sl]
        _same(s.counts(), oracle.count(lat[sl], lon[sl], k, 0, 16))
        for hh, c in s.hourly().items():
            _same(c, oracle.count(lat[sl], lon[sl], k & (h == hh).astype(np.uint8), 0, 16))
        gg, _, z, r, c, cnt = s.rollup("alltime", merge_groups=False)
        m = gg == 3
        _same(Counts(z[m], r[m], c[m], cnt[m], 0, []), oracle.count(lat[sl], lon[sl], k & (g == 3).astype(np.uint8), 0, 16))
        s.close()
