#!/usr/bin/env python3
"""Phase timing of one kernel from s_memtime stamps (HM_STAMPS builds).

    python tools/variants.py build stamps stamps1 stamps2    # here
    python tools/stamps.py [stamps|stamps1|stamps2]          # on the GPU box
Prints the mean/median cycles between consecutive stamps over the first
65536 blocks of the kernel's last launch (stamps: k_partition, stamps1:
k_project_partition, stamps2: k_partition_fr).
"""
import ctypes
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
VAR = sys.argv[1] if len(sys.argv) > 1 else "stamps"
os.environ["HM_LIB_PATH"] = os.path.join(REPO, "heatmap_amd", "_lib", "variants", "lib_%s.so" % VAR)
import torch  # noqa: E402

from heatmap_amd import _lib, device  # noqa: E402

NAMES = {
    "stamps": ["start", "init", "item", "classify", "prefix", "bodies", "pieces", "stream_end", "digit_scan",
               "atomics+gather", "claim", "write+runs"],
    "stamps1": ["start", "issue+lds_setup", "project(loads)", "redo+count_rank", "reserve+scan", "stage",
                "dbase", "copy"],
    "stamps2": ["start", "item+loads_issue+init", "count_rank(loads)", "barrier", "scan+run_atomics", "scatter",
                "copy+runs"],
    "stamps4": ["start", "issue+lds_setup", "project(loads)", "redo+count_rank", "reserve+scan", "stage", "copy"],
    "stamps5": ["start", "zero+item", "count(stream_runs)", "squeeze", "pyramid+emit"],
    "stamps6": [],
    "stamps6w8": [],
    "stamps6w10": [],
    "stamps7": [],
    "stamps7noatom": [],
}[VAR]
K = len(NAMES)
n = int(float(os.environ.get("HM_POINTS", "2.5e8" if not VAR.startswith(("stamps6", "stamps7")) else "1e9")))
lat = torch.empty(n, dtype=torch.float64, device="cuda")
lon = torch.empty(n, dtype=torch.float64, device="cuda")
device.synth(os.environ.get("HM_KIND", "skew" if VAR.startswith("stamps7") else "hotspots"), lat, lon)
bufs = device.CountBuffers(64 << 20)
device.count_device(lat, lon, None, 0, int(os.environ.get("HM_ZMAX", "18")), 0, buffers=bufs)
torch.cuda.synchronize()
L = _lib.load()
L.hm_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
st = np.zeros(65536 * 12, np.uint64)
assert L.hm_debug_stamps(st.ctypes.data, st.nbytes) == 0
st = st.reshape(-1, 12).astype(np.int64)
if VAR.startswith("stamps7"):
    # k_small_pairs: per block, wave 0's (it also makes the atomics) and wave 1's phase cycles summed over its rounds
    w, al = st[:4096, :8], st[4096:8192, :8]
    ok = w[:, 6] > 0
    r = w[ok, 6:7].astype(float)
    print("stamps7 blocks %d rounds/block %.2f batches/block %.2f" % (ok.sum(), r.mean(), w[ok, 7].mean()))
    for i, nm in enumerate(["W0 pass 1", "W0 barrier A wait", "W0 atomics", "W0 barrier B wait", "W0 pass 2"]):
        i = [0, 1, 4, 2, 3][i]
        print("%-24s per round mean %8.0f  median %8.0f" % (nm, (w[ok, i] / r[:, 0]).mean(), np.median(w[ok, i] / r[:, 0])))
    for i, nm in [(0, "W1 pass 1"), (1, "W1 barrier A wait"), (2, "W1 barrier B wait"), (3, "W1 pass 2")]:
        print("%-24s per round mean %8.0f  median %8.0f" % (nm, (al[ok, i] / r[:, 0]).mean(), np.median(al[ok, i] / r[:, 0])))
    sys.exit(0)
if VAR.startswith("stamps6"):
    # k_l1_ws: per block, phase cycles summed over its tiles; slot 11 = its tiles;
    # the writer waves' phases in the rows 4096 + block
    w = st[4096:4096 + 4096, :8]
    st = st[:4096]
    ok = st[:, 11] > 0
    nt = st[ok, 11:12]
    per = st[ok, :6] / nt
    perw = w[ok] / nt
    names = ["C wait+project", "C redo+prefetch+count", "C BAR1 wait", "C scan(3 bar)", "C stage", "C BAR3 wait"]
    namesw = ["W deltas (atomics)", "W rendezvous", "W copy-out", "W BAR1 wait", "W reserve issue", "W scan(3 bar)",
              "W zero+BAR3"]
    print("stamps6 blocks", int(ok.sum()), "tiles/block", nt.mean())
    for k, nm in enumerate(names):
        print("%-24s per tile mean %8.0f  median %8.0f" % (nm, per[:, k].mean(), np.median(per[:, k])))
    for k, nm in enumerate(namesw):
        print("%-24s per tile mean %8.0f  median %8.0f" % (nm, perw[:, k].mean(), np.median(perw[:, k])))
    print("C total per tile %.0f, W total per tile %.0f" % (per.sum(1).mean(), perw[:, :7].sum(1).mean()))
    sys.exit(0)
st_all = st.copy()
extra = st[:, K:K + 3].copy()
st = st[:, :K]
ok = (st[:, 0] > 0) & (st[:, K - 1] > 0)
st = st[ok]
extra = extra[ok]
print(VAR, "blocks", len(st))
# missing intermediate stamps (no chunk) -> carry previous
for k in range(1, K):
    z = st[:, k] == 0
    st[z, k] = st[z, k - 1]
d = np.diff(st, axis=1)
for k in range(K - 1):
    print("%-22s mean %8.0f  median %8.0f" % (NAMES[k + 1], d[:, k].mean(), np.median(d[:, k])))
tot = st[:, K - 1] - st[:, 0]
print("%-16s mean %8.0f  median %8.0f cycles" % ("total", tot.mean(), np.median(tot)))
if VAR == "stamps5":
    # k_aggregate: phase cycles by the item's key count (keys, runs, items of its bucket)
    keys, runs, nit = extra[:, 0], extra[:, 1], extra[:, 2]
    print("items: keys mean %.0f median %.0f; runs mean %.0f median %.0f; multi-item %.3f"
          % (keys.mean(), np.median(keys), runs.mean(), np.median(runs), (nit > 1).mean()))
    # inside the count, first run chunk (0 when the item takes the few-runs path):
    # staged descriptors, prefixes, bodies, pieces
    sub = st_all[ok][:, 8:12].astype(np.int64)
    c0 = st[:, 1]
    many = sub[:, 0] > 0
    if many.any():
        s = sub[many]
        seg = np.diff(np.concatenate([c0[many, None], s], axis=1), axis=1)
        for k, nm in enumerate(["descriptors+barrier", "prefix+barrier", "bodies", "pieces"]):
            print("  first chunk %-20s mean %8.0f  median %8.0f  (%d items)" % (nm, seg[:, k].mean(), np.median(seg[:, k]),
                                                                          many.sum()))
    edges = [0, 1024, 4096, 16384, 65536, 1 << 30]
    for lo, hi in zip(edges[:-1], edges[1:]):
        m = (keys >= lo) & (keys < hi)
        if m.sum():
            print("keys [%7d,%10d): %6d items, runs %7.0f, " % (lo, hi, m.sum(), runs[m].mean())
                  + ", ".join("%s %.0f" % (NAMES[k + 1], d[m, k].mean()) for k in range(K - 1)))
