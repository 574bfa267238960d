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
}[VAR]
K = len(NAMES)
n = int(float(os.environ.get("HM_POINTS", "2.5e8")))
lat = torch.empty(n, dtype=torch.float64, device="cuda")
lon = torch.empty(n, dtype=torch.float64, device="cuda")
device.synth("hotspots", lat, lon)
bufs = device.CountBuffers(64 << 20)
device.count_device(lat, lon, None, 0, int(os.environ.get("HM_ZMAX", "18")), 0, buffers=bufs)
torch.cuda.synchronize()
L = _lib.load()
L.hm_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
st = np.zeros(65536 * 12, np.uint64)
assert L.hm_debug_stamps(st.ctypes.data, st.nbytes) == 0
st = st.reshape(-1, 12).astype(np.int64)
st = st[:, :K]
ok = (st[:, 0] > 0) & (st[:, K - 1] > 0)
st = st[ok]
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
