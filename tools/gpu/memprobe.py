import sys, os, torch
sys.path.insert(0, os.getcwd())
from heatmap_amd import device
free, tot = torch.cuda.mem_get_info(); print("start free %.1f / %.1f GB" % (free/1e9, tot/1e9), flush=True)
n = (1 << 32) + (1 << 20)
lat = torch.empty(n, dtype=torch.float64, device="cuda"); lon = torch.empty(n, dtype=torch.float64, device="cuda")
device.synth("hotspots", lat, lon, seed=7)
free, tot = torch.cuda.mem_get_info(); print("after synth free %.1f GB" % (free/1e9), flush=True)
for chunk in (device.MAX_CALL_POINTS, 3 << 29):
    try:
        m, buf = device.count_device(lat, lon, None, 0, 16, chunk=chunk)
        print("chunk", chunk, "cells", m, flush=True)
    except Exception as e:
        print("chunk", chunk, "FAILED", e, flush=True)
    free, tot = torch.cuda.mem_get_info(); print("  free %.1f GB, torch reserved %.1f GB" % (free/1e9, torch.cuda.memory_reserved()/1e9), flush=True)
