#!/usr/bin/env python3
"""Per-launch and per-step HBM bytes from rocprofv3 FETCH_SIZE / WRITE_SIZE
passes, written into profiles/pmc_summary.json for bench.py.

    python tools/pmc_traffic.py FETCH_DIR WRITE_DIR WORKLOAD_TAG [--out profiles/pmc_summary.json]

(tools/gpu/pmc.sh: FETCH_DIR = gpurun_out/TAG/p1, WRITE_DIR = gpurun_out/TAG/p2.)
FETCH_SIZE and WRITE_SIZE are in KiB.  Per MI355X_MICROARCH.md (HBM section),
FETCH_SIZE counts exactly half the bytes of a 16-B/lane coalesced streaming read
on gfx950, so it is doubled; WRITE_SIZE is taken as is.  One step = one
hm_count (one level-1 k_project_partition<.., 0, true> dispatch); the step's bytes
are every pipeline kernel's bytes of the run divided by the steps (the
synthetic-cloud generator and the bench's own check reduction excluded).
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

EXCLUDE = ("k_synth", "at::native", "__amd_rocclr_copyBuffer", "k_read_stream")   # generator, checks, measured-peak passes


def per_kernel(d, counter):
    f = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    vals = defaultdict(float)
    for row in csv.DictReader(open(f[0])):
        if row["Counter_Name"] != counter:
            continue
        k = row["Kernel_Name"].split("(")[0]
        vals[(k, row.get("Dispatch_Id", row.get("Correlation_Id")))] += float(row["Counter_Value"])
    tot, calls = defaultdict(float), defaultdict(int)
    for (k, _), v in vals.items():
        tot[k] += v
        calls[k] += 1
    return tot, calls


def main():
    fd, wd, tag = sys.argv[1], sys.argv[2], sys.argv[3]
    dst = sys.argv[5] if len(sys.argv) > 5 and sys.argv[4] == "--out" else "profiles/pmc_summary.json"
    fetch, fcalls = per_kernel(fd, "FETCH_SIZE")
    write, wcalls = per_kernel(wd, "WRITE_SIZE")
    # one step = one level-1 launch over whole tiles: k_l1_fast (round 4), or the
    # mode-0 k_project_partition (<OutT, 0, true>; older builds: <OutT, 0>)
    steps = sum(v for k, v in fcalls.items() if k.startswith("void k_l1_fast<"))
    if not steps:
        steps = sum(v for k, v in fcalls.items()
                    if k.startswith("void k_project_partition<") and (k.endswith(", 0>") or k.endswith(", 0, true>")))
    kernels = {}
    step_bytes = 0.0
    for k in sorted(set(fetch) | set(write)):
        n = max(fcalls.get(k, 0), wcalls.get(k, 0), 1)
        fb = fetch.get(k, 0.0) * 1024 * 2
        wb = write.get(k, 0.0) * 1024
        kernels[k] = {"fetch_bytes_corrected": fb / n, "write_bytes": wb / n, "hbm_bytes_per_launch": (fb + wb) / n,
                      "launches": n}
        if not any(k.startswith(e) or e in k for e in EXCLUDE):
            step_bytes += fb / max(fcalls.get(k, 1), 1) * fcalls.get(k, 0) / max(steps, 1) + \
                wb / max(wcalls.get(k, 1), 1) * wcalls.get(k, 0) / max(steps, 1)
    entry = {"source": [fd, wd], "kernels": kernels, "steps_profiled": steps, "hbm_bytes_per_step": step_bytes,
             "note": "FETCH_SIZE x2 (gfx950 16-B streaming-read correction) + WRITE_SIZE, KiB -> B; "
                     "per step = all pipeline kernels of one hm_count"}
    d = json.load(open(dst)) if os.path.exists(dst) else {}
    if "fp64" in d.get(tag, {}):
        entry["fp64"] = d[tag]["fp64"]   # tools/pmc_fp64.py's entry stays
    d[tag] = entry
    json.dump(d, open(dst, "w"), indent=1)
    print("steps %d, HBM bytes per step %.3f GB" % (steps, step_bytes / 1e9))
    for k, v in sorted(kernels.items(), key=lambda kv: -kv[1]["hbm_bytes_per_launch"])[:8]:
        print("%-60s %10.3f GB x %d (fetch %.3f, write %.3f)" % (k[:60], v["hbm_bytes_per_launch"] / 1e9, v["launches"],
                                                               v["fetch_bytes_corrected"] / 1e9, v["write_bytes"] / 1e9))


if __name__ == "__main__":
    main()
