#!/usr/bin/env python3
"""Executed fp64 VALU work per point from a rocprofv3 --pmc pass of
SQ_INSTS_VALU_{ADD,MUL,FMA,TRANS}_F64 and SQ_INSTS_VALU_FLOPS_FP64 (SURVEY.md
8d "FP64 cross-check"), written into profiles/pmc_summary.json[TAG]["fp64"]
for bench.py.

    python tools/pmc_fp64.py PASS_DIR WORKLOAD_TAG POINTS_PER_STEP [--out profiles/pmc_summary.json]

The SQ_INSTS_* counters count wave instructions: x64 gives lane operations
(an upper bound where a wave runs with lanes masked off).  One step = one
level-1 whole-tile launch (k_l1_fast), as in tools/pmc_traffic.py.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

C = ["SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_VALU_TRANS_F64",
     "SQ_INSTS_VALU_FLOPS_FP64"]


def main():
    d, tag, pts = sys.argv[1], sys.argv[2], float(sys.argv[3])
    dst = sys.argv[5] if len(sys.argv) > 5 and sys.argv[4] == "--out" else "profiles/pmc_summary.json"
    f = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)[0]
    per = defaultdict(lambda: defaultdict(float))
    disp = defaultdict(set)
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0]
        per[k][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[k].add(r.get("Dispatch_Id", r.get("Correlation_Id")))
    # one step = one level-1 launch over whole tiles: k_l1_fast (round 4 on),
    # or the mode-0 k_project_partition of older builds
    steps = sum(len(v) for k, v in disp.items() if k.startswith("void k_l1_fast<"))
    if not steps:
        steps = sum(len(v) for k, v in disp.items()
                    if k.startswith("void k_project_partition<") and (k.endswith(", 0>") or k.endswith(", 0, true>")))
    steps = max(steps, 1)
    tot = defaultdict(float)
    k1 = defaultdict(float)
    for k, v in per.items():
        if "k_synth" in k or "at::native" in k:
            continue
        for c in C:
            tot[c] += v.get(c, 0.0)
            if k.startswith(("void k_l1_fast<", "void k_project_partition<", "void k_l1_ws<")):
                k1[c] += v.get(c, 0.0)
    ops = lambda t: 64.0 * (t["SQ_INSTS_VALU_ADD_F64"] + t["SQ_INSTS_VALU_MUL_F64"] + t["SQ_INSTS_VALU_FMA_F64"] +
                            t["SQ_INSTS_VALU_TRANS_F64"]) / steps / pts   # noqa: E731
    out = {"source": d, "steps_profiled": steps,
           "ops_per_point_step": ops(tot), "ops_per_point_level1": ops(k1),
           "flops_counter_per_point_step": tot["SQ_INSTS_VALU_FLOPS_FP64"] / steps / pts,
           "wave_instructions_per_step": {c: tot[c] / steps for c in C},
           "note": "wave instructions x 64 lanes / points (lanes masked off still count); flops counter as reported"}
    dd = json.load(open(dst)) if os.path.exists(dst) else {}
    dd.setdefault(tag, {})["fp64"] = out
    json.dump(dd, open(dst, "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
