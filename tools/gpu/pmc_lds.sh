#!/bin/bash
# One PMC pass of LDS/VALU counters over a short default bench (conflict rate =
# SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE per kernel).   usage: pmc_lds.sh TAG [bench args]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
TAG=${1:-pmclds}; shift
O="$R/gpurun_out/$TAG"
mkdir -p "$O"
cd /tmp
timeout -s KILL 150 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -f csv -d "$O/p" -o run -- python3 "$R/bench.py" --steps 1 --warmup 1 --cpu-sample 0 "$@" > "$O/p.log" 2>&1 || { tail -20 "$O/p.log"; exit 1; }
f=$(find "$O/p" -name "run_counter_collection.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys, collections
acc = collections.defaultdict(lambda: collections.defaultdict(float)); calls = collections.Counter()
for r in csv.DictReader(open(sys.argv[1])):
    k = r["Kernel_Name"][:48]
    acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
for k, c in sorted(acc.items(), key=lambda kv: -kv[1].get("GRBM_GUI_ACTIVE", 0))[:12]:
    lds = c.get("SQ_LDS_IDX_ACTIVE", 0)
    print("%-48s valu %.3g lds %.3g conflict %.2f waves %.3g gui %.3g" % (k, c.get("SQ_INSTS_VALU", 0), c.get("SQ_INSTS_LDS", 0),
          c.get("SQ_LDS_BANK_CONFLICT", 0) / lds if lds else 0, c.get("SQ_WAVES", 0), c.get("GRBM_GUI_ACTIVE", 0)))
PY
