#!/bin/bash
# one PMC pass (LDS / VALU / wave counters) over the exchange alone
# (tools/variants.py mone main): mpmc.sh TAG
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
TAG=$1
O="$R/gpurun_out/$TAG"
mkdir -p "$O"
cd /tmp
export HM_STEPS=2
timeout -s KILL 150 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -f csv -d "$O/p" -o run -- python3 "$R/tools/variants.py" mone main > "$O/p.log" 2>&1 || { tail -20 "$O/p.log"; exit 1; }
f=$(find "$O/p" -name "run_counter_collection.csv" | head -1)
cp "$f" "$O/counters.csv"
python3 - "$f" <<'PY'
import csv, sys, collections
acc = collections.defaultdict(lambda: collections.defaultdict(float)); calls = collections.Counter()
for r in csv.DictReader(open(sys.argv[1])):
    k = r["Kernel_Name"][:40]
    acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
for k, c in sorted(acc.items(), key=lambda kv: -kv[1].get("GRBM_GUI_ACTIVE", 0))[:10]:
    lds = c.get("SQ_LDS_IDX_ACTIVE", 0)
    print("%-40s valu %.3g lds %.3g ldsact %.3g conflict %.2f waves %.3g wcyc %.3g busy %.3g gui %.3g" % (k, c.get("SQ_INSTS_VALU", 0), c.get("SQ_INSTS_LDS", 0), lds,
          c.get("SQ_LDS_BANK_CONFLICT", 0) / lds if lds else 0, c.get("SQ_WAVES", 0), c.get("SQ_WAVE_CYCLES", 0), c.get("SQ_BUSY_CYCLES", 0), c.get("GRBM_GUI_ACTIVE", 0)))
PY
