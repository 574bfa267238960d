#!/bin/bash
# k_small_pairs HBM bytes (FETCH_SIZE / WRITE_SIZE passes) on the skew cloud:
# the shipped build against the timing build without the cursor atomic.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
O="$R/gpurun_out/${1:-r6sppmc}"
mkdir -p "$O"
cd /tmp
for v in main spnoatom; do
  for c in FETCH_SIZE WRITE_SIZE; do
    HM_KIND=skew HM_STEPS=1 timeout -k 10 120 rocprofv3 --kernel-trace --pmc $c -f csv -d "$O/${v}_$c" -o run -- python3 "$R/tools/variants.py" one $v > "$O/${v}_$c.log" 2>&1 || { tail -20 "$O/${v}_$c.log"; exit 1; }
  done
done
python3 - "$O" <<'PY'
import csv, glob, os, sys
from collections import defaultdict
O = sys.argv[1]
for v in ("main", "spnoatom"):
    for c in ("FETCH_SIZE", "WRITE_SIZE"):
        f = glob.glob(os.path.join(O, "%s_%s" % (v, c), "**", "*counter_collection.csv"), recursive=True)[0]
        tot, n = defaultdict(float), defaultdict(set)
        for row in csv.DictReader(open(f)):
            if row["Counter_Name"] != c:
                continue
            k = row["Kernel_Name"].split("(")[0]
            tot[k] += float(row["Counter_Value"])
            n[k].add(row.get("Dispatch_Id", row.get("Correlation_Id")))
        for k in sorted(tot):
            if "small" in k or "aggregate" in k:
                print(v, c, "%-40s launches %d  KiB/launch %.0f" % (k[:40], len(n[k]), tot[k] / len(n[k])))
PY
