#!/bin/bash
# HBM bytes of the grouped count (tools/bench_grouped.py --no-table, 1e8
# points x 10K users, zooms 6-21): FETCH_SIZE and WRITE_SIZE passes.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
O="$R/gpurun_out/${1:-r6gpmc}"
mkdir -p "$O"
cd /tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 200 rocprofv3 --kernel-trace --pmc $c -f csv -d "$O/$c" -o run -- python3 "$R/tools/bench_grouped.py" --steps 1 --warmup 1 --no-table > "$O/$c.log" 2>&1 || { tail -20 "$O/$c.log"; exit 1; }
done
python3 - "$O" <<'PY'
import csv, glob, os, sys
from collections import defaultdict
O = sys.argv[1]
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    f = glob.glob(os.path.join(O, c, "**", "*counter_collection.csv"), recursive=True)[0]
    tot, n = defaultdict(float), defaultdict(set)
    for row in csv.DictReader(open(f)):
        k = row["Kernel_Name"].split("(")[0]
        tot[k] += float(row["Counter_Value"]); n[k].add(row.get("Dispatch_Id"))
    for k in sorted(tot, key=lambda k: -tot[k])[:8]:
        print(c, "%-45s launches %3d  GB total %.3f (KiB x 1024%s)" % (k[:45], len(n[k]), tot[k] * 1024 / 1e9 * (2 if c == "FETCH_SIZE" else 1), ", x2 gfx950 read correction" if c == "FETCH_SIZE" else ""))
PY
