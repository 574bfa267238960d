#!/bin/bash
# kernel stats of the exchange alone (tools/variants.py mone): mks.sh TAG [variant]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
TAG=$1; V=${2:-main}
O="$R/gpurun_out/$TAG"
mkdir -p "$O"
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$O/trace" -o run -- python3 "$R/tools/variants.py" mone "$V" > "$O/trace.log" 2>&1 || { tail -30 "$O/trace.log"; exit 1; }
g=$(find "$O/trace" -name "run_kernel_stats.csv" | head -1); cp "$g" "$O/kernel_stats.csv"
grep '^{' "$O/trace.log" || true
python3 -c "
import csv
r=list(csv.DictReader(open('$O/kernel_stats.csv')))
for x in r[:16]: print(x['Name'][:60].ljust(60), x['Calls'], round(float(x['AverageNs'])/1e3,1), round(float(x['TotalDurationNs'])/1e6,2))
"
