#!/bin/bash
# Kernel-trace stats of the grouped count (tools/bench_grouped.py, device part).
#   usage: prof_grouped.sh TAG [bench_grouped args...]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
TAG=${1:-grouped}; shift
O="$R/gpurun_out/$TAG"
mkdir -p "$O"
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$O/trace_grouped" -o run -- python3 "$R/tools/bench_grouped.py" --no-table --cap-factor 9 --steps 3 "$@" > "$O/trace_grouped.log" 2>&1 || { tail -30 "$O/trace_grouped.log"; exit 1; }
g=$(find "$O/trace_grouped" -name "run_kernel_stats.csv" | head -1); cp "$g" "$O/kernel_stats_grouped.csv"
grep '"part"' "$O/trace_grouped.log" | cut -c1-300
python3 - "$O/kernel_stats_grouped.csv" <<'PY'
import csv, sys
r = list(csv.DictReader(open(sys.argv[1])))
for x in r[:24]:
    print("  %-60s %5s %9.1f us %9.1f us tot" % (x['Name'][:60], x['Calls'], float(x['AverageNs']) / 1e3, float(x['TotalDurationNs']) / 1e3))
PY
