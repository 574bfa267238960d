#!/bin/bash
# Round profile: kernel-trace stats of the default bench and of the other
# clouds (one rocprofv3 run each).   usage: prof_round.sh TAG [kinds...]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
TAG=${1:-prof}; shift
KINDS=${@:-hotspots}
O="$R/gpurun_out/$TAG"
mkdir -p "$O"
cd /tmp
for k in $KINDS; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$O/trace_$k" -o run -- python3 "$R/bench.py" --kind $k --steps 3 --warmup 1 --cpu-sample 0 > "$O/trace_$k.log" 2>&1 || { tail -30 "$O/trace_$k.log"; exit 1; }
  g=$(find "$O/trace_$k" -name "run_kernel_stats.csv" | head -1); cp "$g" "$O/kernel_stats_$k.csv"
  tail -1 "$O/trace_$k.log" > "$O/bench_$k.json"
  python3 - "$O/kernel_stats_$k.csv" <<'PY'
import csv, sys
r = list(csv.DictReader(open(sys.argv[1])))
print(sys.argv[1])
for x in r[:22]:
    print("  %-70s %5s %9.1f us" % (x['Name'][:70], x['Calls'], float(x['AverageNs']) / 1e3))
PY
done
