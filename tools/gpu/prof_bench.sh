#!/bin/bash
# Kernel-trace stats of one bench.py configuration.
#   usage: prof_bench.sh TAG NAME [bench.py args...]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
TAG=${1:-prof}; NAME=${2:-bench}; shift 2
O="$R/gpurun_out/$TAG"
mkdir -p "$O"
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$O/trace_$NAME" -o run -- python3 "$R/bench.py" --steps 3 --warmup 1 --cpu-sample 0 "$@" > "$O/trace_$NAME.log" 2>&1 || { tail -30 "$O/trace_$NAME.log"; exit 1; }
g=$(find "$O/trace_$NAME" -name "run_kernel_stats.csv" | head -1); cp "$g" "$O/kernel_stats_$NAME.csv"
grep "^{" "$O/trace_$NAME.log" | tail -1 > "$O/bench_$NAME.json"
python3 - "$O/kernel_stats_$NAME.csv" "$O/bench_$NAME.json" <<'PY'
import csv, json, sys
r = list(csv.DictReader(open(sys.argv[1])))
d = json.loads(open(sys.argv[2]).read())
print(sys.argv[1], "ms/step %.3f" % d["ms_per_step"], {k: round(v["us"], 1) for k, v in d.get("kernels", {}).items()})
for x in r[:16]:
    print("  %-60s %5s %9.1f us" % (x['Name'][:60], x['Calls'], float(x['AverageNs']) / 1e3))
PY
