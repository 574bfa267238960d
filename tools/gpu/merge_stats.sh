#!/bin/bash
# Exchange cost at the N>1 bench shard (1.25e9 points, world size 1): the
# phase timings of tools/merge_profile.py, then the same run under rocprofv3
# kernel stats (per-kernel averages of the count + exchange kernels).
#   merge_stats.sh TAG [points]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
TAG=${1:-mstats}
P=${2:-1.25e9}
O="$R/gpurun_out/$TAG"
mkdir -p "$O"
cd "$R"
timeout -k 10 240 python3 -u tools/merge_profile.py "$P" > "$O/phases.json" 2> "$O/phases.err" || { tail -20 "$O/phases.err"; exit 1; }
cat "$O/phases.json"
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$O/trace" -o run -- python3 "$R/tools/merge_profile.py" "$P" > "$O/trace.log" 2>&1 || { tail -30 "$O/trace.log"; exit 1; }
g=$(find "$O/trace" -name "run_kernel_stats.csv" | head -1); cp "$g" "$O/kernel_stats.csv"
python3 -c "
import csv
r=list(csv.DictReader(open('$O/kernel_stats.csv')))
for x in r[:30]: print(x['Name'][:60].ljust(60), x['Calls'], round(float(x['AverageNs'])/1e3,1), round(float(x['TotalDurationNs'])/1e6,2))
"
