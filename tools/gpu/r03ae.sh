#!/bin/bash
# grouped (multi-user rows) path: bench + kernel stats at the reference's zooms 6-21 and at 0-18
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
O="$R/gpurun_out/${1:-r03ae}"
mkdir -p "$O"
cd "$R"
for z in "6 21" "0 18"; do
set -- $z
timeout -k 10 300 python -u tools/bench_grouped.py --zmin $1 --zmax $2 > "$O/grouped_z$1-$2.log" 2>&1 || { tail -20 "$O/grouped_z$1-$2.log"; exit 1; }
grep '^{' "$O/grouped_z$1-$2.log" | cut -c1-400
done
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$O/trace" -o run -- python3 "$R/tools/bench_grouped.py" --zmin 6 --zmax 21 > "$O/trace.log" 2>&1 || { tail -30 "$O/trace.log"; exit 1; }
g=$(find "$O/trace" -name "run_kernel_stats.csv" | head -1); cp "$g" "$O/kernel_stats.csv"
python3 -c "
import csv
r=list(csv.DictReader(open('$O/kernel_stats.csv')))
for x in r[:14]: print(x['Name'][:60].ljust(60), x['Calls'], round(float(x['TotalDurationNs'])/1e6,2), round(float(x['AverageNs'])/1e3,1))
"
echo "== done"
