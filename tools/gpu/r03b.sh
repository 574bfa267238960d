#!/bin/bash
# Round 3 profile pass: headline profile set (bench, kernel stats, PMC passes),
# config-5 stream bench + stats, grouped-path kernel stats (csv).
#   usage: r03b.sh TAG
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
TAG=${1:-r03b}
O="$R/gpurun_out/$TAG"
mkdir -p "$O"
export TMPDIR=/tmp
bash tools/gpu/profile_r03.sh "${TAG}_prof" --steps 10 --warmup 3 || exit 1
bash tools/gpu/stream.sh "${TAG}_stream" || exit 1
echo "== grouped path kernel stats"
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$O/prof_grouped" -o run -- python3 "$R/tools/bench_grouped.py" --points 1e8 --users 10000 --zmin 6 --zmax 21 --no-table --steps 3 > "$O/prof_grouped.log" 2>&1 || { tail -20 "$O/prof_grouped.log"; exit 1; }
cd "$R"
f=$(find "$O/prof_grouped" -name "*kernel_stats.csv" | head -1); [ -n "$f" ] && cp "$f" "$O/grouped_kernel_stats.csv" && head -15 "$O/grouped_kernel_stats.csv" | cut -c1-160
echo "== done"
