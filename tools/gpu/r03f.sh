#!/bin/bash
# headline profile set of the current build + rocprofv3 kernel stats of the
# merge phase profile.   usage: r03f.sh TAG
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
TAG=${1:-r03f}
O="$R/gpurun_out/$TAG"
mkdir -p "$O"
export TMPDIR=/tmp
bash tools/gpu/profile_r03.sh "${TAG}_prof" --steps 10 --warmup 3 || exit 1
echo "== merge kernel stats"
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$O/prof_merge" -o run -- python3 "$R/tools/merge_profile.py" > "$O/prof_merge.log" 2>&1 || { tail -20 "$O/prof_merge.log"; exit 1; }
cd "$R"
f=$(find "$O/prof_merge" -name "*kernel_stats.csv" | head -1); [ -n "$f" ] && cp "$f" "$O/merge_kernel_stats.csv" && head -12 "$O/merge_kernel_stats.csv" | cut -c1-160
echo "== done"
