#!/bin/bash
# rocprofv3 kernel-trace summary of a short bench run.   usage: prof.sh TAG [bench args]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
TAG=${1:-prof}; shift
O="$R/gpurun_out/$TAG"
mkdir -p "$O"
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d "$O/prof" -o run -- python3 "$R/bench.py" --steps 5 --warmup 1 --cpu-sample 0 "$@" > "$O/prof.log" 2>&1 || { tail -30 "$O/prof.log"; exit 1; }
tail -1 "$O/prof.log"
f=$(find "$O/prof" -name "*kernel_stats.csv" | head -1)
cp "$f" "$O/kernel_stats.csv"
cut -d, -f1-4 "$f" | head -24
