#!/bin/bash
# stream batch: kernel + HIP API trace (host gaps between launches)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
O="$R/gpurun_out/${1:-r03v}"
mkdir -p "$O"
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --hip-trace -f csv -d "$O/trace" -o run -- python3 "$R/tools/bench_stream.py" --hours 1 --batches 6 --warmup 2 > "$O/trace.log" 2>&1 || { tail -30 "$O/trace.log"; exit 1; }
tail -1 "$O/trace.log" | cut -c1-200
g=$(find "$O/trace" -name "run_kernel_trace.csv" | head -1); cp "$g" "$O/kernel_trace.csv"
g=$(find "$O/trace" -name "run_hip_api_trace.csv" | head -1); cp "$g" "$O/hip_api_trace.csv"
echo "== done"
