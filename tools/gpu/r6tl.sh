#!/bin/bash
# Kernel traces (rocprofv3 --kernel-trace, no counters) of the default bench and
# of the 1-hour stream bench, for tools/timeline.py.   usage: r6tl.sh TAG
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
TAG=${1:-r6tl}
O="$R/gpurun_out/$TAG"
mkdir -p "$O"
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace -f csv -d "$O/kt_bench" -o run -- python3 "$R/bench.py" --steps 3 --warmup 1 --cpu-sample 0 > "$O/kt_bench.log" 2>&1 || { tail -20 "$O/kt_bench.log"; exit 1; }
g=$(find "$O/kt_bench" -name "run_kernel_trace.csv" | head -1); cp "$g" "$O/kernel_trace_bench.csv"; rm -rf "$O/kt_bench"
timeout -k 10 300 rocprofv3 --kernel-trace -f csv -d "$O/kt_stream" -o run -- python3 "$R/tools/bench_stream.py" --batches 6 --warmup 1 --hours 1 > "$O/kt_stream.log" 2>&1 || { tail -20 "$O/kt_stream.log"; exit 1; }
g=$(find "$O/kt_stream" -name "run_kernel_trace.csv" | head -1); cp "$g" "$O/kernel_trace_stream.csv"; rm -rf "$O/kt_stream"
ls -la "$O"
cd "$R"
HM_POINTS=1e7 timeout -k 10 200 python -u tools/stamps.py stamps5 > "$O/stamps5_1e7.txt" 2>&1 || { tail -20 "$O/stamps5_1e7.txt"; exit 1; }
HM_POINTS=1e9 timeout -k 10 200 python -u tools/stamps.py stamps5 > "$O/stamps5_1e9.txt" 2>&1 || { tail -20 "$O/stamps5_1e9.txt"; exit 1; }
grep -v amdgpu.ids "$O/stamps5_1e7.txt"; grep -v amdgpu.ids "$O/stamps5_1e9.txt"
