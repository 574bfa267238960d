#!/bin/bash
# Iteration pass on the GPU box: GPU parity tests, bench (no CPU leg), and a
# rocprofv3 kernel-trace summary of the same bench.   usage: iter.sh TAG [bench args]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
export TMPDIR=/tmp
TAG=${1:-iter}; shift
O="$R/gpurun_out/$TAG"
mkdir -p "$O"
echo "== pytest -m gpu"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$O/pytest_gpu.log" 2>&1 || { tail -40 "$O/pytest_gpu.log"; exit 1; }
tail -2 "$O/pytest_gpu.log"
echo "== bench"
timeout -k 10 400 python -u bench.py --steps 10 --warmup 2 --cpu-sample 0 "$@" > "$O/bench.log" 2>&1 || { tail -30 "$O/bench.log"; exit 1; }
tail -1 "$O/bench.log"
echo "== rocprofv3"
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d "$O/prof" -o run -- python3 "$R/bench.py" --steps 5 --warmup 1 --cpu-sample 0 "$@" > "$O/prof.log" 2>&1 || { tail -30 "$O/prof.log"; exit 1; }
f=$(find "$O/prof" -name "*kernel_stats.csv" | head -1)
cut -d, -f1-4 "$f" | head -20
