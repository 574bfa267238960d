#!/bin/bash
# Round-1 first GPU pass: smoke, GPU parity tests, bench, rocprofv3 kernel stats.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
export TMPDIR=/tmp
mkdir -p gpurun_out
echo "== smoke"
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -30 gpurun_out/smoke.log; exit 1; }
tail -3 gpurun_out/smoke.log
echo "== pytest -m gpu"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -5 gpurun_out/pytest_gpu.log
echo "== bench"
timeout -k 10 400 python -u bench.py --steps 5 --warmup 2 > gpurun_out/bench.log 2>&1 || { tail -30 gpurun_out/bench.log; exit 1; }
tail -2 gpurun_out/bench.log
echo "== rocprofv3 kernel-trace stats"
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof" -o run -- python3 "$R/bench.py" --steps 5 --warmup 2 --cpu-sample 0 > "$R/gpurun_out/prof.log" 2>&1 || { tail -30 "$R/gpurun_out/prof.log"; exit 1; }
tail -2 "$R/gpurun_out/prof.log"
find "$R/gpurun_out/prof" -name "*stats*" | head
