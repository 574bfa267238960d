#!/bin/bash
# The exchange's GPU tests, then its phase timings / kernel stats and the
# 1-rank rehearsal:  xchg.sh TAG
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
TAG=${1:-xchg}
O="$R/gpurun_out/$TAG"
mkdir -p "$O"
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_multigpu.py tests/test_gpu_config3.py > "$O/tests.log" 2>&1 || { tail -40 "$O/tests.log"; exit 1; }
tail -3 "$O/tests.log"
bash tools/gpu/merge_stats.sh "$TAG/m" && bash tools/gpu/dist.sh "$TAG/d"
