#!/bin/bash
# exchange tests (quick) + merge variant timings: xq.sh TAG variants...
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
TAG=$1; shift
O="$R/gpurun_out/$TAG"
mkdir -p "$O"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_multigpu.py tests/test_gpu_config3.py > "$O/tests.log" 2>&1 || { tail -40 "$O/tests.log"; exit 1; }
tail -2 "$O/tests.log"
bash tools/gpu/mvar.sh "$TAG/v" "$@"
