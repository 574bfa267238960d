#!/bin/bash
# GPU test pass: the named test files (default: all) with per-test timeouts.
#   usage: tests.sh TAG [pytest args...]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
TAG=${1:-tests}; shift
O="$R/gpurun_out/$TAG"
mkdir -p "$O"
timeout -k 10 900 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu "${@:-tests}" > "$O/pytest_gpu.log" 2>&1
rc=$?
tail -30 "$O/pytest_gpu.log"
exit $rc
