#!/bin/bash
# stream (cell log) tests, full-size stream parity, stream bench + profile.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
TAG=${1:-r03i}
O="$R/gpurun_out/$TAG"
mkdir -p "$O"
export TMPDIR=/tmp
echo "== stream tests"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_stream.py tests/test_gpu_fullsize.py -k "stream" > "$O/pytest_stream.log" 2>&1
rc=$?; tail -3 "$O/pytest_stream.log"; [ $rc -eq 0 ] || exit $rc
bash tools/gpu/stream.sh "${TAG}_stream" || exit 1
echo "== done"
