#!/bin/bash
# profile set of the hot-tile pipeline, the memory probe of the 2^32-point test, then all GPU tests
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
TAG=${1:-r03c}
O="$R/gpurun_out/$TAG"
mkdir -p "$O"
bash tools/gpu/profile_r03.sh "${TAG}_prof" --steps 10 --warmup 3 || exit 1
echo "== memprobe"
timeout -k 10 300 python -u tools/gpu/memprobe.py > "$O/memprobe.log" 2>&1; cat "$O/memprobe.log" | grep -v amdgpu.ids
echo "== gpu tests"
timeout -k 10 1200 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests > "$O/pytest_gpu.log" 2>&1
rc=$?; tail -15 "$O/pytest_gpu.log"; exit $rc
