#!/bin/bash
# GPU parity tests, then A/B timing of library variants.   usage: k2.sh TAG variant...
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
export TMPDIR=/tmp
TAG=${1:-k2}; shift
O="$R/gpurun_out/$TAG"
mkdir -p "$O"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$O/pytest_gpu.log" 2>&1 || { tail -40 "$O/pytest_gpu.log"; exit 1; }
tail -2 "$O/pytest_gpu.log"
timeout -k 10 500 python -u tools/variants.py run "$@" 2>&1 | tee "$O/variants.jsonl"
for v in ${STAMPS:-}; do timeout -k 10 200 python -u tools/stamps.py $v 2>&1 | grep -v amdgpu.ids | tee -a "$O/stamps.txt"; done
