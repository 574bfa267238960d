#!/bin/bash
# hm_count on stream-sized batches (HM_POINTS, default 1e7) for library variants.
#   usage: small.sh TAG variant...
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O="$R/gpurun_out/${1:-small}"; shift
mkdir -p "$O"
HM_STEPS=${HM_STEPS:-20} HM_POINTS=${HM_POINTS:-1e7} timeout -k 10 400 python -u tools/variants.py run "$@" 2>&1 | grep -v amdgpu.ids | tee "$O/variants.jsonl"
