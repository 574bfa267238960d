#!/bin/bash
# A/B timing of compile-time variants (tools/variants.py) on the GPU box, plus
# the list of PMC counters this rocprofv3 offers.   usage: ab.sh TAG variant...
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
export TMPDIR=/tmp
TAG=${1:-ab}; shift
O="$R/gpurun_out/$TAG"
mkdir -p "$O"
timeout -k 10 600 python -u tools/variants.py run "$@" 2>&1 | tee "$O/variants.jsonl"
