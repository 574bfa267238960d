#!/bin/bash
# hm_count timings of library variants at zooms 0-21: cvar21.sh TAG names...
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
TAG=$1; shift
O="$R/gpurun_out/$TAG"
mkdir -p "$O"
HM_ZMAX=21 timeout -k 10 600 python3 -u tools/variants.py run "$@" > "$O/var.jsonl" 2> "$O/var.err" || { tail -20 "$O/var.err"; cat "$O/var.jsonl"; exit 1; }
cut -c1-260 "$O/var.jsonl"
