#!/bin/bash
# exchange route + merge timings of library variants: mvar.sh TAG names...
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
TAG=$1; shift
O="$R/gpurun_out/$TAG"
mkdir -p "$O"
timeout -k 10 600 python3 -u tools/variants.py mrun "$@" > "$O/mvar.jsonl" 2> "$O/mvar.err" || { tail -20 "$O/mvar.err"; cat "$O/mvar.jsonl"; exit 1; }
cat "$O/mvar.jsonl"
