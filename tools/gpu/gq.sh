#!/bin/bash
# grouped/general GPU tests + the grouped bench line: gq.sh TAG
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
TAG=$1
O="$R/gpurun_out/$TAG"
mkdir -p "$O"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_general.py > "$O/tests.log" 2>&1 || { tail -40 "$O/tests.log"; exit 1; }
tail -2 "$O/tests.log"
timeout -k 10 300 python3 -u tools/bench_grouped.py --steps 5 --no-table > "$O/grouped.jsonl" 2> "$O/grouped.err" || { tail -20 "$O/grouped.err"; exit 1; }
cut -c1-300 "$O/grouped.jsonl"
