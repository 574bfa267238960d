#!/bin/bash
# k_small_pairs timing builds (skew 1e9 z0-18): no cursor atomic, no cell
# stores, no emit pass, against main (batch counter) and spstatic8.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O="$R/gpurun_out/${1:-r6spt}"
mkdir -p "$O"
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_buckets.py tests/test_gpu_smoke.py > "$O/tests.log" 2>&1 || { tail -30 "$O/tests.log"; exit 1; }
tail -1 "$O/tests.log"
HM_KIND=skew timeout -k 10 400 python -u tools/variants.py run main spatomnr spnoatom main spatomnr spnoatom > "$O/skew.jsonl" 2>&1 || { tail -5 "$O/skew.jsonl"; exit 1; }
grep variant "$O/skew.jsonl" | cut -c1-250
