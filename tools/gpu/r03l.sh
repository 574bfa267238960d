#!/bin/bash
# hot-tile threshold knobs (env) and aggregation item sizes (variants).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O="$R/gpurun_out/${1:-r03l}"
mkdir -p "$O"
run() { echo "-- $*"; env "$@" HM_STEPS=5 timeout -k 10 300 python -u tools/variants.py one main 2>&1 | grep '^{' ; }
run HM_HOT_INV_SHARE=2048
run HM_HOT_INV_SHARE=4096
run HM_HOT_INV_SHARE=8192
run HM_HOT_INV_SHARE=8192 HM_HOT_MIN_KEYS=16384
run HM_HOT_INV_SHARE=16384 HM_HOT_MIN_KEYS=16384
HM_STEPS=5 timeout -k 10 400 python -u tools/variants.py run main ta512k ta1m > "$O/var.log" 2>&1 || { tail -20 "$O/var.log"; exit 1; }
grep '^{' "$O/var.log"
HM_KIND=skew HM_STEPS=3 timeout -k 10 400 python -u tools/variants.py run main ta512k ta1m > "$O/var_skew.log" 2>&1 || { tail -20 "$O/var_skew.log"; exit 1; }
grep '^{' "$O/var_skew.log"
echo "== done"
