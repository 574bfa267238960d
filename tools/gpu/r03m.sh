#!/bin/bash
# hot-tile cap / threshold / item size grid (selection by size), skew check, hot tests.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O="$R/gpurun_out/${1:-r03m}"
mkdir -p "$O"
echo "== hot tests"
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_hot.py > "$O/pytest_hot.log" 2>&1
rc=$?; tail -3 "$O/pytest_hot.log"; [ $rc -eq 0 ] || exit $rc
run() { v=$1; shift; echo "-- $v $*"; env "$@" HM_STEPS=5 timeout -k 10 300 python -u tools/variants.py one $v 2>&1 | grep '^{' ; }
for v in main ta1m hot1k hot1kta1m; do
  for sh in 2048 4096 8192; do run $v HM_HOT_INV_SHARE=$sh; done
done
run hot1k HM_HOT_INV_SHARE=16384 HM_HOT_MIN_KEYS=32768
for v in main hot1k; do echo "-- skew $v"; HM_KIND=skew HM_STEPS=3 timeout -k 10 300 python -u tools/variants.py one $v 2>&1 | grep '^{'; done
echo "== done"
