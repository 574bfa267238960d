#!/bin/bash
# level-1 region slack: GPU tests of the partition plans, then skew/hotspots/uniform timings
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O="$R/gpurun_out/${1:-r03s}"
mkdir -p "$O"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_plan.py tests/test_gpu_buckets.py tests/test_gpu_hot.py tests/test_gpu_fullsize.py > "$O/pytest.log" 2>&1
rc=$?; tail -3 "$O/pytest.log"; [ $rc -eq 0 ] || exit $rc
for k in skew hotspots uniform; do
HM_KIND=$k HM_STEPS=3 timeout -k 10 200 python -u tools/variants.py run main > "$O/var_$k.log" 2>&1 || { tail -20 "$O/var_$k.log"; exit 1; }
echo "$k $(grep '^{' "$O/var_$k.log")"
done
