#!/bin/bash
# merge tests + merge phases (two-pass partition), aggregate variants, bench.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
TAG=${1:-r03g}
O="$R/gpurun_out/$TAG"
mkdir -p "$O"
export TMPDIR=/tmp
echo "== gpu tests"
timeout -k 10 900 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests > "$O/pytest_mg.log" 2>&1
rc=$?; tail -3 "$O/pytest_mg.log"; [ $rc -eq 0 ] || exit $rc
echo "== merge phases"
timeout -k 10 300 python -u tools/merge_profile.py > "$O/merge.log" 2>&1 || { tail -20 "$O/merge.log"; exit 1; }
grep '^{' "$O/merge.log" | cut -c1-600
echo "== variants"
HM_STEPS=5 timeout -k 10 400 python -u tools/variants.py run main agslow agm4 agm16 main > "$O/var.log" 2>&1 || { tail -20 "$O/var.log"; exit 1; }
grep '^{' "$O/var.log"
HM_KIND=skew HM_STEPS=3 timeout -k 10 400 python -u tools/variants.py run main agslow > "$O/var_skew.log" 2>&1 || { tail -20 "$O/var_skew.log"; exit 1; }
grep '^{' "$O/var_skew.log"
echo "== dist rehearsal"
bash tools/gpu/dist.sh "$TAG/dist" || exit 1
echo "== done"
