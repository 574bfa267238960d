#!/bin/bash
# all GPU tests, default bench, the 1-rank RCCL rehearsal (dist.sh) and the
# merge phase profile.   usage: r03e.sh TAG
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
TAG=${1:-r03e}
O="$R/gpurun_out/$TAG"
mkdir -p "$O"
export TMPDIR=/tmp
echo "== gpu tests"
timeout -k 10 900 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests > "$O/pytest_gpu.log" 2>&1
rc=$?; tail -3 "$O/pytest_gpu.log"; [ $rc -eq 0 ] || exit $rc
echo "== bench"
timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 > "$O/bench.log" 2>&1 || { tail -20 "$O/bench.log"; exit 1; }
tail -1 "$O/bench.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['value']/1e9, d['roofline']['frac'], d['pipeline'], json.dumps(d['kernels']), json.dumps(d['cpu_baseline']))"
echo "== dist rehearsal"
bash tools/gpu/dist.sh "$TAG/dist" || exit 1
echo "== merge phases"
timeout -k 10 300 python -u tools/merge_profile.py > "$O/merge.log" 2>&1 || { tail -20 "$O/merge.log"; exit 1; }
grep '^{' "$O/merge.log" | cut -c1-600
echo "== done"
