#!/bin/bash
# hot tiles + spread plan: hot/plan tests, full-size digests, benches (hotspots, skew).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
TAG=${1:-r03n}
O="$R/gpurun_out/$TAG"
mkdir -p "$O"
echo "== hot/plan/bucket tests"
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_hot.py tests/test_gpu_plan.py tests/test_gpu_smoke.py > "$O/pytest_hot.log" 2>&1
rc=$?; tail -3 "$O/pytest_hot.log"; [ $rc -eq 0 ] || exit $rc
echo "== benches"
for k in hotspots skew; do
timeout -k 10 300 python -u bench.py --kind $k --steps 5 --warmup 2 --cpu-sample 0 > "$O/bench_$k.log" 2>&1 || { tail -20 "$O/bench_$k.log"; exit 1; }
tail -1 "$O/bench_$k.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['config']['workload'], d['ms_per_step'], d['roofline']['frac'], d['config']['partition_levels'], d['pipeline'], json.dumps(d['kernels']))"
done
echo "== fullsize"
timeout -k 10 900 python -u -m pytest -x -q --timeout 400 --timeout-method thread -m gpu tests/test_gpu_fullsize.py > "$O/pytest_full.log" 2>&1
rc=$?; tail -3 "$O/pytest_full.log"; [ $rc -eq 0 ] || exit $rc
echo "== done"
