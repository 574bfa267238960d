#!/bin/bash
# Hot-tile iteration: hot/plan/bucket GPU tests, then the default bench with
# hot tiles off and on (HM_HOT), and the skew bench.   usage: hot.sh TAG
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
TAG=${1:-hot}
O="$R/gpurun_out/$TAG"
mkdir -p "$O"
echo "== hot tests"
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_hot.py tests/test_gpu_smoke.py > "$O/pytest_hot.log" 2>&1
rc=$?; tail -5 "$O/pytest_hot.log"; [ $rc -eq 0 ] || exit $rc
for h in 0 1; do
  echo "== bench hotspots HM_HOT=$h"
  HM_HOT=$h timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --cpu-sample 0 > "$O/bench_hot$h.log" 2>&1 || { tail -20 "$O/bench_hot$h.log"; exit 1; }
  tail -1 "$O/bench_hot$h.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['roofline']['frac'], d['pipeline'], json.dumps(d['kernels']))"
done
echo "== bench skew"
timeout -k 10 300 python -u bench.py --kind skew --steps 5 --warmup 2 --cpu-sample 0 > "$O/bench_skew.log" 2>&1 || { tail -20 "$O/bench_skew.log"; exit 1; }
tail -1 "$O/bench_skew.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['roofline']['frac'], d['pipeline'], json.dumps(d['kernels']))"
echo "== rest of the gpu tests"
timeout -k 10 900 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests > "$O/pytest_gpu.log" 2>&1
rc=$?; tail -5 "$O/pytest_gpu.log"; [ $rc -eq 0 ] || exit $rc
echo "== done"
