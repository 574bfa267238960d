#!/bin/bash
# all GPU tests, stream bench, default bench, uniform bench.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
TAG=${1:-r03j}
O="$R/gpurun_out/$TAG"
mkdir -p "$O"
export TMPDIR=/tmp
echo "== gpu tests"
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > "$O/pytest_gpu.log" 2>&1
rc=$?; tail -3 "$O/pytest_gpu.log"; [ $rc -eq 0 ] || exit $rc
echo "== stream"
for h in 1 2; do
timeout -k 10 300 python -u tools/bench_stream.py --hours $h > "$O/stream_h$h.log" 2>&1 || { tail -20 "$O/stream_h$h.log"; exit 1; }
tail -1 "$O/stream_h$h.log" | cut -c1-330
done
echo "== bench"
timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 > "$O/bench.log" 2>&1 || { tail -20 "$O/bench.log"; exit 1; }
tail -1 "$O/bench.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['value']/1e9, d['roofline']['frac'], d['pipeline'], json.dumps(d['kernels']))"
for k in uniform skew; do
timeout -k 10 300 python -u bench.py --kind $k --steps 5 --warmup 2 --cpu-sample 0 > "$O/bench_$k.log" 2>&1 || { tail -20 "$O/bench_$k.log"; exit 1; }
tail -1 "$O/bench_$k.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['config']['workload'], d['ms_per_step'], d['roofline']['frac'], json.dumps(d['kernels']))"
done
echo "== done"
