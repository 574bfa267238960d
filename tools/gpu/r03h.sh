#!/bin/bash
# stream profile (1-hour batches) and the uniform / skew benches.  usage: r03h.sh TAG
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
TAG=${1:-r03h}
O="$R/gpurun_out/$TAG"
mkdir -p "$O"
export TMPDIR=/tmp
bash tools/gpu/stream.sh "${TAG}_stream" || exit 1
for k in uniform skew; do
  echo "== bench $k"
  timeout -k 10 300 python -u bench.py --kind $k --steps 5 --warmup 2 --cpu-sample 0 > "$O/bench_$k.log" 2>&1 || { tail -20 "$O/bench_$k.log"; exit 1; }
  tail -1 "$O/bench_$k.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['roofline']['frac'], d['pipeline'], d['config']['partition_levels'], json.dumps(d['kernels']))"
  cd /tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$O/prof_$k" -o run -- python3 "$R/bench.py" --kind $k --steps 3 --warmup 1 --cpu-sample 0 > "$O/prof_$k.log" 2>&1 || { tail -20 "$O/prof_$k.log"; exit 1; }
  cd "$R"
done
echo "== done"
