#!/bin/bash
# Bench on all three synthetic clouds (hotspots = BASELINE config 2) plus the
# small-bucket parity tests; each step under its own time limit.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O="$R/gpurun_out/${1:-kinds}"
mkdir -p "$O"
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_buckets.py tests/test_gpu_smoke.py > "$O/tests.log" 2>&1 || { tail -30 "$O/tests.log"; exit 1; }
tail -2 "$O/tests.log"
for k in hotspots skew uniform; do
  timeout -k 10 300 python -u bench.py --kind $k --steps 5 --warmup 1 --cpu-sample 0 > "$O/bench_$k.log" 2>&1 || { tail -20 "$O/bench_$k.log"; exit 1; }
  python3 - "$O/bench_$k.log" $k <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith('{"metric"'):
        d = json.loads(l)
        print(sys.argv[2], round(d['ms_per_step'], 2), round(d['value'] / 1e9, 1), round(d['roofline']['frac'], 3),
              {k: round(v['us']) for k, v in d.get('kernels', {}).items()})
PY
done
