#!/bin/bash
# GPU round check: the -m gpu tests (stop at the first failure), then the
# default bench line.   usage: check.sh TAG [pytest -k expr]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-check}
O="$R/gpurun_out/$TAG"
mkdir -p "$O"
cd "$R"
K=()
[ -n "$2" ] && K=(-k "$2")
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread "${K[@]}" > "$O/pytest.log" 2>&1
rc=$?
tail -5 "$O/pytest.log"
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --cpu-sample 0 > "$O/bench.log" 2>&1 || { tail -20 "$O/bench.log"; exit 1; }
tail -1 "$O/bench.log" | python3 -c "
import json,sys
d=json.loads(sys.stdin.read())
print('ms/step %.3f frac %.3f' % (d['ms_per_step'], d['roofline']['frac']), {k: round(v['us'],1) for k,v in d['kernels'].items()}, d['pipeline'], 'peak', round(d['roofline']['measured_peak']['GBps']))
"
