#!/bin/bash
# HBM traffic of the default bench step: FETCH_SIZE and WRITE_SIZE rocprofv3
# passes (one counter group per run), summarised by tools/pmc_traffic.py.
#   usage: traffic.sh TAG [--write]   (--write: update profiles/pmc_summary.json)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
TAG=${1:-traffic}
O="$R/gpurun_out/$TAG"
mkdir -p "$O"
cd /tmp
i=0
for p in FETCH_SIZE WRITE_SIZE; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --kernel-trace --pmc $p -f csv -d "$O/p$i" -o run -- python3 "$R/bench.py" --steps 2 --warmup 1 --cpu-sample 0 > "$O/p$i.log" 2>&1 || { tail -20 "$O/p$i.log"; exit 1; }
done
cd "$R"
W=hotspots_1000000000_z0-18          # bench.py's workload tag of the default run
cp profiles/pmc_summary.json "$O/pmc_summary.json"
python3 tools/pmc_traffic.py "$O/p1" "$O/p2" "$W" --out "$O/pmc_summary.json" | tee "$O/traffic.txt"
[ "$2" = "--write" ] && cp "$O/pmc_summary.json" profiles/pmc_summary.json
exit 0
