#!/bin/bash
# Round profile set on the GPU box: bench line, rocprofv3 kernel-trace stats of
# the same command, and the HBM-traffic PMC passes (FETCH_SIZE, WRITE_SIZE in
# separate runs, as MI355X_MICROARCH.md prescribes).   usage: profile_round.sh TAG [bench args]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
TAG=${1:-round}; shift
O="$R/gpurun_out/$TAG"
mkdir -p "$O"
cd "$R"
echo "== bench"
timeout -k 10 400 python -u bench.py "$@" > "$O/bench.log" 2>&1 || { tail -30 "$O/bench.log"; exit 1; }
tail -1 "$O/bench.log"
cd /tmp
echo "== kernel trace"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d "$O/trace" -o run -- python3 "$R/bench.py" --cpu-sample 0 "$@" > "$O/trace.log" 2>&1 || { tail -30 "$O/trace.log"; exit 1; }
for c in FETCH_SIZE WRITE_SIZE; do
  echo "== pmc $c"
  timeout -s KILL 300 rocprofv3 --kernel-trace --pmc $c -f csv -d "$O/pmc_$c" -o run -- python3 "$R/bench.py" --steps 2 --warmup 1 --cpu-sample 0 "$@" > "$O/pmc_$c.log" 2>&1 || { tail -20 "$O/pmc_$c.log"; exit 1; }
done
find "$O" -name "*.csv" | head -20
