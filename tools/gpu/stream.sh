#!/bin/bash
# Config 5 streaming bench (1 and 2 hours per batch) + rocprofv3 kernel stats of
# both.  usage: stream.sh TAG
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
TAG=${1:-stream}
O="$R/gpurun_out/$TAG"
mkdir -p "$O"
cd "$R"
timeout -k 10 300 python -u tools/bench_stream.py --batches 18 --warmup 2 > "$O/bench_stream.log" 2>&1 || { tail -30 "$O/bench_stream.log"; exit 1; }
tail -1 "$O/bench_stream.log"
timeout -k 10 300 python -u tools/bench_stream.py --batches 18 --warmup 2 --hours 2 > "$O/bench_stream_h2.log" 2>&1 || { tail -30 "$O/bench_stream_h2.log"; exit 1; }
tail -1 "$O/bench_stream_h2.log"
cd /tmp
for h in 1 2; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$O/prof_h$h" -o run -- python3 "$R/tools/bench_stream.py" --batches 10 --warmup 1 --hours $h > "$O/prof_h$h.log" 2>&1 || { tail -30 "$O/prof_h$h.log"; exit 1; }
done
echo profiled
