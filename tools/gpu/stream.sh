#!/bin/bash
# Config 5 streaming bench + rocprofv3 kernel stats of the same command.  usage: stream.sh TAG
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
TAG=${1:-stream}
O="$R/gpurun_out/$TAG"
mkdir -p "$O"
cd "$R"
timeout -k 10 300 python -u tools/bench_stream.py --batches 20 --warmup 2 > "$O/bench_stream.log" 2>&1 || { tail -30 "$O/bench_stream.log"; exit 1; }
tail -1 "$O/bench_stream.log"
timeout -k 10 300 python -u tools/bench_stream.py --batches 20 --warmup 2 --hours 2 > "$O/bench_stream_h2.log" 2>&1 || { tail -30 "$O/bench_stream_h2.log"; exit 1; }
tail -1 "$O/bench_stream_h2.log"
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$O/prof" -o run -- python3 "$R/tools/bench_stream.py" --batches 10 --warmup 1 > "$O/prof.log" 2>&1 || { tail -30 "$O/prof.log"; exit 1; }
f=$(find "$O/prof" -name "*kernel_stats.csv" | head -1)
cut -d, -f1-4 "$f" | head -24
