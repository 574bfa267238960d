#!/bin/bash
# stream batches: blocking vs polled waits
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O="$R/gpurun_out/${1:-r03w}"
mkdir -p "$O"
for sp in 0 300 0 300; do
for h in 1 2; do
HM_SYNC_SPIN_US=$sp timeout -k 10 300 python -u tools/bench_stream.py --hours $h > "$O/stream_${sp}_h$h.log" 2>&1 || { tail -20 "$O/stream_${sp}_h$h.log"; exit 1; }
echo "spin $sp h$h $(tail -1 "$O/stream_${sp}_h$h.log" | cut -c1-200)"
done
done
