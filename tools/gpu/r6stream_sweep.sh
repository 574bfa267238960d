#!/bin/bash
# Stream bench (1-hour batches) under aggregation item-size knobs.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O="$R/gpurun_out/${1:-r6ss}"
mkdir -p "$O"
for cfg in "512 16384" "256 16384" "128 16384" "1024 16384" "512 65536" "512 4096" "512 16384"; do
  set -- $cfg
  HM_TA_ITEMS=$1 HM_TA_MIN=$2 timeout -k 10 200 python -u tools/bench_stream.py --batches 18 --warmup 2 > "$O/s_$1_$2.log" 2>&1 || { tail -5 "$O/s_$1_$2.log"; exit 1; }
  echo "ta_items=$1 ta_min=$2 $(tail -1 $O/s_$1_$2.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_batch"],4), d.get("check"))')"
done
