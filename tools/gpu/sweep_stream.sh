#!/bin/bash
# stream 1-hour batch time over aggregation item sizes
set -o pipefail
O=gpurun_out/r06b; mkdir -p $O
for cfg in "16384 512" "8192 512" "4096 512" "8192 1024" "32768 512" "16384 512"; do
  set -- $cfg
  HM_TA_MIN=$1 HM_TA_ITEMS=$2 timeout -k 10 120 python -u tools/bench_stream.py --batches 18 --warmup 2 > $O/s_$1_$2.log 2>&1 || { tail -5 $O/s_$1_$2.log; exit 1; }
  echo "$1 $2 $(grep -o '"ms_per_batch": [0-9.]*' $O/s_$1_$2.log | tail -1)"
done
