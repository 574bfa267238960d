#!/bin/bash
# k_stream_buckets with 16-B loads: the stream GPU tests, then the 1- and
# 2-hour stream bench against the previous commit's library (alternating).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O="$R/gpurun_out/${1:-r6sb}"
mkdir -p "$O"
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_stream.py > "$O/tests.log" 2>&1 || { tail -30 "$O/tests.log"; exit 1; }
tail -1 "$O/tests.log"
OLD="$R/heatmap_amd/_lib/variants/lib_git-36166b6.so"
for r in 1 2; do
  for h in 1 2; do
    timeout -k 10 200 python -u tools/bench_stream.py --batches 18 --warmup 2 --hours $h > "$O/new_h${h}_$r.log" 2>&1 || { tail -5 "$O/new_h${h}_$r.log"; exit 1; }
    echo new h$h $(tail -1 "$O/new_h${h}_$r.log" | cut -c1-150)
    HM_LIB_PATH=$OLD timeout -k 10 200 python -u tools/bench_stream.py --batches 18 --warmup 2 --hours $h > "$O/old_h${h}_$r.log" 2>&1 || { tail -5 "$O/old_h${h}_$r.log"; exit 1; }
    echo old h$h $(tail -1 "$O/old_h${h}_$r.log" | cut -c1-150)
  done
done
