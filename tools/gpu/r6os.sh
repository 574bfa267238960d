#!/bin/bash
# k_rx_onesweep with LDS-only barriers: the grouped / general GPU tests, then
# the grouped bench (1e8 x 10K users, zooms 6-21) against __syncthreads
# barriers (ossync), alternating.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O="$R/gpurun_out/${1:-r6os}"
mkdir -p "$O"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_general.py tests/test_gpu_fullsize.py -k "grouped or general or tiles or exotic or wide" > "$O/tests.log" 2>&1 || { tail -30 "$O/tests.log"; exit 1; }
tail -1 "$O/tests.log"
for r in 1 2 3; do
  timeout -k 10 200 python -u tools/bench_grouped.py --no-table > "$O/main_$r.log" 2>&1 || { tail -5 "$O/main_$r.log"; exit 1; }
  echo main $(grep -h '"part"' "$O/main_$r.log" | head -1 | cut -c1-160)
  HM_LIB_PATH="$R/heatmap_amd/_lib/variants/lib_ossync.so" timeout -k 10 200 python -u tools/bench_grouped.py --no-table > "$O/ossync_$r.log" 2>&1 || { tail -5 "$O/ossync_$r.log"; exit 1; }
  echo ossync $(grep -h '"part"' "$O/ossync_$r.log" | head -1 | cut -c1-160)
done
