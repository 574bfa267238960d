#!/bin/bash
# A/B of library variants on the config-5 stream bench (1- and 2-hour batches),
# interleaved: stream_ab.sh TAG variant...  ("base" = the in-tree library)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
TAG=$1; shift
O="$R/gpurun_out/$TAG"
mkdir -p "$O"
for rep in 1 2; do
  for v in "$@"; do
    for h in 1 2; do
      if [ "$v" = base ]; then L="$R/heatmap_amd/_lib/libheatmap_amd.so"; else L="$R/heatmap_amd/_lib/variants/lib_$v.so"; fi
      HM_LIB_PATH="$L" timeout -k 10 200 python -u tools/bench_stream.py --batches 18 --warmup 2 --hours $h > "$O/${v}_h${h}_$rep.log" 2>&1 || { tail -20 "$O/${v}_h${h}_$rep.log"; exit 1; }
      python3 -c "
import json
d = json.loads(open('$O/${v}_h${h}_$rep.log').read().strip().splitlines()[-1])
print('$v h$h rep$rep', round(d['ms_per_batch'], 4), d.get('check'))" | tee -a "$O/summary.txt"
    done
  done
done
