#!/bin/bash
# level-1 sample size vs region re-runs: skew / hotspots / uniform at 2^18 and 2^20 samples
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O="$R/gpurun_out/${1:-r03q}"
mkdir -p "$O"
for k in skew hotspots uniform; do
for s in 18 20; do
HM_SAMPLE_LOG2=$s HM_KIND=$k HM_STEPS=3 timeout -k 10 200 python -u tools/variants.py run main > "$O/var_${k}_$s.log" 2>&1 || { tail -20 "$O/var_${k}_$s.log"; exit 1; }
echo "$k $s $(grep '^{' "$O/var_${k}_$s.log")"
done
done
