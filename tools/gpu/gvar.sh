#!/bin/bash
# grouped bench (tools/bench_grouped.py) per library variant: gvar.sh TAG names...  ("main": in-tree)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
TAG=$1; shift
O="$R/gpurun_out/$TAG"
mkdir -p "$O"
for v in "$@"; do
  if [ "$v" = main ]; then L=""; else L="$R/heatmap_amd/_lib/variants/lib_$v.so"; fi
  HM_LIB_PATH="$L" timeout -k 10 300 python3 -u tools/bench_grouped.py --steps 5 --no-table > "$O/g_$v.json" 2> "$O/g_$v.err" || { tail -20 "$O/g_$v.err"; exit 1; }
  echo "$v $(python3 -c "import json,sys; d=json.loads(open('$O/g_$v.json').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['check'])")"
done
