#!/bin/bash
# hm_count A/B of library variants on the hotspot, skew and uniform clouds and
# on hotspots at zooms 0-21, interleaved twice: kinds_ab.sh TAG variant...
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
TAG=$1; shift
VARS="$*"
O="$R/gpurun_out/$TAG"
mkdir -p "$O"
for rep in 1 2; do
  for cfg in "hotspots 1e9 18" "skew 1e9 18" "uniform 6e8 18" "hotspots 1e9 21"; do
    read -r k p z <<< "$cfg"
    HM_KIND=$k HM_POINTS=$p HM_ZMAX=$z timeout -k 10 300 python3 -u tools/variants.py run $VARS >> "$O/var.jsonl" 2>> "$O/var.err" || { tail -20 "$O/var.err"; exit 1; }
  done
done
cut -c1-200 "$O/var.jsonl"
