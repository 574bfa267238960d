#!/bin/bash
# Per-user rows (heatmap_table on 1e7 points x 10K users, zooms 6-21; user ids
# as an object array and as an Arrow dictionary column) and the 1-rank RCCL
# rehearsal of the exchange.   usage: r6rows.sh TAG
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O="$R/gpurun_out/${1:-r6rows}"
mkdir -p "$O"
timeout -k 10 300 python -u tools/bench_grouped.py --points 1e8 --users 10000 --zmin 6 --zmax 21 > "$O/grouped.jsonl" 2>&1 || { tail -20 "$O/grouped.jsonl"; exit 1; }
grep '^{' "$O/grouped.jsonl" | cut -c1-400
timeout -k 10 300 python -u tools/bench_grouped.py --points 1e6 --steps 1 --users 10000 --zmin 6 --zmax 21 --arrow > "$O/grouped_arrow.jsonl" 2>&1 || { tail -20 "$O/grouped_arrow.jsonl"; exit 1; }
grep '^{' "$O/grouped_arrow.jsonl" | tail -1 | cut -c1-500
bash tools/gpu/dist.sh "${1:-r6rows}_dist" || exit 1
for t in 1 0 1 0; do HM_TAIL_STREAM=$t timeout -k 10 200 python -u tools/variants.py run main > "$O/tail$t.jsonl" 2>&1 || { tail -5 "$O/tail$t.jsonl"; exit 1; }; echo "tail=$t $(grep variant $O/tail$t.jsonl | cut -c1-200)"; done
for t in 1 0; do HM_TAIL_STREAM=$t timeout -k 10 200 python -u tools/bench_stream.py --batches 18 --warmup 2 > "$O/stream_tail$t.log" 2>&1 || { tail -5 "$O/stream_tail$t.log"; exit 1; }; echo "stream tail=$t $(tail -1 $O/stream_tail$t.log | cut -c1-160)"; done
