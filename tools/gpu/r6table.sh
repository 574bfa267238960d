#!/bin/bash
# heatmap_table (1e7 points x 10K users, zooms 6-21, Arrow user ids), pinned
# and pageable host copies of the text, plus the table parity tests.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O="$R/gpurun_out/${1:-r6table}"
mkdir -p "$O"
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_general.py -k "table" > "$O/tests.log" 2>&1 || { tail -20 "$O/tests.log"; exit 1; }
tail -1 "$O/tests.log"
for pin in 1 1; do
HM_TABLE_THREADED_COPY=$pin timeout -k 10 300 python -u tools/bench_grouped.py --points 1e6 --steps 1 --users 10000 --zmin 6 --zmax 21 --arrow > "$O/table_pin$pin.jsonl" 2>&1 || { tail -20 "$O/table_pin$pin.jsonl"; exit 1; }
echo "threaded=$pin $(grep '"heatmap_table"' $O/table_pin$pin.jsonl | tail -1 | cut -c1-600)"
done
