#!/bin/bash
# row assembly on the GPU: parity tests, then the grouped/table bench at zooms 6-21
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O="$R/gpurun_out/${1:-r03af}"
mkdir -p "$O"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_general.py tests/test_io.py tests/test_gpu_config1.py > "$O/pytest.log" 2>&1
rc=$?; tail -3 "$O/pytest.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/bench_grouped.py --zmin 6 --zmax 21 > "$O/grouped_z6-21.log" 2>&1 || { tail -20 "$O/grouped_z6-21.log"; exit 1; }
grep '^{' "$O/grouped_z6-21.log" | cut -c1-700
echo "== done"
