#!/bin/bash
# Round 3, first GPU pass: GPU tests, default bench, the grouped/row path bench
# and its kernel stats (rocprofv3), the 2-rank spawn check on a 1-GPU box.
#   usage: r03_first.sh TAG
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
TAG=${1:-r03a}
O="$R/gpurun_out/$TAG"
mkdir -p "$O"
export TMPDIR=/tmp
echo "== pytest -m gpu"
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > "$O/pytest_gpu.log" 2>&1
rc=$?; tail -3 "$O/pytest_gpu.log"; [ $rc -eq 0 ] || exit $rc
echo "== bench default"
timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 > "$O/bench_default.log" 2>&1 || { tail -20 "$O/bench_default.log"; exit 1; }
tail -1 "$O/bench_default.log" | cut -c1-600
echo "== bench --gpus 2 on one GPU (must fail loudly)"
timeout -k 10 60 python -u bench.py --gpus 2 > "$O/bench_gpus2.log" 2>&1; echo "rc=$?"; tail -2 "$O/bench_gpus2.log"
echo "== grouped path"
timeout -k 10 300 python -u tools/bench_grouped.py --points 1e8 --users 10000 --zmin 6 --zmax 21 > "$O/grouped_z6-21.log" 2>&1 || { tail -20 "$O/grouped_z6-21.log"; exit 1; }
cat "$O/grouped_z6-21.log" | grep '^{' | cut -c1-700
timeout -k 10 300 python -u tools/bench_grouped.py --points 1e8 --users 10000 --zmin 0 --zmax 18 --no-table > "$O/grouped_z0-18.log" 2>&1 || { tail -20 "$O/grouped_z0-18.log"; exit 1; }
cat "$O/grouped_z0-18.log" | grep '^{' | cut -c1-700
echo "== grouped path kernel stats"
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/prof_grouped" -o run -- python3 "$R/tools/bench_grouped.py" --points 1e8 --users 10000 --zmin 6 --zmax 21 --no-table --steps 3 > "$O/prof_grouped.log" 2>&1 || { tail -20 "$O/prof_grouped.log"; exit 1; }
cd "$R"
find "$O/prof_grouped" -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} "$O/grouped_kernel_stats.csv"
head -15 "$O/grouped_kernel_stats.csv" | cut -c1-200
echo "== done"
