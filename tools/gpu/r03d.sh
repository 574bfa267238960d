#!/bin/bash
# variants (hot-table ways, aggregate skew) on hotspots and skew, then the
# stream and grouped benches after the per-block counter fixes.  usage: r03d.sh TAG
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
TAG=${1:-r03d}
O="$R/gpurun_out/$TAG"
mkdir -p "$O"
export TMPDIR=/tmp
echo "== variants hotspots"
HM_STEPS=5 timeout -k 10 400 python -u tools/variants.py run main hot2 agns hot2agns main > "$O/var_hot.log" 2>&1 || { tail -20 "$O/var_hot.log"; exit 1; }
grep '^{' "$O/var_hot.log"
echo "== variants skew"
HM_KIND=skew HM_STEPS=3 timeout -k 10 400 python -u tools/variants.py run main agns > "$O/var_skew.log" 2>&1 || { tail -20 "$O/var_skew.log"; exit 1; }
grep '^{' "$O/var_skew.log"
echo "== stream"
timeout -k 10 300 python -u tools/bench_stream.py --batches 20 --warmup 2 > "$O/stream_h1.log" 2>&1 || { tail -20 "$O/stream_h1.log"; exit 1; }
tail -1 "$O/stream_h1.log" | cut -c1-400
timeout -k 10 300 python -u tools/bench_stream.py --batches 20 --warmup 2 --hours 2 > "$O/stream_h2.log" 2>&1 || { tail -20 "$O/stream_h2.log"; exit 1; }
tail -1 "$O/stream_h2.log" | cut -c1-400
echo "== grouped"
timeout -k 10 300 python -u tools/bench_grouped.py --points 1e8 --users 10000 --zmin 6 --zmax 21 --no-table > "$O/grouped.log" 2>&1 || { tail -20 "$O/grouped.log"; exit 1; }
grep '^{' "$O/grouped.log" | cut -c1-500
echo "== done"
