#!/bin/bash
# Round-end pass on the GPU box: smoke(), the default bench (with its CPU
# baseline), the round profile set (bench + kernel trace + FETCH/WRITE PMC
# passes), SQ/TCC counter passes, the stream bench + profiles, and the
# 1-rank RCCL merge rehearsal at the N>1 size.   usage: final.sh TAG
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
TAG=${1:-final}
O="$R/gpurun_out/$TAG"
mkdir -p "$O"
echo "== smoke"
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" 2>&1 | grep -v amdgpu.ids | tail -3 || exit 1
echo "== default bench"
timeout -k 10 400 python -u bench.py > "$O/bench_default.log" 2>&1 || { tail -20 "$O/bench_default.log"; exit 1; }
tail -1 "$O/bench_default.log" | cut -c1-400
bash tools/gpu/profile_round.sh "$TAG" || exit 1
bash tools/gpu/pmc.sh "${TAG}_pmc" > /dev/null || exit 1
bash tools/gpu/stream.sh "${TAG}_stream" || exit 1
bash tools/gpu/dist.sh "${TAG}_dist" || exit 1
echo "== final done"
