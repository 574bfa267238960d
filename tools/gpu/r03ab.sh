#!/bin/bash
# everything: all GPU tests, stream, bench (hotspots/uniform/skew), merge phases, 1-rank RCCL rehearsal
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
TAG=${1:-r03ab}
O="$R/gpurun_out/$TAG"
mkdir -p "$O"
bash tools/gpu/r03j.sh "$TAG" || exit $?
echo "== merge phases"
timeout -k 10 300 python -u tools/merge_profile.py > "$O/merge.log" 2>&1 || { tail -20 "$O/merge.log"; exit 1; }
grep '^{' "$O/merge.log" | cut -c1-600
echo "== plain / dist rehearsal"
timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --points 1.25e9 --cpu-sample 0 > "$O/plain.log" 2>&1 || { tail -20 "$O/plain.log"; exit 1; }
{ grep -h '^{"metric"' "$O/plain.log" || true; } | cut -c1-330
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 1 --steps 5 --warmup 1 --points 1.25e9 --cpu-sample 0 --force-dist > "$O/dist1.log" 2>&1 || { tail -30 "$O/dist1.log"; exit 1; }
{ grep -h '^{"metric"' "$O/dist1.log" || true; } | cut -c1-330
echo "== done"
