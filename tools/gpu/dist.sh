#!/bin/bash
# Cost of the RCCL merge path at the N>1 bench size (1.25e9 points per rank):
# the plain bench and the 1-rank torch.distributed.run rehearsal of the same
# step with merge_cells (route + reduce + all-to-all + merge), then robust.sh.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O="$R/gpurun_out/${1:-dist}"
mkdir -p "$O"
timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --points 1.25e9 --cpu-sample 0 > "$O/plain.log" 2>&1 || { tail -20 "$O/plain.log"; exit 1; }
{ grep -h '^{"metric"' "$O/plain.log" || true; } | cut -c1-300
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 1 --steps 5 --warmup 1 --points 1.25e9 --cpu-sample 0 --force-dist > "$O/dist1.log" 2>&1 || { tail -30 "$O/dist1.log"; exit 1; }
{ grep -h '^{"metric"' "$O/dist1.log" || true; } | cut -c1-300
