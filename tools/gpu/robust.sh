#!/bin/bash
# Robustness pass: bench on skew and uniform clouds, and the RCCL merge path
# rehearsed with one rank under torch.distributed.run.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O="$R/gpurun_out/${1:-robust}"
mkdir -p "$O"
for k in skew uniform; do
  echo "== bench $k"
  timeout -k 10 300 python -u bench.py --kind $k --steps 5 --warmup 1 --cpu-sample 0 > "$O/bench_$k.log" 2>&1 || { tail -20 "$O/bench_$k.log"; exit 1; }
  { grep -h '^{"metric"' "$O/bench_$k.log" || true; } | cut -c1-700
done
echo "== torchrun 1 rank, RCCL merge path"
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 1 --steps 3 --warmup 1 --points 2.5e8 --cpu-sample 0 --force-dist > "$O/dist1.log" 2>&1 || { tail -30 "$O/dist1.log"; exit 1; }
{ grep -h '^{"metric"' "$O/dist1.log" || true; } | cut -c1-900
