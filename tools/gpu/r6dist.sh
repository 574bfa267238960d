#!/bin/bash
# 1-rank RCCL rehearsal (1.25e9 points) with and without the count stream at
# the highest priority (HM_COUNT_PRIORITY), beside the plain bench.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O="$R/gpurun_out/${1:-r6dist}"
mkdir -p "$O"
timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --points 1.25e9 --cpu-sample 0 > "$O/plain.log" 2>&1 || { tail -20 "$O/plain.log"; exit 1; }
grep -h '^{"metric"' "$O/plain.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('plain', round(d['ms_per_step'],3))"
for p in 1 0 1 0; do
HM_COUNT_PRIORITY=$p timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 1 --steps 5 --warmup 1 --points 1.25e9 --cpu-sample 0 --force-dist > "$O/dist1_p$p.log" 2>&1 || { tail -30 "$O/dist1_p$p.log"; exit 1; }
grep -h '^{"metric"' "$O/dist1_p$p.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); x=d['distributed']; print('count_priority=$p', round(d['ms_per_step'],3), 'local', round(x['local_ms_per_step'],3), 'merge', round(x['merge_ms_per_step'],3), 'eff', round(x['efficiency_vs_local'],3))"
done
