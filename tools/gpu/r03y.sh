#!/bin/bash
# uniform cloud: kernel stats + two SQ counter passes
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
O="$R/gpurun_out/${1:-r03y}"
mkdir -p "$O"
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$O/trace" -o run -- python3 "$R/bench.py" --kind uniform --steps 3 --warmup 1 --cpu-sample 0 > "$O/trace.log" 2>&1 || { tail -30 "$O/trace.log"; exit 1; }
g=$(find "$O/trace" -name "run_kernel_stats.csv" | head -1); cp "$g" "$O/kernel_stats.csv"
i=0
for p in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES" "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 200 rocprofv3 --kernel-trace --pmc $p -f csv -d "$O/p$i" -o run -- python3 "$R/bench.py" --kind uniform --steps 1 --warmup 0 --cpu-sample 0 --no-check > "$O/p$i.log" 2>&1 || { tail -20 "$O/p$i.log"; exit 1; }
  f=$(find "$O/p$i" -name "run_counter_collection.csv" | head -1); cp "$f" "$O/p$i/run_counter_collection.csv"
done
cd "$R"
python3 tools/pmc_summary.py "$O"/p1/ "$O"/p2/ > "$O/summary.txt" 2>&1
python3 tools/pmc_traffic.py "$O"/p3/ "$O"/p4/ uniform --out "$O/pmc_summary.json" > "$O/traffic.txt" 2>&1 || true
echo "== done"
