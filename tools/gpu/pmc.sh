#!/bin/bash
# PMC passes (one counter group per rocprofv3 run) over a short bench.
#   usage: pmc.sh TAG [bench args]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
TAG=${1:-pmc}; shift
O="$R/gpurun_out/$TAG"
mkdir -p "$O"
cd /tmp
PASSES=(
 "FETCH_SIZE"
 "WRITE_SIZE"
 "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES"
 "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT"
 "SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS_ATOMIC SQ_LDS_ATOMIC_RETURN SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE GRBM_COUNT"
 "TCC_EA0_ATOMIC TCC_EA0_ATOMIC_LEVEL TCC_ATOMIC TCP_ATOMIC_TAGCONFLICT_STALL_CYCLES TCP_WRITE_TAGCONFLICT_STALL_CYCLES TA_ATOMIC_REQ"
 "TCC_EA0_WRREQ TCC_EA0_WRREQ_64B TCC_EA0_WRREQ_STALL TCC_EA0_WRREQ_LEVEL"
)
i=0
for p in "${PASSES[@]}"; do
  i=$((i+1))
  echo "== pass $i: $p"
  timeout -s KILL 150 rocprofv3 --kernel-trace --pmc $p -f csv -d "$O/p$i" -o run -- python3 "$R/bench.py" --steps 1 --warmup 1 --cpu-sample 0 "$@" > "$O/p$i.log" 2>&1 || { tail -20 "$O/p$i.log"; exit 1; }
done
for d in "$O"/p*/; do f=$(find "$d" -name "run_counter_collection.csv" | head -1); [ -n "$f" ] && cp "$f" "$d/run_counter_collection.csv" 2>/dev/null; g=$(find "$d" -name "run_kernel_trace.csv" | head -1); [ -n "$g" ] && cp "$g" "$d/run_kernel_trace.csv" 2>/dev/null; done
python3 "$R/tools/pmc_summary.py" "$O"/p*/ > "$O/summary.txt" 2>&1; head -120 "$O/summary.txt"
