#!/bin/bash
# Round-3 profile set: default bench line, rocprofv3 kernel-trace stats of the
# same command, FETCH/WRITE passes (HBM traffic, separate runs), SQ/LDS/atomic
# counter passes and the fp64 pass.   usage: profile_r03.sh TAG [bench args]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
TAG=${1:-r03}; shift
O="$R/gpurun_out/$TAG"
mkdir -p "$O"
cd "$R"
echo "== bench"
timeout -k 10 400 python -u bench.py "$@" > "$O/bench.log" 2>&1 || { tail -30 "$O/bench.log"; exit 1; }
tail -1 "$O/bench.log" | cut -c1-300
cd /tmp
echo "== kernel trace"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d "$O/trace" -o run -- python3 "$R/bench.py" --cpu-sample 0 "$@" > "$O/trace.log" 2>&1 || { tail -30 "$O/trace.log"; exit 1; }
PASSES=(
 "FETCH_SIZE"
 "WRITE_SIZE"
 "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES"
 "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT"
 "SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS_ATOMIC SQ_LDS_ATOMIC_RETURN SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE GRBM_COUNT"
 "TCC_EA0_ATOMIC TCC_EA0_ATOMIC_LEVEL TCC_ATOMIC TA_ATOMIC_REQ"
 "SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_FLOPS_FP64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64"
)
i=0
for p in "${PASSES[@]}"; do
  i=$((i+1))
  echo "== pass $i: $p"
  timeout -s KILL 200 rocprofv3 --kernel-trace --pmc $p -f csv -d "$O/p$i" -o run -- python3 "$R/bench.py" --steps 2 --warmup 1 --cpu-sample 0 "$@" > "$O/p$i.log" 2>&1 || { tail -20 "$O/p$i.log"; exit 1; }
done
for d in "$O"/p*/; do f=$(find "$d" -name "run_counter_collection.csv" | head -1); [ -n "$f" ] && cp "$f" "$d/run_counter_collection.csv" 2>/dev/null; g=$(find "$d" -name "run_kernel_trace.csv" | head -1); [ -n "$g" ] && cp "$g" "$d/run_kernel_trace.csv" 2>/dev/null; done
cd "$R"
python3 tools/pmc_summary.py "$O"/p3/ "$O"/p4/ "$O"/p5/ "$O"/p6/ "$O"/p7/ > "$O/summary.txt" 2>&1; head -60 "$O/summary.txt"
echo "== done"
