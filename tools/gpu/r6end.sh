#!/bin/bash
# Round-6 end, part 2: the default bench line, its kernel stats and FETCH /
# WRITE passes (profile_round.sh), the fp64 VALU pass and an SQ wait / LDS
# conflict pass of the same bench, kernel stats of the skew cloud and the
# production zooms, the stream bench with kernel stats, and the 1-rank RCCL
# rehearsal.   usage: r6end.sh TAG
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
TAG=${1:-r6_end}
O="$R/gpurun_out/$TAG"
mkdir -p "$O"
cd "$R"
timeout -k 10 400 python -u bench.py > "$O/bench_default.log" 2>&1 || { tail -20 "$O/bench_default.log"; exit 1; }
tail -1 "$O/bench_default.log" | cut -c1-300
bash tools/gpu/profile_round.sh "${TAG}_round" > "$O/profile_round.log" 2>&1 || { tail -20 "$O/profile_round.log"; exit 1; }
cd /tmp
P=1
for p in "SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_FLOPS_FP64" \
         "SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_WAVES"; do
  timeout -s KILL 150 rocprofv3 --kernel-trace --pmc $p -f csv -d "$O/sq$P" -o run -- python3 "$R/bench.py" --steps 2 --warmup 1 --cpu-sample 0 > "$O/sq$P.log" 2>&1 || { tail -20 "$O/sq$P.log"; exit 1; }
  P=$((P+1))
done
run() {   # name, bench args...
  local n=$1; shift
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$O/trace_$n" -o run -- python3 "$R/bench.py" "$@" --cpu-sample 0 > "$O/trace_$n.log" 2>&1 || { tail -30 "$O/trace_$n.log"; return 1; }
  g=$(find "$O/trace_$n" -name "run_kernel_stats.csv" | head -1); cp "$g" "$O/kernel_stats_$n.csv"
  rm -rf "$O/trace_$n"
  grep '^{"metric"' "$O/trace_$n.log" | tail -1 > "$O/bench_$n.json"
  cut -c1-200 "$O/bench_$n.json"
}
run skew --kind skew --steps 5 --warmup 1 || exit 1
run z6-21 --zmin 6 --zmax 21 --steps 5 --warmup 1 || exit 1
cd "$R"
bash tools/gpu/stream.sh "${TAG}_stream" > "$O/stream.log" 2>&1 || { tail -20 "$O/stream.log"; exit 1; }
tail -3 "$O/stream.log" | cut -c1-200
bash tools/gpu/dist.sh "${TAG}_dist" > "$O/dist.log" 2>&1 || { tail -20 "$O/dist.log"; exit 1; }
cut -c1-200 "$O/dist.log"
echo "== r6end done"
