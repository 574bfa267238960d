#!/bin/bash
# Round-6 baseline of every BASELINE config on one GPU: kernel-trace stats of
# the default bench (config 2), the skew cloud (config 4) and the production
# zooms (6-21), plus the stream bench (config 5, 1- and 2-hour batches) with
# its kernel stats.   usage: r6base.sh TAG
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
TAG=${1:-r6base}
O="$R/gpurun_out/$TAG"
mkdir -p "$O"
cd /tmp
run() {   # name, bench args...
  local n=$1; shift
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$O/trace_$n" -o run -- python3 "$R/bench.py" "$@" --cpu-sample 0 > "$O/trace_$n.log" 2>&1 || { tail -30 "$O/trace_$n.log"; return 1; }
  g=$(find "$O/trace_$n" -name "run_kernel_stats.csv" | head -1); cp "$g" "$O/kernel_stats_$n.csv"
  rm -rf "$O/trace_$n"
  grep '^{"metric"' "$O/trace_$n.log" | tail -1 > "$O/bench_$n.json"
  python3 - "$O/bench_$n.json" "$O/kernel_stats_$n.csv" $n <<'PY'
import csv, json, sys
d = json.loads(open(sys.argv[1]).read())
print(sys.argv[3], "ms/step %.3f frac %.3f" % (d['ms_per_step'], d['roofline']['frac']),
      {k: round(v['us']) for k, v in d.get('kernels', {}).items()})
for x in list(csv.DictReader(open(sys.argv[2])))[:14]:
    print("  %-60s %5s %9.1f us" % (x['Name'][:60], x['Calls'], float(x['AverageNs']) / 1e3))
PY
}
run hotspots --steps 5 --warmup 1 || exit 1
run skew --kind skew --steps 5 --warmup 1 || exit 1
run z6-21 --zmin 6 --zmax 21 --steps 5 --warmup 1 || exit 1
cd "$R"
for h in 1 2; do
  timeout -k 10 300 python -u tools/bench_stream.py --batches 18 --warmup 2 --hours $h > "$O/bench_stream_h$h.log" 2>&1 || { tail -30 "$O/bench_stream_h$h.log"; exit 1; }
  tail -1 "$O/bench_stream_h$h.log" | cut -c1-300
done
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$O/prof_h1" -o run -- python3 "$R/tools/bench_stream.py" --batches 10 --warmup 1 --hours 1 > "$O/prof_h1.log" 2>&1 || { tail -30 "$O/prof_h1.log"; exit 1; }
g=$(find "$O/prof_h1" -name "run_kernel_stats.csv" | head -1); cp "$g" "$O/kernel_stats_stream_h1.csv"; rm -rf "$O/prof_h1"
echo done
