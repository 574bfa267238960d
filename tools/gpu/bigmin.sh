#!/bin/bash
# Sweep of the run-copy big-child threshold (HM_RS_BIG_MIN) on hotspot and skew benches.
for b in 4096 2048 1024 512; do
  for k in hotspots skew; do
    HM_RS_BIG_MIN=$b timeout -k 10 200 python -u bench.py --kind $k --steps 5 --warmup 1 --cpu-sample 0 --no-check > gpurun_out/bm_${k}_${b}.log 2>&1 || exit 1
    python3 -c "
import json,sys
for l in open('gpurun_out/bm_${k}_${b}.log'):
    if l.startswith('{\"metric\"'):
        d=json.loads(l); print('$b', '$k', round(d['ms_per_step'],2), {k[:12]:round(v['us']) for k,v in d['kernels'].items()})"
  done
done
