#!/bin/bash
# Small-bucket kernels on the resident grid (HM_SPW_RESIDENT) against the
# fixed 8-waves-per-SIMD grid, and k_small_pairs at 8 waves per SIMD:
# small-bucket / skew parity, then skew, hotspot and z6-21 timing.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O="$R/gpurun_out/${1:-r6grid}"
mkdir -p "$O"
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_buckets.py tests/test_gpu_smoke.py tests/test_gpu_fullsize.py -k "not z6-21 and not grouped and not stream" > "$O/tests.log" 2>&1 || { tail -30 "$O/tests.log"; exit 1; }
tail -1 "$O/tests.log"
HM_KIND=skew timeout -k 10 300 python -u tools/variants.py run main spstatic8 spgrid8 spstatic main spstatic8 spgrid8 spstatic > "$O/skew.jsonl" 2>&1 || { tail -5 "$O/skew.jsonl"; exit 1; }
grep variant "$O/skew.jsonl" | cut -c1-250
timeout -k 10 300 python -u tools/variants.py run main spstatic8 main spstatic8 > "$O/hot.jsonl" 2>&1 || { tail -5 "$O/hot.jsonl"; exit 1; }
grep variant "$O/hot.jsonl" | cut -c1-250
HM_ZMIN=6 HM_ZMAX=21 timeout -k 10 300 python -u tools/variants.py run main spstatic8 main spstatic8 > "$O/z621.jsonl" 2>&1 || { tail -5 "$O/z621.jsonl"; exit 1; }
grep variant "$O/z621.jsonl" | cut -c1-250
