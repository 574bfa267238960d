#!/bin/bash
# k_small_pairs with block-level cursor reservations: parity (small-bucket,
# smoke and full-size digests), then skew / hotspot / z6-21 timing against the
# previous commit (git-1c3613c) and the 8- / 2-wave-block builds, and the
# stream bench.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O="$R/gpurun_out/${1:-r6blk}"
mkdir -p "$O"
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_buckets.py tests/test_gpu_smoke.py tests/test_gpu_fullsize.py -k "not grouped" > "$O/tests.log" 2>&1 || { tail -30 "$O/tests.log"; exit 1; }
tail -1 "$O/tests.log"
HM_KIND=skew timeout -k 10 400 python -u tools/variants.py run main git-7574945 main git-7574945 > "$O/skew.jsonl" 2>&1 || { tail -5 "$O/skew.jsonl"; exit 1; }
grep variant "$O/skew.jsonl" | cut -c1-250
timeout -k 10 300 python -u tools/variants.py run main git-7574945 main git-7574945 main git-7574945 > "$O/hot.jsonl" 2>&1 || { tail -5 "$O/hot.jsonl"; exit 1; }
grep variant "$O/hot.jsonl" | cut -c1-250
HM_ZMIN=6 HM_ZMAX=21 timeout -k 10 300 python -u tools/variants.py run main git-7574945 main git-7574945 main git-7574945 > "$O/z621.jsonl" 2>&1 || { tail -5 "$O/z621.jsonl"; exit 1; }
grep variant "$O/z621.jsonl" | cut -c1-250
timeout -k 10 200 python -u tools/bench_stream.py --batches 18 --warmup 2 > "$O/stream.log" 2>&1 || { tail -5 "$O/stream.log"; exit 1; }
tail -1 "$O/stream.log" | cut -c1-160
