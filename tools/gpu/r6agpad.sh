#!/bin/bash
# k_aggregate histogram row padding 4 words (agpad4) against 8 (main):
# hotspot and z6-21 timing, then SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE of
# k_aggregate for both (one pass each, hotspots z0-18).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
cd "$R"
O="$R/gpurun_out/${1:-r6agpad}"
mkdir -p "$O"
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_buckets.py tests/test_gpu_smoke.py > "$O/tests.log" 2>&1 || true
tail -1 "$O/tests.log"
timeout -k 10 300 python -u tools/variants.py run main agpad4 main agpad4 > "$O/hot.jsonl" 2>&1 || { tail -5 "$O/hot.jsonl"; exit 1; }
grep variant "$O/hot.jsonl" | cut -c1-250
HM_ZMIN=6 HM_ZMAX=21 timeout -k 10 300 python -u tools/variants.py run main agpad4 main agpad4 > "$O/z621.jsonl" 2>&1 || { tail -5 "$O/z621.jsonl"; exit 1; }
grep variant "$O/z621.jsonl" | cut -c1-250
cd /tmp
for v in main agpad4; do
  HM_STEPS=1 timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE -f csv -d "$O/pmc_$v" -o run -- python3 "$R/tools/variants.py" one $v > "$O/pmc_$v.log" 2>&1 || { tail -20 "$O/pmc_$v.log"; exit 1; }
done
python3 - "$O" <<'PY'
import csv, glob, os, sys
from collections import defaultdict
for v in ("main", "agpad4"):
    f = glob.glob(os.path.join(sys.argv[1], "pmc_" + v, "**", "*counter_collection.csv"), recursive=True)[0]
    t = defaultdict(float)
    for r in csv.DictReader(open(f)):
        if r["Kernel_Name"].startswith("k_aggregate("):
            t[r["Counter_Name"]] += float(r["Counter_Value"])
    print(v, "k_aggregate LDS bank conflict / LDS active = %.3f" % (t["SQ_LDS_BANK_CONFLICT"] / max(t["SQ_LDS_IDX_ACTIVE"], 1)), dict(t))
PY
