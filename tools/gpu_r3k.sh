#!/bin/bash
# XCD-aware offset scatter: covis tests, same-box A/B, WRITE_SIZE of the scatter
set -o pipefail
O=gpurun_out/${1:-r3k}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_envab.sh ${1:-r3k}_ab OTTOHIP_POFF_XCD 0 1 tests/test_covis_gpu.py || exit 1
B="bench.py --steps 1 --warmup 0 --knn-steps 0 --cand-steps 0 --no-cpu --no-a6 --no-ingest"
timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/w -o run -- python3 $B > $O/w.log 2>&1 || exit 1
python3 - $O/w/run_counter_collection.csv <<'PY'
import csv, sys, collections
t = collections.defaultdict(float); n = collections.Counter()
for r in csv.DictReader(open(sys.argv[1])):
    k = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("ottohip::", "")
    if "poff" in k or "rows_tile" in k:
        t[k] += float(r["Counter_Value"]); n[k] += 1
for k in t: print(k, n[k], round(t[k] / 1e9, 3), "GB (KiB units per the counter: x1024 -> bytes if so)")
PY
