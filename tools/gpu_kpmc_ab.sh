#!/bin/bash
# Per-kernel SQ counters of one co-visitation build, A/B on an env switch (VAR=AV vs VAR=BV):
#   AV=1 BV=0 tools/gpu_kpmc_ab.sh VAR tag "kernel regex"
set -o pipefail
VAR=$1; O=gpurun_out/$2; K=${3:-.}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
B="bench.py --steps 1 --warmup 0 --knn-steps 0 --cand-steps 0 --no-cpu --no-a6 --no-ingest"
for v in A B; do
  if [ $v = A ]; then export $VAR=${AV:-1}; else export $VAR=${BV:-0}; fi
  timeout -s KILL 180 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD --output-format csv -d $O/$v -o run -- python3 $B > $O/$v.log 2>&1 || { tail -20 $O/$v.log; exit 1; }
  timeout -s KILL 180 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS --output-format csv -d $O/${v}2 -o run -- python3 $B > $O/${v}2.log 2>&1 || { tail -20 $O/${v}2.log; exit 1; }
  timeout -s KILL 180 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${v}k -o run -- python3 $B > $O/${v}k.log 2>&1 || { tail -20 $O/${v}k.log; exit 1; }
done
python3 - "$O" "$K" <<'PY'
import csv, re, sys
from collections import defaultdict
O, K = sys.argv[1], sys.argv[2]
for v in "AB":
    agg = defaultdict(lambda: defaultdict(float)); t = defaultdict(float)
    for f in (v, v + "2"):
        for r in csv.DictReader(open(f"{O}/{f}/run_counter_collection.csv")):
            agg[r["Kernel_Name"].split("(")[0]][r["Counter_Name"]] += float(r["Counter_Value"])
    for r in csv.DictReader(open(f"{O}/{v}k/run_kernel_trace.csv")):
        t[r["Kernel_Name"].split("(")[0]] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
    for k in sorted(agg):
        if re.search(K, k):
            print(v, k[-60:], "ms %.3f" % t.get(k, 0), {c: "%.4g" % x for c, x in sorted(agg[k].items())})
PY
