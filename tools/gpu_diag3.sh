#!/bin/bash
# Reduce diagnostics on the box: per-level task lists and the per-task LDS-hash profile of one
# 220 M build, plus a kernel trace (timeline) of one covis step
set -o pipefail
O=gpurun_out/${1:-diag3}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
ARGS="--steps 1 --warmup 0 --no-cpu --no-a6 --no-ingest --knn-steps 0 --cand-steps 0"
OTTOHIP_DEBUG=1 OTTOHIP_HASH_PROF=1 timeout -k 10 300 python3 -u bench.py $ARGS > $O/dbg.log 2>&1 || { tail -30 $O/dbg.log; exit 1; }
grep -a "level\|hash" $O/dbg.log | head -60
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/kt -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu --no-a6 --no-ingest --knn-steps 0 --cand-steps 0 > $O/kt.log 2>&1 || { tail -30 $O/kt.log; exit 1; }
python3 tools/timeline.py $O/kt/run_kernel_trace.csv > $O/timeline.txt
rm -f $O/kt/run_kernel_trace.csv
tail -80 $O/timeline.txt
