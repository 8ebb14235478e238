#!/bin/bash
# config-5 run with the library's allocation log (OTTOHIP_ALLOC_LOG=1): which device allocations of the timed
# step still reach hipMalloc, and their cost
set -o pipefail
O=gpurun_out/${1:-candalloc}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OTTOHIP_ALLOC_LOG=1 timeout -k 10 400 python3 -u bench.py --no-cpu --no-a6 --no-ingest --steps 1 --warmup 0 --knn-steps 0 > $O/c.log 2> $O/alloc.log || { tail -20 $O/alloc.log; exit 1; }
grep -c "ottohip alloc" $O/alloc.log
