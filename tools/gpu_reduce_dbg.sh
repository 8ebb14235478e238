#!/bin/bash
# reduce level / task-list statistics of one build (OTTOHIP_DEBUG=1: lists per level; OTTOHIP_HASH_PROF=1 with
# OTTOHIP_HASH_FIRST=0: the hash leaves' per-task times)
set -o pipefail
O=gpurun_out/${1:-rdbg}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OTTOHIP_DEBUG=1 OTTOHIP_HASH_FIRST=0 OTTOHIP_HASH_PROF=1 timeout -k 10 300 python3 -u bench.py --no-cpu --no-a6 --no-ingest --steps 1 --warmup 0 --knn-steps 0 --cand-steps 0 > $O/b.log 2> $O/err.log || { tail -20 $O/err.log; exit 1; }
grep -E "level|hash level|P=" $O/err.log | head -60
