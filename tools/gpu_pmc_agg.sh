#!/bin/bash
# SQ counters of the reduce kernels, register sort vs wave hash (one covis build each)
set -o pipefail
O=gpurun_out/r2i
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
C="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU"
B="bench.py --steps 1 --warmup 0 --knn-steps 0 --cand-steps 0 --no-cpu"
OTTOHIP_AGG=sort timeout -s KILL 180 rocprofv3 --pmc $C --output-format csv -d $O/sort -o run -- python3 $B > $O/sort.log 2>&1 || exit 1
timeout -s KILL 240 rocprofv3 --pmc $C --output-format csv -d $O/whash -o run -- python3 $B > $O/whash.log 2>&1 || exit 1
ls -R $O | head -20
