#!/bin/bash
set -o pipefail
O=gpurun_out/r2l
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
B="bench.py --steps 1 --warmup 0 --knn-steps 0 --cand-steps 0 --no-cpu"
timeout -s KILL 180 rocprofv3 --pmc SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_WAVES SQ_INSTS_BRANCH SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d $O/a -o run -- python3 $B > $O/a.log 2>&1 || exit 1
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/f -o run -- python3 $B > $O/f.log 2>&1 || exit 1
timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/w -o run -- python3 $B > $O/w.log 2>&1 || exit 1
