#!/bin/bash
# LDS counters per kernel of one co-visitation build (bench --steps 1 --no-a6 --knn-steps 0 --cand-steps 0)
set -o pipefail
O=gpurun_out/${1:-ldspmc}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -s KILL 240 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_WAVES SQ_INSTS_VALU --output-format csv -d $O/p -o run -- python3 bench.py --no-cpu --no-a6 --no-ingest --steps 1 --warmup 0 --knn-steps 0 --cand-steps 0 > $O/p.log 2>&1 || { tail -20 $O/p.log; exit 1; }
ls $O/p
