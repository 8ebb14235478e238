#!/bin/bash
# LDS / VALU counters per kernel of a bench run with A6 (1 build + 4 A6 passes)
set -o pipefail
O=gpurun_out/${1:-a6lds}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -s KILL 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_WAVES SQ_INSTS_VALU --output-format csv -d $O/p -o run -- python3 bench.py --no-cpu --no-ingest --steps 1 --warmup 0 --knn-steps 0 --cand-steps 0 > $O/p.log 2>&1 || { tail -20 $O/p.log; exit 1; }
ls $O/p
