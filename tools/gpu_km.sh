#!/bin/bash
set -o pipefail
O=gpurun_out/${1:-km}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
KM_MODE=lloyd timeout -k 10 120 python3 tools/km_bench.py 12900000 50 20
KM_MODE=assign timeout -k 10 120 python3 tools/km_bench.py 12900000 50 20
KM_MODE=lloyd timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_INSTS_VALU SQ_WAIT_INST_LDS --output-format csv -d $O/km -o km -- python3 tools/km_bench.py 12900000 50 5 > $O/km.log 2>&1 || { tail -20 $O/km.log; exit 1; }
python3 tools/pmc_sum.py $O/km/km_counter_collection.csv km_assign
