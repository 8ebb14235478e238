#!/bin/bash
# KMeans Lloyd step counters (tools/km_bench.py, KM_MODE=lloyd, 12.9 M x 100, k = 50)
set -o pipefail
O=gpurun_out/${1:-kmpmc}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
KM_MODE=lloyd timeout -s KILL 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_INSTS_VALU SQ_BUSY_CYCLES --output-format csv -d $O/p -o p -- python3 tools/km_bench.py 12900000 50 30 > $O/p.log 2>&1 || { tail -20 $O/p.log; exit 1; }
python3 tools/pmc_sum.py $O/p/p_counter_collection.csv km_
timeout -s KILL 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/k -o k -- python3 tools/km_bench.py 12900000 50 30 > $O/k.log 2>&1 || { tail -20 $O/k.log; exit 1; }
python3 tools/kstats.py $O/k/k_kernel_stats.csv | head -12
