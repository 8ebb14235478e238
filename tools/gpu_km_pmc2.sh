#!/bin/bash
# counters of the KMeans E-step kernels: lockstep group of 4 and one run at a time (tools/km_group_prof.py)
set -o pipefail
O=gpurun_out/${1:-kmpmc2}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for v in 4 1; do
  OTTOHIP_KM_GROUP=$v timeout -s KILL 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_INSTS_VALU SQ_BUSY_CYCLES --output-format csv -d $O/p$v -o p -- python3 tools/km_group_prof.py 12900000 4 5 > $O/p$v.log 2>&1 || { tail -20 $O/p$v.log; exit 1; }
  echo "group $v"; python3 tools/pmc_sum.py $O/p$v/p_counter_collection.csv km_
done
