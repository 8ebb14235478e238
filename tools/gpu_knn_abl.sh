#!/bin/bash
set -o pipefail
O=gpurun_out/${1:-knnabl}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for a in ${ABLS:-0 1 3}; do
  OTTOHIP_KNN_ABLATE=$a timeout -s KILL 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_INSTS_VALU SQ_WAIT_INST_LDS --output-format csv -d $O/p$a -o p -- python3 bench.py --workload knn --steps 1 --warmup 0 --no-cpu > $O/p$a.log 2>&1 || { tail -20 $O/p$a.log; exit 1; }
  echo "ABL=$a"; python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(d['phases_ms'])" $O/p$a.log
  python3 tools/pmc_sum.py $O/p$a/p_counter_collection.csv "knn_main<$a>"
done
