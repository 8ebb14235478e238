#!/bin/bash
# Slot scans at 16 slots per thread (finalize, part heads, rule histograms): covis + merge tests, A6 A/B of the
# in-tree build against otto-recommender_amd/libottohip_ab.so (alternating), then the A6 kernel profile
set -o pipefail
tag=${1:-r4m}
O=gpurun_out/$tag; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_covis_gpu.py tests/test_merge_gpu.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
B=$GRAFT_REPO_ROOT/otto-recommender_amd/libottohip_ab.so
for run in A1 B1 A2 B2; do
  if [ "${run:0:1}" = B ]; then export OTTOHIP_LIB=$B; else unset OTTOHIP_LIB; fi
  timeout -k 10 300 python3 -u bench.py --no-cpu --no-ingest --steps 1 --warmup 0 --knn-steps 0 --cand-steps 0 > "$O/a6_$run.log" 2>&1 || { tail -20 "$O/a6_$run.log"; exit 1; }
  echo "$run"; python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); a=d['a6']; c=a['per_rule']['click_to_click']; print(a['total_ms_runs'], c['stages_ms'])" "$O/a6_$run.log"
done
unset OTTOHIP_LIB
bash tools/gpu_prof_a6.sh ${tag}_prof
