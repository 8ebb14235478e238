#!/bin/bash
# candidate tests + same-box A/B of the config-5 step (A = in-tree lib, B = libottohip_ab.so)
set -o pipefail
O=gpurun_out/${1:-candab}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_candidates_gpu.py tests/test_pipeline_gpu.py tests/test_popularity_gpu.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
B=$GRAFT_REPO_ROOT/otto-recommender_amd/libottohip_ab.so
for run in A1 B1 A2 B2; do
  if [ "${run:0:1}" = B ]; then export OTTOHIP_LIB=$B; else unset OTTOHIP_LIB; fi
  timeout -k 10 400 python3 -u bench.py --workload candidates --steps 2 > $O/$run.log 2>&1 || { tail -20 $O/$run.log; exit 1; }
  echo "$run"; python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); s=d['stages_s']; print(round(d['ms_per_step'],1), {k: s[k] for k in ('C2_kmeans','candidates','knn','merge_click_to_click')})" $O/$run.log
done
