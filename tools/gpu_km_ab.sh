#!/bin/bash
# KMeans tests + same-box A/B of the Lloyd step (A = in-tree lib, B = libottohip_ab.so)
set -o pipefail
O=gpurun_out/${1:-kmab}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_popularity_gpu.py tests/test_pipeline_gpu.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
B=$GRAFT_REPO_ROOT/otto-recommender_amd/libottohip_ab.so
for run in A1 B1 A2 B2; do
  if [ "${run:0:1}" = B ]; then export OTTOHIP_LIB=$B; else unset OTTOHIP_LIB; fi
  KM_MODE=lloyd timeout -k 10 200 python3 tools/km_bench.py 12900000 50 40 > $O/$run.log 2>&1 || { tail -20 $O/$run.log; exit 1; }
  echo "$run $(tail -1 $O/$run.log)"
done
