#!/bin/bash
set -o pipefail
O=gpurun_out/${1:-it4}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_popularity_gpu.py tests/test_pipeline_gpu.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
KM_MODE=lloyd timeout -k 10 120 python3 tools/km_bench.py 12900000 50 20
OTTOHIP_ALLOC_LOG=1 timeout -k 10 400 python3 -u bench.py --workload candidates --steps 1 > $O/cand.log 2>&1 || { tail -20 $O/cand.log; exit 1; }
grep '^{' $O/cand.log | tail -c 1500
