#!/bin/bash
# Round-3 final evidence: pipeline / KMeans GPU tests, default bench line, kernel traces (covis+kNN, config 5),
# PMC traffic per co-visitation phase (full builds only)
set -o pipefail
O=gpurun_out/${1:-ev3f}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_popularity_gpu.py tests/test_pipeline_gpu.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
tools/evidence_r3.sh ${1:-ev3f}
