#!/bin/bash
# rows phase A/B: parity tests with OTTOHIP_ROWS=atomic, then same-box step timings atomic vs sorted rows
set -o pipefail
O=gpurun_out/${1:-rowsab}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OTTOHIP_ROWS=atomic timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_covis_gpu.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
bash tools/gpu_envab.sh ${1:-rowsab}_ab OTTOHIP_ROWS atomic fused
