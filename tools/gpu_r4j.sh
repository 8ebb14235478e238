#!/bin/bash
# A6: boundary files counted together, wave-aggregated tie histograms: part / cut / merge tests, the 220 M
# digest + A6 test, then the A6 kernel profile with per-stage times
set -o pipefail
tag=${1:-r4j}
O=gpurun_out/$tag; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_covis_gpu.py tests/test_merge_gpu.py -k "part or cuts or file_flow or finalize or full_220m" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
bash tools/gpu_prof_a6.sh ${tag}_prof
