#!/bin/bash
# window searches bracketed by the event's own position (emit + prep_count): covis tests, then lib A/B against
# the build without the brackets (otto-recommender_amd/libottohip_ab.so)
set -o pipefail
tag=${1:-r4l}
O=gpurun_out/$tag; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_covis_gpu.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
bash tools/gpu_ab.sh ${tag}_ab || exit 1
