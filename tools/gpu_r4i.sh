#!/bin/bash
# emit flush with two pairs per lane: the record-guard test first (OTTOHIP_DEBUG bounds checks), then the covis /
# shard / dist tests, then OTTOHIP_EMIT_FLUSH2 1 / 0
set -o pipefail
tag=${1:-r4i}
O=gpurun_out/$tag; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_covis_gpu.py -k "guard or kat or golden" > $O/pytest0.log 2>&1 || { tail -40 $O/pytest0.log; exit 1; }
tail -1 $O/pytest0.log
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_covis_gpu.py tests/test_shard_gpu.py tests/test_dist_gpu.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
bash tools/gpu_envab.sh ${tag}_fl2 OTTOHIP_EMIT_FLUSH2 1 0 || exit 1
