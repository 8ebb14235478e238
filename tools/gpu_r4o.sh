#!/bin/bash
# merge big-key extraction (two searches per block): shard tests; then split bucket mean A/Bs on the covis step
set -o pipefail
tag=${1:-r4o}
O=gpurun_out/$tag; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_shard_gpu.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
bash tools/gpu_envab.sh ${tag}_sm200 OTTOHIP_SPLIT_MEAN 420 200 || exit 1
bash tools/gpu_envab.sh ${tag}_sm120 OTTOHIP_SPLIT_MEAN 420 120 || exit 1
timeout -k 10 60 ./tools/mb/mfma_mb
