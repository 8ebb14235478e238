#!/bin/bash
# KMeans large-magnitude determinism probe; symmetric sharded storage tests; emit-check cost A/B (lib B = no check);
# configs[3] at full size with symmetric storage
set -o pipefail
tag=${1:-r5b}
O=gpurun_out/$tag; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 180 python -u tools/dbg/km_range2.py > $O/km.log 2>&1; cat $O/km.log
OTTOHIP_BENCH_PER_FILE=none bash tools/gpu_ab.sh ${tag}_ab tests/test_covis_gpu.py tests/test_merge_gpu.py tests/test_shard_gpu.py tests/test_dist_gpu.py -k "not full_size and not full_220m" || exit 1
bash tools/gpu_envab.sh ${tag}_pf OTTOHIP_BENCH_PER_FILE none click_to_click || exit 1
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 880 --timeout-method thread tests/test_dist_gpu.py -k full_size > $O/p3.log 2>&1 || { tail -60 $O/p3.log; exit 1; }
tail -5 $O/p3.log
