#!/bin/bash
# emit LDS union: covis / merge / shard tests, then A/B in-tree (union) vs libottohip_ab.so (union + 5 waves/EU)
set -o pipefail
O=gpurun_out/${1:-r3i}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_libab.sh ${1:-r3i}_lib tests/test_covis_gpu.py tests/test_merge_gpu.py tests/test_shard_gpu.py || exit 1
