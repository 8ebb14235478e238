#!/bin/bash
# every -m gpu test with the new defaults, then emit A/B (in-tree vs libottohip_ab.so)
set -o pipefail
O=gpurun_out/${1:-r3f}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
tools/gpu_libab.sh ${1:-r3f}_lib || exit 1
