#!/bin/bash
# the new KMeans bounds test, then the per-kernel PMC table of one co-visitation build
set -o pipefail
O=gpurun_out/${1:-r3j}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_popularity_gpu.py -k "invalidated or bounded" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
tools/gpu_pmc_r3.sh ${1:-r3j}_pmc > /dev/null 2>&1 || { echo pmc failed; exit 1; }
head -30 gpurun_out/${1:-r3j}_pmc/pmc_per_kernel.txt
