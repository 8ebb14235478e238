#!/bin/bash
set -o pipefail
O=gpurun_out/$1
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_popularity_gpu.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
KM_MODE=partial timeout -k 10 120 python3 tools/km_bench.py 2>&1 | grep -v amdgpu.ids || exit 1
KM_MODE=partial OTTOHIP_KM_VALU=1 timeout -k 10 120 python3 tools/km_bench.py 2>&1 | grep -v amdgpu.ids || exit 1
KM_MODE=partial timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_VMEM_RD --output-format csv -d $O/pm -o run -- python3 tools/km_bench.py 12900000 50 3 > $O/pm.log 2>&1 || exit 1
