#!/bin/bash
# LDS leaf of the reduce: its tests, a same-box A/B of the covis step (OTTOHIP_LDS_LEAF 1 / 0), the level
# listing of one build with the leaf on, then the 220 M digest + A6 test with the leaf on
set -o pipefail
O=gpurun_out/${1:-r4h}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_reduce_lds_gpu.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
bash tools/gpu_envab.sh ${1:-r4h}_ab OTTOHIP_LDS_LEAF 1 0 || exit 1
OTTOHIP_LDS_LEAF=1 OTTOHIP_DEBUG=1 timeout -k 10 300 python3 -u bench.py --no-cpu --no-a6 --no-ingest --steps 1 --warmup 0 --knn-steps 0 --cand-steps 0 > $O/dbg.log 2>&1 || { tail -20 $O/dbg.log; exit 1; }
grep "level" $O/dbg.log | head -24
OTTOHIP_LDS_LEAF=1 timeout -k 10 900 python -u -m pytest -x -q --timeout 800 --timeout-method thread tests/test_covis_gpu.py -k full_220m > $O/full.log 2>&1 || { tail -30 $O/full.log; exit 1; }
tail -1 $O/full.log
