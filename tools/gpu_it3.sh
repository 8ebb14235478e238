#!/bin/bash
set -o pipefail
O=gpurun_out/${1:-it3}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_covis_gpu.py tests/test_shard_gpu.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 python3 -u bench.py --no-cpu --steps 3 --warmup 1 --knn-steps 0 --cand-steps 0 > $O/b.log 2>&1 || { tail -20 $O/b.log; exit 1; }
python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(d['ms_per_step'], d['phases_ms'])" $O/b.log
KM_MODE=lloyd timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU --output-format csv -d $O/km -o km -- python3 tools/km_bench.py 12900000 50 5 > $O/km.log 2>&1 || { tail -20 $O/km.log; exit 1; }
python3 tools/pmc_sum.py $O/km/km_counter_collection.csv km_assign
