#!/bin/bash
set -o pipefail
O=gpurun_out/${1:-knn}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest -x -q --timeout 250 --timeout-method thread tests/test_knn.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python3 -u bench.py --workload knn --steps 2 --no-cpu > $O/b.log 2>&1 || { tail -20 $O/b.log; exit 1; }
python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(d['value'], d['phases_ms'], d['roofline']['frac'])" $O/b.log
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_INSTS_VALU SQ_WAIT_INST_LDS --output-format csv -d $O/p -o p -- python3 bench.py --workload knn --steps 1 --warmup 0 --no-cpu > $O/p.log 2>&1 || { tail -20 $O/p.log; exit 1; }
python3 tools/pmc_sum.py $O/p/p_counter_collection.csv knn
