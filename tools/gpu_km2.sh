#!/bin/bash
set -o pipefail
O=gpurun_out/${1:-km2}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_popularity_gpu.py tests/test_pipeline_gpu.py tests/test_dist_gpu.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 400 python3 -u bench.py --workload candidates --steps 1 > $O/cand.log 2>&1 || { tail -20 $O/cand.log; exit 1; }
python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(d['value'], d['ms_per_step'], d['stages_s'], d['config'])" $O/cand.log
