#!/bin/bash
# KMeans / pipeline / 2-rank tests, then the config-5 bench (C2 stage and recall)
set -o pipefail
O=gpurun_out/${1:-kmb}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_popularity_gpu.py tests/test_pipeline_gpu.py tests/test_dist_gpu.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 400 python3 -u bench.py --workload candidates --steps 2 > $O/c.log 2>&1 || { tail -20 $O/c.log; exit 1; }
python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); s=d['stages_s']; print(round(d['ms_per_step'],1), s['C2_kmeans'], d['recall@20'])" $O/c.log
