#!/bin/bash
# kNN candidate buffers + KMeans lockstep pairs: their tests, then same-box A/Bs of the kNN search and of
# the config-5 step (env switches OTTOHIP_KNN_BUF / OTTOHIP_KM_PAIR)
set -o pipefail
O=gpurun_out/${1:-r4g}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_knn.py tests/test_popularity_gpu.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for v in 1 0; do
  OTTOHIP_KNN_BUF=$v timeout -k 10 300 python3 -u bench.py --workload knn --no-cpu --knn-steps 2 > $O/knn_$v.log 2>&1 || { tail -20 $O/knn_$v.log; exit 1; }
  echo "KNN_BUF=$v"; python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); k=d.get('knn',d); print(k['phases_ms'], k['roofline']['frac'])" $O/knn_$v.log
done
for v in 1 0; do
  OTTOHIP_KM_PAIR=$v timeout -k 10 400 python3 -u bench.py --workload candidates --no-cpu --steps 1 > $O/cand_$v.log 2>&1 || { tail -20 $O/cand_$v.log; exit 1; }
  echo "KM_PAIR=$v"; python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); c=d.get('candidates',d); print(c['ms_per_step'], c['stages_s'], c['recall@20'])" $O/cand_$v.log
done
