#!/bin/bash
# Split-precision vs exact Lloyd E-steps: KMeans GPU tests, then the config-5 sub-benchmark with each setting
set -o pipefail
O=gpurun_out/${1:-abkm}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_popularity_gpu.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for v in 0 1; do
  OTTOHIP_KM_SPLIT=$([ $v = 0 ] && echo 0 || echo 1) timeout -k 10 400 python3 -u bench.py --workload candidates --steps 1 --warmup 1 > $O/cand$v.log 2>&1 || { tail -20 $O/cand$v.log; exit 1; }
  echo "v=$v (0 exact, 1 split) $(grep '^{' $O/cand$v.log | tail -1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); c=d.get("candidates",d); print(round(c["ms_per_step"],1), c["stages_s"]["C2_kmeans"], c["recall@20"], c["recall_topall"]["total"])')"
done
