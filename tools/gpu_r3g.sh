#!/bin/bash
# grouped KMeans bounds: KMeans GPU tests, rows scored per step, config-5 sub-benchmark without / with bounds
set -o pipefail
O=gpurun_out/${1:-r3g}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_popularity_gpu.py tests/test_pipeline_gpu.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
OTTOHIP_KM_BDBG=1 timeout -k 10 400 python3 -u bench.py --workload candidates --steps 1 --warmup 0 > $O/kmdbg.log 2>&1 || { tail -20 $O/kmdbg.log; exit 1; }
grep -a "kmeans bounds" $O/kmdbg.log | awk 'NR%12==1' | head -30
for v in 0 1; do
  OTTOHIP_KM_BOUNDS=$v timeout -k 10 400 python3 -u bench.py --workload candidates --steps 1 --warmup 1 > $O/cand$v.log 2>&1 || { tail -20 $O/cand$v.log; exit 1; }
  echo "bounds=$v $(grep '^{' $O/cand$v.log | tail -1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); c=d.get("candidates",d); print(round(c["ms_per_step"],1), c["stages_s"]["C2_kmeans"], c["outside_stages_s"], c["recall@20"]["total"], c["recall_topall"]["total"])')"
done
