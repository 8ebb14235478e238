#!/bin/bash
# KMeans bounds A/B: KMeans GPU tests, then per setting the config-5 sub-benchmark and its kernel trace
set -o pipefail
O=gpurun_out/${1:-kmb3}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_popularity_gpu.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for v in 0 1; do
  OTTOHIP_KM_BOUNDS=$v timeout -k 10 400 python3 -u bench.py --workload candidates --steps 1 --warmup 1 > $O/cand$v.log 2>&1 || { tail -20 $O/cand$v.log; exit 1; }
  echo "bounds=$v $(grep '^{' $O/cand$v.log | tail -1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); c=d.get("candidates",d); print(round(c["ms_per_step"],1), c["stages_s"]["C2_kmeans"], c["recall@20"]["total"], c["recall_topall"]["total"])')"
  OTTOHIP_KM_BOUNDS=$v timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kc$v -o run -- python3 bench.py --workload candidates --steps 1 --warmup 0 > $O/kc$v.log 2>&1 || { tail -30 $O/kc$v.log; exit 1; }
  python3 tools/kstats.py $O/kc$v/run_kernel_stats.csv > $O/kc${v}_summary.txt
  rm -f $O/kc$v/run_kernel_trace.csv
  grep "k_km" $O/kc${v}_summary.txt
done
