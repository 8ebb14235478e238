#!/bin/bash
# kernel trace of the config-5 sub-benchmark with split-precision / exact E-steps
set -o pipefail
O=gpurun_out/${1:-profkm}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for v in 0 1; do
  OTTOHIP_KM_SPLIT=$v timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/k$v -o run -- python3 bench.py --workload candidates --steps 1 --warmup 0 > $O/k$v.log 2>&1 || { tail -20 $O/k$v.log; exit 1; }
  python3 tools/kstats.py $O/k$v/run_kernel_stats.csv > $O/k${v}_summary.txt
  rm -f $O/k$v/run_kernel_trace.csv
  echo "split=$v"; grep -E "k_km_|k_knn_main|k_cand" $O/k${v}_summary.txt | head -12
done
