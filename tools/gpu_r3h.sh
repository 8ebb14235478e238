#!/bin/bash
# kernel statistics of the config-5 sub-benchmark with the KMeans bounds on
set -o pipefail
O=gpurun_out/${1:-r3h}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kc -o run -- python3 bench.py --workload candidates --steps 1 --warmup 0 > $O/kc.log 2>&1 || { tail -30 $O/kc.log; exit 1; }
python3 tools/kstats.py $O/kc/run_kernel_stats.csv > $O/kc_summary.txt
rm -f $O/kc/run_kernel_trace.csv
grep "k_km" $O/kc_summary.txt
