#!/bin/bash
# KMeans bounds diagnostics: rows scored per step, and a kernel trace of the config-5 sub-benchmark
set -o pipefail
O=gpurun_out/${1:-kmb2}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OTTOHIP_KM_BDBG=1 timeout -k 10 400 python3 -u bench.py --workload candidates --steps 1 --warmup 0 > $O/dbg.log 2>&1 || { tail -20 $O/dbg.log; exit 1; }
grep -a "kmeans bounds" $O/dbg.log | head -120
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kc -o run -- python3 bench.py --workload candidates --steps 1 --warmup 0 > $O/kc.log 2>&1 || { tail -30 $O/kc.log; exit 1; }
python3 tools/kstats.py $O/kc/run_kernel_stats.csv > $O/kc_summary.txt
rm -f $O/kc/run_kernel_trace.csv
head -25 $O/kc_summary.txt
