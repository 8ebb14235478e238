#!/bin/bash
# kernel trace + stats of the config-5 step (bench --workload candidates, 1 warmup + 1 timed step)
set -o pipefail
O=gpurun_out/${1:-candprof}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/k -o run -- python3 -u bench.py --workload candidates --steps 1 > $O/k.log 2>&1 || { tail -20 $O/k.log; exit 1; }
python3 tools/kstats.py $O/k/run_kernel_stats.csv > $O/summary.txt; head -30 $O/summary.txt
