#!/bin/bash
# Round-2 refresh after the ingest row: default bench line + covis/kNN kernel trace (config-5 trace and
# PMC passes unchanged: tools/evidence_r2.sh)
set -o pipefail
O=gpurun_out/${1:-ev2b}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 700 python3 -u bench.py > $O/bench_default.log 2>&1 || { tail -30 $O/bench_default.log; exit 1; }
grep '^{' $O/bench_default.log | tail -1 > $O/bench_default.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu --knn-steps 2 --cand-steps 0 > $O/kt.log 2>&1 || { tail -30 $O/kt.log; exit 1; }
python3 tools/kstats.py $O/kt/run_kernel_stats.csv > $O/kt_summary.txt
rm -f $O/kt/run_kernel_trace.csv
head -40 $O/kt_summary.txt
