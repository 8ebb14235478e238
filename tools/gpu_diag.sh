#!/bin/bash
# Diagnostics: allocation log of the default line, reduce level statistics, config-5 kernel trace
set -o pipefail
O=gpurun_out/${1:-diag}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OTTOHIP_ALLOC_LOG=1 timeout -k 10 600 python3 -u bench.py --no-cpu --steps 2 --warmup 1 > $O/bench_alloc.log 2>&1 || { tail -40 $O/bench_alloc.log; exit 1; }
OTTOHIP_DEBUG=1 timeout -k 10 300 python3 -u bench.py --no-cpu --steps 1 --warmup 0 --knn-steps 0 --cand-steps 0 > $O/reduce_levels.log 2>&1 || { tail -40 $O/reduce_levels.log; exit 1; }
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_cand -o cand -- python3 bench.py --workload candidates --steps 1 --warmup 0 --no-cpu > $O/cand_prof.log 2>&1 || { tail -40 $O/cand_prof.log; exit 1; }
grep -h '"value"' $O/bench_alloc.log | tail -c 3000
