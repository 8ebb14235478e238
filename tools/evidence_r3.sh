#!/bin/bash
# Round-3 evidence on the box: default bench line, kernel traces (covis+kNN, config 5), PMC traffic
# per co-visitation phase (full builds only: --no-a6 --no-ingest) and per kernel
set -o pipefail
O=gpurun_out/${1:-ev3}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python3 -u bench.py > $O/bench_default.log 2>&1 || { tail -30 $O/bench_default.log; exit 1; }
grep '^{' $O/bench_default.log | tail -1 > $O/bench_default.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu --knn-steps 2 --cand-steps 0 > $O/kt.log 2>&1 || { tail -30 $O/kt.log; exit 1; }
python3 tools/kstats.py $O/kt/run_kernel_stats.csv > $O/kt_summary.txt
rm -f $O/kt/run_kernel_trace.csv
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kc -o run -- python3 bench.py --workload candidates --steps 1 --warmup 1 > $O/kc.log 2>&1 || { tail -30 $O/kc.log; exit 1; }
python3 tools/kstats.py $O/kc/run_kernel_stats.csv > $O/kc_summary.txt
rm -f $O/kc/run_kernel_trace.csv
ARGS="--steps 1 --warmup 0 --no-cpu --no-a6 --no-ingest --knn-steps 1 --cand-steps 0"
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pf -o run -- python3 bench.py $ARGS > $O/pf.log 2>&1 || { tail -30 $O/pf.log; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pw -o run -- python3 bench.py $ARGS > $O/pw.log 2>&1 || { tail -30 $O/pw.log; exit 1; }
python3 tools/pmc_phases.py $O/pf/run_counter_collection.csv $O/pw/run_counter_collection.csv > $O/pmc_traffic.json
cat $O/bench_default.json
head -30 $O/kt_summary.txt
cat $O/pmc_traffic.json
