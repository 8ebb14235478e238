#!/bin/bash
# PMC traffic per co-visitation phase from full 220 M-event builds only (no A6 part recounts, no ingest
# timing in the profiled run): two separate --pmc passes, then tools/pmc_phases.py
set -o pipefail
O=gpurun_out/${1:-pmc2b}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
ARGS="--steps 1 --warmup 0 --no-cpu --no-a6 --no-ingest --knn-steps 1 --cand-steps 0"
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pf -o run -- python3 bench.py $ARGS > $O/pf.log 2>&1 || { tail -30 $O/pf.log; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pw -o run -- python3 bench.py $ARGS > $O/pw.log 2>&1 || { tail -30 $O/pw.log; exit 1; }
python3 tools/pmc_phases.py $O/pf/run_counter_collection.csv $O/pw/run_counter_collection.csv > $O/pmc_traffic.json
python3 tools/kpmc_table.py $O/pf/run_counter_collection.csv $O/pw/run_counter_collection.csv > $O/pmc_per_kernel.txt 2>/dev/null || true
cat $O/pmc_traffic.json
