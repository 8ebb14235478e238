#!/bin/bash
# Kernel traces of the A6 merge: one bench with A6 (1 build + A6 warmup + 3 timed A6 passes) and one without;
# tools/kdb.py prints the per-kernel difference (the A6 kernels) per A6 pass
set -o pipefail
O=gpurun_out/${1:-r4_a6prof}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/with -o run -- python3 -u bench.py --no-cpu --no-ingest --steps 1 --warmup 0 --knn-steps 0 --cand-steps 0 > $O/with.log 2>&1 || { tail -20 $O/with.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/without -o run -- python3 -u bench.py --no-cpu --no-ingest --no-a6 --steps 1 --warmup 0 --knn-steps 0 --cand-steps 0 > $O/without.log 2>&1 || { tail -20 $O/without.log; exit 1; }
a=$(find $O/with -name "*results.db" | head -1); b=$(find $O/without -name "*results.db" | head -1)
python3 tools/kdb.py "$a" "$b" 4 | head -40
echo "---- one build (the --no-a6 run: 1 build)"
python3 tools/kdb.py "$b" | head -30
grep '^{' $O/with.log | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['a6']['per_rule']['click_to_click'])"
