#!/bin/bash
# kept-words part re-fold tests, KMeans range / bounds, emit clamp cost A/B, per-file statistics cost (kernel stats),
# the A6 with the re-fold
set -o pipefail
tag=${1:-r5d}
O=gpurun_out/$tag; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T="python -u -m pytest -x -q --timeout-method thread"
timeout -k 10 600 $T --timeout 300 tests/test_covis_gpu.py tests/test_popularity_gpu.py -k "kept or part_branch or file_cuts or kat or golden or guard or half_rows or split_precision" > $O/p1.log 2>&1 || { tail -50 $O/p1.log; exit 1; }
tail -2 $O/p1.log
OTTOHIP_BENCH_PER_FILE=none bash tools/gpu_ab.sh ${tag}_ab || exit 1
for pf in none click_to_click; do
  OTTOHIP_BENCH_PER_FILE=$pf timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$pf -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu --knn-steps 0 --cand-steps 0 --no-ingest --no-a6 > $O/prof_$pf.log 2>&1 || { tail -20 $O/prof_$pf.log; exit 1; }
done
for pf in none click_to_click; do f=$(find $O/prof_$pf -name "*kernel_stats.csv" | head -1); echo "== $pf"; python3 tools/kstats.py "$f" | head -24; done
timeout -k 10 400 python3 -u bench.py --steps 5 --warmup 2 --no-cpu --knn-steps 0 --cand-steps 0 --no-ingest > $O/bench.log 2>&1 || { tail -c 3000 $O/bench.log; exit 1; }
python3 -c "import json;d=json.loads(open('$O/bench.log').read().strip().splitlines()[-1]);print(d['ms_per_step'],d['phases_ms'],d.get('a6',{}).get('total_ms'),d.get('a6',{}).get('per_rule',{}).get('click_to_click',{}).get('stages_ms'))"
