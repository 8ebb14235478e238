#!/bin/bash
# kernel profile of the A6 stage: the part table re-folded from the kept words vs recounted (OTTOHIP_A6_REFOLD=0)
set -o pipefail
tag=${1:-r5e}
O=gpurun_out/$tag; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for rf in 1 0; do
  OTTOHIP_A6_REFOLD=$rf timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_rf$rf -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu --knn-steps 0 --cand-steps 0 --no-ingest > $O/prof_rf$rf.log 2>&1 || { tail -20 $O/prof_rf$rf.log; exit 1; }
  f=$(find $O/prof_rf$rf -name "*kernel_stats.csv" | head -1); echo "== refold $rf"; python3 tools/kstats.py "$f" | head -40
  python3 -c "import json;d=json.loads([l for l in open('$O/prof_rf$rf.log') if l.startswith('{')][-1]);a=d['a6'];print(a['total_ms'], a['count_ms'], a['per_rule']['click_to_click']['stages_ms'])"
done
