#!/bin/bash
# Same-box A/B of two builds of libottohip (A = in-tree, B = otto-recommender_amd/libottohip_ab.so) on the
# co-visitation step (alternating A B A B, no A6 / kNN / candidates), then one A run with A6 and
# OTTOHIP_ALLOC_LOG=1:  tools/gpu_ab.sh <tag> [pytest files...]
set -o pipefail
tag=$1; shift
O=gpurun_out/$tag; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
if [ $# -gt 0 ]; then
  timeout -k 10 900 python -u -m pytest -x -q --timeout 450 --timeout-method thread "$@" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
  tail -1 $O/pytest.log
fi
B=$GRAFT_REPO_ROOT/otto-recommender_amd/libottohip_ab.so
for run in A1 B1 A2 B2; do
  if [ "${run:0:1}" = B ]; then export OTTOHIP_LIB=$B; else unset OTTOHIP_LIB; fi
  timeout -k 10 300 python3 -u bench.py --no-cpu --no-a6 --no-ingest --steps 5 --warmup 1 --knn-steps 0 --cand-steps 0 > "$O/b_$run.log" 2>&1 || { tail -20 "$O/b_$run.log"; exit 1; }
  echo "$run"; python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(round(d['ms_per_step'],2), d['phases_ms'])" "$O/b_$run.log"
done
unset OTTOHIP_LIB
OTTOHIP_ALLOC_LOG=1 timeout -k 10 300 python3 -u bench.py --no-cpu --no-ingest --steps 3 --warmup 1 --knn-steps 0 --cand-steps 0 > "$O/b_a6.log" 2>&1 || { tail -20 "$O/b_a6.log"; exit 1; }
python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); a=d['a6']; print(a['total_ms_runs'], a.get('warmup_ms'), a['per_rule']['click_to_click'])" "$O/b_a6.log"
