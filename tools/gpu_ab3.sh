#!/bin/bash
# Same-box A/B on the covis line: B = otto-recommender_amd/libottohip_ab.so, A = in-tree (optionally
# with env settings per variant): tools/gpu_ab3.sh <tag> "<variants>" [pytest args...]
#   variants: space-separated list of  B | A | A:VAR=val,VAR2=val
set -o pipefail
tag=$1; variants=$2; shift 2
O=gpurun_out/$tag; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
if [ $# -gt 0 ]; then
  timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread "$@" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
  tail -1 $O/pytest.log
fi
i=0
for v in $variants; do
  i=$((i+1))
  (
    if [ "${v:0:1}" = B ]; then export OTTOHIP_LIB=$GRAFT_REPO_ROOT/otto-recommender_amd/libottohip_ab.so; fi
    if [ "${v:1:1}" = : ]; then for kv in $(echo "${v:2}" | tr ',' ' '); do export "$kv"; done; fi
    timeout -k 10 300 python3 -u bench.py --no-cpu --no-a6 --no-ingest --steps 5 --warmup 2 --knn-steps 0 --cand-steps 0 > "$O/b_$i.log" 2>&1
  ) || { tail -20 "$O/b_$i.log"; exit 1; }
  echo "$v $(python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(round(d['ms_per_step'],2), d['phases_ms'])" "$O/b_$i.log")"
done
