#!/bin/bash
# the co-visitation build under several environment settings (same box, each run twice in rotation):
#   tools/gpu_covis_multi.sh <tag> "A=1,B=2" "A=0" ... [-- pytest args]
set -o pipefail
tag=$1; shift
specs=(); while [ $# -gt 0 ] && [ "$1" != "--" ]; do specs+=("$1"); shift; done
[ "$1" = "--" ] && shift
O=gpurun_out/$tag; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
if [ $# -gt 0 ]; then
  timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread "$@" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
  tail -1 $O/pytest.log
fi
i=0
for spec in "${specs[@]}" "${specs[@]}"; do
  i=$((i + 1))
  ( IFS=','; for kv in $spec; do export "$kv"; done
    timeout -k 10 300 python3 -u bench.py --no-cpu --no-a6 --no-ingest --steps 5 --warmup 1 --knn-steps 0 --cand-steps 0 > "$O/b_$i.log" 2>&1 ) || { tail -20 "$O/b_$i.log"; exit 1; }
  echo "$spec"; python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(round(d['ms_per_step'],2), d['phases_ms'])" "$O/b_$i.log"
done
