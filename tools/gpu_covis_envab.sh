#!/bin/bash
# Co-visitation A/B on an env switch, same box: selected -m gpu tests first (with the switch at its A value),
# then the count step alternating A B A B (no A6 / kNN / candidates), then one A run with A6.
#   AV=1 BV=0 tools/gpu_covis_envab.sh VAR tag [pytest args...]
set -o pipefail
VAR=$1; tag=$2; shift 2
O=gpurun_out/$tag; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export $VAR=${AV:-1}
if [ $# -gt 0 ]; then
  timeout -k 10 900 python -u -m pytest -x -v --timeout 450 --timeout-method thread "$@" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
  tail -2 $O/pytest.log
fi
for run in A1 B1 A2 B2; do
  if [ "${run:0:1}" = A ]; then export $VAR=${AV:-1}; else export $VAR=${BV:-0}; fi
  timeout -k 10 300 python3 -u bench.py --no-cpu --no-a6 --no-ingest --steps 5 --warmup 1 --knn-steps 0 --cand-steps 0 > "$O/b_$run.log" 2>&1 || { tail -20 "$O/b_$run.log"; exit 1; }
  echo "$run $VAR=${!VAR}"; python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(round(d['ms_per_step'],2), d['phases_ms'])" "$O/b_$run.log"
done
export $VAR=${AV:-1}
timeout -k 10 300 python3 -u bench.py --no-cpu --no-ingest --steps 3 --warmup 1 --knn-steps 0 --cand-steps 0 > "$O/b_a6.log" 2>&1 || { tail -20 "$O/b_a6.log"; exit 1; }
python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); a=d['a6']; print(round(d['ms_per_step'],2), a['total_ms_runs'], a['per_rule']['click_to_click'].get('stages_ms'))" "$O/b_a6.log"
