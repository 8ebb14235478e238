#!/bin/bash
# Same-box A/B of an environment switch on the A6 merge (1 build + 3 A6 passes per run):
# tools/gpu_a6envab.sh <tag> <VAR> <A> <B> [pytest files...]
set -o pipefail
tag=$1; var=$2; va=$3; vb=$4; shift 4
O=gpurun_out/$tag; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
if [ $# -gt 0 ]; then
  timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread "$@" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
  tail -1 $O/pytest.log
fi
for run in A1 B1 A2 B2; do
  if [ "${run:0:1}" = A ]; then export $var=$va; else export $var=$vb; fi
  timeout -k 10 300 python3 -u bench.py --no-cpu --no-ingest --steps 1 --warmup 0 --knn-steps 0 --cand-steps 0 > "$O/a6_$run.log" 2>&1 || { tail -20 "$O/a6_$run.log"; exit 1; }
  echo "$run $var=${!var}"; python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); a=d['a6']; c=a['per_rule']['click_to_click']; print(a['total_ms_runs'], c['stages_ms'], c['rows_out'])" "$O/a6_$run.log"
done
