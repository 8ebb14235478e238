#!/bin/bash
# Same-box A/B of an environment switch on the configs[2] kNN (bench --workload knn), alternating A B A B:
# tools/gpu_knn_envab.sh <tag> <VAR> <A> <B> [pytest files...]
set -o pipefail
tag=$1; var=$2; va=$3; vb=$4; shift 4
O=gpurun_out/$tag; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
if [ $# -gt 0 ]; then
  timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread "$@" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
  tail -1 $O/pytest.log
fi
for run in A1 B1 A2 B2; do
  if [ "${run:0:1}" = A ]; then export $var=$va; else export $var=$vb; fi
  timeout -k 10 300 python3 -u bench.py --workload knn --steps 3 --warmup 1 --no-cpu > "$O/k_$run.log" 2>&1 || { tail -20 "$O/k_$run.log"; exit 1; }
  echo "$run $var=${!var}"; python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(round(d['value']), round(d['ms_per_step'],2), d.get('phases_ms'), d.get('roofline',{}).get('frac'))" "$O/k_$run.log"
done
