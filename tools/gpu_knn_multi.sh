#!/bin/bash
# configs[2] kNN under several values of one env switch (same box): tools/gpu_knn_multi.sh <tag> <VAR> <v1> <v2> ... [-- pytest args]
set -o pipefail
tag=$1; var=$2; shift 2
vals=(); while [ $# -gt 0 ] && [ "$1" != "--" ]; do vals+=("$1"); shift; done
[ "$1" = "--" ] && shift
O=gpurun_out/$tag; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
if [ $# -gt 0 ]; then
  timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread "$@" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
  tail -1 $O/pytest.log
fi
for v in "${vals[@]}" "${vals[@]}"; do
  export $var=$v
  timeout -k 10 300 python3 -u bench.py --workload knn --steps 3 --warmup 1 --no-cpu > "$O/k_$v.log" 2>&1 || { tail -20 "$O/k_$v.log"; exit 1; }
  echo "$var=$v"; python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(round(d['value']), round(d['ms_per_step'],2), d.get('phases_ms'), d.get('roofline',{}).get('frac'), d.get('sample_exact_match'))" "$O/k_$v.log"
done
