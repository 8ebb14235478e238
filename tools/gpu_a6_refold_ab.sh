#!/bin/bash
set -o pipefail
O=gpurun_out/r6a6refold; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for v in 1 0; do
  OTTOHIP_A6_REFOLD=$v timeout -k 10 400 python3 -u bench.py --no-cpu --no-ingest --steps 2 --warmup 1 --knn-steps 0 --cand-steps 0 > $O/b_$v.log 2>&1 || { tail -20 $O/b_$v.log; exit 1; }
  echo "REFOLD=$v"; python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); a=d['a6']; print(round(d['ms_per_step'],2), a['total_ms_runs'], a['per_rule']['click_to_click'].get('stages_ms'))" $O/b_$v.log
done
