#!/bin/bash
# kNN with the 8-column last k-step (v_mfma_f32_32x32x8_bf16): kNN tests, then bench --workload knn A/B on
# OTTOHIP_KNN_HALF (1 = 104 columns, 0 = 112)
set -o pipefail
tag=${1:-r4p}
O=gpurun_out/$tag; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_knn.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for run in A1 B1 A2 B2; do
  if [ "${run:0:1}" = A ]; then export OTTOHIP_KNN_HALF=1; else export OTTOHIP_KNN_HALF=0; fi
  timeout -k 10 300 python3 -u bench.py --workload knn --steps 3 --warmup 1 --no-cpu > "$O/k_$run.log" 2>&1 || { tail -20 "$O/k_$run.log"; exit 1; }
  echo "$run HALF=$OTTOHIP_KNN_HALF"; python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(round(d['value']), round(d['ms_per_step'],2), d.get('phases_ms'), d.get('sample_exact_match'), d.get('roofline',{}).get('frac'))" "$O/k_$run.log"
done
