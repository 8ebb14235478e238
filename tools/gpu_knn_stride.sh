#!/bin/bash
# kNN pre-pass stride A/B on one box: bench --workload knn for several OTTOHIP_KNN_PRE_STRIDE values
set -o pipefail
O=gpurun_out/${1:-kst}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_knn.py > $O/pytest.log 2>&1 || { tail -20 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for st in 16 8 24 32 12 16; do
  export OTTOHIP_KNN_PRE_STRIDE=$st
  timeout -k 10 200 python3 -u bench.py --workload knn --steps 3 --warmup 1 --no-cpu > "$O/k_$st.log" 2>&1 || { tail -20 "$O/k_$st.log"; exit 1; }
  echo "stride $st"; python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(round(d['value']), round(d['ms_per_step'],2), d.get('phases_ms'), d.get('sample_exact_match'))" "$O/k_$st.log"
done
