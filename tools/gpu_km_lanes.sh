#!/bin/bash
# KMeans run-lanes: bit-identity test (1/2/3 lanes), then config-5 A/B on OTTOHIP_KM_LANES (1 vs 2)
set -o pipefail
O=gpurun_out/${1:-kmlanes}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OTTOHIP_TEST_KM_LANES=1 timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_popularity_gpu.py -k lanes > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
for run in A1 B1 A2 B2; do
  if [ "${run:0:1}" = A ]; then export OTTOHIP_KM_LANES=1; else export OTTOHIP_KM_LANES=2; fi
  timeout -k 10 400 python3 -u bench.py --no-cpu --no-a6 --no-ingest --steps 1 --warmup 0 --knn-steps 0 > "$O/c_$run.log" 2>&1 || { tail -20 "$O/c_$run.log"; exit 1; }
  echo "$run lanes=$OTTOHIP_KM_LANES"; python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); c=d['candidates']; s=c['stages_s']; print(round(c['ms_per_step'],1), {k: s[k] for k in ('C2_kmeans','candidates','R7_similarity')}, c['recall@20']['total'])" "$O/c_$run.log"
done
