#!/bin/bash
# KMeans rows prepared once per fit: popularity tests (bit-identity with the per-step split), then the config-5
# step at OTTOHIP_KM_PREP 1 / 0 / 1 / 0 (same box)
set -o pipefail
tag=${1:-r4k}
O=gpurun_out/$tag; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_popularity_gpu.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for v in 1 0 1 0; do
  OTTOHIP_KM_PREP=$v timeout -k 10 400 python3 -u bench.py --workload candidates --no-cpu --steps 1 > $O/cand_$v.log 2>&1 || { tail -20 $O/cand_$v.log; exit 1; }
  echo "KM_PREP=$v"; python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); c=d.get('candidates',d); print(c['ms_per_step'], c['stages_s']['C2_kmeans'], c['recall@20'])" $O/cand_$v.log
done
