#!/bin/bash
# covis / merge tests, emit ablations (OTTOHIP_EMIT_DBG 0 / 1 no stores / 2 no expansion), A6 kernel profile
set -o pipefail
tag=${1:-r4g2}
O=gpurun_out/$tag; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_covis_gpu.py tests/test_merge_gpu.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for d in 0 1 2; do
  OTTOHIP_CONSERVATION_WARN=1 OTTOHIP_EMIT_DBG=$d timeout -k 10 300 python3 -u bench.py --no-cpu --no-a6 --no-ingest --steps 3 --warmup 1 --knn-steps 0 --cand-steps 0 > $O/dbg_$d.log 2>&1 || { tail -20 $O/dbg_$d.log; exit 1; }
  echo "EMIT_DBG=$d"; python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(round(d['ms_per_step'],2), d['phases_ms'])" $O/dbg_$d.log
done
bash tools/gpu_prof_a6.sh ${tag}_prof
