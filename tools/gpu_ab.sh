#!/bin/bash
# A/B of env settings on the covis bench: tools/gpu_ab.sh <tag> "<pytest -k expr or ->" "ENV=a" "ENV=b" ...
set -o pipefail
tag=$1; shift; kx=$1; shift
O=gpurun_out/$tag; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
if [ "$kx" != "-" ]; then
  timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_covis_gpu.py tests/test_shard_gpu.py -k "$kx" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
  tail -1 $O/pytest.log
fi
for mode in "$@"; do
  env $mode timeout -k 10 300 python3 -u bench.py --no-cpu --steps 3 --warmup 1 --knn-steps 0 --cand-steps 0 > "$O/b_$mode.log" 2>&1 || { tail -20 "$O/b_$mode.log"; exit 1; }
  echo "$mode"; python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(round(d['ms_per_step'],2), d['phases_ms'])" "$O/b_$mode.log"
done
