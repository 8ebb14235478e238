#!/bin/bash
# covis parity tests + covis-only bench line: tools/gpu_covis.sh <tag> [extra env for bench]
set -o pipefail
tag=$1; shift
O=gpurun_out/$tag
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_covis_gpu.py tests/test_shard_gpu.py tests/test_merge_gpu.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 python3 -u bench.py --steps 3 --warmup 1 --knn-steps 0 --cand-steps 0 --no-cpu > $O/bench.log 2>&1 || { tail -30 $O/bench.log; exit 1; }
python3 -c "import json; d=json.loads(open('$O/bench.log').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['value']/1e9, d['phases_ms'])"
