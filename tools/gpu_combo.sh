#!/bin/bash
# covis parity subset + covis bench + kNN tests + kNN bench (one box call)
set -o pipefail
O=gpurun_out/${1:-combo}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_covis_gpu.py tests/test_shard_gpu.py tests/test_knn.py -k "digest or heavy or hot or three or golden or long or finalize or part or pair or knn" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python3 -u bench.py --no-cpu --steps 3 --warmup 1 --knn-steps 2 --cand-steps 0 > $O/b.log 2>&1 || { tail -20 $O/b.log; exit 1; }
python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(round(d['ms_per_step'],2), d['phases_ms']); k=d['knn']; print(k['value'], k['phases_ms'], k['roofline']['frac'])" $O/b.log
