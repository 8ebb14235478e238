#!/bin/bash
# emit task lists + vectorised slot scans: covis / merge / shard tests, emit A/B (OTTOHIP_EMIT_TASKS 1 / 0),
# then the default bench line (A6 times per stage)
set -o pipefail
tag=${1:-r4e}
O=gpurun_out/$tag; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_covis_gpu.py tests/test_merge_gpu.py tests/test_shard_gpu.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
bash tools/gpu_envab.sh ${tag}_emit OTTOHIP_EMIT_TASKS 1 0 || exit 1
timeout -k 10 600 python3 -u bench.py > $O/bench.log 2>&1 || { tail -30 $O/bench.log; exit 1; }
grep '^{' $O/bench.log | tail -1 > $O/bench.json
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['ms_per_step'], d['phases_ms'], d['knn']['phases_ms'], d['candidates']['ms_per_step'], d['candidates']['stages_s']); a=d['a6']; print(a.get('total_ms_runs'), {k: v['ms'] for k, v in a['per_rule'].items()}, a['per_rule']['click_to_click'].get('stages_ms'))" $O/bench.json
