#!/bin/bash
# KMeans E-step counters (lockstep 4 / single), radix tile A/B (libottohip_ab.so: 32 keys per thread), A6 tests,
# default bench line
set -o pipefail
tag=${1:-r4h2}
O=gpurun_out/$tag; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash tools/gpu_km_pmc2.sh ${tag}_km || exit 1
bash tools/gpu_ab.sh ${tag}_rs || exit 1
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_covis_gpu.py tests/test_merge_gpu.py -k "part or cuts or full_220m or file_flow or finalize" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 600 python3 -u bench.py > $O/bench.log 2>&1 || { tail -30 $O/bench.log; exit 1; }
grep '^{' $O/bench.log | tail -1 > $O/bench.json
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['ms_per_step'], d['phases_ms'], d['knn']['phases_ms'], d['knn']['roofline'].get('search_frac'), d['candidates']['ms_per_step'], d['candidates']['stages_s']); a=d['a6']; print(a.get('total_ms_runs'), {k: v['ms'] for k, v in a['per_rule'].items()}, a['per_rule']['click_to_click'].get('stages_ms'))" $O/bench.json
