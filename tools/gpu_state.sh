#!/bin/bash
# State of the tree on one box: the default bench line, then same-box A/Bs of the covis switches still off
# by default (OTTOHIP_LDS_LEAF, OTTOHIP_ROWS=atomic): tools/gpu_state.sh <tag>
set -o pipefail
tag=${1:-state}
O=gpurun_out/$tag; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python3 -u bench.py > $O/bench.log 2>&1 || { tail -30 $O/bench.log; exit 1; }
grep '^{' $O/bench.log | tail -1 > $O/bench.json
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['ms_per_step'], d['phases_ms'], d['knn']['phases_ms'], d['candidates']['ms_per_step'], d['candidates']['stages_s'], d['a6'].get('total_ms_runs'), d['a6']['per_rule']['click_to_click'])" $O/bench.json
bash tools/gpu_envab.sh ${tag}_lds OTTOHIP_LDS_LEAF 1 0 || exit 1
bash tools/gpu_envab.sh ${tag}_rows OTTOHIP_ROWS atomic fused || exit 1
