#!/bin/bash
# the whole -m gpu suite (slow tests included), then the default bench line
set -o pipefail
tag=${1:-r5f}
O=gpurun_out/$tag; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 1000 python -u -m pytest -x -q --timeout 900 --timeout-method thread -m gpu tests/ > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
timeout -k 10 600 python3 -u bench.py > $O/bench.log 2>&1 || { tail -c 3000 $O/bench.log; exit 1; }
python3 -c "
import json;d=json.loads([l for l in open('$O/bench.log') if l.startswith('{')][-1])
print('step', d['ms_per_step'], d['phases_ms'], 'frac', d['roofline']['frac'])
a=d.get('a6',{}); print('a6', a.get('total_ms'), a.get('count_ms'), a.get('count_plus_merge_ms'), a.get('per_rule',{}).get('click_to_click',{}).get('stages_ms'))
print('cpu', {k: d['cpu_baseline'].get(k) for k in ('value','cores')}, d['cpu_baseline'].get('count_plus_merge',{}).get('value'))
print('knn', d['knn']['ms_per_step'], d['knn']['roofline']['frac'], d['knn']['phases_ms'])
c=d['candidates']; print('cand', c.get('ms_per_step'), c.get('stages_s'))"
