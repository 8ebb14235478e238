#!/bin/bash
# end-of-round check: every -m gpu test and smoke() at HEAD, then the default bench line
set -o pipefail
O=gpurun_out/${1:-final}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
if [ "${2:-bench}" = bench ]; then
  timeout -k 10 600 python3 -u bench.py > $O/bench.log 2>&1 || { tail -30 $O/bench.log; exit 1; }
  grep '^{' $O/bench.log | tail -1 > $O/bench.json
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['ms_per_step'], d['phases_ms'], d['roofline']['frac'], d['knn']['phases_ms'], d['candidates']['ms_per_step'], d['a6']['total_ms'], d['a6']['per_rule']['click_to_click'].get('stages_ms'))" $O/bench.json
fi
