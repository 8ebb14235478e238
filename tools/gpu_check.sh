#!/bin/bash
# One GPU call: selected -m gpu tests, then (optionally) the default bench line.
#   tools/gpu_check.sh <tag> [bench|nobench] [pytest args...]
set -o pipefail
tag=$1; mode=${2:-bench}; shift 2
O=gpurun_out/$tag
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
if [ $# -gt 0 ]; then
  timeout -k 10 900 python -u -m pytest -x -v --timeout 450 --timeout-method thread "$@" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
  tail -3 $O/pytest.log
fi
if [ "$mode" = bench ]; then
  timeout -k 10 600 python3 -u bench.py > $O/bench.log 2>&1 || { tail -30 $O/bench.log; exit 1; }
  grep '^{' $O/bench.log | tail -1 > $O/bench.json
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['ms_per_step'], d['phases_ms'], d['knn']['phases_ms'], d['candidates']['ms_per_step'], d['a6']['total_ms'])" $O/bench.json
fi
