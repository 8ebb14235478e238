#!/bin/bash
# Iteration loop on the box: tools/gpu_iter.sh <tag> "<pytest targets>" [bench args...]
# parity tests first; the covis bench line (no CPU legs) only if they pass
set -o pipefail
tag=$1; shift
tests=$1; shift
O=gpurun_out/$tag
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
if [ -n "$tests" ]; then
  timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread $tests > $O/pytest.log 2>&1
  rc=$?
  tail -15 $O/pytest.log
  [ $rc -ne 0 ] && exit $rc
fi
timeout -k 10 600 python3 -u bench.py --no-cpu "$@" > $O/bench.log 2>&1
rc=$?
grep -v alloc $O/bench.log | tail -c 4000
exit $rc
