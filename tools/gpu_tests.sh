#!/bin/bash
# Run a subset of the -m gpu tests on the box: tools/gpu_tests.sh <tag> <pytest args...>
set -o pipefail
tag=$1; shift
O=gpurun_out/$tag
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread "$@" > $O/pytest.log 2>&1
rc=$?
tail -40 $O/pytest.log
exit $rc
