#!/bin/bash
# Round-2 first GPU check: full -m gpu suite, then the default bench line.
set -o pipefail
O=gpurun_out/r2a
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
timeout -k 10 600 python3 -u bench.py > $O/bench.log 2>&1 || { tail -30 $O/bench.log; exit 1; }
tail -c 3000 $O/bench.log
