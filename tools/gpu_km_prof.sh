#!/bin/bash
# lockstep-group tests, then kernel traces of KMeans fits in lockstep groups of 4 and one run at a time
# (tools/km_group_prof.py)
set -o pipefail
tag=${1:-kmprof}
O=gpurun_out/$tag; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_popularity_gpu.py -k "lockstep or bounded or split" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for v in 4 1; do
  OTTOHIP_KM_GROUP=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/g$v -o run -- python3 -u tools/km_group_prof.py 12900000 4 20 > $O/g$v.log 2>&1 || { tail -20 $O/g$v.log; exit 1; }
  grep group $O/g$v.log
  python3 tools/kdb.py $(find $O/g$v -name "*results.db" | head -1) > $O/g$v.txt; head -8 $O/g$v.txt
done
