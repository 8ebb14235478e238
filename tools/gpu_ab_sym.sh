#!/bin/bash
# A/B of symmetric emission on one box: covis line only (no cpu/a6/ingest/knn/candidates)
set -o pipefail
O=gpurun_out/${1:-absym}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for v in 1 0 1; do
  OTTOHIP_SYMMETRIC=$v timeout -k 10 300 python3 -u bench.py --no-cpu --no-a6 --no-ingest --knn-steps 0 --cand-steps 0 > $O/sym$v.log 2>&1 || { tail -20 $O/sym$v.log; exit 1; }
  echo "sym=$v $(grep '^{' $O/sym$v.log | tail -1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],2), d["phases_ms"])')"
done
