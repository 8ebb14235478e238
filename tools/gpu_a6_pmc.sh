#!/bin/bash
# A6 per-kernel HBM fetch (rocprofv3 --pmc FETCH_SIZE, one pass) of a bench run with A6 (1 build + 4 A6 passes)
set -o pipefail
O=gpurun_out/${1:-a6pmc}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/f -o run -- python3 bench.py --no-cpu --no-ingest --steps 1 --warmup 0 --knn-steps 0 --cand-steps 0 > $O/f.log 2>&1 || { tail -20 $O/f.log; exit 1; }
ls $O/f
