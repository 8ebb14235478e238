set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
KM_MODE=assign timeout -k 10 120 python3 tools/km_bench.py 12900000 50 20
KM_MODE=lloyd timeout -k 10 120 python3 tools/km_bench.py 12900000 50 20
