#!/bin/bash
# Default bench line on the box: tools/gpu_bench.sh <tag> [bench args...]
set -o pipefail
tag=$1; shift
O=gpurun_out/$tag
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
python3 -c "import os; print('cpu_count', os.cpu_count(), 'affinity', len(os.sched_getaffinity(0)))"
cat /sys/fs/cgroup/cpu.max 2>/dev/null; echo "OMP_NUM_THREADS=$OMP_NUM_THREADS"
timeout -k 10 900 python3 -u bench.py "$@" > $O/bench.log 2>&1
rc=$?
tail -c 6000 $O/bench.log
exit $rc
