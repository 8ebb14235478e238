#!/bin/bash
# Kernel-level profile of the configs[1] co-visitation build (1 warmup + 1 timed + 1 phase run).
# usage (on the GPU box): tools/prof_covis.sh <outdir> [extra bench args]
set -e
out=${1:-gpurun_out/prof}
shift || true
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out" -o run -- \
  python3 bench.py --steps 1 --warmup 1 --no-cpu --knn-steps 0 --cand-steps 0 "$@" > "$out/bench.log" 2>&1
python3 tools/kstats.py "$out/run_kernel_stats.csv" > "$out/summary.txt"
