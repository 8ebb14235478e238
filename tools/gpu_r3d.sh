#!/bin/bash
# hash-first A/B on the covis bench, KMeans bound statistics per step, per-kernel PMC table of one build
set -o pipefail
O=gpurun_out/${1:-r3d}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_envab.sh ${1:-r3d}_hf OTTOHIP_HASH_FIRST 0 1 || exit 1
OTTOHIP_KM_BDBG=1 timeout -k 10 400 python3 -u bench.py --workload candidates --steps 1 --warmup 0 > $O/kmdbg.log 2>&1 || { tail -20 $O/kmdbg.log; exit 1; }
grep -a "kmeans bounds" $O/kmdbg.log | awk 'NR%10==1' | head -60
tools/gpu_pmc_r3.sh ${1:-r3d}_pmc > /dev/null 2>&1 || { echo pmc failed; exit 1; }
head -30 gpurun_out/${1:-r3d}_pmc/pmc_per_kernel.txt
