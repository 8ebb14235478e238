#!/bin/bash
# flush microbenchmark, k_cand_build ablation, config-5 kernel profile
set -o pipefail
O=gpurun_out/r5g; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 60 ./tools/dbg/atomic_flush > $O/flush.txt 2>&1 && cat $O/flush.txt &&
timeout -k 10 400 python3 -u tools/cand_ablate.py > $O/ablate.txt 2>&1 && cat $O/ablate.txt &&
bash tools/gpu_cand_prof.sh r5g/prof
