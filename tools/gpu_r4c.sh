#!/bin/bash
# R7 kernel + KMeans pair / kNN buffer A/Bs (tools/gpu_r4g.sh), then the one-GPU emulation of a rank at G = 8 / 4
set -o pipefail
O=gpurun_out/${1:-r4c}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash tools/gpu_r4g.sh ${1:-r4c} || exit 1
for w in 8 4; do
  timeout -k 10 300 python3 -u tools/emulate_rank.py --world $w > $O/emu_$w.log 2>&1 || { tail -20 $O/emu_$w.log; exit 1; }
  echo "world $w"; tail -4 $O/emu_$w.log
done
