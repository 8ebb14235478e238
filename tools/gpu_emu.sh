#!/bin/bash
# one-GPU emulation of rank 0 of the N-GPU co-visitation build (tools/emulate_rank.py), world 8 then 4
set -o pipefail
O=gpurun_out/${1:-emu}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for g in 8 4; do
  timeout -k 10 500 python3 -u tools/emulate_rank.py --world $g --rank 0 --sym ${SYM:-1} > $O/emu_$g.log 2>&1 || { tail -20 $O/emu_$g.log; exit 1; }
  tail -1 $O/emu_$g.log
done
