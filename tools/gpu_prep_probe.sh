#!/bin/bash
# S1-S3 alone (tools/prep_probe.py) for the in-tree library and the ablation builds given as arguments
#   tools/gpu_prep_probe.sh <tag> [lib.so ...]
set -o pipefail
O=gpurun_out/$1; shift; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python3 -u tools/prep_probe.py > $O/in_tree.log 2>&1 || { tail -20 $O/in_tree.log; exit 1; }
tail -1 $O/in_tree.log
OTTOHIP_GROUP=0 timeout -k 10 300 python3 -u tools/prep_probe.py > $O/group0.log 2>&1 || { tail -20 $O/group0.log; exit 1; }
echo group0; tail -1 $O/group0.log
for L in "$@"; do
  OTTOHIP_LIB=$GRAFT_REPO_ROOT/otto-recommender_amd/$L timeout -k 10 300 python3 -u tools/prep_probe.py > $O/$L.log 2>&1 || { tail -20 $O/$L.log; exit 1; }
  tail -1 $O/$L.log
done
