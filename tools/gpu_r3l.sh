#!/bin/bash
# split bucket mean A/B after the symmetric storage: 420 (default) vs 340 and vs 500
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_envab.sh ${1:-r3l}_340 OTTOHIP_SPLIT_MEAN 420 340 || exit 1
tools/gpu_envab.sh ${1:-r3l}_500 OTTOHIP_SPLIT_MEAN 420 500 || exit 1
