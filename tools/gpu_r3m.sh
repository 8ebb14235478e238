#!/bin/bash
# hash-leaf wave priority A/B with the hash-first launch order
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_envab.sh ${1:-r3m} OTTOHIP_HASH_PRIO 0 1 || exit 1
