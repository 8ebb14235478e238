#!/bin/bash
# Grouped record merge (per-(rule, aid) LDS hash): shard / merge / covis tests, A6 A/B against the sort path
# (OTTOHIP_MERGE_GROUPS=0), then the A6 kernel profile
set -o pipefail
tag=${1:-r4n}
bash tools/gpu_a6envab.sh $tag OTTOHIP_MERGE_GROUPS 1 0 tests/test_shard_gpu.py tests/test_merge_gpu.py tests/test_covis_gpu.py || exit 1
bash tools/gpu_prof_a6.sh ${tag}_prof
