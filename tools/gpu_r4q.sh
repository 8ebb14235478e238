#!/bin/bash
# optimistic workgroup hash for the big merge groups: shard tests, then A6 A/B on OTTOHIP_MERGE_OPT (1 / 0)
set -o pipefail
bash tools/gpu_a6envab.sh ${1:-r4q} OTTOHIP_MERGE_OPT 1 0 tests/test_shard_gpu.py tests/test_merge_gpu.py
