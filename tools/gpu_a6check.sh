#!/bin/bash
# A6 check: covis + merge tests, then the A6 timing (four runs of 1 build + 3 A6 passes)
set -o pipefail
bash tools/gpu_a6envab.sh ${1:-a6check} OTTOHIP_MERGE_OPT 1 1 tests/test_covis_gpu.py tests/test_merge_gpu.py
