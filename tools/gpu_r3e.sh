#!/bin/bash
# covis tests, then same-box A/Bs: fused one-chunk split counting, hash-first launch order, 64 records per
# emit flush (libottohip_ab.so); KMeans bound statistics; config-5 time outside the stages
set -o pipefail
O=gpurun_out/${1:-r3e}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_envab.sh ${1:-r3e}_fuse OTTOHIP_SPLIT_FUSE 0 1 tests/test_covis_gpu.py tests/test_merge_gpu.py || exit 1
tools/gpu_envab.sh ${1:-r3e}_hf OTTOHIP_HASH_FIRST 0 1 || exit 1
tools/gpu_libab.sh ${1:-r3e}_lib || exit 1
OTTOHIP_KM_BDBG=1 timeout -k 10 400 python3 -u bench.py --workload candidates --steps 1 --warmup 0 > $O/kmdbg.log 2>&1 || { tail -20 $O/kmdbg.log; exit 1; }
grep -a "kmeans bounds" $O/kmdbg.log | awk 'NR%10==1' | head -40
timeout -k 10 400 python3 -u bench.py --workload candidates --steps 1 --warmup 1 > $O/cand.log 2>&1 || { tail -20 $O/cand.log; exit 1; }
grep '^{' $O/cand.log | tail -1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); c=d.get("candidates",d); print(round(c["ms_per_step"],1), c["outside_stages_s"], c["stages_s"])'
