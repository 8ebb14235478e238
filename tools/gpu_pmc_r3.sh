#!/bin/bash
# Round-3 per-kernel counters of one co-visitation build: kernel trace, FETCH/WRITE, SQ mix
set -o pipefail
O=gpurun_out/${1:-pmc_r3}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
B="bench.py --steps 1 --warmup 0 --knn-steps 0 --cand-steps 0 --no-cpu --no-a6 --no-ingest"
timeout -s KILL 180 rocprofv3 --kernel-trace --stats --output-format csv -d $O/k -o run -- python3 $B > $O/k.log 2>&1 || exit 1
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/f -o run -- python3 $B > $O/f.log 2>&1 || exit 1
timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/w -o run -- python3 $B > $O/w.log 2>&1 || exit 1
timeout -s KILL 180 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD --output-format csv -d $O/a -o run -- python3 $B > $O/a.log 2>&1 || exit 1
ls -R $O | head -30
python3 tools/kpmc_table.py $O 40 > $O/pmc_per_kernel.txt && cat $O/pmc_per_kernel.txt
