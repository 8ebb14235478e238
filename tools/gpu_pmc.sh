#!/bin/bash
# Round evidence (PMC part; tools/gpu_pmc.sh <out tag> <round tag, e.g. r6>): default bench line, kernel traces of the same command (co-visitation + kNN + config 5),
# PMC FETCH / WRITE per phase (profiles/r5_pmc_traffic.json via tools/pmc_phases.py) and per-kernel SQ mix
set -o pipefail
O=gpurun_out/${1:-ev}; R=${2:-r6}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
B="bench.py --steps 1 --warmup 0 --knn-steps 1 --cand-steps 0 --no-cpu --no-a6 --no-ingest"
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/f -o run -- python3 $B > $O/f.log 2>&1 || { tail -20 $O/f.log; exit 1; }
timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/w -o run -- python3 $B > $O/w.log 2>&1 || { tail -20 $O/w.log; exit 1; }
python3 tools/pmc_phases.py $O/f/run_counter_collection.csv $O/w/run_counter_collection.csv > $O/${R}_pmc_traffic.json || exit 1
timeout -s KILL 180 rocprofv3 --kernel-trace --stats --output-format csv -d $O/k -o run -- python3 $B > $O/k.log 2>&1 || { tail -20 $O/k.log; exit 1; }
timeout -s KILL 180 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD --output-format csv -d $O/a -o run -- python3 $B > $O/a.log 2>&1 || { tail -20 $O/a.log; exit 1; }
