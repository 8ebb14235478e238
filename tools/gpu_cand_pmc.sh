#!/bin/bash
# SQ counters of k_cand_build on the config-5 workload (one bench step)
set -o pipefail
O=gpurun_out/${1:-candpmc}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
R="k_cand_build|k_sim16|k_cand_recall"
timeout -s KILL 400 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_WAVES --kernel-include-regex "$R" --output-format csv -d $O/s -o run -- python3 -u bench.py --no-cpu --no-a6 --no-ingest --steps 1 --warmup 0 --knn-steps 0 > $O/s.log 2>&1 || { tail -20 $O/s.log; exit 1; }
timeout -s KILL 400 rocprofv3 --pmc SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_SALU SQ_LDS_IDX_ACTIVE SQ_INSTS_SMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM_RD --kernel-include-regex "$R" --output-format csv -d $O/t -o run -- python3 -u bench.py --no-cpu --no-a6 --no-ingest --steps 1 --warmup 0 --knn-steps 0 > $O/t.log 2>&1 || { tail -20 $O/t.log; exit 1; }
python3 - $O <<'PY'
import csv, sys
from collections import defaultdict
O = sys.argv[1]
agg = defaultdict(lambda: defaultdict(float)); n = defaultdict(set)
for f in ('s', 't'):
    for r in csv.DictReader(open(f'{O}/{f}/run_counter_collection.csv')):
        k = r['Kernel_Name'].split('(')[0].replace('void ', '').replace('ottohip::', '')
        agg[k][r['Counter_Name']] += float(r['Counter_Value']); n[k].add(r['Dispatch_Id'])
for k, c in agg.items():
    d = len(n[k])
    print(k, 'dispatches', d, {cn: round(v / d / 1e6, 3) for cn, v in sorted(c.items())})
PY
