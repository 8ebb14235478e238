#!/bin/bash
# config-5 KMeans E-step evidence: rows scored / near ties / moves per step (OTTOHIP_KM_BDBG), then HBM and SQ
# counters of the split pass, the near-tie kernel and the filter (one bench step each pass)
set -o pipefail
O=gpurun_out/${1:-kmpmc}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_popularity_gpu.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
bash tools/gpu_cand_prof.sh ${1:-kmpmc}/prof || exit 1
export OTTOHIP_KM_BDBG=1
timeout -k 10 400 python3 -u bench.py --workload candidates --steps 1 --warmup 0 > $O/bdbg.log 2>&1 || { tail -20 $O/bdbg.log; exit 1; }
python3 - $O/bdbg.log <<'PY'
import re, sys
sc, nt, mv = [], [], []
for l in open(sys.argv[1]):
    m = re.search(r'kmeans bounds: (\d+) of (\d+)', l)
    if m: sc.append(int(m.group(1))); n = int(m.group(2))
    m = re.search(r'kmeans step: (\d+) near ties, (\d+) split-pass moves', l)
    if m: nt.append(int(m.group(1))); mv.append(int(m.group(2)))
print(f"steps {len(sc)} rows {n}: scored mean {sum(sc)/len(sc):.0f} ({sum(sc)/len(sc)/n:.3f}), near ties mean {sum(nt)/len(nt):.0f}, moves mean {sum(mv)/len(mv):.0f}; first steps moves {mv[:3]}")
PY
R="k_km_(assign_split|ties|filter)"
timeout -s KILL 400 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$R" --output-format csv -d $O/f -o run -- python3 -u bench.py --workload candidates --steps 1 --warmup 0 > $O/f.log 2>&1 || { tail -20 $O/f.log; exit 1; }
timeout -s KILL 400 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$R" --output-format csv -d $O/w -o run -- python3 -u bench.py --workload candidates --steps 1 --warmup 0 > $O/w.log 2>&1 || { tail -20 $O/w.log; exit 1; }
timeout -s KILL 400 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAIT_ANY SQ_INSTS_MFMA --kernel-include-regex "$R" --output-format csv -d $O/s -o run -- python3 -u bench.py --workload candidates --steps 1 --warmup 0 > $O/s.log 2>&1 || { tail -20 $O/s.log; exit 1; }
python3 - $O <<'PY'
import csv, sys
from collections import defaultdict
O = sys.argv[1]
agg = defaultdict(lambda: defaultdict(float)); n = defaultdict(set)
for f in ('f', 'w', 's'):
    for r in csv.DictReader(open(f'{O}/{f}/run_counter_collection.csv')):
        k = r['Kernel_Name'].split('(')[0].replace('void ', '').replace('ottohip::', '')
        agg[k][r['Counter_Name']] += float(r['Counter_Value']); n[k].add(r['Dispatch_Id'])
for k, c in agg.items():
    d = len(n[k])
    print(k, 'dispatches', d, {cn: round(v / d * (2 * 1024 if cn == 'FETCH_SIZE' else 1024 if cn == 'WRITE_SIZE' else 1) / (1e6 if cn.endswith('SIZE') else 1), 3) for cn, v in c.items()})
PY
