#!/bin/bash
# A6 click_to_click probe (tools/a6_probe.py) under a kernel trace: the part count's kernels and A6 stage times
set -o pipefail
O=gpurun_out/${1:-a6probe}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d $O/k -o run -- python3 -u tools/a6_probe.py > $O/a6.log 2>&1 || { tail -20 $O/a6.log; exit 1; }
grep '^{' $O/a6.log | tail -1
python3 - $O <<'PY'
import csv, collections, sys
O = sys.argv[1]
rows = sorted((int(r['Start_Timestamp']), int(r['End_Timestamp']), r['Kernel_Name'].split('(')[0].replace('void ', '').replace('ottohip::', '')[:44])
              for r in csv.DictReader(open(f'{O}/k/run_kernel_trace.csv')))
s0 = [r[0] for r in rows if r[2].startswith('k_prep_count')][-1]  # the last part count (rep 1)
win = [r for r in rows if r[0] >= s0]
t = collections.Counter(); c = collections.Counter()
for r in win:
    t[r[2]] += (r[1] - r[0]) / 1e6; c[r[2]] += 1
print('window ms', round((win[-1][1] - win[0][0]) / 1e6, 2))
for k, v in t.most_common(24):
    print(f"{k:46s} {c[k]:4d} {v:8.2f}")
PY
