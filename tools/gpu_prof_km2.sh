#!/bin/bash
# per-dispatch durations of the KMeans E-step kernels in one config-5 step (split-precision path)
set -o pipefail
O=gpurun_out/${1:-profkm2}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/k -o run -- python3 bench.py --workload candidates --steps 1 --warmup 0 > $O/k.log 2>&1 || { tail -20 $O/k.log; exit 1; }
python3 - "$O/k/run_kernel_trace.csv" > $O/km_dispatch.txt <<'PY'
import csv, sys
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
for name in ("k_km_assign_split", "k_km_assign_mfma"):
    d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in rows if name in r["Kernel_Name"]]
    print(name, len(d), "first 12:", [round(x, 3) for x in d[:12]], "steps 50-61:", [round(x, 3) for x in d[50:62]],
          "last 12:", [round(x, 3) for x in d[-12:]])
PY
rm -f $O/k/run_kernel_trace.csv
cat $O/km_dispatch.txt
