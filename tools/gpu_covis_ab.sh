#!/bin/bash
# co-visitation tests (KAT / goldens / 220 M digest), then the default line's phases with env switches A/B:
# tools/gpu_covis_ab.sh tag "VAR1=0 VAR2=0" (the B side), then WRITE_SIZE per kernel of one build (A side)
set -o pipefail
O=gpurun_out/${1:-covab}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_covis_gpu.py -k "${TESTK:-kat or golden or digest or config1}" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
B="bench.py --steps 10 --warmup 2 --no-cpu --no-a6 --no-ingest --knn-steps 0 --cand-steps 0"
for run in A1 B1 A2 B2; do
  if [ "${run:0:1}" = A ]; then E=""; else E="$2"; fi
  env $E timeout -k 10 300 python3 -u $B > "$O/b_$run.log" 2>&1 || { tail -20 "$O/b_$run.log"; exit 1; }
  echo "$run [$E]"; python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(round(d['ms_per_step'],2), d['phases_ms'])" "$O/b_$run.log"
done
timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/w -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu --no-a6 --no-ingest --knn-steps 0 --cand-steps 0 > $O/w.log 2>&1 || { tail -20 $O/w.log; exit 1; }
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/f -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu --no-a6 --no-ingest --knn-steps 0 --cand-steps 0 > $O/f.log 2>&1 || { tail -20 $O/f.log; exit 1; }
python3 - $O <<'PY'
import csv, sys
from collections import defaultdict
O = sys.argv[1]
agg = defaultdict(lambda: defaultdict(float)); n = defaultdict(set)
for f in ('w', 'f'):
    for r in csv.DictReader(open(f'{O}/{f}/run_counter_collection.csv')):
        k = r['Kernel_Name'].split('(')[0].replace('void ', '').replace('ottohip::', '')
        agg[k][r['Counter_Name']] += float(r['Counter_Value']); n[k].add(r['Dispatch_Id'])
rows = sorted(agg.items(), key=lambda kv: -(kv[1]['WRITE_SIZE'] + 2 * kv[1]['FETCH_SIZE']))[:16]
for k, c in rows:
    print(f"{k[:40]:40s} n={len(n[k]):4d} write {c['WRITE_SIZE'] * 1024 / 2 / 1e9:7.2f} GB  fetch {2 * c['FETCH_SIZE'] * 1024 / 2 / 1e9:7.2f} GB per build")
PY
