#!/bin/bash
# config-5 step at several grids of the KMeans near-tie kernel (OTTOHIP_KM_EGRID blocks; 0 = default)
set -o pipefail
O=gpurun_out/${1:-kmegrid}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for g in 0 128 256 0 128 256; do
  export OTTOHIP_KM_EGRID=$g
  timeout -k 10 400 python3 -u bench.py --workload candidates --steps 1 > $O/g_$g.log 2>&1 || { tail -20 $O/g_$g.log; exit 1; }
  echo "egrid $g"; python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); s=d['stages_s']; print(round(d['ms_per_step'],1), s['C2_kmeans'])" $O/g_$g.log
done
