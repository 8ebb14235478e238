#!/bin/bash
# k_cand_build ablation on the config-5 workload: OTTOHIP_CAND_DBG bits (1 no sort, 2 no popularity list,
# 4 no list expansion), candidates stage time of one bench step each
set -o pipefail
O=gpurun_out/${1:-canddbg}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for d in 0 1 2 4 0; do
  OTTOHIP_CAND_DBG=$d timeout -k 10 400 python3 -u bench.py --no-cpu --no-a6 --no-ingest --steps 1 --warmup 0 --knn-steps 0 > "$O/c_$d.log" 2>&1 || { tail -20 "$O/c_$d.log"; exit 1; }
  echo "dbg $d"; python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); c=d['candidates']; s=c['stages_s']; print(round(c['ms_per_step'],1), {k: s[k] for k in ('candidates','R7_similarity','recall')}, c['config']['candidates'])" "$O/c_$d.log"
done
