#!/bin/bash
# popularity tests, then config-5 A/B on an env switch (VAR=1 / VAR=0, alternating), then a kernel profile
# of the candidates workload with the switch on: tools/gpu_env_ab.sh OTTOHIP_KM_MV tag
set -o pipefail
VAR=$1; O=gpurun_out/${2:-envab}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_popularity_gpu.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for run in A1 B1 A2 B2; do
  if [ "${run:0:1}" = A ]; then export $VAR=${AV:-1}; else export $VAR=${BV:-0}; fi
  timeout -k 10 400 python3 -u bench.py --no-cpu --no-a6 --no-ingest --steps 1 --warmup 0 --knn-steps 0 > "$O/c_$run.log" 2>&1 || { tail -20 "$O/c_$run.log"; exit 1; }
  echo "$run $VAR=${!VAR}"; python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); c=d['candidates']; print(round(c['ms_per_step'],1), c['stages_s']['C2_kmeans'], c['recall@20'], c['config']['candidates'])" "$O/c_$run.log"
done
export $VAR=${AV:-1}
bash tools/gpu_cand_prof.sh ${2:-envab}/prof
