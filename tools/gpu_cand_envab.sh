#!/bin/bash
# candidates + pipeline tests, then config-5 A/B on an env switch (VAR=1 / VAR=0), candidates stage and kernel times
set -o pipefail
VAR=$1; O=gpurun_out/${2:-candenv}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_candidates_gpu.py tests/test_pipeline_gpu.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for run in A1 B1 A2 B2; do
  if [ "${run:0:1}" = A ]; then export $VAR=1; else export $VAR=0; fi
  timeout -k 10 400 python3 -u bench.py --no-cpu --no-a6 --no-ingest --steps 1 --warmup 0 --knn-steps 0 > "$O/c_$run.log" 2>&1 || { tail -20 "$O/c_$run.log"; exit 1; }
  echo "$run $VAR=${!VAR}"; python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); c=d['candidates']; s=c['stages_s']; print(round(c['ms_per_step'],1), {k: s[k] for k in ('C2_kmeans','candidates','R7_similarity')}, c['recall@20']['total'], c['config']['candidates'])" "$O/c_$run.log"
done
export $VAR=1
bash tools/gpu_cand_prof.sh ${2:-candenv}/prof
