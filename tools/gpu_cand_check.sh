#!/bin/bash
# popularity tests, two config-5 runs (C2 and step time), kernel profile of the candidates workload
set -o pipefail
O=gpurun_out/${1:-candcheck}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread ${TESTS:-tests/test_popularity_gpu.py} > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for run in 1 2; do
  timeout -k 10 400 python3 -u bench.py --no-cpu --no-a6 --no-ingest --steps 1 --warmup 0 --knn-steps 0 > "$O/c_$run.log" 2>&1 || { tail -20 "$O/c_$run.log"; exit 1; }
  python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); c=d['candidates']; s=c['stages_s']; print(round(c['ms_per_step'],1), {k: s[k] for k in ('C2_kmeans','candidates','knn','C1_embeddings','R7_similarity')}, c['recall@20']['total'])" "$O/c_$run.log"
done
bash tools/gpu_cand_prof.sh ${1:-candcheck}/prof
