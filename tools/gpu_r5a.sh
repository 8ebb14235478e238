#!/bin/bash
# Round 5 first evidence: always-on emit record check, H16 range refusal, the covis tests, the 220 M digest,
# a covis + A6 bench line, then configs[3] at full size (8 gloo ranks on cuda:0)
set -o pipefail
tag=${1:-r5a}
O=gpurun_out/$tag; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T="python -u -m pytest -x -v --timeout-method thread"
timeout -k 10 120 python -u tools/dbg/km_range.py > $O/km.log 2>&1; cat $O/km.log
timeout -k 10 400 $T --timeout 380 tests/test_covis_gpu.py -k full_220m > $O/p2.log 2>&1 || { tail -40 $O/p2.log; exit 1; }
tail -2 $O/p2.log
timeout -k 10 400 python3 -u bench.py --steps 10 --warmup 3 --no-cpu --knn-steps 0 --cand-steps 0 --no-ingest > $O/bench.log 2>&1 || { tail -c 3000 $O/bench.log; exit 1; }
python3 -c "import json;d=json.loads(open('$O/bench.log').read().strip().splitlines()[-1]);print(d['ms_per_step'],d['phases_ms'],d.get('a6',{}).get('total_ms'),d.get('a6',{}).get('per_rule',{}).get('click_to_click',{}).get('stages_ms'))"
timeout -k 10 900 $T -s --timeout 880 tests/test_dist_gpu.py -k full_size > $O/p3.log 2>&1 || { tail -60 $O/p3.log; exit 1; }
tail -5 $O/p3.log
OTTOHIP_BENCH_PER_FILE=none timeout -k 10 400 python3 -u bench.py --steps 10 --warmup 3 --no-cpu --knn-steps 0 --cand-steps 0 --no-ingest > $O/bench_nopf.log 2>&1 || { tail -c 3000 $O/bench_nopf.log; exit 1; }
python3 -c "import json;d=json.loads(open('$O/bench_nopf.log').read().strip().splitlines()[-1]);print('no per-file', d['ms_per_step'],d['phases_ms'],d.get('a6',{}).get('total_ms'))"
