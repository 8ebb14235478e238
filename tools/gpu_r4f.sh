#!/bin/bash
# part heads + part mode tests, rows A/B (atomic vs sorted), one kernel-trace of the atomic rows, A6 timing
set -o pipefail
O=gpurun_out/${1:-r4f}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_covis_gpu.py tests/test_merge_gpu.py -k "part or cuts or full_220m or file_flow" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
bash tools/gpu_envab.sh ${1:-r4f}_ab OTTOHIP_ROWS atomic fused || exit 1
OTTOHIP_ROWS=atomic timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 -u bench.py --no-cpu --no-a6 --no-ingest --steps 2 --warmup 1 --knn-steps 0 --cand-steps 0 > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
f=$(find $O/prof -name "*kernel_stats.csv" | head -1); python3 tools/kstats.py "$f" 2>/dev/null | head -25 || head -25 "$f"
timeout -k 10 300 python3 -u bench.py --no-cpu --no-ingest --steps 3 --warmup 1 --knn-steps 0 --cand-steps 0 > "$O/b_a6.log" 2>&1 || { tail -20 "$O/b_a6.log"; exit 1; }
python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); a=d['a6']; print(a['total_ms_runs'], a.get('warmup_ms'), a['per_rule']['click_to_click'])" "$O/b_a6.log"
