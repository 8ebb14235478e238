set -o pipefail
O=gpurun_out/it2; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_covis_gpu.py -k "digest or heavy or hot or kat or golden or finalize" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
for mode in "OTTOHIP_AGG=sort" "OTTOHIP_WH_PAIR=0" "OTTOHIP_WH_PAIR=1"; do
  env $mode timeout -k 10 300 python3 -u bench.py --no-cpu --steps 3 --warmup 1 --knn-steps 0 --cand-steps 0 > $O/b_$mode.log 2>&1 || { tail -20 $O/b_$mode.log; exit 1; }
  echo "$mode"; python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(d['ms_per_step'], d['phases_ms'])" $O/b_$mode.log
done
KM_MODE=lloyd timeout -k 10 200 python3 tools/km_bench.py 12900000 50 20
KM_MODE=partial timeout -k 10 200 python3 tools/km_bench.py 12900000 50 20
