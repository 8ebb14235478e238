set -e
O=gpurun_out/ev
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 python3 bench.py > $O/bench_default.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu --knn-steps 2 --cand-steps 0 > $O/kt.log 2>&1
python3 tools/kstats.py $O/kt/run_kernel_stats.csv > $O/kt_summary.txt
rm -f $O/kt/run_kernel_trace.csv
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pf -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu --knn-steps 1 --cand-steps 0 > $O/pf.log 2>&1
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pw -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu --knn-steps 1 --cand-steps 0 > $O/pw.log 2>&1
ls -la $O/pf $O/pw
