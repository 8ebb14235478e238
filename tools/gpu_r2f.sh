#!/bin/bash
# bench rehearsal of N=2 (gloo, both ranks on cuda:0, reduced sizes) + default N=1 line
set -o pipefail
O=gpurun_out/r2f
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 \
  bench.py --gpus 2 --steps 2 --warmup 1 --dist-backend gloo --events 20000000 --cand-sessions 600000 --kmeans-iter 20 --knn-steps 0 --no-cpu \
  > $O/bench_n2.log 2>&1 || { tail -40 $O/bench_n2.log; exit 1; }
tail -c 2500 $O/bench_n2.log
timeout -k 10 900 python3 -u bench.py --pandas-files 0 > $O/bench.log 2>&1 || { tail -40 $O/bench.log; exit 1; }
tail -c 3000 $O/bench.log
