#!/bin/bash
# N=2 rehearsal of the bench contract on one GPU (gloo, both ranks on cuda:0, reduced sizes)
set -o pipefail
O=gpurun_out/${1:-n2}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 500 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 \
  bench.py --gpus 2 --steps 2 --warmup 1 --dist-backend gloo --events 20000000 --cand-sessions 600000 --kmeans-iter 20 --knn-steps 1 --knn-queries 60000 --no-cpu \
  > $O/bench_n2.log 2>&1 || { tail -40 $O/bench_n2.log; exit 1; }
grep '^{' $O/bench_n2.log | tail -c 3000
