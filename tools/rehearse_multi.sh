#!/bin/bash
# One-GPU rehearsal of bench.py's N > 1 path: N ranks share cuda:0 and use gloo
# collectives (FFDDP_BENCH_ONE_GPU=1); checks slicing, max-over-ranks timing,
# the cost / full-trajectory gathers and the rank-0 JSON line, not speed.
# usage: tools/rehearse_multi.sh TAG
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/$1; mkdir -p $O
cd $R
for spec in "2 costs 29533" "4 full 29534"; do
  set -- $spec
  FFDDP_BENCH_ONE_GPU=1 timeout -k 10 240 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node $1 \
    --master-addr 127.0.0.1 --master-port $3 bench.py --gpus $1 --steps 5 --warmup 1 --gather $2 > $O/n$1.log 2>&1
  tail -1 $O/n$1.log | cut -c1-300
done
