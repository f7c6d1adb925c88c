#!/bin/bash
# A/B (alternating) of lib/base (round-5 head) against the in-tree library:
# metric shapes, C5 per-GPU shape, FF.   usage: tools/ab_ldsw_r05.sh TAG
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
TAG=$1
cd $R
BATCHES="4096 1024 512" bash tools/ab_libs.sh $TAG/cls base main main base
BATCHES="1024" BENCH_ARGS="--horizon 100 --contact point3d" bash tools/ab_libs.sh $TAG/c5 base main main base
BATCHES="1024" BENCH_ARGS="--variant ff" bash tools/ab_libs.sh $TAG/ff base main main base
