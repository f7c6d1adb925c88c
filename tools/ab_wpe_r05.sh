#!/bin/bash
# A/B (alternating) of the in-tree library against lib/wpe2 (FW_WPE=2: the
# two-groups-per-row line search compiled for two waves per SIMD, with spills):
# classical 4096/1024/512 and the C5 per-GPU shape.   usage: tools/ab_wpe_r05.sh TAG
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
TAG=$1
cd $R
BATCHES="1024" BENCH_ARGS="--horizon 100 --contact point3d" bash tools/ab_libs.sh $TAG/c5 main wpe2 wpe2 main
BATCHES="4096 1024 512" bash tools/ab_libs.sh $TAG/cls main wpe2 wpe2 main
