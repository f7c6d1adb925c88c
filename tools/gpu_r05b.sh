#!/bin/bash
# Round-5 second pass: GPU tests on the in-tree library, then the
# base-vs-main A/B (tools/ab_ldsw_r05.sh).
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
TAG=${1:-r05b}
O=$R/gpurun_out/$TAG; mkdir -p $O
cd $R
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
echo "step tests done"
bash tools/ab_ldsw_r05.sh $TAG/ab
echo "step ab done"
