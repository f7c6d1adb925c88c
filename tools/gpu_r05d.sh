#!/bin/bash
# GPU tests on the in-tree library, the base-vs-main A/B (tools/ab_ldsw_r05.sh)
# and the C1 tick (tools/c1_breakdown.py) on base and main, alternating.
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
TAG=${1:-r05d}
O=$R/gpurun_out/$TAG; mkdir -p $O
cd $R
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
echo "step tests done"
for name in base main main base; do
  if [ "$name" = main ]; then L=$R/franka-force-feedback-mpc_amd/lib/libffddp.so; else L=$R/franka-force-feedback-mpc_amd/lib/$name/libffddp.so; fi
  FFDDP_LIB=$L timeout -k 10 200 python3 tools/c1_breakdown.py --time 4 > $O/c1_$name.log 2>&1 || { tail -20 $O/c1_$name.log; exit 1; }
  echo "c1 $name $(tail -1 $O/c1_$name.log)"
done
echo "step c1 done"
bash tools/ab_ldsw_r05.sh $TAG/ab
echo "step ab done"
