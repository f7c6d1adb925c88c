#!/bin/bash
# Round-4 GPU check: the steps named in $STEPS (default all), each under its
# own time limit, stopping at the first failure.
#   budget  GPU leg of the extended-precision error budget (tools/ext_budget_gpu.py)
#   c1      configs[0] tick breakdown: solve plan, host-array solve, per-kernel events
#   sq      SQ counters per kernel at B=4096 and B=512 (tools/pmc_sq2.sh)
#   gaps    kernel timelines of one solve at B=1 / 256 / 512 (time between kernels per queue)
#   tests   pytest -m gpu with the parity log
#   bench   one default bench line
# usage: [STEPS="c1 tests"] tools/gpu_r04.sh TAG
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
TAG=${1:-r04}
O=$R/gpurun_out/$TAG; mkdir -p $O
cd $R
STEPS=${STEPS:-"budget c1 sq tests bench"}
for st in $STEPS; do
  case $st in
    budget) timeout -k 10 120 python3 tools/ext_budget_gpu.py $O/ext_gpu.npz > $O/ext.log 2>&1 ;;
    c1) timeout -k 10 200 python3 tools/c1_breakdown.py --time 4 --cpu > $O/c1_plan.log 2>&1
        timeout -k 10 120 python3 tools/c1_breakdown.py --time 4 --no-plan > $O/c1_noplan.log 2>&1
        timeout -k 10 120 python3 tools/c1_breakdown.py --time 4 --profile > $O/c1_prof.log 2>&1
        tail -qn1 $O/c1_plan.log $O/c1_noplan.log $O/c1_prof.log ;;
    sq) BENCH_ARGS="--batch 4096" $R/tools/pmc_sq2.sh $TAG/sq4096 > $O/sq.log 2>&1
        BENCH_ARGS="--batch 512" SQ_CONFIG=classical/normal_1d/B512/N30 $R/tools/pmc_sq2.sh $TAG/sq512 > $O/sq512.log 2>&1 ;;
    gaps) for b in 1 256 512; do $R/tools/diag_timeline_b.sh $TAG/tl$b $b; grep "queue span" $O/tl$b/timeline.txt; done ;;
    tests) rm -f $O/parity.jsonl
        FFDDP_PARITY_LOG=$O/parity.jsonl timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 \
          --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
        tail -1 $O/gpu_tests.log ;;
    bench) timeout -k 10 400 python3 bench.py > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
        tail -1 $O/bench.log | cut -c1-300 ;;
  esac
  echo "step $st done"
done
