#!/bin/bash
# Round-6 closing measurements on one MI355X, in two calls (each under gpurun's limit):
#   part 1: kernel traces + FETCH/WRITE passes + full bench line (gpu_prof.sh), SQ limiter passes at
#           B=4096 / 512 (pmc_sq2.sh), fp64 issue counts classical + FF (pmc_fp64.sh), lane utilisation
#   part 2: every BASELINE config (gpu_configs.sh) and the B=1 phase profile
# The JSON summaries bench.py reads (traffic / sq / fp64 / lanes *_latest.json) come back under
# gpurun_out/TAG and are copied into profiles/ by hand.
# usage: tools/gpu_final_r06.sh TAG 1|2
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
TAG=${1:-r06final}
O=$R/gpurun_out/$TAG; mkdir -p $O
cd $R
if [ "$2" = 1 ]; then
  STEPS="prof sq" bash tools/gpu_r06.sh $TAG
  bash tools/pmc_fp64.sh $TAG/fp64 > $O/fp64.log 2>&1 || { tail -20 $O/fp64.log; exit 1; }
  BENCH_ARGS="--variant ff" FP_CONFIG=ff/normal_1d/B4096/N30 bash tools/pmc_fp64.sh $TAG/fp64ff > $O/fp64ff.log 2>&1 || { tail -20 $O/fp64ff.log; exit 1; }
  STEPS="lanes" bash tools/gpu_r06.sh $TAG
else
  bash tools/gpu_configs.sh $TAG/cfg > $O/configs.log 2>&1 || { tail -20 $O/configs.log; exit 1; }
  tail -12 $O/configs.log
  STEPS="phase" bash tools/gpu_r06.sh $TAG
fi
