#!/bin/bash
# Env-knob A/B at C3 (FF, B=1024) and classical B=1024: start stagger and the
# caller-stream slice, alternating (tools/ab_env.sh).   usage: tools/ab_ff_knobs_r05.sh TAG
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
for rep in 1 2; do
  BATCHES="1024" BENCH_ARGS="--variant ff" bash tools/ab_env.sh $1/ff$rep - FFDDP_STAGGER=1 FFDDP_STAGGER=2 FFDDP_CALLER_SLICE=0
  BATCHES="1024" bash tools/ab_env.sh $1/cls$rep - FFDDP_STAGGER=1 FFDDP_STAGGER=2 FFDDP_CALLER_SLICE=0
done
