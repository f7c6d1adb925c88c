#!/bin/bash
# fp64 VALU work per kernel class over exactly 2 solves of the bench's timed
# configuration (1 warmup + 1 step): one --pmc pass of 8 SQ counters, then
# tools/pmc_fp64.py divides by the device-counted units of the same solves
# (node stages, backward nodes, line-search trial nodes) -> per-unit fp64
# flops for bench.py's roofline.fp64 (profiles/fp64_latest.json).
# usage: [BENCH_ARGS="--batch 512"] [FP_CONFIG=classical/normal_1d/B512/N30] tools/pmc_fp64.sh TAG
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/$1
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_FLOPS_FP64 SQ_INSTS_VALU_FLOPS_FP64_TRANS \
  --output-format csv -d $O/fp -o r -- python3 $R/bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-profile --no-host-io --no-extras $BENCH_ARGS > $O/fp.log 2>&1 || { echo "fp64 pass failed"; tail -5 $O/fp.log; exit 1; }
python3 $R/tools/pmc_fp64.py $O/fp $O/fp.log --config="${FP_CONFIG:-classical/normal_1d/B4096/N30}" --json=$O/fp64.json | tee $O/fp64.txt
