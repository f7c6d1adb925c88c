#!/bin/bash
# SQ instruction / cycle counters per kernel class over exactly 2 solves of the
# bench's timed configuration (1 warmup + 1 step), one --pmc pass per group.
# usage: [BENCH_ARGS="--batch 512"] tools/pmc_sq2.sh TAG
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/$1
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY" "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM" "SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VALU_FMA_F64"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d $O/p$i -o r -- python3 $R/bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-profile --no-host-io --no-extras $BENCH_ARGS > $O/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $O/p$i.log; exit 1; }
done
python3 $R/tools/pmc_summary.py $O --json=$O/sq.json --config="${SQ_CONFIG:-classical/normal_1d/B4096/N30}" --source="tools/pmc_sq2.sh $BENCH_ARGS" > $O/summary.txt
cat $O/summary.txt | head -60
