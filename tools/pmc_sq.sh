#!/bin/bash
# SQ counters per kernel (one --pmc pass per group); summary -> gpurun_out/pmc_sq/summary.txt
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/pmc_sq
mkdir -p $O
[ -n "$BUILD_FLAGS" ] && make -s -C $R/franka-force-feedback-mpc_amd/csrc -B EXTRA="$BUILD_FLAGS" > $O/build.log 2>&1
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY" "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM" "SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY" "SQ_INST_CYCLES_VMEM SQ_WAIT_INST_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_VALU_FMA_F64"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d $O/p$i -o r -- python3 $R/bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-profile --no-host-io $BENCH_ARGS > $O/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $O/p$i.log; }
done
python3 $R/tools/pmc_summary.py $O > $O/summary.txt
cat $O/summary.txt
