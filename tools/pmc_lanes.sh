#!/bin/bash
# VALU lane utilisation per kernel class: one --pmc pass
# of SQ_THREAD_CYCLES_VALU / SQ_ACTIVE_INST_VALU / SQ_INSTS_VALU / SQ_WAVES
# over the lane calibration kernels (tools/micro/lane_util: all 64, 8 and 7
# active lanes), one over exactly 2 solves of the bench's timed
# configuration; tools/pmc_lanes.py normalises by the 64-lane figure.
# usage: [BENCH_ARGS="--batch 512"] [LANE_CONFIG=classical/normal_1d/B512/N30] tools/pmc_lanes.sh TAG
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/$1
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
CNT="SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAVES"
timeout -s KILL 60 rocprofv3 --pmc $CNT --output-format csv -d $O/cal -o r -- $R/tools/micro/lane_util > $O/cal.log 2>&1 || { echo "calibration pass failed"; tail -5 $O/cal.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc $CNT --output-format csv -d $O/run -o r -- python3 $R/bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-profile --no-host-io --no-extras $BENCH_ARGS > $O/run.log 2>&1 || { echo "bench pass failed"; tail -5 $O/run.log; exit 1; }
python3 $R/tools/pmc_lanes.py $O/cal $O/run --config="${LANE_CONFIG:-classical/normal_1d/B4096/N30}" --json=$O/lanes.json
