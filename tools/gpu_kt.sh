#!/bin/bash
# Kernel trace of the timed bench configuration + per-iteration timeline of one solve.
# usage: tools/gpu_kt.sh TAG [bench args...]
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
TAG=$1; shift
O=$R/gpurun_out/$TAG; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o kt -- python3 $R/bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-profile --no-extras --no-host-io "$@" > $O/kt_bench.log 2>&1
tail -1 $O/kt_bench.log | cut -c1-200
python3 $R/tools/timeline.py $O/kt 3 > $O/timeline.txt
grep totals $O/timeline.txt
