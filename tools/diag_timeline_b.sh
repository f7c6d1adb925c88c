#!/bin/bash
# Kernel timeline of one solve of the bench's timed configuration at batch B.
# usage: tools/diag_timeline_b.sh TAG B
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/$1; rm -rf $O; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/kt -o kt -- python3 $R/bench.py --batch $2 --steps 2 --warmup 1 --no-cpu-baseline --no-host-io --no-profile --no-extras > $O/kt_bench.log 2>&1
python3 $R/tools/timeline.py $O/kt > $O/timeline.txt
rm -rf $O/kt
