#!/bin/bash
# Diagnostics: full kernel trace of a short bench (per-iteration timeline),
# solver-work histogram, then the phase-profiled build of instance 0.
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/diag
rm -rf $O; mkdir -p $O
timeout -k 10 120 python3 $R/tools/iter_hist.py 4096 classical > $O/iter_hist.txt 2>&1
timeout -k 10 120 python3 $R/tools/iter_hist.py 4096 ff >> $O/iter_hist.txt 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/kt -o kt -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-host-io --no-profile > $O/kt_bench.log 2>&1
python3 $R/tools/timeline.py $O/kt > $O/timeline.txt
rm -rf $O/kt
cd $R
make -s -C franka-force-feedback-mpc_amd/csrc -B EXTRA=-DFFDDP_PHASE_PROF > $O/build.log 2>&1
timeout -k 10 120 python3 tools/phase_prof.py 4096 classical > $O/phase.txt 2>&1
