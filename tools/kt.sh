#!/bin/bash
# kernel-trace stats of a short bench run -> gpurun_out/kt/summary.txt
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/kt
rm -rf $O; mkdir -p $O
[ -n "$BUILD_FLAGS" ] && make -s -C $R/franka-force-feedback-mpc_amd/csrc -B EXTRA="$BUILD_FLAGS" > $O/build.log 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o kt -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-host-io $BENCH_ARGS > $O/bench.log 2>&1
python3 - $O <<'PY'
import csv,sys,glob
f=glob.glob(sys.argv[1]+"/**/kt_kernel_stats.csv",recursive=True)[0]
for r in csv.DictReader(open(f)):
    print("%-60s calls %5s avg_us %9.1f pct %6s" % (r["Name"][:60], r["Calls"], float(r["AverageNs"])/1e3, r["Percentage"]))
PY
