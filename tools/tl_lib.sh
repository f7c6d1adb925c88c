#!/bin/bash
# Kernel timeline of one solve at batch B with the library variant NAME
# (lib/NAME/libffddp.so; "main" = the in-tree library).  usage: tl_lib.sh TAG B NAME
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/$1; rm -rf $O; mkdir -p $O
if [ "$3" = main ]; then L=$R/franka-force-feedback-mpc_amd/lib/libffddp.so; else L=$R/franka-force-feedback-mpc_amd/lib/$3/libffddp.so; fi
cd /tmp && export TMPDIR=/tmp
FFDDP_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/kt -o kt -- python3 $R/bench.py --batch $2 --steps 2 --warmup 1 --no-cpu-baseline --no-host-io --no-profile --no-extras > $O/kt_bench.log 2>&1
python3 $R/tools/rawtl.py $O/kt > $O/raw.txt
rm -rf $O/kt
