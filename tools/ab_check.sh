#!/bin/bash
# Bit-for-bit check of the in-tree library against lib/base (tools/lib_dump.py)
# and a short A/B bench of both at each batch in $BATCHES.
# usage: tools/ab_check.sh TAG
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
TAG=${1:-abc}
O=$R/gpurun_out/$TAG; mkdir -p $O
cd $R
FFDDP_LIB=$R/franka-force-feedback-mpc_amd/lib/base/libffddp.so timeout -k 10 200 python3 tools/lib_dump.py $O/a.npz > $O/dump_a.log 2>&1
timeout -k 10 200 python3 tools/lib_dump.py $O/b.npz > $O/dump_b.log 2>&1
python3 tools/lib_dump.py --compare $O/a.npz $O/b.npz; rm -f $O/a.npz $O/b.npz
BATCHES=${BATCHES:-4096 1024 512} bash tools/ab_libs.sh $TAG base main
