#!/bin/bash
# Bit comparison of the in-tree library against lib/head, GPU tests, and the
# FF A/B head vs main (C3 and B=4096).
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
TAG=${1:-r05h}
O=$R/gpurun_out/$TAG; mkdir -p $O
cd $R
FFDDP_LIB=$R/franka-force-feedback-mpc_amd/lib/head/libffddp.so timeout -k 10 200 python3 tools/lib_dump.py $O/a.npz > $O/dump_a.log 2>&1
timeout -k 10 200 python3 tools/lib_dump.py $O/b.npz > $O/dump_b.log 2>&1
python3 tools/lib_dump.py --compare $O/a.npz $O/b.npz | tee $O/bits.txt; rm -f $O/a.npz $O/b.npz
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
BATCHES="1024 4096" BENCH_ARGS="--variant ff" bash tools/ab_libs.sh $TAG/ff head main main head
