#!/bin/bash
# Bits (in-tree vs lib/head), GPU tests, and the classical A/B head vs main
# (B = 4096 / 1024 / 512 and the C5 per-GPU shape).
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
TAG=${1:-r05i}
O=$R/gpurun_out/$TAG; mkdir -p $O
cd $R
FFDDP_LIB=$R/franka-force-feedback-mpc_amd/lib/head/libffddp.so timeout -k 10 200 python3 tools/lib_dump.py $O/a.npz > $O/dump_a.log 2>&1
timeout -k 10 200 python3 tools/lib_dump.py $O/b.npz > $O/dump_b.log 2>&1
python3 tools/lib_dump.py --compare $O/a.npz $O/b.npz | tee $O/bits.txt; rm -f $O/a.npz $O/b.npz
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
BATCHES="4096 1024 512" bash tools/ab_libs.sh $TAG/cls head main main head
BATCHES="1024" BENCH_ARGS="--horizon 100 --contact point3d" bash tools/ab_libs.sh $TAG/c5 head main main head
