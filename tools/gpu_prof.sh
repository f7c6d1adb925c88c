#!/bin/bash
# GPU profile recipe: GPU tests, kernel-trace stats of the timed configuration
# (4 slices) and of the single-stream profiling step, FETCH_SIZE / WRITE_SIZE
# in separate --pmc passes, then the full default bench line.
# usage: tools/gpu_prof.sh TAG [skip-tests]
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
TAG=${1:-prof}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
if [ "$2" != "skip-tests" ]; then
  (cd $R && timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1)
  echo "tests done"; tail -3 $O/gpu_tests.log
fi
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o kt -- python3 $R/bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-profile --no-extras --no-host-io > $O/kt_bench.log 2>&1
echo "kernel trace (timed config) done"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt1 -o kt1 -- python3 $R/bench.py --profile-only > $O/kt1_bench.log 2>&1
echo "kernel trace (single stream) done"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o f -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-profile --no-extras --no-host-io > $O/fetch_bench.log 2>&1
echo "fetch done"
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o w -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-profile --no-extras --no-host-io > $O/write_bench.log 2>&1
echo "write done"
python3 $R/tools/pmc_traffic.py $O/fetch $O/write classical/normal_1d/B4096/N30 3 $O/traffic_latest.json > /dev/null
cp $O/traffic_latest.json $R/profiles/traffic_latest.json
timeout -k 10 400 python3 $R/bench.py > $O/bench_full.log 2>&1
echo "bench done"; tail -1 $O/bench_full.log
