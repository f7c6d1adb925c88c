#!/bin/bash
# Round-1 profiling recipe: kernel-trace stats, then FETCH_SIZE and WRITE_SIZE
# in separate --pmc passes, then a full bench line that picks up the traffic.
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r01prof
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o r01 -- python3 $R/bench.py --steps 5 --warmup 1 --no-cpu-baseline > $O/kt_bench.log 2>&1
echo "kernel trace done"
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o r01 -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-profile > $O/fetch_bench.log 2>&1
echo "fetch done"
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o r01 -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-profile > $O/write_bench.log 2>&1
echo "write done"
python3 $R/tools/pmc_traffic.py $O/fetch $O/write classical/normal_1d/B4096/N30 3 $O/traffic_latest.json
cp $O/traffic_latest.json $R/profiles/traffic_latest.json
timeout -k 10 400 python3 $R/bench.py > $O/bench_full.log 2>&1
echo "bench done"
