#!/bin/bash
# Round-1 (final) profiling recipe: kernel-trace stats of a bench run, then
# FETCH_SIZE and WRITE_SIZE in separate --pmc passes (per-launch HBM traffic of
# each kernel class -> profiles/traffic_latest.json, read by bench.py), then the
# default bench line.  Everything lands in gpurun_out/r01b/.
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r01b
rm -rf $O; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o r01 -- python3 $R/bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-host-io > $O/kt_bench.log 2>&1
echo "kernel trace done"
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o r01 -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-profile --no-host-io > $O/fetch_bench.log 2>&1
echo "fetch done"
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o r01 -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-profile --no-host-io > $O/write_bench.log 2>&1
echo "write done"
python3 $R/tools/pmc_traffic.py $O/fetch $O/write classical/normal_1d/B4096/N30 3 $O/traffic_latest.json 1024
cp $O/traffic_latest.json $R/profiles/traffic_latest.json
for f in $(find $O/kt -name "*kernel_stats.csv"); do cp $f $O/kernel_stats.csv; done
for f in $(find $O/fetch -name "*counter_collection.csv"); do cp $f $O/pmc_fetch_size.csv; done
for f in $(find $O/write -name "*counter_collection.csv"); do cp $f $O/pmc_write_size.csv; done
rm -rf $O/kt $O/fetch $O/write
cd $R
timeout -k 10 400 python3 bench.py > $O/bench.log 2>&1
tail -1 $O/bench.log
