set -e
O=gpurun_out/diag2; rm -rf $O; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /root/repo/$O/kt -o kt -- python3 /root/repo/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-host-io --no-profile > /root/repo/$O/kt_bench.log 2>&1
python3 /root/repo/tools/timeline.py /root/repo/$O/kt > /root/repo/$O/timeline.txt
rm -rf /root/repo/$O/kt
