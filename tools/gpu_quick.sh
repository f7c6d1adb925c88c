#!/bin/bash
# Quick GPU check of the in-tree library: GPU tests (optional) + short bench lines.
# usage: tools/gpu_quick.sh TAG [tests|notests] [extra bench args...]
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
TAG=${1:-quick}; shift || true
MODE=${1:-tests}; shift || true
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
if [ "$MODE" = "tests" ]; then
  timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
  tail -2 $O/gpu_tests.log
fi
for B in 4096 1024 512; do
  timeout -k 10 200 python3 bench.py --batch $B --no-cpu-baseline --no-extras --no-host-io "$@" > $O/bench_$B.log 2>&1
  python3 -c "import json,sys; d=json.loads(open('$O/bench_$B.log').read().strip().splitlines()[-1]); k=d['kernels']; print($B, round(d['value']), 'ms/step %.2f'%d['ms_per_step'], ' '.join('%s=%.0f'%(n,v['avg_launch_ms']*1e3) for n,v in k.items()))"
done
