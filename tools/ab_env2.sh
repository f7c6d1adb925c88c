#!/bin/bash
# A/B of one environment knob over values, alternating runs (noise control).
# usage: [BENCH_ARGS="--horizon 100 ..."] tools/ab_env2.sh TAG VAR "v1 v2 ..." "B1 B2 ..." [reps]
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
TAG=$1; VAR=$2; VALS=$3; BS=$4; REPS=${5:-2}
O=$R/gpurun_out/$TAG; mkdir -p $O
cd $R
for rep in $(seq $REPS); do
  for B in $BS; do
    for v in $VALS; do
      env $VAR=$v timeout -k 10 200 python3 bench.py --batch $B --steps 10 --no-cpu-baseline --no-extras --no-host-io $BENCH_ARGS > $O/${v}_${B}_$rep.log 2>&1 || { echo "bench failed: $v $B"; tail -20 $O/${v}_${B}_$rep.log; exit 1; }
      python3 -c "import json; d=json.loads(open('$O/${v}_${B}_$rep.log').read().strip().splitlines()[-1]); k=d['kernels'] or {}; print('$VAR=%-4s'%'$v', $B, round(d['value']), 'ms/step %.2f'%d['ms_per_step'], ' '.join('%s=%.0f'%(n,v['avg_launch_ms']*1e3) for n,v in k.items() if n not in ('init','finalize','commit')))"
    done
  done
done
