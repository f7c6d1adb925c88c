#!/bin/bash
# A/B of environment settings on the in-tree library: for each quoted setting
# (e.g. "FFDDP_FW_SCALAR_IT=2"; "-" = none) a short bench at each batch in
# $BATCHES (default "4096 512").   usage: tools/ab_env.sh TAG setting1 setting2 ...
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
TAG=$1; shift
O=$R/gpurun_out/$TAG; mkdir -p $O
cd $R
i=0
for cfg in "$@"; do
  i=$((i+1))
  [ "$cfg" = "-" ] && e="" || e="$cfg"
  for B in ${BATCHES:-4096 512}; do
    env $e timeout -k 10 200 python3 bench.py --batch $B --steps ${STEPS:-10} --no-cpu-baseline --no-extras --no-host-io $BENCH_ARGS > $O/v${i}_$B.log 2>&1 || { echo "bench failed: $cfg $B"; tail -20 $O/v${i}_$B.log; exit 1; }
    python3 -c "import json,sys; d=json.loads(open('$O/v${i}_$B.log').read().strip().splitlines()[-1]); k=d['kernels'] or {}; print('%-28s'%'$cfg', $B, round(d['value']), 'ms/step %.2f'%d['ms_per_step'], 'it %.2f ok %.3f'%(d['solver']['mean_iter'], d['solver']['ok_frac']), ' '.join('%s=%.0f'%(n,v['avg_launch_ms']*1e3) for n,v in k.items() if n not in ('init','finalize')))"
  done
done
