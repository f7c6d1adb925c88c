#!/bin/bash
# A/B of prebuilt library variants (built on the CPU host into
# franka-force-feedback-mpc_amd/lib/<name>/libffddp.so): for each name, a short
# bench at each batch in $BATCHES (default "4096 512"), one summary line each.
# usage: tools/ab_libs.sh TAG name1 name2 ...   (name "main" = lib/libffddp.so)
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
TAG=$1; shift
O=$R/gpurun_out/$TAG; mkdir -p $O
cd $R
for name in "$@"; do
  if [ "$name" = main ]; then L=$R/franka-force-feedback-mpc_amd/lib/libffddp.so; else L=$R/franka-force-feedback-mpc_amd/lib/$name/libffddp.so; fi
  for B in ${BATCHES:-4096 512}; do
    FFDDP_LIB=$L timeout -k 10 200 python3 bench.py --batch $B --steps ${STEPS:-10} --no-cpu-baseline --no-extras --no-host-io $BENCH_ARGS > $O/${name}_$B.log 2>&1 || { echo "bench failed: $name $B"; tail -20 $O/${name}_$B.log; exit 1; }
    python3 -c "import json,sys; d=json.loads(open('$O/${name}_$B.log').read().strip().splitlines()[-1]); k=d['kernels'] or {}; print('%-10s'%'$name', $B, round(d['value']), 'ms/step %.2f'%d['ms_per_step'], 'it %.2f ok %.3f'%(d['solver']['mean_iter'], d['solver']['ok_frac']), ' '.join('%s=%.0f'%(n,v['avg_launch_ms']*1e3) for n,v in k.items() if n not in ('init','finalize')))"
  done
done
