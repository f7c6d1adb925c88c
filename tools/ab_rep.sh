#!/bin/bash
# Alternating A/B of lib/base vs the in-tree library, REPS rounds per batch
# (noise control).  usage: BATCHES="4096 2048" REPS=3 tools/ab_rep.sh TAG
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
TAG=${1:-abr}
O=$R/gpurun_out/$TAG; mkdir -p $O
cd $R
for B in ${BATCHES:-4096}; do
  for r in $(seq ${REPS:-3}); do
    for name in base main; do
      if [ "$name" = main ]; then L=$R/franka-force-feedback-mpc_amd/lib/libffddp.so; else L=$R/franka-force-feedback-mpc_amd/lib/$name/libffddp.so; fi
      FFDDP_LIB=$L timeout -k 10 200 python3 bench.py --batch $B --steps ${STEPS:-20} --no-cpu-baseline --no-extras --no-host-io --no-profile $BENCH_ARGS > $O/${name}_${B}_$r.log 2>&1 || { echo "bench failed: $name $B"; tail -5 $O/${name}_${B}_$r.log; exit 1; }
      python3 -c "import json; d=json.loads(open('$O/${name}_${B}_$r.log').read().strip().splitlines()[-1]); print('%-6s'%'$name', $B, $r, round(d['value']), 'ms/step %.3f'%d['ms_per_step'])"
    done
  done
done
