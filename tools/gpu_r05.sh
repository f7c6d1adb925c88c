#!/bin/bash
# Round-5 GPU steps named in $STEPS, each under its own time limit, stopping
# at the first failure.
#   peak    measured fp64 FMA throughput (tools/micro/fp64_peak, built on the CPU host)
#   fp64    fp64 PMC pass per kernel class, classical B=4096 and FF B=4096 (tools/pmc_fp64.sh)
#   bits    in-tree library vs lib/base bit for bit (tools/lib_dump.py)
#   nccl    one-process RCCL group: bench at B=4096 / 512 with --gather none / costs / full
#   queue   RCCL communicator vs the slice streams' hardware queues (tools/nccl_queue.py)
#   tests   pytest -m gpu with the parity log
#   ext     error-budget cases through each library in $EXTLIBS -> ext_<lib>.npz (tools/ext_budget.py reads them)
#   sq      SQ counter passes at B=4096 and B=512 (tools/pmc_sq2.sh)
#   prof    kernel-trace stats (timed and single-stream), FETCH/WRITE traffic, full bench line (tools/gpu_prof.sh)
#   bench   one default bench line
#   ab      lib/base vs the in-tree library, then line-search layout thresholds (FFDDP_LS_ROW_MAX)
#   abrnd   the same A/B in the random-x0 regime (B = 1024 / 4096)
#   abff    the same A/B for the force-feedback variant (B = 4096 / 1024)
#   phase   per-phase cycles of instance 0 at B = 1 and 512 (lib/prof: build with -DFFDDP_PHASE_PROF)
#   forced  bench with a forced one-process RCCL group vs without (gather none)
#   small   configs[4] per-GPU shape (N=100 point3d B=1024) and the C1 tick breakdown, lib/base vs in-tree
#   quick   short bench lines at B = 4096 / 1024 / 512 (no extras)
# usage: [STEPS="tests bench"] tools/gpu_r05.sh TAG
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
TAG=${1:-r05}
O=$R/gpurun_out/$TAG; mkdir -p $O
cd $R
STEPS=${STEPS:-"peak fp64 tests bench"}
for st in $STEPS; do
  case $st in
    peak) timeout -k 10 60 tools/micro/fp64_peak > $O/fp64_peak.txt 2>&1; cat $O/fp64_peak.txt ;;
    fp64) BENCH_ARGS="--batch 4096" $R/tools/pmc_fp64.sh $TAG/fp4096 > $O/fp.log 2>&1; cat $O/fp.log
          BENCH_ARGS="--batch 4096 --variant ff" FP_CONFIG=ff/normal_1d/B4096/N30 $R/tools/pmc_fp64.sh $TAG/fpff > $O/fpff.log 2>&1; cat $O/fpff.log ;;
    bits) FFDDP_LIB=$R/franka-force-feedback-mpc_amd/lib/base/libffddp.so timeout -k 10 200 python3 tools/lib_dump.py $O/a.npz > $O/dump_a.log 2>&1
          timeout -k 10 200 python3 tools/lib_dump.py $O/b.npz > $O/dump_b.log 2>&1
          python3 tools/lib_dump.py --compare $O/a.npz $O/b.npz | tee $O/bits.txt; rm -f $O/a.npz $O/b.npz ;;
    nccl) for B in 4096 512; do for g in none costs full; do
            timeout -k 10 200 python3 bench.py --batch $B --force-collective --gather $g --steps 20 --warmup 3 \
              --no-cpu-baseline --no-extras --no-host-io --no-profile > $O/nccl_${B}_$g.log 2>&1 || { tail -20 $O/nccl_${B}_$g.log; exit 1; }
            python3 -c "import json; d=json.loads(open('$O/nccl_${B}_$g.log').read().strip().splitlines()[-1]); print($B, '$g', round(d['value']), 'ms/step %.3f' % d['ms_per_step'])" | tee -a $O/nccl.txt
          done; done ;;
    queue) for B in 4096 512; do for m in ${QMODES:-none rccl_first solver_first bench_order}; do for g in ${QGATHER:-none full}; do
            [ $m = none ] && [ $g = full ] && continue
            timeout -k 10 120 python3 tools/nccl_queue.py --mode $m --batch $B --gather $g > $O/q_${m}_${B}_$g.log 2>&1 || { tail -20 $O/q_${m}_${B}_$g.log; exit 1; }
            tail -1 $O/q_${m}_${B}_$g.log | tee -a $O/queue.txt
          done; done; done ;;
    tests) rm -f $O/parity.jsonl
        FFDDP_PARITY_LOG=$O/parity.jsonl timeout -k 10 1000 python3 -u -m pytest tests -m gpu ${TESTX--x} -v --timeout 300 \
          --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
        tail -1 $O/gpu_tests.log ;;
    ext) for L in ${EXTLIBS:-base main}; do
          if [ $L = main ]; then LIB=$R/franka-force-feedback-mpc_amd/lib/libffddp.so; else LIB=$R/franka-force-feedback-mpc_amd/lib/$L/libffddp.so; fi
          FFDDP_LIB=$LIB timeout -k 10 200 python3 tools/ext_budget_gpu.py $O/ext_$L.npz > $O/ext_$L.log 2>&1 || { tail -20 $O/ext_$L.log; exit 1; }
        done ;;
    sq) $R/tools/pmc_sq2.sh $TAG/sq4096 > $O/sq4096.log 2>&1 || { tail -20 $O/sq4096.log; exit 1; }
        BENCH_ARGS="--batch 512" SQ_CONFIG=classical/normal_1d/B512/N30 $R/tools/pmc_sq2.sh $TAG/sq512 > $O/sq512.log 2>&1 || { tail -20 $O/sq512.log; exit 1; }
        head -12 $O/sq4096/summary.txt; head -12 $O/sq512/summary.txt ;;
    prof) bash $R/tools/gpu_prof.sh $TAG/prof skip-tests > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
        tail -3 $O/prof.log | cut -c1-300 ;;
    bench) timeout -k 10 400 python3 bench.py > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
        tail -1 $O/bench.log | cut -c1-300 ;;
    ab) STEPS=10 BATCHES="${ABB:-4096 1024 512}" bash tools/ab_libs.sh $TAG/ab ${LIBS:-base main} ;;
    abff) STEPS=10 BATCHES="${ABB:-4096 1024}" BENCH_ARGS="--variant ff" bash tools/ab_libs.sh $TAG/abff ${LIBS:-base main} ;;
    phase) for B in 1 512; do echo "== prof B=$B"; FFDDP_LIB=$R/franka-force-feedback-mpc_amd/lib/prof/libffddp.so timeout -k 10 200 python3 tools/phase_prof.py $B 2>&1 | grep -v amdgpu.ids; done | tee $O/phase_prof.txt ;;
    abrow) STEPS=10 BATCHES="${ABB:-4096 1024 512}" bash tools/ab_env.sh $TAG/abe ${ROWS:-"FFDDP_LS_ROW_MAX=0" "-" "FFDDP_LS_ROW_MAX=128" "FFDDP_LS_ROW_MAX=1024"} ;;
    abrnd) STEPS=10 BATCHES="${ABB:-1024 4096}" BENCH_ARGS="--regime random" bash tools/ab_libs.sh $TAG/abrnd ${LIBS:-base main} ;;
    forced) for B in 4096 512; do
          timeout -k 10 200 python3 bench.py --batch $B --force-collective --gather none --steps 20 --warmup 3 \
            --no-cpu-baseline --no-extras --no-host-io --no-profile > $O/forced_$B.log 2>&1 || { tail -20 $O/forced_$B.log; exit 1; }
          python3 -c "import json; d=json.loads(open('$O/forced_$B.log').read().strip().splitlines()[-1]); print('forced', $B, round(d['value']))"
          timeout -k 10 200 python3 bench.py --batch $B --gather none --steps 20 --warmup 3 \
            --no-cpu-baseline --no-extras --no-host-io --no-profile > $O/plain_$B.log 2>&1 || { tail -20 $O/plain_$B.log; exit 1; }
          python3 -c "import json; d=json.loads(open('$O/plain_$B.log').read().strip().splitlines()[-1]); print('plain', $B, round(d['value']))"
        done ;;
    small) for L in base main; do
          if [ $L = main ]; then LIB=$R/franka-force-feedback-mpc_amd/lib/libffddp.so; else LIB=$R/franka-force-feedback-mpc_amd/lib/$L/libffddp.so; fi
          FFDDP_LIB=$LIB timeout -k 10 200 python3 bench.py --horizon 100 --contact point3d --batch 1024 --no-extras --no-cpu-baseline --no-host-io > $O/c5_$L.log 2>&1 || { tail -20 $O/c5_$L.log; exit 1; }
          python3 -c "import json; d=json.loads(open('$O/c5_$L.log').read().strip().splitlines()[-1]); k=d['kernels']; print('c5', '$L', round(d['value']), ' '.join('%s=%.0f'%(n,v['avg_launch_ms']*1e3) for n,v in k.items()))"
          FFDDP_LIB=$LIB timeout -k 10 200 python3 tools/c1_breakdown.py --time 4 > $O/c1_$L.log 2>&1 || { tail -20 $O/c1_$L.log; exit 1; }
          echo "c1 $L $(tail -1 $O/c1_$L.log | cut -c1-400)"
        done ;;
    quick) for B in 4096 1024 512; do
        timeout -k 10 200 python3 bench.py --batch $B --no-cpu-baseline --no-extras --no-host-io > $O/q_$B.log 2>&1 || { tail -20 $O/q_$B.log; exit 1; }
        python3 -c "import json; d=json.loads(open('$O/q_$B.log').read().strip().splitlines()[-1]); k=d['kernels']; print($B, round(d['value']), 'ms/step %.2f'%d['ms_per_step'], ' '.join('%s=%.0f'%(n,v['avg_launch_ms']*1e3) for n,v in k.items()))"
      done ;;
  esac
  echo "step $st done"
done
