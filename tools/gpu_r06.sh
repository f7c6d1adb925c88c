#!/bin/bash
# Round-6 GPU steps named in $STEPS, each under its own time limit, stopping
# at the first failure.  Steps not listed here are tools/gpu_r05.sh's.
#   hostio   host entry point timeline at B=4096: stage-in / enqueue / per-slice done and
#            copied times (FFDDP_HOSTIO_TIMING), pageable and page-locked outputs (tools/hostio.py)
#   avail    the SQ counters this box's rocprofv3 exposes (lane-utilisation candidates)
#   lanes    VALU lane utilisation per kernel class (tools/pmc_lanes.sh)
# usage: [STEPS="bits tests hostio"] tools/gpu_r06.sh TAG
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
TAG=${1:-r06}
O=$R/gpurun_out/$TAG; mkdir -p $O
cd $R
STEPS=${STEPS:-"tests bench"}
for st in $STEPS; do
  case $st in
    hostio) for L in ${HOSTIO_LIBS:-base main}; do
              if [ $L = main ]; then LIB=$R/franka-force-feedback-mpc_amd/lib/libffddp.so; else LIB=$R/franka-force-feedback-mpc_amd/lib/$L/libffddp.so; fi
              FFDDP_LIB=$LIB HOSTIO_CONFIGS=${HOSTIO_CONFIGS:-pageable:0,pinned:0} timeout -k 10 200 python3 tools/hostio.py 4096 ${HOSTIO_REPS:-5} \
                > $O/hostio_$L.txt 2>&1 || { tail -20 $O/hostio_$L.txt; exit 1; }
              echo "== $L"; grep -v amdgpu.ids $O/hostio_$L.txt | tail -14 | cut -c1-600
            done ;;
    probe) timeout -k 10 200 python3 tools/hostio_probe.py 4096 6 > $O/probe.txt 2>&1 || { tail -20 $O/probe.txt; exit 1; }
           grep -v amdgpu.ids $O/probe.txt ;;
    rehearse) bash $R/tools/rehearse_multi.sh $TAG/rehearse ;;
    phase) for spec in "1 tracking" "1 random" "1024 random"; do set -- $spec; echo "== prof B=$1 $2"
             FFDDP_LIB=$R/franka-force-feedback-mpc_amd/lib/prof/libffddp.so timeout -k 10 200 python3 tools/phase_prof.py $1 classical "" $2 2>&1 | grep -v amdgpu.ids; done | tee $O/phase_prof.txt ;;
    avail) (cd /tmp && export TMPDIR=/tmp && timeout -k 10 120 rocprofv3 --list-avail > $O/avail.txt 2>&1) || { tail -5 $O/avail.txt; exit 1; }
           grep -o -E "SQ_[A-Z0-9_]*(THREAD|LANE|ACTIVE|VALU)[A-Z0-9_]*" $O/avail.txt | sort -u | tr '\n' ' '; echo ;;
    lanes) BENCH_ARGS="${LANE_ARGS:---batch 4096}" bash $R/tools/pmc_lanes.sh $TAG/lanes > $O/lanes.log 2>&1 || { tail -20 $O/lanes.log; exit 1; }
           cat $O/lanes.log ;;
    *) STEPS=$st bash $R/tools/gpu_r05.sh $TAG ;;
  esac
  echo "step $st done"
done
