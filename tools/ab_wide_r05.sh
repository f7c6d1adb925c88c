set -e
cd $GRAFT_REPO_ROOT
BENCH_ARGS="--horizon 100 --contact point3d" bash tools/ab_env2.sh wm_c5 FFDDP_FW_WIDE_MAX "256 204 128" "1024" 2
bash tools/ab_env2.sh wm_c2 FFDDP_FW_WIDE_MAX "256 204 128" "1024 512 4096" 2
BENCH_ARGS="--regime random" bash tools/ab_env2.sh wm_rnd FFDDP_FW_WIDE_MAX "256 204 128" "1024" 2
