set -e
make -s -C franka-force-feedback-mpc_amd/csrc -B > /dev/null 2>&1
FFDDP_FW=group timeout -k 10 400 python -m pytest tests/test_gpu_parity.py -x -q -k solve > gpurun_out/fw_tests.log 2>&1 || { tail -30 gpurun_out/fw_tests.log; exit 1; }
tail -1 gpurun_out/fw_tests.log
NO_TESTS=1 bash tools/ab.sh FFDDP_FW=lane "FFDDP_FW=group FFDDP_FW_FIRST=10" "FFDDP_FW=group FFDDP_FW_FIRST=3" "FFDDP_FW=group FFDDP_FW_FIRST=2" "FFDDP_FW=group FFDDP_FW_FIRST=1"
