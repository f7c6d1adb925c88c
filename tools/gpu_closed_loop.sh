#!/bin/bash
# GPU: plant + closed-loop tests, then the BASELINE configs[0] closed loop
# (classical, flat, 20 s) on the HIP solver + HIP plant, then all 5 scenarios
# for 4 s each.  Logs under gpurun_out/closed_loop/.
set -e
O=gpurun_out/closed_loop
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_plant.py -x -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 400 python -u -c "import ffddp_path; from ffddp.closed_loop import main; main(['--scenario','flat','--time','20','--no-viewer','--results-dir','$O/runs'])" > $O/flat20.log 2>&1 || { tail -30 $O/flat20.log; exit 1; }
tail -1 $O/flat20.log
timeout -k 10 400 python -u -c "import ffddp_path; from ffddp.closed_loop import main; main(['--scenario','all','--time','4','--no-viewer','--results-dir','$O/runs'])" > $O/all4.log 2>&1 || { tail -30 $O/all4.log; exit 1; }
grep "RMS" $O/all4.log
