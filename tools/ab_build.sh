#!/bin/bash
# Build-variant A/B: for each quoted EXTRA flag set, rebuild libffddp.so on the
# box, run the solve parity tests once (first variant only) and a short bench.
set -e
mkdir -p gpurun_out
first=1
for flags in "$@"; do
  make -s -C franka-force-feedback-mpc_amd/csrc -B EXTRA="$flags" > gpurun_out/ab_build.log 2>&1 || { tail -20 gpurun_out/ab_build.log; exit 1; }
  if [ $first = 1 ] && [ -z "$NO_TESTS" ]; then
    timeout -k 10 400 python -m pytest tests/test_gpu_parity.py -x -q > gpurun_out/ab_tests.log 2>&1 || { tail -30 gpurun_out/ab_tests.log; exit 1; }
    tail -1 gpurun_out/ab_tests.log
  fi
  first=0
  timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-host-io $BENCH_ARGS $AB_ARGS > gpurun_out/ab_bench.log 2>&1 || { tail -20 gpurun_out/ab_bench.log; exit 1; }
  python - "$flags" <<'PY'
import json,sys
l=[x for x in open("gpurun_out/ab_bench.log") if x.startswith("{")][-1]
j=json.loads(l)
print(repr(sys.argv[1]), "value %.0f" % j["value"], "ms %.2f" % j["ms_per_step"], " ".join("%s=%.2f" % (k, v["ms_per_solve"]) for k, v in (j["kernels"] or {}).items() if v["ms_per_solve"] > 0.2), "ok=%.3f it=%.2f" % (j["solver"]["ok_frac"], j["solver"]["mean_iter"]))
PY
done
