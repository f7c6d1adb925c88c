#!/bin/bash
# A/B timing helper: runs the GPU parity tests, then bench.py once per
# environment setting given as arguments (e.g. FFDDP_BW=group), printing the
# per-kernel ms/step.
set -e
mkdir -p gpurun_out
if [ -z "$NO_TESTS" ]; then timeout -k 10 400 python -m pytest tests/test_gpu_parity.py -x -q > gpurun_out/ab_tests.log 2>&1 || { tail -30 gpurun_out/ab_tests.log; exit 1; }; fi
[ -z "$NO_TESTS" ] && tail -2 gpurun_out/ab_tests.log || true
for cfg in "$@"; do
  env $cfg timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-host-io $BENCH_ARGS $AB_ARGS > gpurun_out/ab_bench.log 2>&1 || { tail -20 gpurun_out/ab_bench.log; exit 1; }
  python - "$cfg" <<'PY'
import json,sys
l=[x for x in open("gpurun_out/ab_bench.log") if x.startswith("{")][-1]
j=json.loads(l)
print(sys.argv[1], "value %.0f" % j["value"], "ms %.2f" % j["ms_per_step"], " ".join("%s=%.2f" % (k, v["ms_per_solve"]) for k, v in (j["kernels"] or {}).items()), "ok=%.3f it=%.2f" % (j["solver"]["ok_frac"], j["solver"]["mean_iter"]))
PY
done
