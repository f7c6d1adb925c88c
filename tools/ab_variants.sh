#!/bin/bash
# Build-variant A/B with parity: for each quoted EXTRA flag set, rebuild
# libffddp.so on the box, run the GPU solve-parity tests, then a short bench;
# prints one summary line per variant (value, per-kernel ms per solve).
set -e
mkdir -p gpurun_out
i=0
for flags in "$@"; do
  i=$((i+1))
  make -s -C franka-force-feedback-mpc_amd/csrc -B EXTRA="$flags" > gpurun_out/ab_build_$i.log 2>&1 || { echo "build failed: $flags"; tail -20 gpurun_out/ab_build_$i.log; exit 1; }
  if [ -z "$NO_TESTS" ]; then
    timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/ab_tests_$i.log 2>&1 || { echo "TESTS FAILED: $flags"; tail -30 gpurun_out/ab_tests_$i.log; exit 1; }
  fi
  timeout -k 10 200 python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-host-io $BENCH_ARGS > gpurun_out/ab_bench_$i.log 2>&1 || { echo "bench failed: $flags"; tail -20 gpurun_out/ab_bench_$i.log; exit 1; }
  python - "$flags" "$i" <<'PY'
import json,sys
l=[x for x in open("gpurun_out/ab_bench_%s.log" % sys.argv[2]) if x.startswith("{")][-1]
j=json.loads(l)
t=[x for x in open("gpurun_out/ab_tests_%s.log" % sys.argv[2])][-1].strip() if __import__("os").path.exists("gpurun_out/ab_tests_%s.log" % sys.argv[2]) else ""
print(repr(sys.argv[1]), "value %.0f" % j["value"], "ms %.2f" % j["ms_per_step"], " ".join("%s=%.2f" % (k, v["ms_per_solve"]) for k, v in (j["kernels"] or {}).items() if v["ms_per_solve"] > 0.2), "ok=%.3f it=%.2f" % (j["solver"]["ok_frac"], j["solver"]["mean_iter"]), "|", t)
PY
done
