#!/bin/bash
# Round-3 GPU check: GPU test suite (parity log), smoke, one default bench line.
# usage: tools/gpu_r03.sh TAG [notests]
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
TAG=${1:-r03}
O=$R/gpurun_out/$TAG; mkdir -p $O
cd $R
if [ "$2" != "notests" ]; then
  rm -f $O/parity.jsonl
  FFDDP_PARITY_LOG=$O/parity.jsonl timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
  tail -2 $O/gpu_tests.log
  timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
fi
timeout -k 10 400 python3 bench.py > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
python3 - <<PY
import json
d = json.loads(open("$O/bench.log").read().strip().splitlines()[-1])
print("value", round(d["value"]), "ms/step %.3f" % d["ms_per_step"], "frac %.3f" % d["roofline"]["frac"],
      "ok %.3f it %.2f" % (d["solver"]["ok_frac"], d["solver"]["mean_iter"]))
print("host_io", json.dumps(d["host_io"]))
print("cpu", d["cpu_baseline"]["value"] if d["cpu_baseline"] else None, "random", d.get("random_regime"))
print(" ".join("%s=%.0f" % (n, v["avg_launch_ms"] * 1e3) for n, v in (d["kernels"] or {}).items()))
PY
