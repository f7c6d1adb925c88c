#!/bin/bash
# Every BASELINE.json config on one MI355X:
#   metric  classical N=30 B=4096 (bench default, with CPU baseline + extras)
#   C2      classical N=30 B=1024 random x0 (configs[1]) and tracking x0
#   C3      force-feedback N=30 B=1024
#   C5      classical point3d N=100, per-GPU shape B=1024 (8192 over 8 GPUs)
#   C4      5 scenarios x 256 seeds closed loops (tools/sweep_c4.py, 1 rank)
#   C1      flat 20 s closed loop, 1 instance
# usage: tools/gpu_configs.sh TAG
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
TAG=${1:-cfg}
O=$R/gpurun_out/$TAG; mkdir -p $O
cd $R
run() { local name=$1; shift; timeout -k 10 400 python3 "$@" > $O/$name.log 2>&1 || { echo "FAILED: $name"; tail -20 $O/$name.log; exit 1; }; echo "$name done"; }
run metric bench.py
run c2_random bench.py --batch 1024 --regime random --no-extras
run c2_tracking bench.py --batch 1024 --no-extras
run c3_ff bench.py --variant ff --batch 1024 --no-extras
run c5_n100_point3d bench.py --horizon 100 --contact point3d --batch 1024 --no-extras --cpu-budget 20
run c4_sweep tools/sweep_c4.py --seeds 256 --time 4
run c1_flat -u -c "import ffddp_path; from ffddp.closed_loop import main; main(['--scenario','flat','--time','20','--no-viewer','--results-dir','$O/results'])"
python3 - "$O" <<'PY'
import json, sys, pathlib
o = pathlib.Path(sys.argv[1]); out = {}
for f in sorted(o.glob("*.log")):
    lines = [l for l in f.read_text().splitlines() if l.startswith("{")]
    if lines:
        out[f.stem] = json.loads(lines[-1])
(o / "summary.json").write_text(json.dumps(out, indent=1))
for k, v in out.items():
    if "value" in v:
        cb = v.get("cpu_baseline") or {}
        print(k, round(v["value"]), "ms/step %.2f" % v["ms_per_step"], "frac %.3f" % v["roofline"]["frac"],
              "cpu", round(cb.get("value", 0)), "ok", round(v["solver"]["ok_frac"], 3), "it", round(v["solver"]["mean_iter"], 2))
    else:
        print(k, json.dumps(v)[:300])
PY
