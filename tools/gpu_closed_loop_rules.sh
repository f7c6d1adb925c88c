#!/bin/bash
# Closed loops under both ascent-direction comparators (include/ffddp.h
# FFDDP_NEGSTEP_*: 0 Crocoddyl's, 1 bounded rise) on one MI355X:
#   C1  flat 20 s, one instance (BASELINE configs[0])
#   C4  5 scenarios x 256 seeds x 4 s (configs[3], tools/sweep_c4.py)
# -> gpurun_out/TAG/closed_loop_rules.json
# usage: tools/gpu_closed_loop_rules.sh TAG
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
TAG=${1:-clr}
O=$R/gpurun_out/$TAG; mkdir -p $O
cd $R
for rule in 0 1; do
  timeout -k 10 300 python3 -u -c "
import json, ffddp_path
from ffddp.closed_loop import run_single
s = run_single('flat', 20.0, verbose=False, log=False, neg_step_rule=$rule)
keys = ('rms_tangential_error', 'rms_tangential_error_contact_phase', 'avg_abs_force_err',
        'contact_loss_contact_phase_pct', 'unstable_ticks', 'neg_accepted_ticks', 'neg_accepted_total', 'solve_not_ok_ticks', 'controller_s', 'ticks')
print(json.dumps({'config': 'c1_flat_20s', 'neg_step_rule': $rule, **{k: s[k] for k in keys}}))
" > $O/c1_rule$rule.log 2>&1 || { tail -20 $O/c1_rule$rule.log; exit 1; }
  echo "c1 rule $rule done"
  timeout -k 10 300 python3 tools/sweep_c4.py --seeds 256 --time 4 --neg-step-rule $rule > $O/c4_rule$rule.log 2>&1 \
    || { tail -20 $O/c4_rule$rule.log; exit 1; }
  echo "c4 rule $rule done"
done
python3 - "$O" <<'PY'
import json, sys, pathlib
o = pathlib.Path(sys.argv[1]); out = {}
for f in sorted(o.glob("c[14]_rule*.log")):
    lines = [l for l in f.read_text().splitlines() if l.startswith("{")]
    out[f.stem] = json.loads(lines[-1])
(o / "closed_loop_rules.json").write_text(json.dumps(out, indent=1))
for k, v in out.items():
    if "scenarios" in v:
        for s, m in v["scenarios"].items():
            print(k, s, "rms_tan med %.4f" % m["rms_tangential_error"]["median"],
                  "contact-phase med %.4f" % m["rms_tangential_error_contact_phase"]["median"],
                  "loss mean %.2f" % m["contact_loss_contact_phase_pct"]["mean"],
                  "unstable mean %.2f" % m["unstable_ticks"]["mean"], "neg ticks mean %.2f" % m["neg_accepted_ticks"]["mean"],
                  "not-ok ticks mean %.1f" % m["solve_not_ok_ticks"]["mean"])
    else:
        print(k, json.dumps(v))
PY
