"""Committed closed-loop outcomes (tests/golden/closed_loop_outcome.json).

The reference's product is closed-loop task quality (run_classical.py:513-556:
RMS tangential error, force error, contact loss); these pins make a change of
it visible in the tests.  Sources:
  gpu  profiles/r04_closed_loop_rules.json (tools/gpu_closed_loop_rules.sh on
       one MI355X: C1 flat 20 s and the C4 5 x 256 x 4 s sweep under both
       ascent-direction comparators, include/ffddp.h FFDDP_NEGSTEP_*)
  cpu  tools/closed_loop_cpu.py (C1 flat 2.5 s on the CPU checkers: the C++
       BoxFDDP of oracle/cpu + oracle/plant.py), run here.

usage: python tests/golden/make_closed_loop_outcome.py
"""
from __future__ import annotations

import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT / "tools"))

C1_KEYS = ("rms_tangential_error", "rms_tangential_error_contact_phase", "avg_abs_force_err",
           "contact_loss_contact_phase_pct", "unstable_ticks", "neg_accepted_ticks", "solve_not_ok_ticks")
C4_KEYS = (("rms_tangential_error_contact_phase", "median"), ("rms_tangential_error", "median"),
           ("avg_abs_force_err", "median"), ("contact_loss_contact_phase_pct", "mean"), ("unstable_ticks", "mean"),
           ("solve_not_ok_ticks", "mean"))
CPU_TIME = 2.5


def main():
    import closed_loop_cpu

    g = json.loads((ROOT / "profiles" / "r04_closed_loop_rules.json").read_text())
    out = {"source": {"gpu": "profiles/r04_closed_loop_rules.json", "cpu": "tools/closed_loop_cpu.py"}}
    for rule in (0, 1):
        c1 = g[f"c1_rule{rule}"]
        out[f"gpu_c1_flat_20s_rule{rule}"] = {k: c1[k] for k in C1_KEYS}
        sc = g[f"c4_rule{rule}"]["scenarios"]
        out[f"gpu_c4_4s_rule{rule}"] = {s: {f"{k}_{stat}": m[k][stat] for k, stat in C4_KEYS} for s, m in sc.items()}
        s = closed_loop_cpu.run_cpu("flat", CPU_TIME, rule)
        out[f"cpu_c1_flat_{CPU_TIME}s_rule{rule}"] = {k: s[k] for k in C1_KEYS}
    path = Path(__file__).resolve().parent / "closed_loop_outcome.json"
    path.write_text(json.dumps(out, indent=1) + "\n")
    print("wrote", path)


if __name__ == "__main__":
    main()
