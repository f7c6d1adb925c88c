"""Closed-loop outcome pinned on the CPU (a 3-5x regression of
the closed loop went unnoticed because nothing pinned it).

The reference's product is closed-loop task quality (run_classical.py:513-556).
Here BASELINE configs[0]'s flat scenario runs for 2.5 s (approach, contact
onset and 1.5 s of the circle) through the product controller
(ffddp.controller.ClassicalCrocoddylMPC, ffddp.closed_loop.run_single) on
the CPU checkers: the C++ BoxFDDP of oracle/cpu and the numpy plant
oracle/plant.py (tools/closed_loop_cpu.py).  Both ascent-direction
comparators (include/ffddp.h FFDDP_NEGSTEP_*) are pinned against
tests/golden/closed_loop_outcome.json; the GPU runs of the same closed loops
at full length are tests/test_gpu_configs.py::test_c1_flat_outcome /
test_c4_outcome.
"""
from __future__ import annotations

import sys
from pathlib import Path

import pytest

from helpers import check_outcome, closed_loop_pins

sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "tools"))


@pytest.mark.parametrize("rule", [0, 1])
def test_c1_flat_outcome_cpu(rule):
    import closed_loop_cpu

    pin = closed_loop_pins()[f"cpu_c1_flat_2.5s_rule{rule}"]
    s = closed_loop_cpu.run_cpu("flat", 2.5, rule)
    check_outcome(s, pin, f"cpu/c1/rule{rule}")


def test_crocoddyl_comparator_cost_is_recorded():
    """What following Crocoddyl's comparator costs the closed loop
    (DESIGN.md §3): in the committed GPU runs the default rule leaves the
    approach-phase solves infeasible (ok = False) and triples the RMS
    tangential error of C1 and the contact-phase error of C4, with no
    instability fallback in either."""
    g = closed_loop_pins()
    c0, c1 = g["gpu_c1_flat_20s_rule0"], g["gpu_c1_flat_20s_rule1"]
    assert c0["rms_tangential_error"] > 2.5 * c1["rms_tangential_error"]
    assert c0["solve_not_ok_ticks"] > 100 and c1["solve_not_ok_ticks"] == 0
    assert c0["unstable_ticks"] == 0 and c1["unstable_ticks"] == 0
    for s, m0 in g["gpu_c4_4s_rule0"].items():
        m1 = g["gpu_c4_4s_rule1"][s]
        assert m0["rms_tangential_error_contact_phase_median"] > 1.5 * m1["rms_tangential_error_contact_phase_median"]
