"""GPU: solve plans (include/ffddp.h ffddp_plan_*) -- the per-tick solve of a
receding-horizon loop captured once as a HIP graph and replayed.  A plan's
run equals BatchedBoxFDDP.solve (the host entry point) on the same inputs,
bit for bit: one instance (the controllers' B = 1, classical and FF), and
batches that take the multi-slice schedule (several streams inside the
capture).  The plan's arrays are refilled in place between runs, and solver
properties set after the capture apply to later runs."""
from __future__ import annotations

import numpy as np
import pytest

from ffddp import BatchedBoxFDDP, FfddpError

from helpers import make_batch, product_cfg

pytestmark = pytest.mark.gpu

OUT = ("xs", "us", "K", "cost", "iter", "ok", "fn_pred", "stats")


def _same(a, p, tag):
    for name in OUT:
        x, y = getattr(a, name), getattr(p, name)
        assert np.array_equal(x, y, equal_nan=True), (tag, name)


@pytest.mark.parametrize("variant,B,N", [("classical", 1, 36), ("ff", 1, 40), ("classical", 300, 30),
                                         ("classical", 1030, 30)])
def test_plan_bit_identical_to_solve(variant, B, N):
    cfg = product_cfg(variant, N)
    ref = BatchedBoxFDDP(cfg, max_batch=B)
    s = BatchedBoxFDDP(cfg, max_batch=B)
    plan = s.plan(B, maxiter=10)
    for seed in (5, 6):  # two runs of one plan, inputs refilled in place
        batch = make_batch(variant, B, N, seed=seed, surface=seed % 2)
        ref.solve(batch, maxiter=10)
        plan.fill(batch)
        plan.run()
        _same(ref, plan, (variant, B, seed))
    plan.close()
    s.close()
    ref.close()


def test_plan_solver_params_and_errors():
    N, B = 30, 4
    cfg = product_cfg("classical", N)
    batch = make_batch("classical", B, N, seed=101, regime="random")
    s = BatchedBoxFDDP(cfg, max_batch=B)
    ref = BatchedBoxFDDP(cfg, max_batch=B)
    plan = s.plan(B, maxiter=10)
    for rule in (1, 0):  # a property changed after the capture applies to the next run
        s.neg_step_rule = rule
        ref.neg_step_rule = rule
        ref.solve(batch, maxiter=10)
        plan.fill(batch)
        plan.run()
        _same(ref, plan, ("rule", rule))
    plan.close()
    with pytest.raises(FfddpError):
        plan.run()
    with pytest.raises(FfddpError):
        s.plan(B + 1)
    s.close()
    ref.close()
