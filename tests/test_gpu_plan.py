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

from ffddp import BatchedBoxFDDP, FfddpError, _abi

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


def test_plan_lifetime_rules():
    """a plan's graph holds the handle's workspace and trace
    pointer.  Tracing cannot change while a plan is alive; closing the solver
    closes its plans first (no dangling handle); a plan's run after an
    asynchronous device solve on another stream waits for it."""
    import torch

    N, B = 30, 8
    cfg = product_cfg("classical", N)
    batch = make_batch("classical", B, N, seed=7)
    s = BatchedBoxFDDP(cfg, max_batch=B)
    ref = BatchedBoxFDDP(cfg, max_batch=B)
    plan = s.plan(B, maxiter=10)
    with pytest.raises(FfddpError, match="plans"):
        s.trace_enable(8)
    with pytest.raises(FfddpError):
        s.setCallbacks([lambda solver, tr: None])
    plan.close()
    s.trace_enable(8)  # no live plan: allowed again
    s.trace_enable(0)

    # device solve on a side stream, then the plan in program order: the
    # plan's graph waits for it on the device, so both results stay exact
    dev = torch.device("cuda", 0)
    f64 = dict(dtype=torch.float64, device=dev)
    other = make_batch("classical", B, N, seed=8)
    t = dict(x0=torch.tensor(other.x0, **f64), node_ref=torch.tensor(other.node_ref, **f64),
             inst_ref=torch.tensor(other.inst_ref, **f64),
             surface=torch.tensor(other.surface, dtype=torch.uint8, device=dev),
             xs_init=torch.tensor(other.xs_init, **f64), us_init=torch.tensor(other.us_init, **f64),
             xs=torch.zeros((B, N + 1, 14), **f64), us=torch.zeros((B, N, 7), **f64),
             K=torch.zeros((B, N, 7, 14), **f64), cost=torch.zeros(B, **f64),
             iters=torch.zeros(B, dtype=torch.int32, device=dev), ok=torch.zeros(B, dtype=torch.uint8, device=dev),
             fn_pred=torch.zeros((B, 2), **f64),
             stats=torch.zeros((B, _abi.NSTATS), dtype=torch.int32, device=dev))
    side = torch.cuda.Stream(dev)
    plan = s.plan(B, maxiter=10)
    plan.fill(batch)
    s.solve_dev(t, maxiter=10, stream=side.cuda_stream)
    plan.run()
    torch.cuda.synchronize(dev)
    ref.solve(batch, maxiter=10)
    _same(ref, plan, "plan after side-stream solve")
    ref.solve(other, maxiter=10)
    assert np.array_equal(t["xs"].cpu().numpy(), ref.xs) and np.array_equal(t["K"].cpu().numpy(), ref.K)

    # closing the solver closes the plan first; the plan then refuses to run
    s.close()
    with pytest.raises(FfddpError):
        plan.run()
    plan.close()  # idempotent
    ref.close()


def test_host_and_device_solves_after_side_stream_solve():
    """the host entry point (caller slice on the null stream) and
    a device solve on a second non-blocking stream both reuse the workspace of
    a device solve still running on a non-blocking side stream; each waits for
    it on the device.  Results equal fresh handles' bit for bit."""
    import torch

    N, B = 30, 300  # several slices: the slice streams fork from the caller's stream
    cfg = product_cfg("classical", N)
    dev = torch.device("cuda", 0)
    f64 = dict(dtype=torch.float64, device=dev)

    def dev_inputs(b):
        return dict(x0=torch.tensor(b.x0, **f64), node_ref=torch.tensor(b.node_ref, **f64),
                    inst_ref=torch.tensor(b.inst_ref, **f64),
                    surface=torch.tensor(b.surface, dtype=torch.uint8, device=dev),
                    xs_init=torch.tensor(b.xs_init, **f64), us_init=torch.tensor(b.us_init, **f64),
                    xs=torch.zeros((B, N + 1, 14), **f64), us=torch.zeros((B, N, 7), **f64),
                    K=torch.zeros((B, N, 7, 14), **f64), cost=torch.zeros(B, **f64),
                    iters=torch.zeros(B, dtype=torch.int32, device=dev),
                    ok=torch.zeros(B, dtype=torch.uint8, device=dev), fn_pred=torch.zeros((B, 2), **f64),
                    stats=torch.zeros((B, _abi.NSTATS), dtype=torch.int32, device=dev))

    b1 = make_batch("classical", B, N, seed=21, regime="random")  # long solves: still running when the next is enqueued
    b2 = make_batch("classical", B, N, seed=22)
    b3 = make_batch("classical", B, N, seed=23, surface=0)
    s = BatchedBoxFDDP(cfg, max_batch=B)
    t1, t3 = dev_inputs(b1), dev_inputs(b3)
    side1, side2 = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    s.solve_dev(t1, maxiter=10, stream=side1.cuda_stream)
    s.solve(b2, maxiter=10)  # host entry point right behind it
    host = {k: np.copy(getattr(s, k)) for k in ("xs", "us", "K", "cost", "iter", "stats")}
    s.solve_dev(t1, maxiter=10, stream=side1.cuda_stream)
    s.solve_dev(t3, maxiter=10, stream=side2.cuda_stream)  # another non-blocking stream
    torch.cuda.synchronize(dev)
    for b, got in ((b1, {k: t1[k].cpu().numpy() for k in ("xs", "us", "K", "cost", "stats")}), (b2, host),
                   (b3, {k: t3[k].cpu().numpy() for k in ("xs", "us", "K", "cost", "stats")})):
        ref = BatchedBoxFDDP(cfg, max_batch=B)
        ref.solve(b, maxiter=10)
        for k, v in got.items():
            assert np.array_equal(v, getattr(ref, k), equal_nan=True), k
        ref.close()
    s.close()
