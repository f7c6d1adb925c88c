"""HIP path vs the oracle on identical seeded inputs (run through the C-ABI).

Tolerances (fp64, north_star "stated fp64 tolerance"):
  * per-node calcDiff blocks (Fx, Fu, Lx, Lu, Lxx, Lxu, Luu, cost, xnext,
    lambda): max|gpu - oracle| <= 1e-9 * max(1, max|oracle block|)
    (forward-mode tangents vs complex-step derivatives: two independent
    exact-derivative methods, agreement limited by rounding only);
  * full solves: identical discrete path (iterations, ok) and
    xs / us / K / cost within 1e-6 relative (10 nonlinear iterations
    amplify rounding differences of the two implementations).
"""
import numpy as np
import pytest

from ffddp import BatchedBoxFDDP
from oracle import ocp

from helpers import make_batch, oracle_cfg, oracle_problem, oracle_solve, product_cfg, rel_err

pytestmark = pytest.mark.gpu

TOL_NODE = 1e-9
TOL_SOLVE = 1e-6

CASES = [
    ("classical", "normal_1d", 1),
    ("classical", "normal_1d", 0),
    ("classical", "point3d", 1),
    ("ff", "normal_1d", 1),
    ("ff", "normal_1d", 0),
    ("ff", "point3d", 1),
]


@pytest.mark.parametrize("variant,contact,surf", CASES)
def test_calc_diff_matches_oracle(variant, contact, surf):
    N, B = 4, 3
    cfg = product_cfg(variant, N, contact)
    ocfg = oracle_cfg(cfg)
    b = make_batch(variant, B, N, seed=11 + surf, surface=surf)
    rng = np.random.default_rng(7)
    xs = b.xs_init + 0.02 * rng.normal(size=b.xs_init.shape)
    us = b.us_init + 0.5 * rng.normal(size=b.us_init.shape)
    solver = BatchedBoxFDDP(cfg, max_batch=B)
    out = solver.calc_diff(b, xs, us)
    for i in range(B):
        prob = oracle_problem(b, i, N)
        run = ocp.running_eval(ocfg, prob, slice(0, N), xs[i, :N], us[i], True)
        term = ocp.terminal_eval(ocfg, prob, xs[i, N], True)
        for key in ("Fx", "Fu", "Lx", "Lu", "Lxx", "Lxu", "Luu"):
            assert rel_err(out[key][i, :N], run[key]) < TOL_NODE, (key, rel_err(out[key][i, :N], run[key]))
        assert rel_err(out["cost"][i, :N], run["cost"]) < TOL_NODE
        assert rel_err(out["xnext"][i], run["xnext"]) < TOL_NODE
        assert rel_err(out["Lx"][i, N], term["Lx"]) < TOL_NODE
        assert rel_err(out["Lxx"][i, N], term["Lxx"]) < TOL_NODE
        assert rel_err(out["cost"][i, N], term["cost"]) < TOL_NODE
        if surf:
            nc = ocfg.nc
            assert rel_err(out["lam"][i, :N, :nc], run["lam"]) < TOL_NODE


@pytest.mark.parametrize("variant,contact,surf", CASES)
def test_solve_matches_oracle(variant, contact, surf):
    N = 30 if contact == "normal_1d" else 12
    B = 4
    cfg = product_cfg(variant, N, contact)
    b = make_batch(variant, B, N, seed=21 + surf, surface=surf)
    solver = BatchedBoxFDDP(cfg, max_batch=B)
    ok = solver.solve(b, maxiter=10, is_feasible=False)
    for i in range(B):
        ok_o, s = oracle_solve(cfg, b, i)
        assert bool(ok[i]) == bool(ok_o)
        assert int(solver.iter[i]) == int(s.iter), (i, solver.iter[i], s.iter)
        assert rel_err(solver.cost[i], s.cost) < TOL_SOLVE
        assert rel_err(solver.xs[i], s.xs) < TOL_SOLVE
        assert rel_err(solver.us[i], s.us) < TOL_SOLVE
        assert rel_err(solver.K[i], s.K) < TOL_SOLVE * 10
        assert int(solver.stats[i, 0]) == s.stats.iters_run - s.stats.reg_retries or s.stats.reg_retries > 0


def test_gravity_torque_dev_matches_oracle():
    import torch
    from ffddp import _abi
    from oracle import panda as P

    cfg = product_cfg("classical", 4)
    solver = BatchedBoxFDDP(cfg, max_batch=8)
    rng = np.random.default_rng(3)
    q = P.Q_NEUTRAL + rng.uniform(-0.5, 0.5, size=(64, 7))
    qd = torch.tensor(q, device="cuda")
    td = torch.zeros_like(qd)
    import ctypes

    rc = solver._lib.ffddp_gravity_torque_dev(solver._h, 64, ctypes.c_void_p(qd.data_ptr()), ctypes.c_void_p(td.data_ptr()), None)
    assert rc == 0
    torch.cuda.synchronize()
    assert rel_err(td.cpu().numpy(), P.gravity_torque(q)) < 1e-12


@pytest.mark.parametrize("box,regime", [(False, "tracking"), (True, "random")])
def test_solve_variants_match_oracle(box, regime):
    """Plain FDDP (use_box_fddp=False: Cholesky gains, no clamping, th_stop 1e-9)
    and the SURVEY-literal random x0 regime."""
    N, B = 20, 4
    cfg = product_cfg("classical", N)
    cfg.use_box_fddp = box
    b = make_batch("classical", B, N, seed=33, surface=1, regime=regime)
    solver = BatchedBoxFDDP(cfg, max_batch=B)
    ok = solver.solve(b, maxiter=10, is_feasible=False)
    for i in range(B):
        ok_o, s = oracle_solve(cfg, b, i, box=box)
        assert bool(ok[i]) == bool(ok_o)
        assert int(solver.iter[i]) == int(s.iter), (i, solver.iter[i], s.iter)
        assert rel_err(solver.cost[i], s.cost) < TOL_SOLVE
        assert rel_err(solver.xs[i], s.xs) < TOL_SOLVE
        assert rel_err(solver.us[i], s.us) < TOL_SOLVE
        assert rel_err(solver.K[i], s.K) < TOL_SOLVE * 10


def test_long_horizon_point3d_matches_oracle():
    """BASELINE config 5 shape: horizon 100, point3d contact, maxiter 10."""
    N, B = 100, 2
    cfg = product_cfg("classical", N, "point3d")
    b = make_batch("classical", B, N, seed=55, surface=1)
    solver = BatchedBoxFDDP(cfg, max_batch=B)
    ok = solver.solve(b, maxiter=10, is_feasible=False)
    for i in range(B):
        ok_o, s = oracle_solve(cfg, b, i)
        assert bool(ok[i]) == bool(ok_o)
        assert int(solver.iter[i]) == int(s.iter), (i, solver.iter[i], s.iter)
        assert rel_err(solver.cost[i], s.cost) < TOL_SOLVE
        assert rel_err(solver.xs[i], s.xs) < TOL_SOLVE
        assert rel_err(solver.us[i], s.us) < TOL_SOLVE
        assert rel_err(solver.K[i], s.K) < TOL_SOLVE * 10
