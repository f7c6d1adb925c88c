"""Oracle self-consistency: model data vs the MJCF, dynamics identities,
finite-difference checks of every calcDiff block, an LQR known answer and
the BoxQP KKT conditions.  (CPU only.)"""
import re
import xml.etree.ElementTree as ET
from pathlib import Path

import numpy as np
import pytest

from ffddp import robot as R
from oracle import fddp, ocp, panda as P

from helpers import make_batch, oracle_cfg, oracle_problem, product_cfg

MJCF = Path("/root/reference/assets/scenes/panda_robot.xml")


@pytest.mark.skipif(not MJCF.exists(), reason="reference tree absent (GPU box)")
def test_model_parameters_match_mjcf():
    root = ET.parse(MJCF).getroot()
    bodies = {b.get("name"): b for b in root.iter("body")}
    for i in range(7):
        b = bodies[f"link{i + 1}"]
        pos = np.array([float(v) for v in (b.get("pos") or "0 0 0").split()])
        assert np.allclose(pos, P.JOINT_PLACEMENT_P[i]) and np.allclose(pos, R.JOINT_P[i])
        qw = np.array([float(v) for v in (b.get("quat") or "1 0 0 0").split()])
        qw = qw / np.linalg.norm(qw)
        w, x, y, z = qw
        Rq = np.array(
            [[1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)],
             [2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)],
             [2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)]]
        )
        assert np.allclose(Rq, P.JOINT_PLACEMENT_R[i], atol=1e-12) and np.allclose(Rq, R.JOINT_R[i], atol=1e-12)
        inert = b.find("inertial")
        assert np.isclose(float(inert.get("mass")), P.LINK_MASS[i]) and np.isclose(float(inert.get("mass")), R.MASS[i])
        com = np.array([float(v) for v in inert.get("pos").split()])
        assert np.allclose(com, P.LINK_COM[i]) and np.allclose(com, R.COM[i])
        f = [float(v) for v in inert.get("fullinertia").split()]
        I = np.array([[f[0], f[3], f[4]], [f[3], f[1], f[5]], [f[4], f[5], f[2]]])
        assert np.allclose(I, P.LINK_INERTIA[i]) and np.allclose(I, R.INERTIA[i])
    key = [k for k in root.iter("key") if k.get("name") == "neutral"][0]
    assert np.allclose([float(v) for v in key.get("qpos").split()], R.Q_NEUTRAL)
    tool = bodies["tool"]
    assert np.allclose([float(v) for v in tool.get("pos").split()], R.EE_P)


def _rand_state(rng):
    q = P.Q_NEUTRAL + rng.uniform(-0.4, 0.4, 7)
    return q, rng.normal(0, 0.5, 7)


def test_mass_matrix_spd_and_rnea_consistency():
    rng = np.random.default_rng(0)
    for _ in range(5):
        q, v = _rand_state(rng)
        M = P.crba(q)
        assert np.allclose(M, M.T, atol=1e-14) and np.all(np.linalg.eigvalsh(M) > 0)
        # CRBA columns == RNEA(q, 0, e_j) - g(q)
        g = P.gravity_torque(q)
        for j in range(7):
            e = np.zeros(7)
            e[j] = 1.0
            assert np.allclose(P.rnea(q, np.zeros(7), e) - g, M[:, j], atol=1e-12)
        tau = rng.normal(0, 5, 7)
        a = np.linalg.solve(M, tau - P.rnea(q, v, np.zeros(7)))
        assert np.allclose(P.rnea(q, v, a), tau, atol=1e-11)


def test_power_balance():
    """dE/dt = v . tau for the conservative arm (energy from M and gravity)."""
    rng = np.random.default_rng(1)
    q, v = _rand_state(rng)
    tau = rng.normal(0, 3, 7)
    M = P.crba(q)
    a = np.linalg.solve(M, tau - P.rnea(q, v, np.zeros(7)))

    def energy(q, v):
        oR, op, _, _ = P.forward_kinematics(q)
        c = op + np.einsum("kij,kj->ki", oR, P.LINK_COM)
        return 0.5 * v @ P.crba(q) @ v - np.sum(P.LINK_MASS * (c @ P.GRAVITY))

    h = 1e-6
    dE = (energy(q + h * v, v + h * a) - energy(q - h * v, v - h * a)) / (2 * h)
    assert abs(dE - v @ tau) < 1e-6 * max(1.0, abs(v @ tau))


def test_contact_kkt_residuals():
    cfg = oracle_cfg(product_cfg("classical", 4))
    rng = np.random.default_rng(2)
    q, v = _rand_state(rng)
    tau = P.gravity_torque(q) + rng.normal(0, 2, 7)
    pstar = np.array([0.5, 0.0, 0.34])
    d = ocp.dynamics(cfg, q, v, tau, True, pstar)
    Jc, gam = ocp._contact_terms(cfg, q, v, np.zeros(7), pstar)
    lam = d["lam"]
    M = P.crba(q)
    b = P.rnea(q, v, np.zeros(7))
    assert np.allclose(M @ d["a"] + b - Jc.T @ lam, tau, atol=1e-10)
    assert np.allclose(Jc @ d["a"] + gam, -cfg.contact_inv_damping * lam, atol=1e-9)


CASES = [(v, c, s, 0) for v in ("classical", "ff") for c in ("normal_1d", "point3d") for s in (0, 1)]
# point3d with the friction cone on (ClassicalMPCConfig defaults w = 2e2, mu = 0.6)
CASES += [("classical", "point3d", 1, 1), ("ff", "point3d", 1, 1)]


def cone_cfg(variant, N, contact="point3d"):
    c = product_cfg(variant, N, contact)
    c.w_friction_cone, c.mu = 2.0e2, 0.6
    return c


@pytest.mark.parametrize("variant,contact,surf,cone", CASES)
def test_node_derivatives_finite_differences(variant, contact, surf, cone):
    N = 3
    cfg = oracle_cfg(cone_cfg(variant, N, contact) if cone else product_cfg(variant, N, contact))
    b = make_batch(variant, 1, N, seed=4, surface=surf)
    prob = oracle_problem(b, 0, N)
    rng = np.random.default_rng(9)
    nx = cfg.nx
    x = b.x0[0] + 0.03 * rng.normal(size=nx)
    u = b.us_init[0, 0] + 0.3 * rng.normal(size=7)
    if cone:
        # the cone's facet rows must be active at this point for the test to bite
        lam = ocp.running_eval(cfg, prob, 1, x, u, False)["lam"]
        A, lb, ub = ocp.friction_cone(cfg)
        r = A @ lam
        assert np.any(r > ub) or np.any(r < lb), (lam, r)
    d = ocp.running_eval(cfg, prob, 1, x, u, True)
    h = 1e-6

    def f(xx, uu):
        e = ocp.running_eval(cfg, prob, 1, xx, uu, False)
        return e["xnext"], e["cost"]

    Fx = np.zeros((nx, nx))
    Lx = np.zeros(nx)
    for j in range(nx):
        e = np.zeros(nx)
        e[j] = h
        (a1, c1), (a2, c2) = f(x + e, u), f(x - e, u)
        Fx[:, j] = (a1 - a2) / (2 * h)
        Lx[j] = (c1 - c2) / (2 * h)
    Fu = np.zeros((nx, 7))
    Lu = np.zeros(7)
    for j in range(7):
        e = np.zeros(7)
        e[j] = h
        (a1, c1), (a2, c2) = f(x, u + e), f(x, u - e)
        Fu[:, j] = (a1 - a2) / (2 * h)
        Lu[j] = (c1 - c2) / (2 * h)
    scale = lambda A: max(1.0, np.abs(A).max())
    assert np.abs(d["Fx"] - Fx).max() / scale(Fx) < 1e-7
    assert np.abs(d["Fu"] - Fu).max() / scale(Fu) < 1e-7
    cost_scale = max(1.0, abs(float(d["cost"])))
    assert np.abs(d["Lx"] - Lx).max() < 1e-5 * cost_scale
    assert np.abs(d["Lu"] - Lu).max() < 1e-5 * cost_scale
    # Gauss-Newton Hessians: symmetric positive semi-definite
    H = np.block([[d["Lxx"], d["Lxu"]], [d["Lxu"].T, d["Luu"]]])
    assert np.allclose(H, H.T, atol=1e-9)
    assert np.linalg.eigvalsh(H).min() > -1e-8 * np.abs(H).max()


def _lqr(rng, nx=4, nu=2, N=12):
    A = np.eye(nx) + 0.1 * rng.normal(size=(nx, nx))
    B = 0.2 * rng.normal(size=(nx, nu))
    c = 0.05 * rng.normal(size=nx)
    Q = np.diag(rng.uniform(0.5, 2.0, nx))
    R_ = np.diag(rng.uniform(0.1, 1.0, nu))
    return ocp.LQRProblem(A, B, c, Q, 0.1 * rng.normal(size=nx), R_, 0.1 * rng.normal(size=nu),
                          3 * Q, np.zeros(nx), rng.normal(size=nx), N)


def _lqr_direct(m):
    """Direct KKT solve of the equality-constrained QP (independent of DDP)."""
    N, nx, nu = m.N, m.nx, m.nu
    nz = (N + 1) * nx + N * nu
    H = np.zeros((nz, nz))
    g = np.zeros(nz)
    xi = lambda t: slice(t * nx, (t + 1) * nx)
    ui = lambda t: slice((N + 1) * nx + t * nu, (N + 1) * nx + (t + 1) * nu)
    for t in range(N):
        H[xi(t), xi(t)] = m.Q
        g[xi(t)] = m.q
        H[ui(t), ui(t)] = m.R
        g[ui(t)] = m.r
    H[xi(N), xi(N)] = m.Qf
    g[xi(N)] = m.qf
    Aeq = np.zeros(((N + 1) * nx, nz))
    beq = np.zeros((N + 1) * nx)
    Aeq[0:nx, xi(0)] = np.eye(nx)
    beq[0:nx] = m.x0
    for t in range(N):
        r = slice((t + 1) * nx, (t + 2) * nx)
        Aeq[r, xi(t + 1)] = np.eye(nx)
        Aeq[r, xi(t)] = -m.A
        Aeq[r, ui(t)] = -m.B
        beq[r] = m.c
    K = np.block([[H, Aeq.T], [Aeq, np.zeros((Aeq.shape[0], Aeq.shape[0]))]])
    sol = np.linalg.solve(K, np.concatenate([-g, beq]))
    z = sol[:nz]
    return z[: (N + 1) * nx].reshape(N + 1, nx), z[(N + 1) * nx:].reshape(N, nu)


def test_fddp_lqr_known_answer():
    """Linear dynamics + quadratic cost: the first full step closes the gaps and
    lands on the optimum; the solver then stops (iter 1, ok).  Closing the
    gaps of this LQR raises the cost (dVexp < 0) and the quadratic model is
    exact (dV = dVexp), so the step is accepted only by the bounded-rise
    comparator (neg_step_rule 1); Crocoddyl's own comparator
    (dV < 2 dVexp) rejects it, and every shorter step too."""
    rng = np.random.default_rng(3)
    m = _lqr(rng)
    xs_ref, us_ref = _lqr_direct(m)
    s = fddp.SolverBoxFDDP(m, box=False, consts=fddp.Consts(neg_step_rule=1))
    ok = s.solve(np.zeros((m.N + 1, m.nx)), np.zeros((m.N, m.nu)), maxiter=10)
    assert ok and s.iter == 1
    assert np.allclose(s.xs, xs_ref, atol=1e-10) and np.allclose(s.us, us_ref, atol=1e-10)
    # the first iteration took the ascent branch with an exact model
    it0 = s.trace[0]
    assert it0[9] < 0 and abs(it0[8] - it0[9]) <= 1e-6 * abs(it0[9]) and it0[6] == 1.0
    c = fddp.SolverBoxFDDP(m, box=False)
    c.solve(np.zeros((m.N + 1, m.nx)), np.zeros((m.N, m.nu)), maxiter=1)
    assert c.stats.neg_branch == 10 and not c.is_feasible  # every step length rejected


def test_boxfddp_lqr_with_bounds_is_feasible_and_bounded():
    rng = np.random.default_rng(5)
    m = _lqr(rng)
    xs_ref, us_ref = _lqr_direct(m)
    bound = 0.5 * np.abs(us_ref).max()
    m.u_lb, m.u_ub = -bound * np.ones(m.nu), bound * np.ones(m.nu)
    # closing this LQR's gaps raises the cost: bounded-rise comparator (see above)
    s = fddp.SolverBoxFDDP(m, box=True, consts=fddp.Consts(neg_step_rule=1))
    s.solve(np.zeros((m.N + 1, m.nx)), np.zeros((m.N, m.nu)), maxiter=20)
    assert np.all(s.us <= bound + 1e-12) and np.all(s.us >= -bound - 1e-12)
    # dynamics satisfied (feasible rollout)
    for t in range(m.N):
        assert np.allclose(s.xs[t + 1], m.A @ s.xs[t] + m.B @ s.us[t] + m.c, atol=1e-10)


def _qp_bruteforce(H, q, lb, ub):
    """Exact box-QP minimiser by active-set enumeration (n <= 7)."""
    import itertools

    n = len(q)
    best = None
    for st in itertools.product((0, 1, 2), repeat=n):  # 0 free, 1 at lb, 2 at ub
        x = np.where(np.array(st) == 1, lb, np.where(np.array(st) == 2, ub, 0.0))
        f = [i for i in range(n) if st[i] == 0]
        if f:
            c = [i for i in range(n) if st[i] != 0]
            rhs = -q[f] - (H[np.ix_(f, c)] @ x[c] if c else 0.0)
            x[f] = np.linalg.solve(H[np.ix_(f, f)], rhs)
        if np.all(x >= lb - 1e-12) and np.all(x <= ub + 1e-12):
            val = 0.5 * x @ H @ x + q @ x
            if best is None or val < best[0] - 1e-14:
                best = (val, x)
    return best[1]


@pytest.mark.parametrize("seed", range(6))
def test_boxqp_matches_bruteforce(seed):
    rng = np.random.default_rng(seed)
    n = 7
    Aq = rng.normal(size=(n, n))
    H = Aq @ Aq.T + 0.5 * np.eye(n)
    q = 3.0 * rng.normal(size=n)
    lb, ub = -np.ones(n), np.ones(n)
    x, free, clamped, Hinv = fddp.boxqp(H, q, lb, ub, rng.normal(size=n), fddp.Consts())
    xb = _qp_bruteforce(H, q, lb, ub)
    assert np.allclose(x, xb, atol=1e-6)
    if free:
        assert np.allclose(Hinv, np.linalg.inv(H[np.ix_(free, free)]), atol=1e-10)


def test_boxqp_stagnation_exit():
    """The kernel's BoxQP (boxqp_lanes) stops at the first projected-Newton
    iteration whose line search accepts no step length; crocoddyl::BoxQP::solve
    runs on to maxiter with x unchanged.  On a QP from the random-x0 batch
    where this happens (tests/golden/make_boxqp_stagnation.py), stopping there
    returns exactly what the full 100 iterations return."""
    g = np.load(Path(__file__).parent / "golden" / "boxqp_stagnation.npz")
    args = (g["H"], g["q"], g["lb"], g["ub"], g["xinit"], fddp.Consts())
    i_full, i_stop = {}, {}
    full = fddp.boxqp(*args, info=i_full)
    stop = fddp.boxqp(*args, stall_exit=True, info=i_stop)
    assert i_full["stalled"] and i_full["iters"] == fddp.Consts().qp_maxiter
    assert i_stop["iters"] == i_full["stall_iter"] + 1 == int(g["stall_iter"]) + 1 < 10
    assert np.array_equal(full[0], stop[0])
    assert full[1] == stop[1] and full[2] == stop[2]
    assert np.array_equal(full[3], stop[3])


def test_backward_failure_raises_regularisation():
    """A non-convex Luu makes the first LLT fail: preg grows (SolverFDDP retry)."""
    rng = np.random.default_rng(6)
    m = _lqr(rng)
    m.R = -0.5 * np.eye(m.nu)
    s = fddp.SolverBoxFDDP(m, box=False)
    s.solve(np.zeros((m.N + 1, m.nx)), np.zeros((m.N, m.nu)), maxiter=3)
    assert s.stats.reg_retries > 0


def test_accept_step_rule():
    """SolverFDDP::solve acceptance (oracle.fddp.accept_step, the rule the HIP
    kernel's trial_accepted implements), both ascent-branch comparators."""
    c = fddp.Consts()
    assert c.neg_step_rule == 0  # Crocoddyl's comparator is the default
    # descent direction: sufficient decrease
    assert fddp.accept_step(c, False, dV=0.2, d0=1.0, dVexp=1.0)
    assert not fddp.accept_step(c, False, dV=0.05, d0=1.0, dVexp=1.0)
    assert fddp.accept_step(c, True, dV=-1.0, d0=1e-13, dVexp=1e-13)  # |d0| < th_grad
    # ascent direction while infeasible, Crocoddyl: dV < 2 dVexp
    assert not fddp.accept_step(c, False, dV=-1.5, d0=-1.0, dVexp=-1.0)
    assert fddp.accept_step(c, False, dV=-2.5, d0=-1.0, dVexp=-1.0)
    # bounded rise: dV > 2 dVexp
    b = fddp.Consts(neg_step_rule=1)
    assert fddp.accept_step(b, False, dV=-1.5, d0=-1.0, dVexp=-1.0)
    assert not fddp.accept_step(b, False, dV=-2.5, d0=-1.0, dVexp=-1.0)
    # ascent direction once feasible: never (`!is_feasible_ && ...`), either rule
    for cc in (c, b):
        assert not fddp.accept_step(cc, True, dV=-0.5, d0=-1.0, dVexp=-1.0)
        assert not fddp.accept_step(cc, True, dV=+0.5, d0=-1.0, dVexp=-1.0)
        assert not fddp.accept_step(cc, True, dV=-2.5, d0=-1.0, dVexp=-1.0)
