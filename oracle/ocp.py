"""ORACLE — test infrastructure only.  Never imported by the product path.

numpy fp64 restatement of the per-node action models the reference builds in
src/mpc/crocoddyl_classical.py:521-728 and src/mpc/crocoddyl_force_feedback.py:
149-290, 776-1009, i.e. Crocoddyl's
  IntegratedActionModelEuler( DifferentialActionModel{Free,Contact}FwdDynamics(
      StateMultibody, ActuationModelFull, ContactModel{1D,3D}, CostModelSum ) )
and the Python _AugmentedLPFActionModel wrapper.

Semantics restated (Crocoddyl >= 2.0, public algorithms):
  * Euler: dx = [v dt + a dt^2, a dt], xnext = x + dx, cost = dt * l(x,u);
    terminal calc(x): xnext = x, cost = l_T(x) UNSCALED (R1).
  * Free dynamics: a = M^-1 (tau - b);  Fx = -M^-1 dRNEA/dx, Fu = M^-1
    (computeABADerivatives).
  * Contact dynamics: KKT [[M, J^T],[J, -eps I]] [a; -lambda] = [tau - b; -a0]
    with a0 = classical EE acceleration (LWA) + Kp (p - p*) + Kd v_p;
    calcDiff with Kinv = KKT^-1:  Fx = -Kinv_aa dRNEA(q,v,a,fext=lambda)/dx
    - Kinv_al da0/dx, Fu = Kinv_aa, df/dx = Kinv_la dRNEA/dx + Kinv_ll da0/dx,
    df/du = -Kinv_la.  (DifferentialActionModelContactFwdDynamics::calcDiff)
  * lambda = world-aligned contact force ON the robot; for the 1D model it is
    the world-z component (R3 resolution: r = lambda_n - fref).
  * Terminal contact-force residuals (classical terminal calc(x)) read
    zero-initialised contact data: lambda_T = 0, zero Jacobian (R2).
  * Costs: Gauss-Newton, L = sum_i w_i a_i(r_i), Lx = R^T A_r, Lxx = R^T A_rr R.
  * Activations: Quad, WeightedQuad, QuadraticBarrier (beta = 1):
    a = 0.5|min(r-lb,0)|^2 + 0.5|max(r-ub,0)|^2,
    A_rr = diag((r-lb <= 0) + (r-ub >= 0)).
The partial derivatives that Pinocchio computes analytically (dRNEA/dq,
dRNEA/dv, frame acceleration / velocity derivatives) are obtained here by
complex-step differentiation (exact to machine precision for these analytic
functions) -- an independent method from the forward-mode tangents of the HIP
kernels.
"""
from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np

from . import panda as P

INF = np.inf


@dataclass
class OCPConfig:
    """Benchmark-mode classical preset (src/run/run_classical.py:269-315) by default."""

    variant: str = "classical"  # "classical" | "ff"
    horizon: int = 30
    dt: float = 0.01
    contact_model: str = "normal_1d"  # "normal_1d" | "point3d"
    z_press: float = 0.0065
    w_ee_pos: float = 1.2e3
    w_ee_ori: float = 5.0e1
    ori_weights: np.ndarray = field(default_factory=lambda: np.array([2.4, 2.4, 0.3]))
    w_posture: float = 1.5e-1
    w_v: float = 8.0e-2
    v_damp_weights: np.ndarray = field(default_factory=lambda: np.array([1.0, 1.0, 1.0, 1.0, 0.4, 0.4, 0.4]))
    w_tau: float = 8.0e-4
    w_tau_soft_limits: float = 2.0
    tau_soft_limit_margin: float = 0.2
    w_q_soft_limits: float = 8.0
    q_soft_limit_margin: float = 0.05
    w_tangent_pos: float = 2.6e3
    w_tangent_vel: float = 7.0e2
    w_plane_z: float = 1.2e3
    w_vz: float = 5.0e2
    w_unilateral: float = 3.0e1
    friction_margin: float = 1e-3
    w_friction_cone: float = 0.0  # run_classical.py:292 (benchmark presets: off)
    mu: float = 1.0  # run_classical.py:294
    w_fn: float = 2.8e1
    fn_des: float = 22.0
    w_wdamp: float = 6.0e1
    w_wdamp_weights: np.ndarray = field(default_factory=lambda: np.array([1.8, 1.8, 0.3]))
    contact_gains: np.ndarray = field(default_factory=lambda: np.array([140.0, 80.0]))
    contact_inv_damping: float = 1.0e-8
    tau_limits: np.ndarray = field(default_factory=lambda: np.array([87.0, 87, 87, 87, 12, 12, 12]))
    R_des: np.ndarray = field(default_factory=lambda: np.eye(3))
    # force-feedback augmentation (crocoddyl_force_feedback.py:149-290)
    ff_alpha: float = 0.0
    w_w: float = 0.0
    w_w_soft_limits: float = 0.0
    w_y: float = 0.0
    y_weights: np.ndarray = field(default_factory=lambda: np.zeros(21))
    use_inner_state_reg: bool = True
    use_inner_tau_reg: bool = True

    @property
    def nc(self) -> int:
        return 3 if self.contact_model in ("point3d", "3d", "rigid3d", "route_a_3d") else 1

    @property
    def nx(self) -> int:
        return 21 if self.variant == "ff" else 14


def ff_preset(horizon: int = 30, contact_model: str = "normal_1d") -> OCPConfig:
    """Force-feedback benchmark preset (src/run/run_force_feedback.py:272-330)."""
    wc = 2.0 * np.pi * 25.0
    alpha = float(np.clip(np.exp(-wc * 0.01), 0.0, 0.999999))  # _ff_alpha_ocp, :493-497
    return OCPConfig(
        variant="ff",
        horizon=horizon,
        contact_model=contact_model,
        z_press=0.0065,
        w_ee_pos=1.2e3,
        w_ee_ori=4.5e1,
        ori_weights=np.array([2.2, 2.2, 0.3]),
        w_posture=1.0e-1,
        w_v=5.0e-2,
        w_tau=8.0e-4,
        w_tau_soft_limits=1.5,
        w_q_soft_limits=8.0,
        w_tangent_pos=3.6e3,
        w_tangent_vel=1.2e3,
        w_plane_z=9.0e2,
        w_vz=3.0e2,
        w_unilateral=3.0e1,
        w_fn=3.0e1,
        fn_des=22.0,
        w_wdamp=7.0e1,
        w_wdamp_weights=np.array([1.8, 1.8, 0.3]),
        contact_gains=np.array([145.0, 85.0]),
        ff_alpha=alpha,
        w_w=6.0e-4,
        w_w_soft_limits=2.0,
        w_y=8.0e-4,
        y_weights=np.concatenate(
            [[0.15] * 4 + [0.08] * 3, [0.05] * 4 + [0.03] * 3, [0.12] * 4 + [0.08] * 3]
        ).astype(float),
    )


@dataclass
class Problem:
    """One OCP instance: what _build_problem feeds ShootingProblem (crocoddyl_classical.py:521-556)."""

    x0: np.ndarray  # (nx,)  (FF: y0 = [q, v, tau_hat])
    p_ref: np.ndarray  # (N+1, 3) Pinocchio-frame EE position refs per node
    v_ref: np.ndarray  # (N+1, 3)
    x_reg_ref: np.ndarray  # (14,)
    tau_ref: np.ndarray  # (7,)
    surface: bool


# ---------------------------------------------------------------------------
# dense solves: LAPACK for fp64 (and complex128), else (np.longdouble, the
# extended-precision error-budget runs, tools/ext_budget.py) Gaussian
# elimination with partial pivoting in the array's own precision
# ---------------------------------------------------------------------------
_LAPACK = (np.dtype(np.float64), np.dtype(np.complex128))


def solve(A, b):
    """np.linalg.solve(A, b) for batched A (..., n, n), b (..., n, k)."""
    if A.dtype in _LAPACK and b.dtype in _LAPACK:
        return np.linalg.solve(A, b)
    dt = np.result_type(A, b)
    A = np.array(A, dtype=dt, copy=True)
    X = np.array(np.broadcast_to(b, A.shape[:-2] + b.shape[-2:]), dtype=dt, copy=True)
    n = A.shape[-1]
    for j in range(n):
        piv = j + np.argmax(np.abs(A[..., j:, j]), axis=-1)  # (...)
        idx = np.indices(piv.shape)
        rows_j = A[..., j, :].copy()
        A[..., j, :] = A[(*idx, piv)]
        A[(*idx, piv)] = rows_j
        xj = X[..., j, :].copy()
        X[..., j, :] = X[(*idx, piv)]
        X[(*idx, piv)] = xj
        for i in range(j + 1, n):
            f = A[..., i, j] / A[..., j, j]
            A[..., i, :] = A[..., i, :] - f[..., None] * A[..., j, :]
            X[..., i, :] = X[..., i, :] - f[..., None] * X[..., j, :]
    for j in range(n - 1, -1, -1):
        acc = X[..., j, :]
        for m in range(j + 1, n):
            acc = acc - A[..., j, m][..., None] * X[..., m, :]
        X[..., j, :] = acc / A[..., j, j][..., None]
    return X


def inv(A):
    if A.dtype in _LAPACK:
        return np.linalg.inv(A)
    return solve(A, np.broadcast_to(np.eye(A.shape[-1], dtype=A.dtype), A.shape))


def cholesky(A):
    """Lower Cholesky factor of batched SPD A (..., n, n), any float dtype."""
    n = A.shape[-1]
    L = np.zeros_like(A)
    for j in range(n):
        d = A[..., j, j] - np.sum(L[..., j, :j] * L[..., j, :j], -1)
        L[..., j, j] = np.sqrt(d)
        for i in range(j + 1, n):
            L[..., i, j] = (A[..., i, j] - np.sum(L[..., i, :j] * L[..., j, :j], -1)) / L[..., j, j]
    return L


def tri_lower_solve(L, B):
    """L^-1 B (forward substitution), L (..., n, n) lower, B (..., n, k)."""
    n = L.shape[-1]
    X = np.array(np.broadcast_to(B, L.shape[:-2] + B.shape[-2:]), dtype=np.result_type(L, B), copy=True)
    for i in range(n):
        acc = X[..., i, :]
        for m in range(i):
            acc = acc - L[..., i, m][..., None] * X[..., m, :]
        X[..., i, :] = acc / L[..., i, i][..., None]
    return X


def tri_upper_solve(L, B):
    """L^-T B (back substitution with the transpose of lower L)."""
    n = L.shape[-1]
    X = np.array(np.broadcast_to(B, L.shape[:-2] + B.shape[-2:]), dtype=np.result_type(L, B), copy=True)
    for i in range(n - 1, -1, -1):
        acc = X[..., i, :]
        for m in range(i + 1, n):
            acc = acc - L[..., m, i][..., None] * X[..., m, :]
        X[..., i, :] = acc / L[..., i, i][..., None]
    return X


def chol_solve(L, B):
    return tri_upper_solve(L, tri_lower_solve(L, B))


# ---------------------------------------------------------------------------
# activations (crocoddyl ActivationModel{Quad,WeightedQuad,QuadraticBarrier})
# ---------------------------------------------------------------------------
def act_quad(r):
    return 0.5 * np.sum(r * r, -1), r, np.ones_like(r)


def act_wquad(w):
    def f(r):
        return 0.5 * np.sum(w * r * r, -1), w * r, np.broadcast_to(w, r.shape).copy()

    return f


def act_barrier(lb, ub):
    def f(r):
        dl = r - lb
        du = r - ub
        rlb = np.minimum(dl, 0.0)
        rub = np.maximum(du, 0.0)
        a = 0.5 * np.sum(rlb * rlb, -1) + 0.5 * np.sum(rub * rub, -1)
        Arr = (dl <= 0.0).astype(float) + (du >= 0.0).astype(float)
        return a, rlb + rub, Arr

    return f


def q_soft_limit_terms(cfg: OCPConfig):
    """_make_q_soft_limit_cost (crocoddyl_classical.py:487-519)."""
    q_lb, q_ub = P.Q_LOWER, P.Q_UPPER
    q_ref = 0.5 * (q_lb + q_ub)
    m = max(cfg.q_soft_limit_margin, 0.0)
    lbs, ubs = q_lb + m, q_ub - m
    bad = lbs > ubs
    mid = 0.5 * (q_lb + q_ub)
    lbs = np.where(bad, mid - 1e-3, lbs)
    ubs = np.where(bad, mid + 1e-3, ubs)
    lb = np.concatenate([lbs - q_ref, np.full(7, -INF)])
    ub = np.concatenate([ubs - q_ref, np.full(7, INF)])
    x_ref = np.concatenate([q_ref, np.zeros(7)])
    return x_ref, lb, ub


def tau_soft_bounds(cfg: OCPConfig):
    """_make_tau_soft_limit_activation (crocoddyl_classical.py:478-485)."""
    lim = np.asarray(cfg.tau_limits, float)
    margin = min(max(cfg.tau_soft_limit_margin, 0.0), float(np.min(lim) - 1e-6))
    return -lim + margin, lim - margin


# ---------------------------------------------------------------------------
# differential action model: dynamics + costs, batched over nodes
# ---------------------------------------------------------------------------
def _contact_terms(cfg, q, v, a, p_star):
    """Contact Jacobian rows and drift a0 (LOCAL_WORLD_ALIGNED ContactModel1D/3D)."""
    kin = P.rnea_full(q, v, a)
    J, _, _ = P.frame_jacobian_lwa(q)
    Kp, Kd = cfg.contact_gains
    a0 = kin["acc_ee"] + Kp * (kin["p_ee"] - p_star) + Kd * kin["v_ee"]
    if cfg.nc == 1:
        return J[..., 2:3, :], a0[..., 2:3]
    return J[..., 0:3, :], a0


def _force_vec(cfg, lam):
    if cfg.nc == 1:
        z = np.zeros(lam.shape[:-1] + (2,), dtype=lam.dtype)
        return np.concatenate([z, lam], -1)
    return lam


def contact_star(cfg, p_ref):
    """z_target = p_ref_z - z_press;  p_contact = [p_ref_x, p_ref_y, z_target]  (:630-632)."""
    ps = np.array(p_ref, dtype=float, copy=True)
    ps[..., 2] = ps[..., 2] - cfg.z_press
    return ps


def dynamics(cfg, q, v, tau, surface, p_star):
    """Forward dynamics.  Free: a = M^-1 (tau - b).  Contact: the KKT system
    [[M, Jc^T], [Jc, -eps I]] [a; -lam] = [tau - b; -gamma], solved as
    pinocchio::forwardDynamics(model, data, q, v, tau, J, gamma, inv_damping)
    does it (Crocoddyl's ContactFwdDynamics calc): Cholesky of M, Y = L^-1
    Jc^T, S = Jc M^-1 Jc^T + eps I = Y^T Y + eps I, lam = -S^-1 (Jc M^-1
    (tau - b) + gamma), a = M^-1 (tau - b + Jc^T lam).  (A dense LU of the
    eps = 1e-8 KKT matrix loses ~8 digits: tools/ext_budget.py.)"""
    M = P.crba(q)
    b = P.rnea(q, v, np.zeros_like(q))
    L = cholesky(M)
    r = (tau - b)[..., None]
    Mr = chol_solve(L, r)  # M^-1 (tau - b)
    if not surface:
        return dict(a=Mr[..., 0], lam=None, M=M, L=L)
    Jc, gam = _contact_terms(cfg, q, v, np.zeros_like(q), p_star)
    nc = cfg.nc
    Y = tri_lower_solve(L, np.swapaxes(Jc, -1, -2))  # (..., 7, nc)
    S = P.mm(np.swapaxes(Y, -1, -2), Y) + cfg.contact_inv_damping * np.eye(nc)
    Ls = cholesky(S)
    lam = -chol_solve(Ls, P.mm(Jc, Mr) + gam[..., None])  # (..., nc, 1)
    a = Mr + chol_solve(L, P.mm(np.swapaxes(Jc, -1, -2), lam))
    return dict(a=a[..., 0], lam=lam[..., 0], M=M, L=L, Jc=Jc, Ls=Ls)


def dynamics_derivatives(cfg, q, v, dyn, surface, p_star):
    """Fx (…,7,14), Fu (…,7,7), df_dx (…,nc,14), df_du (…,nc,7)."""
    a = dyn["a"]
    x = np.concatenate([q, v], -1)
    eye7 = np.broadcast_to(np.eye(7, dtype=dyn["L"].dtype), dyn["L"].shape)
    Minv = chol_solve(dyn["L"], eye7)
    if not surface:
        tau_fn = lambda X: P.rnea(X[..., :7], X[..., 7:], a.astype(X.dtype))
        dtau = P.complex_step_jacobian(tau_fn, x)
        return dict(Fx=-P.mm(Minv, dtau), Fu=Minv, dfdx=None, dfdu=None)
    lam = dyn["lam"]
    fvec = _force_vec(cfg, lam)
    tau_fn = lambda X: P.rnea(X[..., :7], X[..., 7:], a.astype(X.dtype), fvec.astype(X.dtype))
    dtau = P.complex_step_jacobian(tau_fn, x)
    a0_fn = lambda X: _contact_terms(cfg, X[..., :7], X[..., 7:], a.astype(X.dtype), p_star)[1]
    da0 = P.complex_step_jacobian(a0_fn, x)
    # KKT inverse in the block form of pinocchio::getKKTContactDynamicMatrixInverse:
    # [[Minv - Minv Jc^T S^-1 Jc Minv, Minv Jc^T S^-1], [S^-1 Jc Minv, -S^-1]]
    Jc, Ls = dyn["Jc"], dyn["Ls"]
    nc = Jc.shape[-2]
    Sinv = chol_solve(Ls, np.broadcast_to(np.eye(nc, dtype=Ls.dtype), Ls.shape))
    MJt = P.mm(Minv, np.swapaxes(Jc, -1, -2))  # (..., 7, nc)
    Kal = P.mm(MJt, Sinv)
    Kla = np.swapaxes(Kal, -1, -2)
    Kaa = Minv - P.mm(Kal, np.swapaxes(MJt, -1, -2))
    Kll = -Sinv
    Fx = -P.mm(Kaa, dtau) - P.mm(Kal, da0)
    dfdx = P.mm(Kla, dtau) + P.mm(Kll, da0)
    return dict(Fx=Fx, Fu=Kaa, dfdx=dfdx, dfdu=-Kla)


def friction_cone(cfg):
    """crocoddyl.FrictionCone(R=I, mu, nf=4, inner_appr=False) as the reference
    builds it (crocoddyl_classical.py:999-1018, crocoddyl_force_feedback.py:1428-1447;
    Crocoddyl 2.x FrictionCone::update:
    facet rows (-mu e_z +- t_i)^T R^T with t_i = (cos th_i, sin th_i, 0),
    th_i = i 2 pi / nf, bounds (-inf, 0]; row nf = R e_z with bounds
    [min_nforce = 0, inf)), and the barrier bounds of
    _make_friction_barrier_activation (:891-903): finite bounds moved inwards by
    friction_margin."""
    nf = 4
    theta = 2.0 * np.pi / nf
    A = np.zeros((nf + 1, 3))
    for i in range(nf // 2):
        t = np.array([np.cos(theta * i), np.sin(theta * i), 0.0])
        mn = np.array([0.0, 0.0, -cfg.mu])
        A[2 * i] = mn + t
        A[2 * i + 1] = mn - t
    A[nf] = [0.0, 0.0, 1.0]
    lb = np.full(nf + 1, -INF)
    ub = np.zeros(nf + 1)
    lb[nf], ub[nf] = 0.0, INF
    eps = max(cfg.friction_margin, 0.0)
    lb = np.where(np.isfinite(lb), lb + eps, lb)
    ub = np.where(np.isfinite(ub), ub - eps, ub)
    return A, lb, ub


def cost_stack(cfg, surface, terminal):
    """Ordered cost list of _make_dam (crocoddyl_classical.py:567-718).

    Each entry: (name, residual kind, weight, activation builder args)."""
    costs = []
    x_ref_q, q_lb, q_ub = q_soft_limit_terms(cfg)
    if cfg.variant != "ff" or cfg.use_inner_state_reg:
        costs.append(("posture", "state_xreg", cfg.w_posture, ("quad",)))
        costs.append(("v_damp", "state_zero", cfg.w_v, ("wquad", np.concatenate([np.zeros(7), cfg.v_damp_weights]))))
    if cfg.w_q_soft_limits > 0.0:
        costs.append(("q_soft_limits", ("state_fixed", x_ref_q), cfg.w_q_soft_limits, ("barrier", q_lb, q_ub)))
    costs.append(("ee_ori", "frame_rot", cfg.w_ee_ori, ("wquad", np.asarray(cfg.ori_weights, float))))
    ww = np.asarray(cfg.w_wdamp_weights, float)
    costs.append(("w_damp", ("frame_vel", "zero"), cfg.w_wdamp, ("wquad", np.array([0, 0, 0, ww[0], ww[1], ww[2]]))))
    if not terminal and (cfg.variant != "ff" or cfg.use_inner_tau_reg):
        costs.append(("tau_reg", "control_tauref", cfg.w_tau, ("quad",)))
        if cfg.w_tau_soft_limits > 0.0:
            lb, ub = tau_soft_bounds(cfg)
            costs.append(("tau_soft_limits", "control_zero", cfg.w_tau_soft_limits, ("barrier", lb, ub)))
    if not surface:
        costs.append(("ee_pos", ("frame_trans", "pref"), cfg.w_ee_pos, ("wquad", np.array([1.0, 1.0, 2.5]))))
        return costs
    costs.append(("ee_xy", ("frame_trans", "pref"), cfg.w_tangent_pos, ("wquad", np.array([1.0, 1.0, 0.0]))))
    costs.append(("ee_vxy", ("frame_vel", "vref_xy"), cfg.w_tangent_vel, ("wquad", np.array([1.0, 1, 0, 0, 0, 0]))))
    if cfg.w_plane_z > 0.0:
        costs.append(("plane_z", ("frame_trans", "pcontact"), cfg.w_plane_z, ("wquad", np.array([0.0, 0.0, 1.0]))))
    if cfg.w_vz > 0.0:
        costs.append(("vz_damp", ("frame_vel", "zero"), cfg.w_vz, ("wquad", np.array([0.0, 0, 1, 0, 0, 0]))))
    nc = cfg.nc
    if nc == 3 and cfg.w_friction_cone > 0.0:
        A, lb, ub = friction_cone(cfg)
        costs.append(("friction_cone", ("force_cone", A), cfg.w_friction_cone, ("barrier", lb, ub)))
    if cfg.w_unilateral > 0.0:
        if nc == 1:
            lb, ub = np.array([cfg.friction_margin]), np.array([INF])
        else:
            lb, ub = np.array([-INF, -INF, cfg.friction_margin]), np.array([INF, INF, INF])
        costs.append(("unilateral", ("force", 0.0), cfg.w_unilateral, ("barrier", lb, ub)))
    if cfg.w_fn > 0.0:
        w = np.array([1.0]) if nc == 1 else np.array([0.0, 0.0, 1.0])
        costs.append(("fn_track", ("force", cfg.fn_des), cfg.w_fn, ("wquad", w)))
    return costs


def _activation(spec):
    if spec[0] == "quad":
        return act_quad
    if spec[0] == "wquad":
        return act_wquad(spec[1])
    return act_barrier(spec[1], spec[2])


def dam_eval(cfg, prob_refs, x, u, surface, mode, diff):
    """Evaluate the differential action model on a batch of nodes.

    prob_refs: dict with p_ref (...,3), v_ref (...,3), x_reg_ref (14), tau_ref (7)
    mode: "running" | "terminal_x" (classical terminal calc(x)) |
          "terminal_u" (FF terminal: running semantics, terminal cost set)
    Returns dict with a, lam, cost (DAM, unscaled), and if diff: Fx, Fu, Lx, Lu, Lxx, Lxu, Luu.
    """
    q, v = x[..., :7], x[..., 7:14]
    batch = x.shape[:-1]
    p_ref, v_ref = prob_refs["p_ref"], prob_refs["v_ref"]
    p_star = contact_star(cfg, p_ref)
    terminal = mode != "running"
    with_dyn = mode != "terminal_x"
    nc = cfg.nc
    out = {}
    dyn = None
    if with_dyn:
        dyn = dynamics(cfg, q, v, u, surface, p_star)
        out["a"], out["lam"] = dyn["a"], dyn["lam"]
    kin = P.rnea_full(q, v, np.zeros_like(q))
    J, R_ee, p_ee = P.frame_jacobian_lwa(q)
    v_frame = np.concatenate([kin["v_ee"], kin["w_ee"]], -1)
    if diff:
        def _vel(X):
            k = P.rnea_full(X[..., :7], X[..., 7:], np.zeros(X.shape[:-1] + (7,), dtype=X.dtype))
            return np.concatenate([k["v_ee"], k["w_ee"]], -1)

        dvel = P.complex_step_jacobian(_vel, x[..., :14])  # (...,6,14)
        ddyn = dynamics_derivatives(cfg, q, v, dyn, surface, p_star) if with_dyn else None
    cost = np.zeros(batch)
    Lx = np.zeros(batch + (14,))
    Lu = np.zeros(batch + (7,))
    Lxx = np.zeros(batch + (14, 14))
    Lxu = np.zeros(batch + (14, 7))
    Luu = np.zeros(batch + (7, 7))
    for name, kind, w, aspec in cost_stack(cfg, surface, terminal):
        act = _activation(aspec)
        Rx = Ru = None
        if kind == "state_xreg":
            r = x[..., :14] - prob_refs["x_reg_ref"]
            Rx = np.broadcast_to(np.eye(14), batch + (14, 14))
        elif kind == "state_zero":
            r = x[..., :14].copy()
            Rx = np.broadcast_to(np.eye(14), batch + (14, 14))
        elif isinstance(kind, tuple) and kind[0] == "state_fixed":
            r = x[..., :14] - kind[1]
            Rx = np.broadcast_to(np.eye(14), batch + (14, 14))
        elif kind == "control_tauref":
            r = u - prob_refs["tau_ref"]
            Ru = np.broadcast_to(np.eye(7), batch + (7, 7))
        elif kind == "control_zero":
            r = u.copy()
            Ru = np.broadcast_to(np.eye(7), batch + (7, 7))
        elif kind == "frame_rot":
            Rrel = P.mm(np.swapaxes(np.broadcast_to(cfg.R_des, R_ee.shape), -1, -2), R_ee)
            r, th = P.log3(Rrel)
            if diff:
                Jloc = P.mm(np.swapaxes(R_ee, -1, -2), J[..., 3:6, :])
                Rx = np.concatenate([P.mm(P.jlog3(r, th), Jloc), np.zeros(batch + (3, 7))], -1)
        elif kind[0] == "frame_trans":
            ref = p_ref if kind[1] == "pref" else p_star
            r = p_ee - ref
            if diff:
                Rx = np.concatenate([J[..., 0:3, :], np.zeros(batch + (3, 7))], -1)
        elif kind[0] == "frame_vel":
            if kind[1] == "zero":
                ref = np.zeros(batch + (6,))
            else:
                ref = np.concatenate([v_ref[..., 0:2], np.zeros(batch + (4,))], -1)
            r = v_frame - ref
            if diff:
                Rx = dvel
        elif kind[0] == "force_cone":
            # ResidualModelContactFrictionCone: r = A lambda (world-aligned force)
            A = kind[1]
            if mode == "terminal_x" or not surface:
                lam = np.zeros(batch + (nc,))
            else:
                lam = dyn["lam"]
            r = np.einsum("kr,...r->...k", A, lam)
            if diff:
                if mode == "terminal_x":
                    Rx = np.zeros(batch + (A.shape[0], 14))
                else:
                    Rx = np.einsum("kr,...ri->...ki", A, ddyn["dfdx"])
                    Ru = np.einsum("kr,...ri->...ki", A, ddyn["dfdu"])
        elif kind[0] == "force":
            fref = kind[1]
            if mode == "terminal_x" or not surface:
                lam = np.zeros(batch + (nc,))
            else:
                lam = dyn["lam"]
            if nc == 1:
                r = lam - fref
            else:
                r = lam - np.array([0.0, 0.0, fref])
            if diff:
                if mode == "terminal_x":
                    Rx = np.zeros(batch + (nc, 14))
                else:
                    Rx, Ru = ddyn["dfdx"], ddyn["dfdu"]
        else:
            raise ValueError(kind)
        a_val, Ar, Arr = act(r)
        cost = cost + w * a_val
        if diff:
            if Rx is not None:
                Lx = Lx + w * np.einsum("...ri,...r->...i", Rx, Ar)
                Lxx = Lxx + w * np.einsum("...ri,...r,...rj->...ij", Rx, Arr, Rx)
            if Ru is not None:
                Lu = Lu + w * np.einsum("...ri,...r->...i", Ru, Ar)
                Luu = Luu + w * np.einsum("...ri,...r,...rj->...ij", Ru, Arr, Ru)
            if Rx is not None and Ru is not None:
                Lxu = Lxu + w * np.einsum("...ri,...r,...rj->...ij", Rx, Arr, Ru)
    out["cost"] = cost
    if diff:
        out.update(Lx=Lx, Lu=Lu, Lxx=Lxx, Lxu=Lxu, Luu=Luu)
        if with_dyn:
            out["Fx"], out["Fu"] = ddyn["Fx"], ddyn["Fu"]
    return out


# ---------------------------------------------------------------------------
# integrated (Euler) action model, and the FF augmentation
# ---------------------------------------------------------------------------
def iam_eval(cfg, refs, x, u, surface, mode, diff):
    """IntegratedActionModelEuler.calc / calcDiff.  x (…,14), u (…,7)."""
    dt = cfg.dt
    d = dam_eval(cfg, refs, x, u, surface, mode, diff)
    out = dict(lam=d.get("lam"))
    if mode == "terminal_x":
        out["xnext"] = x.copy()
        out["cost"] = d["cost"]
        if diff:
            out.update(Lx=d["Lx"], Lxx=d["Lxx"])
        return out
    a = d["a"]
    v = x[..., 7:14]
    out["xnext"] = np.concatenate([x[..., :7] + v * dt + a * dt * dt, v + a * dt], -1)
    out["cost"] = dt * d["cost"]
    if diff:
        Fa_x, Fa_u = d["Fx"], d["Fu"]
        batch = x.shape[:-1]
        Fx = np.broadcast_to(np.eye(14, dtype=np.result_type(x, Fa_x)), batch + (14, 14)).copy()
        Fx[..., :7, :] += dt * dt * Fa_x
        Fx[..., 7:, :] += dt * Fa_x
        Fx[..., :7, 7:] += dt * np.eye(7)
        Fu = np.concatenate([dt * dt * Fa_u, dt * Fa_u], -2)
        out.update(
            Fx=Fx, Fu=Fu, Lx=dt * d["Lx"], Lu=dt * d["Lu"], Lxx=dt * d["Lxx"], Lxu=dt * d["Lxu"], Luu=dt * d["Luu"]
        )
    return out


def _ff_soft(cfg, w):
    """_AugmentedLPFActionModel._soft_limit_terms (crocoddyl_force_feedback.py:195-209)."""
    lim = np.maximum(np.asarray(cfg.tau_limits, float) - max(cfg.tau_soft_limit_margin, 0.0), 1.0e-9)
    over = np.maximum(np.abs(w) - lim, 0.0)
    active = over > 0.0
    cost = 0.5 * np.sum(over * over, -1)
    grad = np.where(active, over * np.sign(w), 0.0)
    return cost, grad, active.astype(float)


def ff_augment(cfg, inner, y, w, yref, diff):
    """Augmentation algebra of _AugmentedLPFActionModel.calc / calcDiff
    (crocoddyl_force_feedback.py:211-290) given the inner IAM results
    `inner` (xnext, cost and, if diff, Fx, Fu, Lx, Lu, Lxx, Lxu, Luu)."""
    alpha = float(np.clip(cfg.ff_alpha, 0.0, 0.999999))
    beta = 1.0 - alpha
    tau = y[..., 14:21]
    out = dict(lam=inner.get("lam"))
    out["xnext"] = np.concatenate([inner["xnext"], alpha * tau + beta * w], -1)
    cost = inner["cost"]
    Wy2 = np.square(np.asarray(cfg.y_weights, float))
    dy = y - yref
    w_y = max(cfg.w_y, 0.0)
    w_w = max(cfg.w_w, 0.0)
    w_s = max(cfg.w_w_soft_limits, 0.0)
    if w_y > 0.0:
        cost = cost + 0.5 * w_y * np.sum(Wy2 * dy * dy, -1)
    if w_w > 0.0:
        cost = cost + 0.5 * w_w * np.sum(w * w, -1)
    if w_s > 0.0:
        c_soft, g_soft, h_soft = _ff_soft(cfg, w)
        cost = cost + w_s * c_soft
    out["cost"] = cost
    if diff:
        batch = y.shape[:-1]
        fdt = np.result_type(y, inner["Fx"])
        Fx = np.zeros(batch + (21, 21), dtype=fdt)
        Fx[..., :14, :14] = inner["Fx"]
        Fx[..., :14, 14:] = inner["Fu"]
        Fx[..., 14:, 14:] = alpha * np.eye(7)
        Fu = np.zeros(batch + (21, 7), dtype=fdt)
        Fu[..., 14:, :] = beta * np.eye(7)
        Lx = np.concatenate([inner["Lx"], inner["Lu"]], -1)
        Lxx = np.zeros(batch + (21, 21), dtype=fdt)
        Lxx[..., :14, :14] = inner["Lxx"]
        Lxx[..., :14, 14:] = inner["Lxu"]
        Lxx[..., 14:, :14] = np.swapaxes(inner["Lxu"], -1, -2)
        Lxx[..., 14:, 14:] = inner["Luu"]
        Lu = np.zeros(batch + (7,))
        Luu = np.zeros(batch + (7, 7))
        if w_y > 0.0:
            Lx = Lx + w_y * (Wy2 * dy)
            Lxx = Lxx + w_y * np.diag(Wy2)
        if w_w > 0.0:
            Lu = Lu + w_w * w
            Luu = Luu + w_w * np.eye(7)
        if w_s > 0.0:
            Lu = Lu + w_s * g_soft
            Luu = Luu + w_s * (h_soft[..., :, None] * np.eye(7))
        out.update(Fx=Fx, Fu=Fu, Lx=Lx, Lu=Lu, Lxx=Lxx, Lxu=np.zeros(batch + (21, 7)), Luu=Luu)
    return out


def ff_eval(cfg, refs, y, w, surface, terminal, diff):
    """_AugmentedLPFActionModel around the inner IAM.  Terminal nodes are
    called by the solver without u -> w = 0 and the inner IAM is evaluated
    with running semantics at u = tau (R1)."""
    tau = y[..., 14:21]
    if terminal:
        w = np.zeros_like(tau)
    inner = iam_eval(cfg, refs, y[..., :14], tau, surface, "terminal_u" if terminal else "running", diff)
    return ff_augment(cfg, inner, y, w, refs["y_ref"], diff)


def node_refs(prob: Problem, idx):
    return dict(
        p_ref=prob.p_ref[idx],
        v_ref=prob.v_ref[idx],
        x_reg_ref=prob.x_reg_ref,
        tau_ref=prob.tau_ref,
        y_ref=prob.x0,
    )


def running_eval(cfg, prob, idx, x, u, diff):
    refs = node_refs(prob, idx)
    if cfg.variant == "ff":
        return ff_eval(cfg, refs, x, u, prob.surface, False, diff)
    return iam_eval(cfg, refs, x, u, prob.surface, "running", diff)


def terminal_eval(cfg, prob, x, diff):
    N = cfg.horizon
    refs = node_refs(prob, N)
    if cfg.variant == "ff":
        return ff_eval(cfg, refs, x, None, prob.surface, True, diff)
    return iam_eval(cfg, refs, x, None, prob.surface, "terminal_x", diff)


class RobotOCP:
    """The reference's ShootingProblem for one instance, as the solver sees it."""

    def __init__(self, cfg: OCPConfig, prob: Problem):
        self.cfg, self.prob = cfg, prob
        self.N, self.nx, self.nu = cfg.horizon, cfg.nx, 7
        self.x0 = prob.x0
        self.u_lb = -np.asarray(cfg.tau_limits, float)
        self.u_ub = np.asarray(cfg.tau_limits, float)

    def running(self, idx, x, u, diff):
        return running_eval(self.cfg, self.prob, idx, x, u, diff)

    def terminal(self, x, diff):
        return terminal_eval(self.cfg, self.prob, x, diff)


class LQRProblem:
    """Linear dynamics x+ = A x + B u + c, cost 0.5 x'Qx + q'x + 0.5 u'Ru + r'u per
    running node (terminal: Qf, qf) — a known-answer model for the solver."""

    def __init__(self, A, B, c, Q, q, R, r, Qf, qf, x0, N, u_lb=None, u_ub=None):
        self.A, self.B, self.c, self.Q, self.q, self.R, self.r, self.Qf, self.qf = A, B, c, Q, q, R, r, Qf, qf
        self.x0, self.N = np.asarray(x0, float), int(N)
        self.nx, self.nu = A.shape[0], B.shape[1]
        inf = np.full(self.nu, np.inf)
        self.u_lb = -inf if u_lb is None else np.asarray(u_lb, float)
        self.u_ub = inf if u_ub is None else np.asarray(u_ub, float)

    def running(self, idx, x, u, diff):
        xn = x @ self.A.T + u @ self.B.T + self.c
        cost = 0.5 * np.einsum("...i,ij,...j->...", x, self.Q, x) + x @ self.q
        cost = cost + 0.5 * np.einsum("...i,ij,...j->...", u, self.R, u) + u @ self.r
        out = dict(xnext=xn, cost=cost, lam=None)
        if diff:
            b = x.shape[:-1]
            out.update(
                Fx=np.broadcast_to(self.A, b + self.A.shape).copy(), Fu=np.broadcast_to(self.B, b + self.B.shape).copy(),
                Lx=x @ self.Q + self.q, Lu=u @ self.R + self.r,
                Lxx=np.broadcast_to(self.Q, b + self.Q.shape).copy(), Luu=np.broadcast_to(self.R, b + self.R.shape).copy(),
                Lxu=np.zeros(b + (self.nx, self.nu)),
            )
        return out

    def terminal(self, x, diff):
        out = dict(xnext=x.copy(), cost=0.5 * x @ self.Qf @ x + self.qf @ x, lam=None)
        if diff:
            out.update(Lx=self.Qf @ x + self.qf, Lxx=self.Qf.copy())
        return out
