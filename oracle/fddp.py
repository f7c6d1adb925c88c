"""ORACLE — test infrastructure only.  Never imported by the product path.

numpy fp64 restatement of crocoddyl::SolverBoxFDDP (and SolverFDDP) as called
by the reference at src/mpc/crocoddyl_classical.py:367 and
src/mpc/crocoddyl_force_feedback.py:605:

    ok = solver.solve(xs_init, us_init, max_iters, False)

Crocoddyl is not vendored in /root/reference and is not installed here
(SURVEY.md §8(c)); the algorithm restated below is the public Crocoddyl 2.x
one: SolverDDP::backwardPass / computeGains,
SolverFDDP::solve / forwardPass / updateExpectedImprovement /
expectedImprovement, SolverBoxFDDP::computeGains / forwardPass, BoxQP::solve.
Every constant lives in `Consts`.

Documented deviations:
  * calcDiff is always evaluated fresh at (xs, us); Crocoddyl re-uses the
    datas of the last tried line-search step after a fully rejected line
    search (R7 edge case).
  * BoxQP warm start x_init = clamp(k_prev) with k = 0 at solve start.
Parity against real Crocoddyl: UNPINNED (pinned by the LQR known answer,
the BoxQP KKT conditions and finite-difference tests in tests/).
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field

import numpy as np

from . import ocp


@dataclass
class Consts:
    th_stop_box: float = 5e-5  # SolverBoxFDDP constructor
    th_stop_fddp: float = 1e-9  # SolverAbstract default
    th_grad: float = 1e-12
    th_acceptstep: float = 0.1
    th_acceptnegstep: float = 2.0
    # ascent-direction comparator (include/ffddp.h FFDDP_NEGSTEP_*):
    # 0 = Crocoddyl's `dV < th_acceptnegstep * dVexp`, 1 = bounded rise `>`
    neg_step_rule: int = 0
    th_stepdec: float = 0.5
    th_stepinc: float = 0.01
    reg_min: float = 1e-9
    reg_max: float = 1e9
    reg_incfactor: float = 10.0
    reg_decfactor: float = 10.0
    alphas: tuple = tuple(1.0 / 2.0**n for n in range(10))
    qp_maxiter: int = 100
    qp_th_acceptstep: float = 0.1
    qp_th_grad: float = 1e-5
    qp_reg: float = 0.0
    # feasible-iteration gains on the BoxQP free set: "crocoddyl" = K =
    # Quu_inv Qxu^T with the explicit Hff_inv (SolverBoxFDDP::computeGains),
    # "solve" = Cholesky solves with Hff's factor, the HIP kernel's evaluation
    # order.  Same mathematics; the explicit inverse carries ~100x more
    # rounding error (tools/ext_budget.py, profiles/r03_ext_budget.jsonl).
    gains_form: str = "crocoddyl"


class BackwardError(Exception):
    pass


class ForwardError(Exception):
    pass


def raise_if_nan(value: float) -> bool:
    """crocoddyl::raiseIfNaN."""
    return bool(math.isnan(value) or math.isinf(value) or value >= 1e30)


def llt(H):
    """Eigen::LLT: fails if a pivot is <= 0 (or NaN)."""
    n = H.shape[0]
    L = np.zeros_like(H)
    for j in range(n):
        d = H[j, j] - np.dot(L[j, :j], L[j, :j])
        if not (d > 0.0):
            raise BackwardError("llt")
        L[j, j] = np.sqrt(d)
        for i in range(j + 1, n):
            L[i, j] = (H[i, j] - np.dot(L[i, :j], L[j, :j])) / L[j, j]
    return L


def llt_solve(L, B):
    Y = ocp.solve(L, B if B.ndim == 2 else B[:, None])
    X = ocp.solve(L.T, Y)
    return X if B.ndim == 2 else X[:, 0]


def boxqp(H, q, lb, ub, xinit, c: Consts, stall_exit: bool = False, info: dict | None = None):
    """crocoddyl::BoxQP::solve (projected Newton).  Returns x, free, clamped, Hff_inv.

    stall_exit: stop at the first iteration whose line search accepts no step
    length (the kernel's rule, boxqp_lanes); Crocoddyl runs on to maxiter with
    x unchanged.  info (optional dict) receives the iterations run and whether
    the loop stopped that way."""
    n = q.shape[0]
    x = np.maximum(np.minimum(xinit, ub), lb)
    free, clamped, Hff_inv = list(range(n)), [], None
    if info is not None:
        info.update(iters=0, stalled=False)
    for _ in range(c.qp_maxiter):
        if info is not None:
            info["iters"] += 1
        g = q + H @ x
        free, clamped = [], []
        for j in range(n):
            if (x[j] == lb[j] and g[j] > 0.0) or (x[j] == ub[j] and g[j] < 0.0):
                clamped.append(j)
            else:
                free.append(j)
        nf = len(free)
        Hff = H[np.ix_(free, free)].copy()
        if c.qp_reg != 0.0:
            Hff[np.diag_indices(nf)] += c.qp_reg
        L = llt(Hff) if nf > 0 else np.zeros((0, 0))
        Hff_inv = llt_solve(L, np.eye(nf, dtype=H.dtype)) if nf > 0 else np.zeros((0, 0))
        dxf = -q[free]
        if clamped:
            dxf = dxf - H[np.ix_(free, clamped)] @ x[clamped]
        dxf = llt_solve(L, dxf) if nf > 0 else dxf
        dxf = dxf - x[free]
        dx = np.zeros(n, dtype=np.result_type(H, q))
        dx[free] = dxf
        if np.max(np.abs(dx)) < c.qp_th_grad:
            break
        fold = 0.5 * x @ (H @ x) + q @ x
        for a in c.alphas:
            xn = np.maximum(np.minimum(x + a * dx, ub), lb)
            fnew = 0.5 * xn @ (H @ xn) + q @ xn
            if fold - fnew > c.qp_th_acceptstep * (g @ (x - xn)):
                x = xn
                break
        else:
            if info is not None and not info["stalled"]:
                info["stall_iter"] = info["iters"] - 1
            if info is not None:
                info["stalled"] = True
            if stall_exit:
                break
    return x, free, clamped, Hff_inv


def accept_step(c: Consts, is_feasible: bool, dV: float, d0: float, dVexp: float) -> bool:
    """SolverFDDP::solve step acceptance for one trial.
    Descent direction (dVexp >= 0): |d0| < th_grad or dV > th_acceptstep dVexp.
    Ascent direction (dVexp < 0, closing the gaps may raise the cost): only
    while infeasible (`!is_feasible_ && ...`), with Crocoddyl's comparator
    `dV < th_acceptnegstep * dVexp` (neg_step_rule 0, the default), or the
    bounded-rise alternative `dV > th_acceptnegstep * dVexp` (rule 1: a rise
    of at most th_acceptnegstep x the predicted one; the only one of the two
    that accepts the exact LQR step whose cost must rise, see
    tests/test_oracle.py::test_fddp_lqr_known_answer).  The HIP kernel's
    trial_accepted and oracle/cpu implement the same switch."""
    if dVexp >= 0:
        return abs(d0) < c.th_grad or dV > c.th_acceptstep * dVexp
    if is_feasible:
        return False
    if c.neg_step_rule == 0:
        return dV < c.th_acceptnegstep * dVexp
    return dV > c.th_acceptnegstep * dVexp


@dataclass
class Stats:
    iters_run: int = 0  # calcDiff+backward executions (I)
    trials: int = 0  # line-search trials a sequential solver executes (L)
    reg_retries: int = 0
    forward_errors: int = 0  # line-search trials rejected as non-finite (raiseIfNaN)
    neg_branch: int = 0  # trials judged by the ascent-direction (dVexp < 0) branch
    neg_accepted: int = 0  # ... and accepted by it
    clamped: int = 0  # BoxQP solutions with at least one active bound


class SolverBoxFDDP:
    """Per-instance solver on one ocp.Problem (setProblem + solve surface)."""

    def __init__(self, cfg_or_model, prob: ocp.Problem | None = None, box: bool = True, consts: Consts | None = None,
                 dtype=np.float64):
        """SolverBoxFDDP(problem): either (OCPConfig, Problem) for the reference
        OCP, or a model object with running()/terminal()/x0/N/nx/nu/u_lb/u_ub.
        dtype: the solver's working precision (np.longdouble for the
        extended-precision error budget, tools/ext_budget.py); fp64 results
        are unchanged by it."""
        model = ocp.RobotOCP(cfg_or_model, prob) if prob is not None else cfg_or_model
        self.model, self.box = model, box
        self.cfg, self.prob = getattr(model, "cfg", None), getattr(model, "prob", None)
        self.c = consts or Consts()
        self.th_stop = self.c.th_stop_box if box else self.c.th_stop_fddp
        N, nx, nu = model.N, model.nx, model.nu
        self.N, self.nx, self.nu = N, nx, nu
        self.dt = np.dtype(dtype)
        self.x0 = np.asarray(model.x0, self.dt)
        self.u_lb = np.asarray(model.u_lb, float)
        self.u_ub = np.asarray(model.u_ub, float)
        self.k = np.zeros((N, nu), self.dt)
        self.K = np.zeros((N, nu, nx), self.dt)
        self.stats = Stats()

    def _num(self, v):
        """A scalar in the working precision (a Python float for fp64)."""
        return float(v) if self.dt == np.float64 else self.dt.type(v)

    # --- problem evaluations -------------------------------------------------
    def _calc_diff(self):
        N = self.N
        run = self.model.running(slice(0, N), self.xs[:N], self.us, True)
        term = self.model.terminal(self.xs[N], True)
        self.run, self.term = run, term
        self.cost = self._num(np.sum(run["cost"]) + term["cost"])  # ShootingProblem::calcDiff sum
        self.fs = np.zeros((N + 1, self.nx), self.dt)
        if not self.is_feasible:
            self.fs[0] = self.x0 - self.xs[0]
            self.fs[1:] = run["xnext"] - self.xs[1:]
        self.ffeas = self._num(np.max(np.abs(self.fs)))  # ||ffeas||_inf of this calcDiff

    def _backward(self):
        N, c = self.N, self.c
        run, term = self.run, self.term
        preg = self.preg
        Vxx = [None] * (N + 1)
        Vx = [None] * (N + 1)
        Qu = np.zeros((N, self.nu), self.dt)
        Quu = np.zeros((N, self.nu, self.nu), self.dt)
        K = self.K  # Crocoddyl overwrites K_/k_ in place (a retried pass sees partial updates)
        k = self.k
        Vxx[N] = term["Lxx"].copy() + preg * np.eye(self.nx)
        Vx[N] = term["Lx"].copy()
        if not self.is_feasible:
            Vx[N] = Vx[N] + Vxx[N] @ self.fs[N]
        for t in range(N - 1, -1, -1):
            Fx, Fu = run["Fx"][t], run["Fu"][t]
            Vxx_p, Vx_p = Vxx[t + 1], Vx[t + 1]
            FxTV = Fx.T @ Vxx_p
            Qx = run["Lx"][t] + Fx.T @ Vx_p
            Qxx = run["Lxx"][t] + FxTV @ Fx
            FuTV = Fu.T @ Vxx_p
            Qu_t = run["Lu"][t] + Fu.T @ Vx_p
            Quu_t = run["Luu"][t] + FuTV @ Fu
            Qxu = run["Lxu"][t] + FxTV @ Fu
            Quu_t = Quu_t + preg * np.eye(self.nu)
            if (not self.box) or (not self.is_feasible):
                L = llt(Quu_t)
                K[t] = llt_solve(L, Qxu.T)
                k[t] = llt_solve(L, Qu_t)
            else:
                lb = self.u_lb - self.us[t]
                ub = self.u_ub - self.us[t]
                x, free, clamped, Hff_inv = boxqp(Quu_t, Qu_t, lb, ub, self.k[t], c)
                Quu_inv = np.zeros((self.nu, self.nu), self.dt)
                if free:
                    Quu_inv[np.ix_(free, free)] = Hff_inv
                if c.gains_form == "crocoddyl" or not free:
                    K[t] = Quu_inv @ Qxu.T
                else:  # "solve": K_f = Hff^-1 Qxu_f^T by the Cholesky factor (the HIP kernel's order)
                    K[t] = 0.0
                    K[t][free] = llt_solve(llt(Quu_t[np.ix_(free, free)]), Qxu.T[free])
                k[t] = -x
                if clamped:
                    self.stats.clamped += 1
                Qu_t = Qu_t.copy()
                Qu_t[clamped] = 0.0
            Vx_t = Qx - K[t].T @ Qu_t
            Vxx_t = Qxx - Qxu @ K[t]
            Vxx_t = 0.5 * (Vxx_t + Vxx_t.T)
            Vxx_t = Vxx_t + preg * np.eye(self.nx)
            if not self.is_feasible:
                Vx_t = Vx_t + Vxx_t @ self.fs[t]
            if raise_if_nan(float(np.max(np.abs(Vx_t)))) or raise_if_nan(float(np.max(np.abs(Vxx_t)))):
                raise BackwardError("nan")
            Vxx[t], Vx[t] = Vxx_t, Vx_t
            Qu[t], Quu[t] = Qu_t, Quu_t
        self.Vxx, self.Vx, self.Qu, self.Quu = Vxx, Vx, Qu, Quu

    def _update_expected_improvement(self):
        dg = dq = 0.0
        N = self.N
        if not self.is_feasible:
            dg -= self.Vx[N] @ self.fs[N]
            dq += self.fs[N] @ (self.Vxx[N] @ self.fs[N])
        for t in range(N):
            dg += self.Qu[t] @ self.k[t]
            dq -= self.k[t] @ (self.Quu[t] @ self.k[t])
            if not self.is_feasible:
                dg -= self.Vx[t] @ self.fs[t]
                dq += self.fs[t] @ (self.Vxx[t] @ self.fs[t])
        self.dg, self.dq = dg, dq

    def _expected_improvement(self, xs_try):
        dv = 0.0
        if not self.is_feasible:
            for t in range(self.N + 1):
                dx = self.xs[t] - xs_try[t]
                dv -= self.fs[t] @ (self.Vxx[t] @ dx)
        return self.dg + dv, self.dq - 2.0 * dv

    def _forward(self, alpha):
        N = self.N
        xs_try = np.zeros_like(self.xs)
        us_try = np.zeros_like(self.us)
        cost_try = self._num(0.0)
        xnext = self.x0.copy()
        gap = not (self.is_feasible or alpha == 1.0)
        for t in range(N):
            xs_try[t] = xnext + self.fs[t] * (alpha - 1.0) if gap else xnext
            dx = xs_try[t] - self.xs[t]
            u = self.us[t] - self.k[t] * alpha - self.K[t] @ dx
            if self.box:
                u = np.minimum(np.maximum(u, self.u_lb), self.u_ub)
            us_try[t] = u
            d = self.model.running(t, xs_try[t], us_try[t], False)
            xnext = d["xnext"]
            cost_try += self._num(d["cost"])
            if raise_if_nan(float(cost_try)) or raise_if_nan(float(np.max(np.abs(xnext)))):
                raise ForwardError("nan")
        xs_try[N] = xnext + self.fs[N] * (alpha - 1.0) if gap else xnext
        d = self.model.terminal(xs_try[N], False)
        cost_try += self._num(d["cost"])
        if raise_if_nan(float(cost_try)):
            raise ForwardError("nan")
        return xs_try, us_try, cost_try

    def _increase_reg(self):
        self.preg = min(self.preg * self.c.reg_incfactor, self.c.reg_max)

    def _decrease_reg(self):
        self.preg = max(self.preg / self.c.reg_decfactor, self.c.reg_min)

    # --- SolverFDDP::solve -----------------------------------------------------
    def solve(self, xs_init, us_init, maxiter: int = 10, is_feasible: bool = False, init_reg: float = float("nan")):
        c = self.c
        self.xs = np.array(xs_init, dtype=self.dt, copy=True)
        self.us = np.array(us_init, dtype=self.dt, copy=True)
        self.is_feasible = bool(is_feasible)
        self.preg = c.reg_min if math.isnan(init_reg) else float(init_reg)
        self.was_feasible = False
        self.k = np.zeros((self.N, self.nu), self.dt)
        self.K = np.zeros((self.N, self.nu, self.nx), self.dt)
        self.stats = Stats()
        self.stop = float("nan")
        # CallbackVerbose records (include/ffddp.h ffddp_trace_*): iter, cost,
        # stop, grad = -d1, preg, dreg, step, ffeas, dV, dVexp
        self.trace = []
        self.ffeas = 0.0
        recalc = True
        self.iter = 0
        for it in range(maxiter):
            self.iter = it
            while True:
                try:
                    if recalc:
                        self._calc_diff()
                    self.stats.iters_run += 1
                    self._backward()
                except BackwardError:
                    recalc = False
                    self.stats.reg_retries += 1
                    self._increase_reg()
                    if self.preg == c.reg_max:
                        return False
                    continue
                break
            self._update_expected_improvement()
            steplength = c.alphas[0]
            tdV = tdVexp = td1 = float("nan")
            for steplength in c.alphas:
                self.stats.trials += 1
                try:
                    xs_try, us_try, cost_try = self._forward(steplength)
                except ForwardError:
                    self.stats.forward_errors += 1
                    continue
                dV = self.cost - cost_try
                d0, d1 = self._expected_improvement(xs_try)
                dVexp = steplength * (d0 + 0.5 * steplength * d1)
                tdV, tdVexp, td1 = dV, dVexp, d1
                if dVexp < 0:
                    self.stats.neg_branch += 1
                ok = accept_step(c, self.is_feasible, dV, d0, dVexp)
                if ok and dVexp < 0:
                    self.stats.neg_accepted += 1
                if ok:
                    self.was_feasible = self.is_feasible
                    self.xs, self.us = xs_try, us_try
                    self.is_feasible = self.was_feasible or steplength == 1.0
                    self.cost = cost_try
                    recalc = True
                    break
            if steplength > c.th_stepdec:
                self._decrease_reg()
            if steplength <= c.th_stepinc:
                self._increase_reg()
                if self.preg == c.reg_max:
                    return False
            self.stop = self._num(np.sum(self.Qu * self.Qu))
            self.trace.append((it, self.cost, self.stop, -td1, self.preg, self.preg, steplength, self.ffeas, tdV, tdVexp))
            if self.was_feasible and self.stop < self.th_stop:
                return True
        self.iter = maxiter
        return False

    def contact_force(self, t: int):
        """lambda at knot t evaluated at the final (xs, us) (fn_pred source, R7)."""
        d = self.model.running(t, self.xs[t], self.us[t], False)
        return d["lam"]
