#!/usr/bin/env python3
"""Generate golden vectors by executing the REFERENCE's own code (numpy-only
parts) in this container.  Output: tests/golden/reference_vectors.npz.

What runs (all under /root/reference/src, read-only, never copied):
  * src/tasks/trajectories.py::make_approach_then_circle  (plain import)
  * src/mpc/crocoddyl_force_feedback.py::_AugmentedLPFActionModel.calc/calcDiff
    with a synthetic inner model (fixed random Fx, Fu, L*, xnext, cost)
  * ForceFeedbackCrocoddylMPC._shift_guess / _policy_control / _safe_tau /
    _ff_alpha_ocp / _ff_alpha_ctrl / _policy_epsilon / _align_logged_force_prediction
  * ClassicalCrocoddylMPC._shift_guess / _policy_control / _safe_tau
The controller modules import crocoddyl, pinocchio and example_robot_data at
module level; none is installed, so inert placeholder
modules are registered in sys.modules solely to let the import succeed.  The
methods exercised here use numpy only (plus the placeholder base classes
ActionModelAbstract / ActionDataAbstract / StateVector, which just store
attributes).  Controller objects are created with object.__new__ and only the
attributes those methods read.

Run:  python tests/golden/make_golden.py   (needs /root/reference)
"""
from __future__ import annotations

import sys
import types
from pathlib import Path

import numpy as np

REF = Path("/root/reference")
OUT = Path(__file__).resolve().parent / "reference_vectors.npz"


def _install_placeholders():
    croc = types.ModuleType("crocoddyl")

    class StateVector:
        def __init__(self, nx):
            self.nx = int(nx)
            self.ndx = int(nx)

    class ActionModelAbstract:
        def __init__(self, state, nu, nr=1):
            self.state = state
            self.nu = nu
            self.nr = nr

    class ActionDataAbstract:
        def __init__(self, model):
            self.model = model

    croc.StateVector = StateVector
    croc.ActionModelAbstract = ActionModelAbstract
    croc.ActionDataAbstract = ActionDataAbstract
    pin = types.ModuleType("pinocchio")
    pin.Model = object
    pin.Data = object
    erd = types.ModuleType("example_robot_data")
    erd.load = None
    sys.modules.setdefault("crocoddyl", croc)
    sys.modules.setdefault("pinocchio", pin)
    sys.modules.setdefault("example_robot_data", erd)


def main():
    if not REF.exists():
        raise SystemExit("needs /root/reference")
    sys.path.insert(0, str(REF))
    _install_placeholders()
    from src.tasks.trajectories import make_approach_then_circle
    from src.mpc import crocoddyl_force_feedback as FFM
    from src.mpc import crocoddyl_classical as CLM

    rng = np.random.default_rng(20261015)
    out = {}

    # ---- trajectories: benchmark parameters (run_classical.py:221-255) and a raw variant
    ee_start = np.array([-0.29997502, 0.0, 0.63314633])
    center = np.array([-0.5, 0.0, 0.342])
    tb = make_approach_then_circle(center=center, radius=0.10, omega=1.5, z_pre=0.392, z_contact=0.342,
                                   t_approach=0.55, ee_start=ee_start, t_pre=0.25)
    tr = make_approach_then_circle(center=center, radius=0.07, omega=2.0, z_contact=0.35, t_approach=1.0)
    ts = np.concatenate([np.linspace(0.0, 2.0, 401), rng.uniform(0.0, 20.0, 200)])
    for name, f in (("traj_bench", tb), ("traj_raw", tr)):
        P = np.zeros((ts.size, 3))
        V = np.zeros((ts.size, 3))
        Sf = np.zeros(ts.size)
        for i, t in enumerate(ts):
            p, v, s = f(float(t))
            P[i], V[i], Sf[i] = p, v, float(s)
        out[f"{name}_t"] = ts
        out[f"{name}_p"] = P
        out[f"{name}_v"] = V
        out[f"{name}_surf"] = Sf
    out["traj_bench_args"] = np.concatenate([center, [0.10, 1.5, 0.392, 0.342, 0.55, 0.25], ee_start])

    # ---- _AugmentedLPFActionModel algebra (crocoddyl_force_feedback.py:149-290)
    class Inner:
        def __init__(self, seed):
            r = np.random.default_rng(seed)
            self.xnext = r.normal(size=14)
            self.cost = float(r.uniform(1, 5))
            self.Fx = r.normal(size=(14, 14))
            self.Fu = r.normal(size=(14, 7))
            self.Lx = r.normal(size=14)
            self.Lu = r.normal(size=7)
            A = r.normal(size=(21, 21))
            H = A @ A.T
            self.Lxx, self.Lxu, self.Luu = H[:14, :14], H[:14, 14:], H[14:, 14:]

        def createData(self):
            return types.SimpleNamespace()

        def _fill(self, data):
            for k in ("xnext", "cost", "Fx", "Fu", "Lx", "Lu", "Lxx", "Lxu", "Luu"):
                setattr(data, k, getattr(self, k))

        def calc(self, data, x, u):
            self.last_calc = (np.array(x), np.array(u))
            self._fill(data)

        def calcDiff(self, data, x, u):
            self._fill(data)

    tau_lim = np.array([87.0, 87, 87, 87, 12, 12, 12])
    cases = []
    for c in range(6):
        inner = Inner(100 + c)
        alpha = float(rng.uniform(0.1, 0.9))
        w_reg, w_soft, w_y = float(rng.uniform(0, 1e-2)), float(rng.uniform(0.5, 3)), float(rng.uniform(0, 1e-2))
        y_ref = rng.normal(size=21)
        y_w = rng.uniform(0.01, 0.5, size=21)
        m = FFM._AugmentedLPFActionModel(inner, 14, 7, alpha, w_reg, w_soft, tau_lim, 0.2, w_y, y_ref, y_w)
        d = m.createData()
        x = rng.normal(size=21)
        u = rng.normal(size=7) * np.array([50, 50, 50, 50, 14, 14, 14])  # some entries beyond the soft limits
        terminal = c == 5
        if terminal:
            m.calc(d, x)
            m.calcDiff(d, x)
            u = np.zeros(7)
        else:
            m.calc(d, x, u)
            m.calcDiff(d, x, u)
        rec = np.concatenate([
            [alpha, w_reg, w_soft, w_y, float(terminal)], y_ref, y_w, x, u,
            inner.xnext, [inner.cost], inner.Fx.ravel(), inner.Fu.ravel(), inner.Lx, inner.Lu,
            inner.Lxx.ravel(), inner.Lxu.ravel(), inner.Luu.ravel(),
            d.xnext, [d.cost], d.Fx.ravel(), d.Fu.ravel(), d.Lx, d.Lu, d.Lxx.ravel(), d.Luu.ravel(), d.Lxu.ravel(),
            inner.last_calc[1],
        ])
        cases.append(rec)
    out["ff_aug"] = np.stack(cases)

    # ---- FF controller helpers
    def ff_ctrl(cutoff=25.0, dt=0.005, dt_ocp=0.01, scale=0.55, interp=True, inverse=True):
        o = object.__new__(FFM.ForceFeedbackCrocoddylMPC)
        o.cfg = FFM.ForceFeedbackMPCConfig(horizon=6, dt=dt, dt_ocp=dt_ocp, ff_cutoff_hz=cutoff,
                                           feedback_gain_scale=scale, ff_use_tau_interpolation=interp,
                                           ff_inverse_actuation_model=inverse)
        o.sim = types.SimpleNamespace(dt=dt)
        o.nx_mb, o.ndx_mb, o.nx_aug = 14, 14, 21
        o.actuation = types.SimpleNamespace(nu=7)
        o._warned_keys = set()
        o._tau_prev = rng.normal(size=7)
        o._fn_pred_hist_raw, o._fn_pred_hist_meas, o._fn_pred_corr = [], [], np.nan
        return o

    o = ff_ctrl()
    out["ff_alpha"] = np.array([o._ff_alpha_ocp(), o._ff_alpha_ctrl(), o._policy_epsilon()])
    N = 6
    xs = [rng.normal(size=21) for _ in range(N + 1)]
    us = [rng.normal(size=7) for _ in range(N)]
    Ks = [rng.normal(size=(7, 21)) for _ in range(N)]
    y_now = rng.normal(size=21)
    o.xs, o.us, o.Ks = xs, us, Ks
    tau_pol, _ = o._policy_control(y_now)
    xi, ui = o._shift_guess(y_now, N)
    o.xs = None
    xi_c, ui_c = o._shift_guess(y_now, N)
    out["ff_policy_in"] = np.concatenate([np.ravel(xs), np.ravel(us), np.ravel(Ks), y_now])
    out["ff_policy_out"] = np.concatenate([tau_pol, np.ravel(xi), np.ravel(ui), np.ravel(xi_c), np.ravel(ui_c)])
    # safe tau (no command filter)
    tt = rng.normal(size=(5, 7)) * 60.0
    tt[2, 3] = np.nan
    st = []
    for row in tt:
        st.append(o._safe_tau(row))
    out["safe_tau_in"] = tt
    out["safe_tau_out"] = np.stack(st)
    # force-prediction alignment (rolling affine fit), 150 samples
    oa = ff_ctrl()
    raw = 20 + 3 * np.sin(np.linspace(0, 9, 150)) + rng.normal(0, 0.2, 150)
    meas = 0.8 * np.roll(raw, 3) + 4 + rng.normal(0, 0.1, 150)
    al = [oa._align_logged_force_prediction(float(r), float(mm), True) for r, mm in zip(raw, meas)]
    out["align_in"] = np.stack([raw, meas])
    out["align_out"] = np.array(al)

    # ---- classical controller helpers
    oc = object.__new__(CLM.ClassicalCrocoddylMPC)
    oc.cfg = CLM.ClassicalMPCConfig(horizon=N, feedback_gain_scale=0.55)
    oc._tau_prev = rng.normal(size=7)
    cx = [rng.normal(size=14) for _ in range(N + 1)]
    cu = [rng.normal(size=7) for _ in range(N)]
    cK = [rng.normal(size=(7, 14)) for _ in range(N)]
    x_now = rng.normal(size=14)
    oc.xs, oc.us, oc.Ks = cx, cu, cK
    u_pol, _ = oc._policy_control(x_now)
    cxi, cui = oc._shift_guess(x_now, N)
    out["cl_policy_in"] = np.concatenate([np.ravel(cx), np.ravel(cu), np.ravel(cK), x_now, oc._tau_prev])
    out["cl_policy_out"] = np.concatenate([u_pol, np.ravel(cxi), np.ravel(cui)])

    np.savez_compressed(OUT, **out)
    print("wrote", OUT, {k: v.shape for k, v in out.items()})


if __name__ == "__main__":
    main()
