"""Golden vectors produced by the reference's own Python (tests/golden/
make_golden.py) against the product host code and the oracle.  CPU only; the
fixtures are data, the reference is not needed at test time."""
from __future__ import annotations

import types
from pathlib import Path

import numpy as np
import pytest

from ffddp import controller as CT
from ffddp import trajectory as TR
from oracle import ocp

G = np.load(Path(__file__).resolve().parent / "golden" / "reference_vectors.npz")


def _traj_check(name, f):
    ts = G[f"{name}_t"]
    for i, t in enumerate(ts):
        p, v, s = f(float(t))
        np.testing.assert_allclose(p, G[f"{name}_p"][i], rtol=0, atol=1e-14)
        np.testing.assert_allclose(v, G[f"{name}_v"][i], rtol=0, atol=1e-14)
        assert bool(s) == bool(G[f"{name}_surf"][i])


def test_trajectory_benchmark_params():
    a = G["traj_bench_args"]
    f = TR.make_approach_then_circle(center=a[0:3], radius=a[3], omega=a[4], z_pre=a[5], z_contact=a[6],
                                     t_approach=a[7], ee_start=a[9:12], t_pre=a[8])
    _traj_check("traj_bench", f)


def test_trajectory_raw_defaults():
    f = TR.make_approach_then_circle(center=np.array([-0.5, 0.0, 0.342]), radius=0.07, omega=2.0, z_contact=0.35,
                                     t_approach=1.0)
    _traj_check("traj_raw", f)


def _split(rec, sizes):
    out, o = [], 0
    for s in sizes:
        out.append(rec[o:o + s])
        o += s
    assert o == rec.size
    return out


@pytest.mark.parametrize("case", range(6))
def test_ff_augmentation_vs_reference(case):
    """oracle.ocp.ff_augment == _AugmentedLPFActionModel.calc/calcDiff
    (crocoddyl_force_feedback.py:211-290) on synthetic inner-model data."""
    rec = G["ff_aug"][case]
    (hdr, yref, yw, x, u, ixn, icost, iFx, iFu, iLx, iLu, iLxx, iLxu, iLuu,
     xn, cost, Fx, Fu, Lx, Lu, Lxx, Luu, Lxu, u_inner) = _split(
        rec, [5, 21, 21, 21, 7, 14, 1, 196, 98, 14, 7, 196, 98, 49, 21, 1, 441, 147, 21, 7, 441, 49, 147, 7])
    alpha, w_reg, w_soft, w_y, terminal = hdr
    cfg = ocp.OCPConfig(variant="ff", ff_alpha=alpha, w_w=w_reg, w_w_soft_limits=w_soft, w_y=w_y,
                        y_weights=yw, tau_soft_limit_margin=0.2)
    inner = dict(xnext=ixn, cost=icost[0], Fx=iFx.reshape(14, 14), Fu=iFu.reshape(14, 7), Lx=iLx, Lu=iLu,
                 Lxx=iLxx.reshape(14, 14), Lxu=iLxu.reshape(14, 7), Luu=iLuu.reshape(7, 7))
    out = ocp.ff_augment(cfg, inner, x, u, yref, diff=True)
    # the inner model is driven with tau = y[14:21] as its control
    np.testing.assert_array_equal(u_inner, x[14:21])
    tol = dict(rtol=1e-13, atol=1e-12)
    np.testing.assert_allclose(out["xnext"], xn, **tol)
    np.testing.assert_allclose(out["cost"], cost[0], **tol)
    np.testing.assert_allclose(out["Fx"], Fx.reshape(21, 21), **tol)
    np.testing.assert_allclose(out["Fu"], Fu.reshape(21, 7), **tol)
    np.testing.assert_allclose(out["Lx"], Lx, **tol)
    np.testing.assert_allclose(out["Lu"], Lu, **tol)
    np.testing.assert_allclose(out["Lxx"], Lxx.reshape(21, 21), **tol)
    np.testing.assert_allclose(out["Luu"], Luu.reshape(7, 7), **tol)
    np.testing.assert_allclose(out["Lxu"], Lxu.reshape(21, 7), **tol)
    if terminal:
        assert np.all(u == 0.0)


# ---- controller host algebra -------------------------------------------------------------
def _ff_ctrl(tau_prev=None, **kw):
    o = object.__new__(CT.ForceFeedbackCrocoddylMPC)
    o.cfg = CT.ForceFeedbackMPCConfig(horizon=6, dt=0.005, dt_ocp=0.01, ff_cutoff_hz=25.0, feedback_gain_scale=0.55,
                                      ff_use_tau_interpolation=True, ff_inverse_actuation_model=True, **kw)
    o.sim = types.SimpleNamespace(dt=0.005)
    o._warned_keys = set()
    o._tau_prev = np.zeros(7) if tau_prev is None else tau_prev
    o._fn_pred_hist_raw, o._fn_pred_hist_meas, o._fn_pred_corr = [], [], np.nan
    return o


def test_ff_filter_constants():
    o = _ff_ctrl()
    np.testing.assert_allclose([o._ff_alpha_ocp(), o._ff_alpha_ctrl(), o._policy_epsilon()], G["ff_alpha"],
                               rtol=1e-15, atol=0)


def test_ff_policy_and_shift():
    N = 6
    xs, us, Ks, y = _split(G["ff_policy_in"], [21 * (N + 1), 7 * N, 7 * 21 * N, 21])
    tau, xi, ui, xic, uic = _split(G["ff_policy_out"], [7, 21 * (N + 1), 7 * N, 21 * (N + 1), 7 * N])
    o = _ff_ctrl()
    o.xs = list(xs.reshape(N + 1, 21))
    o.us = list(us.reshape(N, 7))
    o.Ks = list(Ks.reshape(N, 7, 21))
    t, idx = o._policy_control(y)
    assert idx == 0
    np.testing.assert_allclose(t, tau, rtol=1e-14, atol=1e-13)
    a, b = o._shift_guess(y, N)
    np.testing.assert_array_equal(np.ravel(a), xi)
    np.testing.assert_array_equal(np.ravel(b), ui)
    o.xs = None
    a, b = o._shift_guess(y, N)
    np.testing.assert_array_equal(np.ravel(a), xic)
    np.testing.assert_array_equal(np.ravel(b), uic)


def test_safe_tau():
    # row 2 holds a NaN: the command falls back to the previous (clipped) one
    tin, tout = G["safe_tau_in"], G["safe_tau_out"]
    o = _ff_ctrl(tau_prev=np.zeros(7))
    for r in range(tin.shape[0]):
        np.testing.assert_array_equal(o._safe_tau(tin[r]), tout[r])


def test_force_prediction_alignment():
    raw, meas = G["align_in"]
    o = _ff_ctrl()
    out = np.array([o._align_logged_force_prediction(float(r), float(m), True) for r, m in zip(raw, meas)])
    np.testing.assert_allclose(out, G["align_out"], rtol=1e-12, atol=1e-12)


def test_classical_policy_and_shift():
    N = 6
    xs, us, Ks, x, tau_prev = _split(G["cl_policy_in"], [14 * (N + 1), 7 * N, 7 * 14 * N, 14, 7])
    u, xi, ui = _split(G["cl_policy_out"], [7, 14 * (N + 1), 7 * N])
    o = object.__new__(CT.ClassicalCrocoddylMPC)
    o.cfg = CT.ClassicalMPCConfig(horizon=N, feedback_gain_scale=0.55)
    o._tau_prev = tau_prev
    o.xs, o.us, o.Ks = list(xs.reshape(N + 1, 14)), list(us.reshape(N, 7)), list(Ks.reshape(N, 7, 14))
    got, idx = o._policy_control(x)
    assert idx == 0
    np.testing.assert_allclose(got, u, rtol=1e-14, atol=1e-13)
    a, b = o._shift_guess(x, N)
    np.testing.assert_array_equal(np.ravel(a), xi)
    np.testing.assert_array_equal(np.ravel(b), ui)
