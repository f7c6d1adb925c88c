"""Controller mirrors (ffddp.controller) driven tick by tick.

CPU: the HIP solver is swapped for an oracle-backed stand-in (test-only) so
the host control flow — problem packing, warm-start shift, feedback policy,
solve period / rollout shift, mode-switch invalidation, instability fallback —
is checked without a GPU.  GPU: the real controller (HIP solver, B = 1) against
the same controller running on the oracle stand-in, tick by tick."""
from __future__ import annotations

import types

import numpy as np
import pytest

from ffddp import _abi, controller as CT, robot as R, trajectory as TR
from helpers import oracle_cfg
from oracle import fddp, ocp


def _rot_to_quat_wxyz(Rm):
    w = np.sqrt(max(1e-16, 1.0 + np.trace(Rm))) / 2.0
    return np.array([w, (Rm[2, 1] - Rm[1, 2]) / (4 * w), (Rm[0, 2] - Rm[2, 0]) / (4 * w), (Rm[1, 0] - Rm[0, 1]) / (4 * w)])


class FakeSim:
    """Kinematically consistent observations from the product FK (no physics):
    site = EE frame origin, site rotation = R_SITE_FROM_EE (MJCF tool quat)."""

    dt = 0.01

    def __init__(self, q, dq=None, fn=0.0):
        self.q = np.asarray(q, float)
        self.dq = np.zeros(7) if dq is None else np.asarray(dq, float)
        self.fn = fn

    def get_observation(self, with_ee=True, with_jacobian=False):
        Rp, pp = _abi.frame_placement(self.q)
        g = _abi.gravity_torque(self.q[None])[0]
        Rs = R.R_MJ_FROM_PIN @ Rp @ R.R_SITE_FROM_EE
        return types.SimpleNamespace(
            q=self.q.copy(), dq=self.dq.copy(), tau_bias=g, tau_cmd=g.copy(), tau_meas_act_filt=g.copy(),
            ee_pos=R.R_MJ_FROM_PIN @ pp, ee_quat=_rot_to_quat_wxyz(Rs), f_contact_normal=self.fn,
        )


class OracleSolver:
    """BatchedBoxFDDP stand-in over the numpy oracle (test infrastructure only)."""

    calls: list = []

    def __init__(self, cfg, max_batch, device=0):
        self.cfg = cfg
        self.N = cfg.horizon
        OracleSolver.last_cfg = cfg

    def solve(self, batch, maxiter=10, is_feasible=False, xs_init=None, us_init=None):
        N = self.N
        prob = ocp.Problem(batch.x0[0], batch.node_ref[0, :, :3], batch.node_ref[0, :, 3:], batch.inst_ref[0, :14],
                           batch.inst_ref[0, 14:], bool(batch.surface[0]))
        s = fddp.SolverBoxFDDP(oracle_cfg(self.cfg), prob, box=self.cfg.use_box_fddp)
        ok = s.solve(xs_init[0], us_init[0], maxiter, is_feasible)
        OracleSolver.calls.append((batch, xs_init[0].copy(), us_init[0].copy()))
        self.xs, self.us, self.K = s.xs[None], s.us[None], s.K[None]
        self.cost, self.iter = np.array([s.cost]), np.array([s.iter])
        nc = 3 if self.cfg.nc == 3 else 1
        sel = 0 if nc == 1 else 2
        fn = [s.contact_force(t)[sel] if batch.surface[0] else np.nan for t in range(min(2, N))]
        self.fn_pred = np.array([fn + [np.nan] * (2 - len(fn))])
        self.ok = np.array([bool(ok)])
        return self.ok

    def close(self):
        pass


def _traj():
    ee0 = R.R_MJ_FROM_PIN @ _abi.frame_placement(R.Q_NEUTRAL)[1]
    return TR.make_approach_then_circle(center=np.array([-0.5, 0.0, 0.3]) + np.array([0, 0, 0.042]), radius=0.10,
                                       omega=1.5, z_pre=0.392, z_contact=0.342, t_approach=0.55, ee_start=ee0,
                                       t_pre=0.25)


def _make(variant, monkeypatch=None, **kw):
    if monkeypatch is not None:
        monkeypatch.setattr(CT, "BatchedBoxFDDP", OracleSolver)
    sim = FakeSim(R.Q_NEUTRAL)
    if variant == "ff":
        cfg = CT.ff_benchmark_config(dt=0.01, z_contact=0.342, max_iters=3, horizon=6, **kw)
        return CT.ForceFeedbackCrocoddylMPC(sim, _traj(), cfg), sim
    cfg = CT.classical_benchmark_config(dt=0.01, z_contact=0.342, max_iters=3, horizon=6, **kw)
    return CT.ClassicalCrocoddylMPC(sim, _traj(), cfg), sim


def test_calibration_recovers_model_frames(monkeypatch):
    c, _ = _make("classical", monkeypatch)
    np.testing.assert_allclose(c.R_site_from_pin_ee, R.R_SITE_FROM_EE, atol=1e-12)
    np.testing.assert_allclose(c.p_site_minus_frame_pin, 0.0, atol=1e-12)
    np.testing.assert_allclose(c.R_des, R.default_R_des(), atol=1e-12)


@pytest.mark.parametrize("variant", ["classical", "ff"])
def test_compute_control_flow_cpu(monkeypatch, variant):
    OracleSolver.calls = []
    c, sim = _make(variant, monkeypatch, phase_source="trajectory")
    c.cfg.mpc_update_steps = 2
    taus = []
    for k, t in enumerate([0.0, 0.01, 0.02]):
        taus.append(c.compute_control(sim.get_observation(), t))
        assert c.last_info["solved_now"] == (k != 1)
        assert np.all(np.abs(taus[-1]) <= R.TAU_LIMITS + 1e-12)
        assert not c.last_info["unstable"]
    assert len(OracleSolver.calls) == 2
    # problem packing: knot refs from traj(t0 + k dt_ocp), posture ref q_nom, torque ref gravity(q0)
    b0, xs0, us0 = OracleSolver.calls[0]
    p, v, _ = _traj()(0.0 + 3 * 0.01)
    np.testing.assert_allclose(b0.node_ref[0, 3, :3], R.R_MJ_FROM_PIN.T @ p, atol=1e-12)
    np.testing.assert_allclose(b0.node_ref[0, 3, 3:], R.R_MJ_FROM_PIN.T @ v, atol=1e-12)
    np.testing.assert_allclose(b0.inst_ref[0, :7], R.Q_NEUTRAL)
    np.testing.assert_allclose(b0.inst_ref[0, 14:], _abi.gravity_torque(R.Q_NEUTRAL[None])[0], atol=1e-12)
    # cold start holds x0 and the initial torque
    assert np.all(xs0 == xs0[0])
    # second solve warm-starts from the solution shifted once by the rollout and once by _shift_guess
    _, xs1, us1 = OracleSolver.calls[1]
    assert xs1.shape == xs0.shape and us1.shape == us0.shape
    assert np.all(np.isfinite(xs1)) and np.all(np.isfinite(us1))


def test_unstable_fallback(monkeypatch):
    c, sim = _make("classical", monkeypatch)
    c.cfg.max_solver_cost = -1.0  # every solve counts as diverged
    obs = sim.get_observation()
    tau = c.compute_control(obs, 0.0)
    assert c.last_info["unstable"] and c.xs is None and c.us is None
    np.testing.assert_allclose(tau, np.clip(obs.tau_bias - 5.0 * obs.dq, -R.TAU_LIMITS, R.TAU_LIMITS))


def test_mode_switch_invalidates_warm_start(monkeypatch):
    c, sim = _make("classical", monkeypatch)
    c.compute_control(sim.get_observation(), 0.0)
    assert c.xs is not None and not c.last_info["surface_mode"]
    OracleSolver.calls = []
    c.compute_control(sim.get_observation(), 1.0)  # in contact from t = 0.8 s
    assert c.last_info["surface_mode"]
    _, xs_init, _ = OracleSolver.calls[0]
    assert np.all(xs_init == xs_init[0])  # cold start after the switch
    assert np.isfinite(c.last_info["fn_pred"])


@pytest.mark.parametrize("contact_model", ["normal_1d", "point3d"])
def test_default_config_builds_with_friction_cone(monkeypatch, contact_model):
    """ClassicalMPCConfig() (w_friction_cone = 2e2, mu = 0.6) builds like the
    reference's; the cone weight and mu reach the OCP, which adds the cone only
    for nc = 3 (crocoddyl_classical.py:678)."""
    monkeypatch.setattr(CT, "BatchedBoxFDDP", OracleSolver)
    cfg = CT.ClassicalMPCConfig(contact_model=contact_model, horizon=4, max_iters=2)
    c = CT.ClassicalCrocoddylMPC(FakeSim(R.Q_NEUTRAL), _traj(), cfg)
    tau = c.compute_control(c.sim.get_observation(), 1.0)
    assert np.all(np.isfinite(tau))
    ocfg = oracle_cfg(c._solver.cfg)
    assert ocfg.w_friction_cone == 2.0e2 and ocfg.mu == 0.6
    names = [n for n, *_ in ocp.cost_stack(ocfg, surface=True, terminal=False)]
    assert ("friction_cone" in names) == (contact_model == "point3d")


@pytest.mark.gpu
@pytest.mark.parametrize("variant", ["classical", "ff"])
def test_controller_gpu_matches_oracle(variant):
    """HIP-backed controller vs the same controller on the oracle, 4 ticks across
    the contact switch; tolerance 1e-6 relative on the torque command."""
    import pytest as _pt

    mp = _pt.MonkeyPatch()
    c_gpu, sim = _make(variant)
    c_ref, _ = _make(variant, mp)
    try:
        for t in (0.70, 0.71, 0.85, 0.86):
            obs = sim.get_observation()
            tg = c_gpu.compute_control(obs, t)
            tr = c_ref.compute_control(obs, t)
            scale = max(1.0, float(np.max(np.abs(tr))))
            assert np.max(np.abs(tg - tr)) / scale < 1e-6, (t, tg, tr)
            assert c_gpu.last_info["iters"] == c_ref.last_info["iters"]
            assert c_gpu.last_info["ok"] == c_ref.last_info["ok"]
            fg, fr = c_gpu.last_info["fn_pred"], c_ref.last_info["fn_pred"]
            assert (np.isnan(fg) and np.isnan(fr)) or abs(fg - fr) <= 1e-6 * max(1.0, abs(fr))
    finally:
        mp.undo()
        c_gpu.close()
