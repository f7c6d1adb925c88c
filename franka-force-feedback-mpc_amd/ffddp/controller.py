"""Receding-horizon controllers around the HIP solver (SURVEY.md §8 "next"
row: the callers of the hot path).

ClassicalCrocoddylMPC / ForceFeedbackCrocoddylMPC keep the reference
controllers' public surface — constructor (sim, traj_fn, config),
compute_control(obs, t) -> tau_cmd, last_info, xs/us/Ks — and their host-side
algebra (warm-start shift, feedback policy, command safety, force-prediction
logging), but the OCP is never built as Python objects: each tick packs the
problem data (x0, per-knot EE references, posture/torque references, surface
flag) into the flat arrays the C-ABI takes and runs ONE batched solve with
B = 1 on the GPU.  Many robots / scenarios at once go through
BatchedBoxFDDP directly.

Reference: src/mpc/crocoddyl_classical.py:12-445, 733-780, 905-942 and
src/mpc/crocoddyl_force_feedback.py:12-146, 293-720, 1014-1093, 1219-1371.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Callable, List, Optional, Set, Tuple

import numpy as np

from . import _abi
from . import robot as R
from .callbacks import CallbackVerbose
from .config import OcpConfig
from .solver import BatchedBoxFDDP
from .workload import Batch

Traj = Callable[[float], Tuple[np.ndarray, np.ndarray, bool]]


def _arr(*v):
    return field(default_factory=lambda: np.array(v, dtype=float))


@dataclass
class ClassicalMPCConfig:
    """ClassicalMPCConfig (crocoddyl_classical.py:12-110), same names and defaults."""

    horizon: int = 20
    dt: float = 0.01
    dt_ocp: Optional[float] = None
    w_ee_pos: float = 2.0e2
    w_ee_ori: float = 1.0e1
    ori_weights: np.ndarray = _arr(2.0, 2.0, 0.15)
    w_posture: float = 5.0e-1
    w_v: float = 2.5e-1
    w_tau: float = 1.0e-3
    w_tau_smooth: float = 5.0e-2
    posture_ref_mode: str = "x0"
    torque_ref_mode: str = "gravity_x0"
    w_tau_soft_limits: float = 0.0
    tau_soft_limit_margin: float = 0.2
    w_q_soft_limits: float = 0.0
    q_soft_limit_margin: float = 0.05
    z_contact: float = 0.35
    z_press: float = 0.0020
    w_plane_z: float = 0.0
    w_vz: float = 0.0
    w_tangent_pos: float = 2.0e2
    w_tangent_vel: float = 1.0e2
    contact_name: str = "ee_contact"
    contact_model: str = "normal_1d"
    mu: float = 0.6
    friction_margin: float = 1e-3
    w_friction_cone: float = 2.0e2
    w_unilateral: float = 5.0e1
    contact_gains: np.ndarray = _arr(0.0, 60.0)
    contact_inv_damping: float = 1.0e-8
    strict_force_residual_dim: bool = True
    fn_des: float = 8.0
    w_fn: float = 2.0e1
    w_wdamp: float = 2.0e1
    w_wdamp_weights: np.ndarray = _arr(1.5, 1.5, 0.2)
    phase_source: str = "trajectory"
    fn_contact_on: float = 2.0
    fn_contact_off: float = 0.5
    z_contact_band: float = 0.01
    tau_limits: np.ndarray = _arr(87, 87, 87, 87, 12, 12, 12)
    tau_rate_limit: np.ndarray = _arr(450, 450, 450, 450, 180, 180, 180)
    tau_trust_inf: float = 40.0
    tau_smoothing_alpha: float = 0.35
    apply_command_filter: bool = False
    v_damp_weights: np.ndarray = _arr(1.0, 1.0, 1.0, 1.0, 0.4, 0.4, 0.4)
    max_iters: int = 20
    use_box_fddp: bool = True
    mpc_update_steps: int = 1
    use_feedback_policy: bool = True
    feedback_gain_scale: float = 1.0
    verbose: bool = False
    debug_every: int = 25
    max_solver_cost: float = 1.0e8
    max_tau_raw_inf: float = 3.0e2
    fallback_dq_damping: float = 5.0
    contact_release_steps: int = 25
    # Not a field of the reference's config: the comparator of the solver's
    # ascent-direction acceptance (include/ffddp.h FFDDP_NEGSTEP_*), which the
    # reference leaves at Crocoddyl's own (0).  1 = bounded rise; its effect on
    # the closed loop is in DESIGN.md §3.
    neg_step_rule: int = 0


@dataclass
class ForceFeedbackMPCConfig(ClassicalMPCConfig):
    """ForceFeedbackMPCConfig (crocoddyl_force_feedback.py:12-146): the classical
    fields with the FF defaults, plus the augmentation / policy knobs."""

    w_w: float = 8.0e-4
    w_y: float = 3.0e-3
    y_q_weights: np.ndarray = _arr(0.2, 0.2, 0.2, 0.2, 0.1, 0.1, 0.1)
    y_v_weights: np.ndarray = _arr(0.08, 0.08, 0.08, 0.08, 0.05, 0.05, 0.05)
    y_tau_weights: np.ndarray = _arr(0.35, 0.35, 0.35, 0.35, 0.2, 0.2, 0.2)
    use_inner_state_reg: bool = True
    use_inner_tau_reg: bool = True
    w_tau_soft_limits: float = 1.5
    w_w_soft_limits: float = 2.0
    w_q_soft_limits: float = 8.0
    feedback_gain_scale: float = 0.35
    ff_cutoff_hz: float = 18.0
    ff_alpha_override: Optional[float] = None
    ff_use_tau_meas_filt: bool = True
    ff_tau_state_source: str = "tau_meas_act_filt"
    ff_use_tau_interpolation: bool = True
    ff_align_force_prediction: bool = True
    ff_align_window: int = 240
    ff_align_min_samples: int = 80
    ff_align_corr_threshold: float = 0.05
    ff_align_max_lag: int = 8
    ff_inverse_actuation_model: bool = False
    ff_tau_feedback_gain: float = 1.0


def classical_benchmark_config(dt: float, z_contact: float, max_iters: int = 10, horizon: int = 36,
                               contact_model: str = "normal_1d", phase_source: str = "trajectory",
                               neg_step_rule: int = 0):
    """Benchmark-mode ClassicalMPCConfig of src/run/run_classical.py:269-315."""
    return ClassicalMPCConfig(
        horizon=horizon, dt=dt, dt_ocp=0.01, z_contact=z_contact, z_press=0.0065, w_ee_pos=1.2e3,
        w_ee_ori=5.0e1, ori_weights=np.array([2.4, 2.4, 0.3]), w_posture=1.5e-1, w_v=8.0e-2,
        posture_ref_mode="q_nom", w_tau=8.0e-4, torque_ref_mode="gravity_x0", w_tau_soft_limits=2.0,
        w_q_soft_limits=8.0, q_soft_limit_margin=0.05, w_tau_smooth=0.0, w_tangent_pos=2.6e3,
        w_tangent_vel=7.0e2, w_plane_z=1.2e3, w_vz=5.0e2, w_friction_cone=0.0, w_unilateral=3.0e1, mu=1.0,
        contact_gains=np.array([140.0, 80.0]), fn_des=22.0, w_fn=2.8e1, w_wdamp=6.0e1,
        w_wdamp_weights=np.array([1.8, 1.8, 0.3]), fn_contact_on=1.0, fn_contact_off=0.1, z_contact_band=0.012,
        max_iters=max_iters, mpc_update_steps=1, use_feedback_policy=True, feedback_gain_scale=0.55,
        max_solver_cost=1.0e8, max_tau_raw_inf=3.0e2, contact_release_steps=60, contact_model=contact_model,
        phase_source=phase_source, apply_command_filter=False, debug_every=100, neg_step_rule=neg_step_rule,
    )


def ff_benchmark_config(dt: float, z_contact: float, max_iters: int = 10, horizon: int = 40,
                        contact_model: str = "normal_1d", phase_source: str = "trajectory",
                        ff_tau_state_source: str = "tau_meas_act_filt", neg_step_rule: int = 0):
    """Benchmark-mode ForceFeedbackMPCConfig of src/run/run_force_feedback.py:272-330."""
    return ForceFeedbackMPCConfig(
        horizon=horizon, dt=dt, dt_ocp=0.01, z_contact=z_contact, z_press=0.0065, w_ee_pos=1.2e3,
        w_ee_ori=4.5e1, ori_weights=np.array([2.2, 2.2, 0.3]), w_posture=1.0e-1, w_v=5.0e-2,
        posture_ref_mode="q_nom", w_tau=8.0e-4, w_w=6.0e-4, w_w_soft_limits=2.0, w_y=8.0e-4,
        y_q_weights=np.array([0.15] * 4 + [0.08] * 3), y_v_weights=np.array([0.05] * 4 + [0.03] * 3),
        y_tau_weights=np.array([0.12] * 4 + [0.08] * 3), use_inner_state_reg=True, use_inner_tau_reg=True,
        torque_ref_mode="gravity_x0", w_tau_soft_limits=1.5, w_q_soft_limits=8.0, q_soft_limit_margin=0.05,
        w_tau_smooth=0.0, w_tangent_pos=3.6e3, w_tangent_vel=1.2e3, w_plane_z=9.0e2, w_vz=3.0e2,
        w_friction_cone=0.0, w_unilateral=3.0e1, mu=1.0, contact_gains=np.array([145.0, 85.0]), fn_des=22.0,
        w_fn=3.0e1, w_wdamp=7.0e1, w_wdamp_weights=np.array([1.8, 1.8, 0.3]), fn_contact_on=1.0,
        fn_contact_off=0.1, z_contact_band=0.012, max_iters=max_iters, mpc_update_steps=1,
        use_feedback_policy=True, feedback_gain_scale=0.55, max_solver_cost=1.0e8, max_tau_raw_inf=3.0e2,
        contact_release_steps=80, contact_model=contact_model, phase_source=phase_source,
        apply_command_filter=False, ff_tau_state_source=ff_tau_state_source, ff_cutoff_hz=25.0,
        ff_inverse_actuation_model=True, ff_tau_feedback_gain=1.0, debug_every=500, neg_step_rule=neg_step_rule,
    )


_OCP_FIELDS = (
    "z_press", "w_ee_pos", "w_ee_ori", "ori_weights", "w_posture", "w_v", "v_damp_weights", "w_tau",
    "w_tau_soft_limits", "tau_soft_limit_margin", "w_q_soft_limits", "q_soft_limit_margin", "w_tangent_pos",
    "w_tangent_vel", "w_plane_z", "w_vz", "w_unilateral", "friction_margin", "w_fn", "fn_des", "w_wdamp",
    "w_wdamp_weights", "contact_gains", "contact_inv_damping", "tau_limits", "contact_model", "use_box_fddp",
    "w_friction_cone", "mu",
)


def _quat_wxyz_to_R(q) -> np.ndarray:
    """_quat_wxyz_to_R (crocoddyl_classical.py:228-239)."""
    q = np.asarray(q, dtype=float).reshape(4)
    q = q / (np.linalg.norm(q) + 1e-12)
    w, x, y, z = q
    return np.array(
        [
            [1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)],
            [2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)],
            [2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)],
        ]
    )


class _MPCBase:
    variant = "classical"

    def __init__(self, sim, traj_fn: Traj, config, device: int = 0, use_plan: bool = True, calibration_obs=None):
        """use_plan: run each tick's solve through a captured solve plan
        (BatchedBoxFDDP.plan: one graph launch per tick, bit-identical to
        solve()); False: the plain host-array solve.
        calibration_obs: the observation the site calibration
        (_calibrate_site_rotation / _calibrate_site_position_offset) is taken
        from; default the sim's initial observation, as the reference does
        (crocoddyl_classical.py:199-226).  The calibration is a rigid offset,
        so another posture changes it at rounding level only; the fleet
        controller calibrates once for all its instances, and its tick-for-tick
        comparisons pass the fleet's observation here."""
        cfg = config
        self.sim = sim
        self.traj_fn = traj_fn
        self.cfg = cfg
        self._k = 0
        self._warned_keys: Set[str] = set()
        self.R_mj_from_pin = R.R_MJ_FROM_PIN.copy()
        self.nq = self.nv = self.nu = 7
        self.nx_mb = 14
        obs0 = sim.get_observation(with_ee=True, with_jacobian=False)
        self.q_nom = np.asarray(obs0.q, dtype=float).copy()
        obs_cal = obs0 if calibration_obs is None else calibration_obs
        self.R_site_from_pin_ee = self._calibrate_site_rotation(obs_cal)
        self.p_site_minus_frame_pin = self._calibrate_site_position_offset(obs_cal)
        self.R_des = self._rot_mj_to_pin(R.vertical_down_rotation_mj())
        self.xs: Optional[List[np.ndarray]] = None
        self.us: Optional[List[np.ndarray]] = None
        self.Ks: Optional[List[np.ndarray]] = None
        self.ks = None
        self._tau_prev = np.asarray(self._initial_tau(obs0), dtype=float).copy()
        self._last_solve_step = -1_000_000_000
        self._last_solve_ok = False
        self._last_solve_cost = np.nan
        self._last_solve_iters = -1
        self._last_neg = (0, 0)
        self._surface_latched = False
        self._contact_loss_count = 0
        self._prev_surface_mode: Optional[bool] = None
        self.last_info = {"ok": False, "cost": np.nan, "iters": -1, "tau_raw_inf": np.nan, "tau_cmd_inf": np.nan,
                          "surface_mode": False, "unstable": False, "fn_pred": np.nan}
        self.ocp = self._ocp_config()
        self._solver = BatchedBoxFDDP(self.ocp, max_batch=1, device=device)
        self._solver.neg_step_rule = int(getattr(self.cfg, "neg_step_rule", 0))
        self._use_plan = bool(use_plan) and hasattr(self._solver, "plan")
        self._plan = None
        self._res = self._solver  # where the last solve's outputs live (solver or plan)
        if self.cfg.verbose:  # crocoddyl_classical.py:352-353, 360-361
            self._solver.setCallbacks([CallbackVerbose()], max_iters=max(int(self.cfg.max_iters), 1))

    # -- frames (crocoddyl_classical.py:199-258) -------------------------------------
    @property
    def _dt_ocp(self) -> float:
        return float(self.cfg.dt_ocp) if self.cfg.dt_ocp is not None else float(self.cfg.dt)

    def _calibrate_site_rotation(self, obs0) -> np.ndarray:
        R_pin_ee = _abi.frame_placement(np.asarray(obs0.q, float))[0]
        if getattr(obs0, "ee_quat", None) is not None:
            R_mj_site = _quat_wxyz_to_R(obs0.ee_quat)
        else:
            R_mj_site = self.R_mj_from_pin @ R_pin_ee @ R.R_SITE_FROM_EE
        return R_pin_ee.T @ self.R_mj_from_pin.T @ R_mj_site

    def _calibrate_site_position_offset(self, obs0) -> np.ndarray:
        p_pin_ee = _abi.frame_placement(np.asarray(obs0.q, float))[1]
        if getattr(obs0, "ee_pos", None) is None:
            return np.zeros(3)
        p_pin_site = self.R_mj_from_pin.T @ np.asarray(obs0.ee_pos, float).reshape(3)
        return p_pin_site - p_pin_ee

    def _pos_mj_to_pin(self, p_mj) -> np.ndarray:
        return self.R_mj_from_pin.T @ np.asarray(p_mj, float) - self.p_site_minus_frame_pin

    def _vel_mj_to_pin(self, v_mj) -> np.ndarray:
        return self.R_mj_from_pin.T @ np.asarray(v_mj, float)

    def _rot_mj_to_pin(self, R_mj_site) -> np.ndarray:
        return self.R_mj_from_pin.T @ np.asarray(R_mj_site, float) @ self.R_site_from_pin_ee.T

    # -- OCP data ---------------------------------------------------------------------
    def _ocp_config(self) -> OcpConfig:
        c = OcpConfig(variant=self.variant, horizon=int(self.cfg.horizon), dt=self._dt_ocp, R_des=self.R_des)
        for f in _OCP_FIELDS:
            setattr(c, f, getattr(self.cfg, f))
        c.tau_limits = np.asarray(self.cfg.tau_limits, float).copy()
        return c

    def _gravity_torque(self, q) -> np.ndarray:
        return _abi.gravity_torque(np.asarray(q, float).reshape(1, 7))[0]

    def _compute_tau_reference(self, q_now) -> np.ndarray:
        """crocoddyl_classical.py:453-460."""
        mode = str(self.cfg.torque_ref_mode).strip().lower()
        if mode == "zero":
            return np.zeros(7)
        if mode == "gravity_qnom":
            return self._gravity_torque(self.q_nom)
        return self._gravity_torque(q_now)

    def _compute_posture_reference(self, x0) -> np.ndarray:
        """crocoddyl_classical.py:462-466 (classical: anything but "q_nom" -> x0)."""
        mode = str(self.cfg.posture_ref_mode).strip().lower()
        if mode == "q_nom":
            return np.concatenate([self.q_nom, np.zeros(7)])
        return np.asarray(x0[:14], float).copy()

    def _problem_arrays(self, t0: float, x0: np.ndarray, surface_now: bool) -> Batch:
        """Everything _build_problem (crocoddyl_classical.py:521-556) feeds the
        action models, as flat arrays: knot k uses traj(t0 + k dt_ocp)."""
        N, dt = int(self.cfg.horizon), self._dt_ocp
        node_ref = np.zeros((1, N + 1, 6))
        sample = getattr(self.traj_fn, "sample", None)
        if sample is not None:
            # all knots at once (trajectory.sample: the same arithmetic per
            # knot; R_MJ_FROM_PIN is a signed permutation, so the frame maps
            # below are exact in either order)
            P, V, _ = sample(np.array([t0 + k * dt for k in range(N + 1)]))
            node_ref[0, :, :3] = P @ self.R_mj_from_pin - self.p_site_minus_frame_pin
            node_ref[0, :, 3:] = V @ self.R_mj_from_pin
        else:
            for k in range(N + 1):
                p, v, _ = self.traj_fn(t0 + k * dt)
                node_ref[0, k, :3] = self._pos_mj_to_pin(p)
                node_ref[0, k, 3:] = self._vel_mj_to_pin(v)
        inst = np.concatenate([self._compute_posture_reference(x0), self._compute_tau_reference(x0[:7])])
        return Batch(x0[None].copy(), node_ref, inst[None], np.array([1 if surface_now else 0], np.uint8),
                     None, None, np.array([t0]))

    # -- phase (crocoddyl_classical.py:286-303) ---------------------------------------
    def _detect_surface(self, obs, t: float, surf_hint: bool) -> bool:
        fn = float(getattr(obs, "f_contact_normal", 0.0))
        ee_z = float(obs.ee_pos[2]) if getattr(obs, "ee_pos", None) is not None else float("inf")
        near = np.isfinite(ee_z) and (ee_z <= float(self.cfg.z_contact) + float(self.cfg.z_contact_band))
        if self._surface_latched:
            lost = fn < self.cfg.fn_contact_off
            self._contact_loss_count = self._contact_loss_count + 1 if lost else 0
            if self._contact_loss_count >= int(self.cfg.contact_release_steps):
                self._surface_latched = False
                self._contact_loss_count = 0
        elif (fn > self.cfg.fn_contact_on) or (surf_hint and near):
            self._surface_latched = True
            self._contact_loss_count = 0
        return self._surface_latched

    def _surface_mode(self, obs, t: float) -> bool:
        _, _, hint = self.traj_fn(t)
        if str(self.cfg.phase_source).strip().lower() == "force_latch":
            return self._detect_surface(obs, t, hint)
        return bool(hint)

    def _invalidate(self):
        self.xs = self.us = self.Ks = self.ks = None
        self._last_solve_step = -1_000_000_000

    # -- command safety (crocoddyl_classical.py:260-284) ------------------------------
    def _safe_tau(self, tau_target) -> np.ndarray:
        tau_target = np.asarray(tau_target, dtype=float).copy()
        lim = np.asarray(self.cfg.tau_limits, float)
        if not np.all(np.isfinite(tau_target)):
            tau_target = self._tau_prev.copy()
        tau_target = np.clip(tau_target, -lim, lim)
        if not bool(self.cfg.apply_command_filter):
            self._tau_prev = tau_target.copy()
            return tau_target
        d = np.clip(tau_target - self._tau_prev, -self.cfg.tau_trust_inf, self.cfg.tau_trust_inf)
        dt = float(getattr(self.sim, "dt", self.cfg.dt))
        max_step = np.asarray(self.cfg.tau_rate_limit, float) * dt
        d = np.clip(d, -max_step, max_step)
        a = float(np.clip(self.cfg.tau_smoothing_alpha, 0.0, 1.0))
        tau_cmd = np.clip((1.0 - a) * self._tau_prev + a * (self._tau_prev + d), -lim, lim)
        self._tau_prev = tau_cmd.copy()
        return tau_cmd

    # -- warm start (crocoddyl_classical.py:733-757) -----------------------------------
    def _cold_control(self, x0) -> np.ndarray:
        return self._tau_prev.copy()

    def _shift_guess(self, x0, N: int):
        if self.xs is None or self.us is None or len(self.us) < N:
            return [x0.copy() for _ in range(N + 1)], [self._cold_control(x0) for _ in range(N)]
        xs_prev, us_prev = self.xs, self.us
        xs_init = [x0.copy()] + [xs_prev[i].copy() for i in range(1, min(len(xs_prev), N + 1))]
        while len(xs_init) < N + 1:
            xs_init.append(xs_prev[-1].copy())
        us_init = [us_prev[i].copy() for i in range(1, min(len(us_prev), N))]
        while len(us_init) < N:
            us_init.append(us_prev[-1].copy())
        return xs_init, us_init

    # -- one solve ------------------------------------------------------------------
    def _solve(self, t: float, x0: np.ndarray, surface_now: bool):
        N = int(self.cfg.horizon)
        prob = self._problem_arrays(t, x0, surface_now)
        xs_init, us_init = self._shift_guess(x0, N)
        s = self._solver
        if self._use_plan:
            if self._plan is None:
                self._plan = s.plan(1, maxiter=int(self.cfg.max_iters), is_feasible=False)
            s = self._plan
            s.fill(prob, xs_init=np.asarray(xs_init)[None], us_init=np.asarray(us_init)[None])
            ok = bool(s.run()[0])
        else:
            ok = bool(s.solve(prob, maxiter=int(self.cfg.max_iters), is_feasible=False,
                              xs_init=np.asarray(xs_init)[None], us_init=np.asarray(us_init)[None])[0])
        self._res = s
        cost, iters = float(s.cost[0]), int(s.iter[0])
        st = getattr(s, "stats", None)
        # ascent-direction branch (dVexp < 0): trials judged / accepted in this solve
        self._last_neg = (int(st[0, 8]), int(st[0, 9])) if st is not None and st.shape[1] > 9 else (0, 0)
        self._last_solve_step = self._k
        self._last_solve_ok, self._last_solve_cost, self._last_solve_iters = ok, cost, iters
        if N > 0 and np.all(np.isfinite(s.us[0, 0])):
            self.xs = [x.copy() for x in s.xs[0]]
            self.us = [u.copy() for u in s.us[0]]
            self.Ks = [k.copy() for k in s.K[0]]
            self.ks = None
        return ok, cost, iters

    def _rollout_shift(self):
        """Receding-horizon shift between solves (crocoddyl_classical.py:430-438)."""
        if self.us is not None and self.xs is not None:
            if len(self.us) > 1:
                self.us = self.us[1:] + [self.us[-1]]
            if len(self.xs) > 1:
                self.xs = self.xs[1:] + [self.xs[-1]]
            if self.Ks is not None and len(self.Ks) > 1:
                self.Ks = self.Ks[1:] + [self.Ks[-1]]
            self.ks = None

    def _need_solve(self) -> bool:
        period = max(1, int(self.cfg.mpc_update_steps))
        return self.us is None or self.xs is None or (self._k - self._last_solve_step) >= period

    def _track_mode(self, surface_now: bool):
        if self._prev_surface_mode is None:
            self._prev_surface_mode = bool(surface_now)
        elif bool(surface_now) != bool(self._prev_surface_mode):
            self._invalidate()
            self._prev_surface_mode = bool(surface_now)

    def close(self):
        if self._plan is not None:
            self._plan.close()
            self._plan = None
        self._solver.close()


class ClassicalCrocoddylMPC(_MPCBase):
    """Classical EE MPC (crocoddyl_classical.py:113-445); OCP state x=(q,v), control tau."""

    variant = "classical"

    def __init__(self, sim, traj_fn: Traj, config: Optional[ClassicalMPCConfig] = None, device: int = 0,
                 use_plan: bool = True, calibration_obs=None):
        super().__init__(sim, traj_fn, config if config is not None else ClassicalMPCConfig(), device, use_plan,
                         calibration_obs)

    def _initial_tau(self, obs0):
        return obs0.tau_bias

    def _policy_control(self, x_now) -> Tuple[np.ndarray, int]:
        """crocoddyl_classical.py:759-779: u = us[0] + scale * K[0] (x_now - xs[0])."""
        if self.us is None or len(self.us) == 0:
            return self._tau_prev.copy(), -1
        i = 0
        u = np.asarray(self.us[i], dtype=float).copy()
        if (self.cfg.use_feedback_policy and self.Ks is not None and self.xs is not None
                and i < len(self.Ks) and i < len(self.xs)):
            dx = np.asarray(x_now - self.xs[i], dtype=float)
            u += float(self.cfg.feedback_gain_scale) * (np.asarray(self.Ks[i], float) @ dx)
        return u, i

    def compute_control(self, obs, t: float) -> np.ndarray:
        """crocoddyl_classical.py:305-440."""
        self._k += 1
        q = np.asarray(obs.q, dtype=float)
        v = np.asarray(obs.dq, dtype=float)
        x0 = np.concatenate([q, v])
        surface_now = self._surface_mode(obs, t)
        self._track_mode(surface_now)
        solved_now = False
        ok, cost, iters = self._last_solve_ok, float(self._last_solve_cost), int(self._last_solve_iters)
        fn_pred = float(self.last_info.get("fn_pred", np.nan))
        if self._need_solve():
            ok, cost, iters = self._solve(t, x0, surface_now)
            # _extract_predicted_normal_force: world-z contact force at knot 0 (R7)
            fn_pred = float(self._res.fn_pred[0, 0]) if surface_now else np.nan
            solved_now = True
        tau_raw, policy_idx = self._policy_control(x0)
        tau_raw_inf = float(np.max(np.abs(tau_raw)))
        unstable = (not np.isfinite(cost)) or cost > float(self.cfg.max_solver_cost) or \
            tau_raw_inf > float(self.cfg.max_tau_raw_inf)
        if unstable:
            tau_raw = np.asarray(obs.tau_bias, dtype=float) - float(self.cfg.fallback_dq_damping) * v
            self._invalidate()
        tau_cmd = self._safe_tau(tau_raw)
        self.last_info = {
            "ok": bool(ok), "cost": float(cost), "iters": iters, "tau_raw_inf": tau_raw_inf,
            "tau_cmd_inf": float(np.max(np.abs(tau_cmd))), "surface_mode": bool(surface_now),
            "unstable": bool(unstable), "fn_pred": float(fn_pred) if np.isfinite(fn_pred) else np.nan,
            "solved_now": bool(solved_now), "policy_idx": int(policy_idx),
            "neg_branch": self._last_neg[0] if solved_now else 0, "neg_accepted": self._last_neg[1] if solved_now else 0,
        }
        if (self._k % self.cfg.debug_every) == 0:  # crocoddyl_classical.py:420-428
            fn = float(getattr(obs, "f_contact_normal", 0.0))
            ee_z = float(obs.ee_pos[2]) if getattr(obs, "ee_pos", None) is not None else np.nan
            print(
                f"[MPC] t={t:6.3f} ok={ok} cost={cost:.2e} iters={iters:2d} "
                f"|tau_raw|∞={np.max(np.abs(tau_raw)):.2f} |tau_cmd|∞={np.max(np.abs(tau_cmd)):.2f} "
                f"surf={int(surface_now)} fn={fn:.2f} fn_pred={fn_pred:.2f} ee_z={ee_z:.4f} "
                f"solve={int(solved_now)} i={int(policy_idx)} unstable={int(unstable)}"
            )
        if not solved_now:
            self._rollout_shift()
        return tau_cmd


class ForceFeedbackCrocoddylMPC(_MPCBase):
    """Force-feedback EE MPC (crocoddyl_force_feedback.py:293-1093): OCP state
    y=(q,v,tau_filtered), control w; torque policy of Eq. 14-18."""

    variant = "ff"

    def __init__(self, sim, traj_fn: Traj, config: Optional[ForceFeedbackMPCConfig] = None, device: int = 0,
                 use_plan: bool = True):
        self.nx_aug = 21
        self._fn_pred_hist_raw: list = []
        self._fn_pred_hist_meas: list = []
        self._fn_pred_corr = np.nan
        super().__init__(sim, traj_fn, config if config is not None else ForceFeedbackMPCConfig(), device, use_plan)

    def _initial_tau(self, obs0):
        return obs0.tau_cmd

    def _ocp_config(self) -> OcpConfig:
        c = super()._ocp_config()
        c.ff_alpha = self._ff_alpha_ocp()
        c.w_w = float(self.cfg.w_w)
        c.w_w_soft_limits = float(self.cfg.w_w_soft_limits)
        c.w_y = float(self.cfg.w_y)
        c.y_weights = np.concatenate([self.cfg.y_q_weights, self.cfg.y_v_weights, self.cfg.y_tau_weights]).astype(float)
        c.use_inner_state_reg = bool(self.cfg.use_inner_state_reg)
        c.use_inner_tau_reg = bool(self.cfg.use_inner_tau_reg)
        return c

    # -- filter constants (crocoddyl_force_feedback.py:493-510) ----------------------
    def _ff_alpha_ocp(self) -> float:
        if self.cfg.ff_alpha_override is not None:
            return float(np.clip(float(self.cfg.ff_alpha_override), 0.0, 0.999999))
        wc = 2.0 * np.pi * float(max(self.cfg.ff_cutoff_hz, 0.0))
        return float(np.clip(np.exp(-wc * self._dt_ocp), 0.0, 0.999999))

    def _ff_alpha_ctrl(self) -> float:
        if self.cfg.ff_alpha_override is not None:
            return float(np.clip(float(self.cfg.ff_alpha_override), 0.0, 0.999999))
        dt_mpc = float(getattr(self.sim, "dt", self.cfg.dt))
        wc = 2.0 * np.pi * float(max(self.cfg.ff_cutoff_hz, 0.0))
        return float(np.clip(np.exp(-wc * dt_mpc), 0.0, 0.999999))

    def _policy_epsilon(self) -> float:
        dt_mpc = float(getattr(self.sim, "dt", self.cfg.dt))
        return float(np.clip(dt_mpc / self._dt_ocp, 0.0, 1.0))

    # -- measured torque state (crocoddyl_force_feedback.py:512-540) ------------------
    def _tau_state_from_obs(self, obs) -> np.ndarray:
        src = str(self.cfg.ff_tau_state_source).strip().lower()
        if src == "auto":
            src = "tau_meas_filt" if bool(self.cfg.ff_use_tau_meas_filt) else "tau_meas"
        keys = {
            "tau_meas_act_filt": ("tau_meas_act_filt", "tau_meas_act", "tau_cmd"),
            "tau_meas_act": ("tau_meas_act", "tau_cmd"),
            "tau_cmd": ("tau_cmd",),
            "tau_meas_filt": ("tau_meas_filt", "tau_meas"),
            "tau_meas": ("tau_meas",),
            "tau_total": ("tau_total", "tau_meas"),
        }.get(src, ("tau_meas_act_filt", "tau_meas_act", "tau_cmd", "tau_meas"))
        for key in keys:
            if not hasattr(obs, key):
                continue
            tau = np.asarray(getattr(obs, key), dtype=float).reshape(7)
            if np.all(np.isfinite(tau)):
                return tau
        tau = np.asarray(getattr(obs, "tau_cmd", np.zeros(7)), dtype=float).reshape(7)
        return tau if np.all(np.isfinite(tau)) else np.zeros(7)

    def _tau_from_aug_state(self, y) -> np.ndarray:
        return np.asarray(y, float).reshape(21)[14:21].copy()

    def _cold_control(self, y0) -> np.ndarray:
        return self._tau_from_aug_state(y0)

    def _compute_posture_reference(self, y0) -> np.ndarray:
        """crocoddyl_force_feedback.py:717-721 (FF: "x0" -> y0[:14], else q_nom)."""
        if str(self.cfg.posture_ref_mode).strip().lower() == "x0":
            return np.asarray(y0[:14], float).copy()
        return np.concatenate([self.q_nom, np.zeros(7)])

    # -- Eq. 14-18 (crocoddyl_force_feedback.py:1041-1093) ----------------------------
    def _policy_control(self, y_now) -> Tuple[np.ndarray, int]:
        if self.us is None or self.xs is None or len(self.us) == 0 or len(self.xs) == 0:
            return self._tau_from_aug_state(y_now), -1
        i = 0
        alpha = self._ff_alpha_ocp()
        eps = self._policy_epsilon() if bool(self.cfg.ff_use_tau_interpolation) else 0.0
        y0_nom = np.asarray(self.xs[i], dtype=float)
        tau0 = self._tau_from_aug_state(y0_nom)
        if len(self.xs) > i + 1:
            tau1 = self._tau_from_aug_state(self.xs[i + 1])
        else:
            tau1 = alpha * tau0 + (1.0 - alpha) * np.asarray(self.us[i], float).reshape(7)
        tau_cmd = tau0 + eps * (tau1 - tau0)
        if self.cfg.use_feedback_policy and self.Ks is not None and i < len(self.Ks):
            K0 = np.asarray(self.Ks[i], dtype=float)
            if K0.ndim == 1:
                K0 = K0.reshape(1, -1)
            if K0.shape[1] >= 21:
                Kx, Ktau = K0[:, :14], K0[:, 14:21]
                x_err = y0_nom[:14] - np.asarray(y_now[:14], float)
                tau_err = tau0 - np.asarray(y_now[14:21], float)
                I7 = np.eye(7)
                K_tilde_x = eps * (1.0 - alpha) * Kx
                K_tilde_tau = I7 + eps * (1.0 - alpha) * (Ktau - I7)
                tau_cmd = tau_cmd + float(self.cfg.feedback_gain_scale) * (K_tilde_x @ x_err + K_tilde_tau @ tau_err)
            elif "ff_policy_gain_dim" not in self._warned_keys:
                self._warned_keys.add("ff_policy_gain_dim")
                print(f"[WARN] FF policy gain shape {K0.shape} incompatible with ndx_aug=21; interpolation only.")
        return np.asarray(tau_cmd, float).reshape(7), i

    # -- force prediction (crocoddyl_force_feedback.py:1219-1243, 1301-1371) ----------
    def _predicted_normal_force_next_step(self) -> float:
        N = int(self.cfg.horizon)
        f0 = abs(float(self._res.fn_pred[0, 0]))
        if N == 1:
            return f0
        f1 = abs(float(self._res.fn_pred[0, 1]))
        if not np.isfinite(f0):
            return f1
        if not np.isfinite(f1):
            return f0
        dt_mpc = float(getattr(self.sim, "dt", self.cfg.dt))
        if dt_mpc >= self._dt_ocp - 1.0e-9:
            return f0
        eps = self._policy_epsilon()
        return float((1.0 - eps) * f0 + eps * f1)

    def _align_logged_force_prediction(self, fn_pred_raw: float, fn_meas: float, surface_now: bool) -> float:
        if not np.isfinite(fn_pred_raw):
            return np.nan
        if (not bool(surface_now)) or (not bool(self.cfg.ff_align_force_prediction)):
            self._fn_pred_corr = np.nan
            return float(fn_pred_raw)
        if np.isfinite(fn_meas):
            self._fn_pred_hist_raw.append(float(fn_pred_raw))
            self._fn_pred_hist_meas.append(float(fn_meas))
            win = int(max(self.cfg.ff_align_window, 16))
            if len(self._fn_pred_hist_raw) > win:
                self._fn_pred_hist_raw = self._fn_pred_hist_raw[-win:]
                self._fn_pred_hist_meas = self._fn_pred_hist_meas[-win:]
        min_n = int(max(self.cfg.ff_align_min_samples, 8))
        raw = np.asarray(self._fn_pred_hist_raw, float)
        meas = np.asarray(self._fn_pred_hist_meas, float)
        n = int(min(raw.size, meas.size))
        if n < min_n:
            self._fn_pred_corr = np.nan
            return float(fn_pred_raw)
        max_lag = min(int(max(self.cfg.ff_align_max_lag, 0)), n - min_n)
        corr_min = float(max(self.cfg.ff_align_corr_threshold, 0.0))
        best = None  # (rmse, lag, corr, a, b)
        for lag in range(max_lag + 1):
            x = raw[:-lag] if lag > 0 else raw
            y = meas[lag:] if lag > 0 else meas
            if x.size < min_n or y.size < min_n:
                continue
            xc, yc = x - float(np.mean(x)), y - float(np.mean(y))
            den = float(np.linalg.norm(xc) * np.linalg.norm(yc))
            if den < 1.0e-9:
                continue
            corr = float(np.dot(xc, yc) / den)
            if abs(corr) < corr_min:
                continue
            try:
                a, b = np.linalg.lstsq(np.column_stack([x, np.ones_like(x)]), y, rcond=None)[0]
            except np.linalg.LinAlgError:
                continue
            rmse = float(np.sqrt(np.mean((a * x + b - y) ** 2)))
            if best is None or rmse < best[0]:
                best = (rmse, lag, corr, float(a), float(b))
        if best is None:
            self._fn_pred_corr = np.nan
            return float(fn_pred_raw)
        _, lag, corr, a, b = best
        self._fn_pred_corr = corr
        x_cur = float(raw[max(0, raw.size - 1 - int(lag))])
        return float(max(a * x_cur + b, 0.0))

    def compute_control(self, obs, t: float) -> np.ndarray:
        """crocoddyl_force_feedback.py:542-695."""
        self._k += 1
        q = np.asarray(obs.q, dtype=float)
        v = np.asarray(obs.dq, dtype=float)
        tau_hat = self._tau_state_from_obs(obs)
        y0 = np.concatenate([q, v, tau_hat])
        surface_now = self._surface_mode(obs, t)
        self._track_mode(surface_now)
        solved_now = False
        ok, cost, iters = self._last_solve_ok, float(self._last_solve_cost), int(self._last_solve_iters)
        fn_pred_raw = float(self.last_info.get("fn_pred_raw", self.last_info.get("fn_pred", np.nan)))
        if self._need_solve():
            ok, cost, iters = self._solve(t, y0, surface_now)
            fn_pred_raw = self._predicted_normal_force_next_step() if surface_now else np.nan
            solved_now = True
        tau_des, policy_idx = self._policy_control(y0)
        tau_raw = np.asarray(tau_des, float).copy()
        if bool(self.cfg.ff_inverse_actuation_model):
            a_c = self._ff_alpha_ctrl()
            tau_raw = (tau_raw - a_c * tau_hat) / max(1.0e-6, 1.0 - a_c)
        tau_des_inf = float(np.max(np.abs(tau_des)))
        tau_raw_inf = float(np.max(np.abs(tau_raw)))
        unstable = (not np.isfinite(cost)) or cost > float(self.cfg.max_solver_cost) or \
            tau_raw_inf > float(self.cfg.max_tau_raw_inf)
        if unstable:
            tau_raw = np.asarray(obs.tau_bias, dtype=float) - float(self.cfg.fallback_dq_damping) * v
            self._invalidate()
        tau_cmd = self._safe_tau(tau_raw)
        fn_pred = self._align_logged_force_prediction(fn_pred_raw, float(getattr(obs, "f_contact_normal", np.nan)),
                                                      surface_now)
        fin = lambda z: float(z) if np.isfinite(z) else np.nan
        self.last_info = {
            "ok": bool(ok), "cost": float(cost), "iters": iters, "tau_des_inf": tau_des_inf,
            "tau_meas_state_inf": float(np.max(np.abs(tau_hat))), "tau_raw_inf": tau_raw_inf,
            "tau_cmd_inf": float(np.max(np.abs(tau_cmd))), "surface_mode": bool(surface_now),
            "unstable": bool(unstable), "fn_pred": fin(fn_pred), "fn_pred_raw": fin(fn_pred_raw),
            "fn_pred_corr": fin(self._fn_pred_corr), "solved_now": bool(solved_now), "policy_idx": int(policy_idx),
            "neg_branch": self._last_neg[0] if solved_now else 0, "neg_accepted": self._last_neg[1] if solved_now else 0,
        }
        if (self._k % self.cfg.debug_every) == 0:  # crocoddyl_force_feedback.py:673-683
            fn = float(getattr(obs, "f_contact_normal", 0.0))
            ee_z = float(obs.ee_pos[2]) if getattr(obs, "ee_pos", None) is not None else np.nan
            print(
                f"[MPC] t={t:6.3f} ok={ok} cost={cost:.2e} iters={iters:2d} "
                f"|tau_des|∞={np.max(np.abs(tau_des)):.2f} "
                f"|tau_raw|∞={np.max(np.abs(tau_raw)):.2f} |tau_cmd|∞={np.max(np.abs(tau_cmd)):.2f} "
                f"|tau_state|∞={np.max(np.abs(tau_hat)):.2f} "
                f"surf={int(surface_now)} fn={fn:.2f} fn_pred={fn_pred:.2f} corr={self._fn_pred_corr:.2f} "
                f"ee_z={ee_z:.4f} solve={int(solved_now)} i={int(policy_idx)} unstable={int(unstable)}"
            )
        if not solved_now:
            self._rollout_shift()
        return tau_cmd
