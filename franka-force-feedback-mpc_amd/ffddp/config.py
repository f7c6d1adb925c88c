"""OCP configuration mirroring the reference's controller configs.

`OcpConfig` carries exactly the ClassicalMPCConfig / ForceFeedbackMPCConfig
fields that _build_problem/_make_dam read (crocoddyl_classical.py:12-110,
521-728; crocoddyl_force_feedback.py:12-146, 776-1009).  `classical_preset`
and `ff_preset` are the benchmark-mode presets of src/run/run_classical.py:
269-315 and src/run/run_force_feedback.py:272-330.
"""
from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np

from . import _abi
from . import robot as R


@dataclass
class OcpConfig:
    variant: str = "classical"  # "classical" | "ff"
    horizon: int = 30
    dt: float = 0.01
    contact_model: str = "normal_1d"
    use_box_fddp: bool = True
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
    # friction cone (built only for point3d, crocoddyl_classical.py:678); the
    # benchmark presets switch it off (run_classical.py:292-294: weight 0, mu 1)
    w_friction_cone: float = 0.0
    mu: float = 1.0
    w_fn: float = 2.8e1
    fn_des: float = 22.0
    w_wdamp: float = 6.0e1
    w_wdamp_weights: np.ndarray = field(default_factory=lambda: np.array([1.8, 1.8, 0.3]))
    contact_gains: np.ndarray = field(default_factory=lambda: np.array([140.0, 80.0]))
    contact_inv_damping: float = 1.0e-8
    tau_limits: np.ndarray = field(default_factory=lambda: R.TAU_LIMITS.copy())
    R_des: np.ndarray = field(default_factory=R.default_R_des)
    # force feedback
    ff_alpha: float = 0.0
    w_w: float = 0.0
    w_w_soft_limits: float = 0.0
    w_y: float = 0.0
    y_weights: np.ndarray = field(default_factory=lambda: np.zeros(21))
    use_inner_state_reg: bool = True
    use_inner_tau_reg: bool = True

    @property
    def nc(self) -> int:
        return 3 if str(self.contact_model).strip().lower() in ("point3d", "3d", "rigid3d", "route_a_3d") else 1

    @property
    def nx(self) -> int:
        return 21 if self.variant == "ff" else 14

    def to_struct(self) -> _abi.OcpConfig:
        c = _abi.OcpConfig()
        c.variant = _abi.FFDDP_FORCE_FEEDBACK if self.variant == "ff" else _abi.FFDDP_CLASSICAL
        c.horizon = int(self.horizon)
        c.nc = self.nc
        c.use_box = 1 if self.use_box_fddp else 0
        c.dt = max(float(self.dt), 1.0e-6)
        for name in (
            "z_press", "w_ee_pos", "w_ee_ori", "w_posture", "w_v", "w_tau", "w_tau_soft_limits",
            "tau_soft_limit_margin", "w_q_soft_limits", "q_soft_limit_margin", "w_tangent_pos", "w_tangent_vel",
            "w_plane_z", "w_vz", "w_unilateral", "friction_margin", "w_fn", "fn_des", "w_wdamp",
            "contact_inv_damping", "ff_alpha", "w_w", "w_w_soft_limits", "w_y", "w_friction_cone", "mu",
        ):
            setattr(c, name, float(getattr(self, name)))
        _abi._fill(c.ori_weights, self.ori_weights)
        _abi._fill(c.v_damp_weights, self.v_damp_weights)
        _abi._fill(c.q_lower, R.Q_LOWER)
        _abi._fill(c.q_upper, R.Q_UPPER)
        _abi._fill(c.w_wdamp_weights, self.w_wdamp_weights)
        _abi._fill(c.contact_gains, self.contact_gains)
        _abi._fill(c.tau_limits, self.tau_limits)
        _abi._fill(c.R_des, np.asarray(self.R_des, float).reshape(9))
        _abi._fill(c.y_weights, self.y_weights)
        c.use_inner_state_reg = 1 if self.use_inner_state_reg else 0
        c.use_inner_tau_reg = 1 if self.use_inner_tau_reg else 0
        return c


def classical_preset(horizon: int = 30, contact_model: str = "normal_1d") -> OcpConfig:
    """run_classical.py:269-315 (benchmark mode).  The reference preset uses N=36; BASELINE uses 30 (R9)."""
    return OcpConfig(variant="classical", horizon=horizon, contact_model=contact_model)


def ff_alpha_ocp(cutoff_hz: float, dt_ocp: float) -> float:
    """_ff_alpha_ocp (crocoddyl_force_feedback.py:493-497)."""
    wc = 2.0 * np.pi * float(max(cutoff_hz, 0.0))
    return float(np.clip(np.exp(-wc * float(dt_ocp)), 0.0, 0.999999))


def ff_preset(horizon: int = 30, contact_model: str = "normal_1d") -> OcpConfig:
    """run_force_feedback.py:272-330 (benchmark mode).  The reference preset uses N=40 (R9)."""
    return OcpConfig(
        variant="ff",
        horizon=horizon,
        contact_model=contact_model,
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
        ff_alpha=ff_alpha_ocp(25.0, 0.01),
        w_w=6.0e-4,
        w_w_soft_limits=2.0,
        w_y=8.0e-4,
        y_weights=np.concatenate([[0.15] * 4 + [0.08] * 3, [0.05] * 4 + [0.03] * 3, [0.12] * 4 + [0.08] * 3]),
    )
