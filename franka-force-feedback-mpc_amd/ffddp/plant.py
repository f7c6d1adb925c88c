"""Closed-loop plant stand-in on the GPU.

The reference closes its MPC loop around MuJoCo: ``FrankaMujocoSim``
(src/sim/franka_sim.py:40-354) in torque mode on
assets/scenes/panda_table_scene.xml, with a hidden table tilt per scenario
(run_classical.py:94-107).  MuJoCo is not available here, so this module
provides the same observation interface over a HIP kernel
(csrc/ffddp_plant.hpp, C-ABI ``ffddp_plant_*``) that integrates the arm with
armature/damping, the tool sphere and the table_contact plane as MuJoCo's soft
frictionless contact, implicitfast, ``n_substeps`` physics steps per control
step.  Parity with MuJoCo is unpinned.

``PandaTablePlant``  one plant with FrankaMujocoSim's methods (reset, step,
                     get_observation, bias_torque, dt, tau_meas_lpf_alpha)
``BatchedPlant``     B plants stepped by one launch (per-instance tilt), for
                     batched closed loops.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass
from typing import Optional

import numpy as np

from . import _abi
from . import robot as R

# scene constants (panda_table_scene.xml:15-29, panda_robot.xml:9, 189-199, 233)
TABLE_BODY_POS = np.array([-0.5, 0.0, 0.3])
TABLE_CONTACT_OFFSET = np.array([0.0, 0.0, 0.02])  # table_contact plane in the table body
TABLE_TOP_HALF = np.array([0.35, 0.35, 0.02])  # table_top box half-sizes (at the body origin)
R_TOOL = 0.03
CONTACT_MARGIN = 0.001
JOINT_ARMATURE = 0.1
JOINT_DAMPING = 1.0
KEYFRAMES = {"neutral": R.Q_NEUTRAL.copy(), "home": np.array([0.0, 0.0, 0.0, -1.57079, 0.0, 1.57079, -0.7853])}
DEFAULT_TIMESTEP = 0.002  # MuJoCo default (the scene sets none); benchmark protocol uses 0.001


@dataclass
class Observation:
    """Same fields as the reference's Observation (franka_sim.py:11-37)."""

    q: np.ndarray
    dq: np.ndarray
    tau_meas: np.ndarray
    tau_meas_filt: np.ndarray
    tau_meas_act: np.ndarray
    tau_meas_act_filt: np.ndarray
    tau_cmd: np.ndarray
    tau_act: np.ndarray
    tau_constraint: np.ndarray
    tau_total: np.ndarray
    tau_bias: np.ndarray
    f_contact_world: np.ndarray
    f_contact_normal: float
    f_contact_normal_world_z: float
    f_contact_tangent: float
    contact_count_ee: int
    contact_count_table: int
    table_normal_world: np.ndarray
    ee_pos: Optional[np.ndarray] = None
    ee_quat: Optional[np.ndarray] = None
    J_pos: Optional[np.ndarray] = None
    J_rot: Optional[np.ndarray] = None
    ee_vel: Optional[np.ndarray] = None


def mat_to_quat_wxyz(Rm: np.ndarray) -> np.ndarray:
    """Rotation matrix -> unit quaternion (w, x, y, z), Shepperd's branch on
    the largest diagonal term (same convention as franka_sim.py:317-354)."""
    Rm = np.asarray(Rm, dtype=float).reshape(3, 3)
    tr = Rm[0, 0] + Rm[1, 1] + Rm[2, 2]
    if tr > 0.0:
        s = 2.0 * np.sqrt(tr + 1.0)
        q = [0.25 * s, (Rm[2, 1] - Rm[1, 2]) / s, (Rm[0, 2] - Rm[2, 0]) / s, (Rm[1, 0] - Rm[0, 1]) / s]
    else:
        if Rm[0, 0] > Rm[1, 1] and Rm[0, 0] > Rm[2, 2]:
            s = 2.0 * np.sqrt(1.0 + Rm[0, 0] - Rm[1, 1] - Rm[2, 2])
            q = [(Rm[2, 1] - Rm[1, 2]) / s, 0.25 * s, (Rm[0, 1] + Rm[1, 0]) / s, (Rm[0, 2] + Rm[2, 0]) / s]
        elif Rm[1, 1] > Rm[2, 2]:
            s = 2.0 * np.sqrt(1.0 + Rm[1, 1] - Rm[0, 0] - Rm[2, 2])
            q = [(Rm[0, 2] - Rm[2, 0]) / s, (Rm[0, 1] + Rm[1, 0]) / s, 0.25 * s, (Rm[1, 2] + Rm[2, 1]) / s]
        else:
            s = 2.0 * np.sqrt(1.0 + Rm[2, 2] - Rm[0, 0] - Rm[1, 1])
            q = [(Rm[1, 0] - Rm[0, 1]) / s, (Rm[0, 2] + Rm[2, 0]) / s, (Rm[1, 2] + Rm[2, 1]) / s, 0.25 * s]
    q = np.asarray(q, dtype=float)
    return q / (np.linalg.norm(q) + 1e-12)


def table_plane(tilt_deg: float = 0.0):
    """(normal, point) of the table_contact plane in the MuJoCo world with the
    table body rotated by tilt_deg about world y (_apply_table_tilt,
    run_classical.py:94-107)."""
    a = np.deg2rad(float(tilt_deg))
    Ry = np.array([[np.cos(a), 0.0, np.sin(a)], [0.0, 1.0, 0.0], [-np.sin(a), 0.0, np.cos(a)]])
    return Ry[:, 2].copy(), TABLE_BODY_POS + Ry @ TABLE_CONTACT_OFFSET


def plant_params(timestep: float = DEFAULT_TIMESTEP, n_substeps: int = 1) -> _abi.PlantParams:
    p = _abi.PlantParams()
    p.timestep = float(timestep)
    p.n_substeps = int(n_substeps)
    _abi._fill(p.armature, np.full(7, JOINT_ARMATURE))
    _abi._fill(p.damping, np.full(7, JOINT_DAMPING))
    p.r_tool = R_TOOL
    p.margin = CONTACT_MARGIN
    _abi._fill(p.solref, [0.02, 1.0])
    _abi._fill(p.solimp, [0.9, 0.95, 0.001, 0.5, 2.0])
    _abi._fill(p.site_R, [np.cos(np.deg2rad(135.0)), np.sin(np.deg2rad(135.0))])
    return p


def observation_from_record(rec, tau_cmd=None, tilt_deg: float = 0.0) -> Observation:
    """Observation of one FFDDP_PLANT_OBS record (no torque filters: the
    tau_meas* fields hold the unfiltered tau_total)."""
    rec = np.asarray(rec, dtype=float)
    tau_cmd = np.zeros(7) if tau_cmd is None else np.asarray(tau_cmd, dtype=float).copy()
    tau_c = rec[21:28].copy()
    total = tau_cmd + tau_c
    ncon = int(round(rec[47]))
    fw = rec[43:46].copy()
    return Observation(
        q=rec[0:7].copy(), dq=rec[7:14].copy(), tau_meas=total.copy(), tau_meas_filt=total.copy(),
        tau_meas_act=tau_cmd.copy(), tau_meas_act_filt=tau_cmd.copy(), tau_cmd=tau_cmd, tau_act=np.zeros(7),
        tau_constraint=tau_c, tau_total=total, tau_bias=rec[14:21].copy(), f_contact_world=fw,
        f_contact_normal=abs(float(rec[46])) if ncon else 0.0, f_contact_normal_world_z=max(float(fw[2]), 0.0),
        f_contact_tangent=0.0, contact_count_ee=ncon, contact_count_table=ncon,
        table_normal_world=table_plane(tilt_deg)[0], ee_pos=rec[28:31].copy(),
        ee_quat=mat_to_quat_wxyz(rec[34:43].reshape(3, 3)), J_pos=rec[48:69].reshape(3, 7).copy(), J_rot=None,
        ee_vel=rec[31:34].copy(),
    )


class BatchedPlant:
    """B plant instances on one device; host-array stepping (one launch per
    control step).  ``obs`` rows follow FFDDP_PLANT_OBS (ffddp_plant.hpp)."""

    def __init__(self, B: int, timestep: float = DEFAULT_TIMESTEP, n_substeps: int = 1, device: int = 0):
        self.lib = _abi.load()
        self.B = int(B)
        self.params = plant_params(timestep, n_substeps)
        h = C.c_void_p()
        rc = self.lib.ffddp_plant_create(C.byref(_abi.robot_struct()), C.byref(self.params), int(device), self.B,
                                         C.byref(h))
        if rc:
            raise RuntimeError(f"ffddp_plant_create failed ({rc}); a HIP device is required")
        self._h = h
        self.q = np.tile(R.Q_NEUTRAL, (self.B, 1))
        self.v = np.zeros((self.B, 7))
        self.plane = np.tile(np.concatenate(table_plane(0.0)), (self.B, 1))
        self.obs = np.zeros((self.B, _abi.PLANT_OBS))

    @property
    def dt(self) -> float:
        return float(self.params.timestep * self.params.n_substeps)

    def set_tilt(self, tilt_deg):
        tilt = np.broadcast_to(np.asarray(tilt_deg, dtype=float), (self.B,))
        self.plane = np.stack([np.concatenate(table_plane(t)) for t in tilt])

    def step(self, tau, integrate: bool = True) -> np.ndarray:
        tau = np.ascontiguousarray(np.broadcast_to(np.asarray(tau, dtype=float), (self.B, 7)))
        self.q = np.ascontiguousarray(self.q)
        self.v = np.ascontiguousarray(self.v)
        self.plane = np.ascontiguousarray(self.plane)
        rc = self.lib.ffddp_plant_step(self._h, self.B, _abi.dptr(self.q), _abi.dptr(self.v), _abi.dptr(tau),
                                       _abi.dptr(self.plane), 1 if integrate else 0, _abi.dptr(self.obs))
        if rc:
            raise RuntimeError(f"ffddp_plant_step failed ({rc})")
        return self.obs

    def close(self):
        if getattr(self, "_h", None):
            self.lib.ffddp_plant_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class PandaTablePlant:
    """FrankaMujocoSim (torque mode) counterpart for one arm: the methods and
    Observation fields the controllers and runners use (franka_sim.py:40-237)."""

    def __init__(self, n_substeps: int = 1, timestep: float = DEFAULT_TIMESTEP, tau_meas_lpf_alpha: float = 0.2,
                 device: int = 0):
        self.n_substeps = int(n_substeps)
        self.tau_meas_lpf_alpha = float(np.clip(tau_meas_lpf_alpha, 0.0, 1.0))
        self._bp = BatchedPlant(1, timestep, n_substeps, device)
        self.tilt_deg = 0.0
        self._tau_cmd = np.zeros(7)
        self._filt = np.zeros(7)
        self._filt_act = np.zeros(7)
        self._bp.step(np.zeros(7), integrate=False)

    @property
    def dt(self) -> float:
        return self._bp.dt

    @property
    def timestep(self) -> float:
        return float(self._bp.params.timestep)

    def set_table_tilt(self, tilt_deg: float):
        """_apply_table_tilt (run_classical.py:94-107) + mj_forward."""
        self.tilt_deg = float(tilt_deg)
        self._bp.set_tilt(self.tilt_deg)
        self._bp.step(self._tau_cmd, integrate=False)

    def table_geometry(self):
        """(center, half sizes, z_top) of table_top (_table_geometry_world, run_classical.py:42-50)."""
        c = TABLE_BODY_POS.copy()
        return c, TABLE_TOP_HALF.copy(), float(c[2] + TABLE_TOP_HALF[2])

    def reset(self, keyframe: str = "neutral") -> Observation:
        if keyframe not in KEYFRAMES:
            raise ValueError(f"Keyframe '{keyframe}' not found.")
        self._bp.q[0] = KEYFRAMES[keyframe]
        self._bp.v[0] = 0.0
        self._tau_cmd = np.zeros(7)
        rec = self._bp.step(self._tau_cmd, integrate=False)[0]
        tau_c = rec[21:28]
        self._filt = self._tau_cmd + tau_c
        self._filt_act = self._tau_cmd.copy()
        return self.get_observation(with_ee=True, with_jacobian=True)

    def step(self, u) -> Observation:
        u = np.asarray(u, dtype=np.float64).reshape(-1).copy()
        if u.shape != (7,):
            raise ValueError(f"torque mode expects (7,), got {u.shape}")
        self._tau_cmd = u
        self._bp.step(u, integrate=True)
        return self.get_observation(with_ee=True, with_jacobian=True)

    def set_state(self, q, v=None) -> Observation:
        """Write qpos / qvel and run the forward pass (data.qpos[...] = q; mj_forward)."""
        self._bp.q[0] = np.asarray(q, float).reshape(7)
        self._bp.v[0] = 0.0 if v is None else np.asarray(v, float).reshape(7)
        self._bp.step(self._tau_cmd, integrate=False)
        return self.get_observation(with_ee=True, with_jacobian=True)

    def bias_torque(self) -> np.ndarray:
        return self._bp.obs[0, 14:21].copy()

    def get_observation(self, with_ee: bool = True, with_jacobian: bool = False) -> Observation:
        rec = self._bp.obs[0]
        q, dq = rec[0:7].copy(), rec[7:14].copy()
        tau_bias, tau_c = rec[14:21].copy(), rec[21:28].copy()
        tau_cmd = self._tau_cmd.copy()
        tau_act = np.zeros(7)  # torque mode: actuators zeroed (franka_sim.py:117-124)
        tau_meas_act = tau_cmd + tau_act
        tau_total = tau_cmd + tau_act + tau_c
        a = self.tau_meas_lpf_alpha
        self._filt = (1.0 - a) * self._filt + a * tau_total
        self._filt_act = (1.0 - a) * self._filt_act + a * tau_meas_act
        fw = rec[43:46].copy()
        fn = float(rec[46])
        ncon = int(round(rec[47]))
        n_tab, _ = table_plane(self.tilt_deg)
        ee_pos = ee_quat = ee_vel = J_pos = None
        if with_ee:
            ee_pos = rec[28:31].copy()
            ee_quat = mat_to_quat_wxyz(rec[34:43].reshape(3, 3))
            ee_vel = rec[31:34].copy()
        if with_jacobian:
            J_pos = rec[48:69].reshape(3, 7).copy()
        return Observation(
            q=q, dq=dq, tau_meas=tau_total.copy(), tau_meas_filt=self._filt.copy(), tau_meas_act=tau_meas_act,
            tau_meas_act_filt=self._filt_act.copy(), tau_cmd=tau_cmd, tau_act=tau_act, tau_constraint=tau_c,
            tau_total=tau_total, tau_bias=tau_bias, f_contact_world=fw, f_contact_normal=abs(fn) if ncon else 0.0,
            f_contact_normal_world_z=max(float(fw[2]), 0.0), f_contact_tangent=0.0, contact_count_ee=ncon,
            contact_count_table=ncon, table_normal_world=n_tab, ee_pos=ee_pos, ee_quat=ee_quat, J_pos=J_pos,
            J_rot=None, ee_vel=ee_vel,
        )

    def close(self):
        self._bp.close()
