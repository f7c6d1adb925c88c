"""Synthetic batched OCP instances (BASELINE.json configs).

Per instance (seeded numpy PCG64), regime "tracking" (default):
  t0  ~ U(0, 20) s;  q = IK(p_ref(t0), R_des) + U(-0.03, 0.03), i.e. the arm
        near its reference as in the closed loop (the only states the
        reference's solver ever sees), v ~ N(0, 0.05^2).
Regime "random" (SURVEY.md §8(d) literal):
  q   = q_neutral + U(-0.15, 0.15), clipped to [q_lo + 0.05, q_hi - 0.05]
        (panda_robot.xml:9,122,137,156,233), v ~ N(0, 0.1^2).  In contact
        mode this puts the EE ~30 cm above the contact plane; classical
        BoxFDDP then frequently diverges.
Common:
  FF: tau_hat = g(q) + N(0, 0.5^2)
  t0  ~ U(0, 20) s;  p_ref_k, v_ref_k = traj(t0 + k dt_ocp), k = 0..N, from the
        benchmark trajectory (run_classical.py:221-264), mapped MuJoCo->Pinocchio
        (crocoddyl_classical.py:250-255);  surface = traj(t0).surf.
  x_reg_ref = [q_nom, 0] (posture_ref_mode="q_nom", :462-466),
  tau_ref   = g(q0)      (torque_ref_mode="gravity_x0", :447-460),
  cold warm start xs_init = [x0]*(N+1), us_init = [g(q0)]*N (:740-743;
  FF: us_init = [tau_hat]*N, crocoddyl_force_feedback.py:1021-1025).
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

from . import robot as R
from .trajectory import benchmark_traj


@dataclass
class Batch:
    x0: np.ndarray  # (B, nx)
    node_ref: np.ndarray  # (B, N+1, 6)  p_ref, v_ref (Pinocchio frame)
    inst_ref: np.ndarray  # (B, 21)      x_reg_ref (14), tau_ref (7)
    surface: np.ndarray  # (B,) uint8
    xs_init: np.ndarray  # (B, N+1, nx)
    us_init: np.ndarray  # (B, N, 7)
    t0: np.ndarray  # (B,)

    @property
    def B(self) -> int:
        return int(self.x0.shape[0])

    def slice(self, sl) -> "Batch":
        return Batch(*(getattr(self, f)[sl] for f in ("x0", "node_ref", "inst_ref", "surface", "xs_init", "us_init", "t0")))


def pos_mj_to_pin(p_mj, p_site_minus_frame=np.zeros(3)):
    """_pos_mj_to_pin (crocoddyl_classical.py:250-252)."""
    return np.asarray(p_mj, float) @ R.R_MJ_FROM_PIN - p_site_minus_frame  # R^T p (R diagonal)


def vel_mj_to_pin(v_mj):
    return np.asarray(v_mj, float) @ R.R_MJ_FROM_PIN


def _log3(Rm):
    c = np.clip((np.trace(Rm) - 1.0) / 2.0, -1.0, 1.0)
    th = np.arccos(c)
    t = 0.5 if th < 1e-6 else th / (2.0 * np.sin(th))
    return t * np.array([Rm[2, 1] - Rm[1, 2], Rm[0, 2] - Rm[2, 0], Rm[1, 0] - Rm[0, 1]])


def ik_pose(fk, p_target, R_target, q_init, iters: int = 60, damping: float = 1e-4):
    """Damped least-squares IK on (position, orientation log error); fk(q)->(R,p)."""
    q = np.array(q_init, float)
    for _ in range(iters):
        Rq, pq = fk(q)
        e = np.concatenate([p_target - pq, Rq @ _log3(Rq.T @ R_target)])
        if np.max(np.abs(e)) < 1e-10:
            break
        J = np.zeros((6, 7))
        h = 1e-7
        for j in range(7):
            dq = np.zeros(7)
            dq[j] = h
            R2, p2 = fk(q + dq)
            J[:3, j] = (p2 - pq) / h
            J[3:, j] = Rq @ _log3(Rq.T @ R2) / h
        dq = J.T @ np.linalg.solve(J @ J.T + damping * np.eye(6), e)
        dq += 0.05 * (np.eye(7) - np.linalg.pinv(J) @ J) @ (R.Q_NEUTRAL - q)
        q = np.clip(q + dq, R.Q_LOWER + 0.02, R.Q_UPPER - 0.02)
    return q


_IK_CACHE: dict = {}


def _ik_grid(traj, fk, R_des, t_max: float, n: int):
    key = (id(fk), t_max, n)
    if key not in _IK_CACHE:
        ts = np.linspace(0.0, t_max, n)
        qs = np.zeros((n, 7))
        q = R.Q_NEUTRAL.copy()
        for i, t in enumerate(ts):
            q = ik_pose(fk, pos_mj_to_pin(traj(t)[0]), R_des, q)
            qs[i] = q
        _IK_CACHE[key] = (ts, qs)
    return _IK_CACHE[key]


def make_batch(
    B: int,
    horizon: int,
    variant: str,
    gravity_fn,
    ee_start_mj,
    seed: int = 0,
    dt_ocp: float = 0.01,
    t_range=(0.0, 20.0),
    surface_override=None,
    regime: str = "tracking",
    fk=None,
    R_des=None,
) -> Batch:
    """Build B synthetic instances.  gravity_fn(q (B,7)) -> (B,7); fk(q) -> (R, p)
    (needed by the "tracking" regime)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    N = horizon
    t0 = rng.uniform(t_range[0], t_range[1], size=B)
    if regime == "random":
        q = R.Q_NEUTRAL + rng.uniform(-0.15, 0.15, size=(B, 7))
        q = np.clip(q, R.Q_LOWER + 0.05, R.Q_UPPER - 0.05)
        v = rng.normal(0.0, 0.1, size=(B, 7))
    elif regime == "tracking":
        if fk is None:
            raise ValueError("regime='tracking' needs fk")
        traj_ik, meta = benchmark_traj(ee_start_mj)
        # contact phase is periodic in the circle angle: IK on a 1/128-period grid
        period = 2.0 * np.pi / 1.5
        t_c = meta["t_contact_phase"] + 0.2
        ts_a, qs_a = _ik_grid(traj_ik, fk, R.default_R_des() if R_des is None else R_des, t_c, 48)
        ts_c, qs_c = _ik_grid(lambda t: traj_ik(t_c + t), fk, R.default_R_des() if R_des is None else R_des, period, 129)
        q = np.zeros((B, 7))
        for b in range(B):
            if t0[b] < t_c:
                q[b] = qs_a[int(np.argmin(np.abs(ts_a - t0[b])))]
            else:
                ph = (t0[b] - t_c) % period
                q[b] = qs_c[int(np.argmin(np.abs(ts_c - ph)))]
        q = np.clip(q + rng.uniform(-0.03, 0.03, size=(B, 7)), R.Q_LOWER + 0.02, R.Q_UPPER - 0.02)
        v = rng.normal(0.0, 0.05, size=(B, 7))
    else:
        raise ValueError(regime)
    g = np.asarray(gravity_fn(q), float).reshape(B, 7)
    if variant == "ff":
        tau_hat = g + rng.normal(0.0, 0.5, size=(B, 7))
        x0 = np.concatenate([q, v, tau_hat], 1)
        u_init = tau_hat
    else:
        x0 = np.concatenate([q, v], 1)
        u_init = g
    traj, _ = benchmark_traj(ee_start_mj)
    node_ref = np.zeros((B, N + 1, 6))
    surface = np.zeros(B, np.uint8)
    for b in range(B):
        surface[b] = 1 if traj(t0[b])[2] else 0
        for k in range(N + 1):
            p, vr, _ = traj(t0[b] + k * dt_ocp)
            node_ref[b, k, 0:3] = pos_mj_to_pin(p)
            node_ref[b, k, 3:6] = vel_mj_to_pin(vr)
    if surface_override is not None:
        surface[:] = np.uint8(surface_override)
    x_reg = np.concatenate([np.broadcast_to(R.Q_NEUTRAL, (B, 7)), np.zeros((B, 7))], 1)
    inst_ref = np.concatenate([x_reg, g], 1)
    xs_init = np.repeat(x0[:, None, :], N + 1, axis=1).copy()
    us_init = np.repeat(u_init[:, None, :], N, axis=1).copy()
    return Batch(x0, node_ref, inst_ref, surface, xs_init, us_init, t0)
