"""EE reference trajectories sampled per OCP node.

Restates src/tasks/trajectories.py:8-93 (make_approach_then_circle) and the
benchmark-mode wrapper of src/run/run_classical.py:221-264 (contact height,
pre/approach timing and the 0.2 s hold at contact onset).  Pinned by golden
vectors generated from the reference module itself (tests/golden/
make_golden.py -> reference_vectors.npz).
"""
from __future__ import annotations

from typing import Callable, Tuple

import numpy as np

Traj = Callable[[float], Tuple[np.ndarray, np.ndarray, bool]]


def _smoothstep(s: float) -> float:
    s = min(max(s, 0.0), 1.0)
    return s * s * (3.0 - 2.0 * s)


def _dsmoothstep(s: float) -> float:
    s = min(max(s, 0.0), 1.0)
    return 6.0 * s * (1.0 - s)


def make_approach_then_circle(
    center,
    radius: float,
    omega: float,
    z_contact: float,
    t_approach: float = 2.0,
    ee_start=None,
    z_pre=None,
    t_pre: float = 0.0,
) -> Traj:
    """traj(t) -> (p_ref[3], v_ref[3], surface_mode) (trajectories.py:8-93)."""
    center = np.asarray(center, dtype=float).reshape(3).copy()
    radius, omega, z_contact = float(radius), float(omega), float(z_contact)
    t_approach = max(float(t_approach), 1.0e-6)
    t_pre = max(float(t_pre), 0.0)

    p_contact_start = center.copy()
    p_contact_start[0] += radius
    p_contact_start[2] = z_contact
    if ee_start is None:
        p_start = p_contact_start.copy()
        p_start[2] += 0.08
    else:
        p_start = np.asarray(ee_start, dtype=float).reshape(3).copy()
    if z_pre is None:
        z_pre = max(z_contact + 0.05, p_start[2])
    z_pre = float(z_pre)
    p_pre = p_contact_start.copy()
    p_pre[2] = z_pre

    def blend(p0, p1, tau, T):
        s_lin = tau / T
        s = _smoothstep(s_lin)
        dsdt = _dsmoothstep(s_lin) / T
        return (1.0 - s) * p0 + s * p1, dsdt * (p1 - p0)

    def traj(t: float):
        t = float(t)
        if t_pre > 0.0 and t < t_pre:
            p, v = blend(p_start, p_pre, t, t_pre)
            return p, v, False
        if t < t_pre + t_approach:
            p0 = p_pre if t_pre > 0.0 else p_start
            p, v = blend(p0, p_contact_start, t - t_pre, t_approach)
            return p, v, False
        th = omega * (t - (t_pre + t_approach))
        p = center.copy()
        p[0] += radius * np.cos(th)
        p[1] += radius * np.sin(th)
        p[2] = z_contact
        v = np.zeros(3)
        v[0] = -radius * omega * np.sin(th)
        v[1] = radius * omega * np.cos(th)
        return p, v, True

    def sample(ts):
        """traj at every time of ts at once: (P [n][3], V [n][3], surface [n]),
        element for element the same arithmetic as traj (so the same bits)."""
        t = np.asarray(ts, dtype=float).reshape(-1)
        P, V = np.empty((t.size, 3)), np.empty((t.size, 3))
        m_pre = (t < t_pre) if t_pre > 0.0 else np.zeros(t.size, bool)
        m_app = ~m_pre & (t < t_pre + t_approach)
        m_cir = ~(m_pre | m_app)

        def blend_v(sel, p0, p1, tau, T):
            s_lin = tau / T
            sc = np.minimum(np.maximum(s_lin, 0.0), 1.0)
            s_ = sc * sc * (3.0 - 2.0 * sc)
            dsdt = 6.0 * sc * (1.0 - sc) / T
            P[sel] = (1.0 - s_)[:, None] * p0 + s_[:, None] * p1
            V[sel] = dsdt[:, None] * (p1 - p0)

        if m_pre.any():
            blend_v(m_pre, p_start, p_pre, t[m_pre], t_pre)
        if m_app.any():
            blend_v(m_app, p_pre if t_pre > 0.0 else p_start, p_contact_start, t[m_app] - t_pre, t_approach)
        if m_cir.any():
            th = omega * (t[m_cir] - (t_pre + t_approach))
            P[m_cir, 0] = center[0] + radius * np.cos(th)
            P[m_cir, 1] = center[1] + radius * np.sin(th)
            P[m_cir, 2] = z_contact
            V[m_cir, 0] = -radius * omega * np.sin(th)
            V[m_cir, 1] = radius * omega * np.cos(th)
            V[m_cir, 2] = 0.0
        return P, V, m_cir.copy()

    traj.sample = sample
    return traj


def with_contact_hold(base: Traj, t_contact_phase: float, t_hold: float = 0.2) -> Traj:
    """The benchmark runner's wrapper (run_classical.py:246-264): for t_hold
    after the contact onset the reference holds the onset point with zero
    velocity.  Keeps base's vectorised sample()."""
    t_cp, t_end = float(t_contact_phase), float(t_contact_phase) + float(t_hold)

    def traj(t: float):
        p, v, s = base(t)
        if s and float(t) < t_end:
            return np.asarray(base(t_cp)[0], float), np.zeros(3), True
        return p, v, s

    if hasattr(base, "sample"):
        p_hold = np.asarray(base(t_cp)[0], float)

        def sample(ts):
            t = np.asarray(ts, dtype=float).reshape(-1)
            P, V, S = base.sample(t)
            h = S & (t < t_end)
            P[h] = p_hold
            V[h] = 0.0
            return P, V, S

        traj.sample = sample
    return traj


# Benchmark scene constants (assets/scenes/panda_table_scene.xml:17-29,
# panda_robot.xml:189-199) and run_classical.py:221-255.
TABLE_CENTER = np.array([-0.5, 0.0, 0.3])
TABLE_HALF_Z = 0.02
TOOL_RADIUS = 0.03


def benchmark_traj(ee_start_mj, radius: float = 0.10, omega: float = 1.5) -> Tuple[Traj, dict]:
    """The benchmark-mode trajectory of run_classical.py:221-264 (MuJoCo world)."""
    z_top = TABLE_CENTER[2] + TABLE_HALF_Z
    z_contact = z_top + TOOL_RADIUS - 8.0e-3
    z_pre = z_contact + 0.05
    center = np.array([TABLE_CENTER[0], TABLE_CENTER[1], z_contact])
    t_approach, t_pre = 0.55, 0.25
    base = make_approach_then_circle(
        center=center, radius=radius, omega=omega, z_pre=z_pre, z_contact=z_contact,
        t_approach=t_approach, ee_start=np.asarray(ee_start_mj, float), t_pre=t_pre,
    )
    t_contact_phase = t_pre + t_approach
    traj = with_contact_hold(base, t_contact_phase, 0.2)
    meta = dict(z_contact=z_contact, z_pre=z_pre, center=center, t_contact_phase=t_contact_phase)
    return traj, meta
