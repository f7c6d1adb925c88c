"""ORACLE — test infrastructure only.  Never imported by the product path.

numpy (fp64) restatement of the closed-loop plant stand-in
(franka-force-feedback-mpc_amd/csrc/ffddp_plant.hpp), i.e. the subset of
MuJoCo the reference's closed loop exercises (src/sim/franka_sim.py:144-169,
torque mode, assets/scenes/panda_table_scene.xml):

  * arm dynamics with joint armature 0.1 and damping 1 (panda_robot.xml:9),
  * the tool sphere (r = 0.03, panda_robot.xml:191-198) against the
    table_contact plane (condim 1, margin 0.001, panda_table_scene.xml:17-22)
    as one soft frictionless constraint (solref / solimp defaults),
  * implicitfast integration with n_substeps physics steps per control step.

Built on oracle/panda.py (independent of the HIP code).  Parity with MuJoCo
itself: UNPINNED (MuJoCo is not installed).  Checked by physical identities in
tests/test_plant.py (static contact equilibrium, free-fall energy, constraint
force = MuJoCo's closed form for a single contact).
"""
from __future__ import annotations

import numpy as np

from . import panda as P

R_MJ = np.diag([-1.0, -1.0, 1.0])
_C135, _S135 = np.cos(np.deg2rad(135.0)), np.sin(np.deg2rad(135.0))
R_SITE = np.array([[_C135, -_S135, 0.0], [_S135, _C135, 0.0], [0.0, 0.0, 1.0]])


def default_params(timestep=0.001, n_substeps=5):
    return dict(timestep=timestep, n_substeps=n_substeps, armature=np.full(7, 0.1), damping=np.full(7, 1.0),
                r_tool=0.03, margin=0.001, solref=(0.02, 1.0), solimp=(0.9, 0.95, 0.001, 0.5, 2.0))


def impedance(solimp, pos):
    d0, dmax, width, mid, pw = solimp
    x = abs(pos) / width
    if x >= 1.0:
        return dmax
    y = x ** pw / mid ** (pw - 1.0) if x <= mid else 1.0 - (1.0 - x) ** pw / (1.0 - mid) ** (pw - 1.0)
    return d0 + y * (dmax - d0)


def contact_force(prm, A, a_unc, vel, dist):
    """Soft frictionless unilateral contact, one constraint row (MuJoCo)."""
    pos = dist - prm["margin"]
    imp = impedance(prm["solimp"], pos)
    dmax = prm["solimp"][1]
    tc, dr = prm["solref"]
    K = 1.0 / (dmax * dmax * tc * tc * dr * dr)
    Bd = 2.0 / (dmax * tc)
    aref = -Bd * vel - K * imp * pos
    Rr = (1.0 - imp) / imp * A
    return max(0.0, (aref - a_unc) / (A + Rr))


def forward(prm, q, v, tau, n_mj, p0_mj):
    """One mj_forward: returns qfrc pieces, contact and site kinematics."""
    n = R_MJ @ np.asarray(n_mj, float)
    p0 = R_MJ @ np.asarray(p0_mj, float)
    z7 = np.zeros(7)
    out = P.rnea_full(q, v, z7)
    bias = out["tau"]
    M = P.crba(q) + np.diag(prm["armature"])
    fs = tau - bias - prm["damping"] * v
    qs = np.linalg.solve(M, fs)
    J6, R_ee, p_ee = P.frame_jacobian_lwa(q)
    Jl = J6[:3]
    dist = float(n @ (p_ee - p0)) - prm["r_tool"]
    f = 0.0
    qc = np.zeros(7)
    active = dist < prm["margin"]
    if active:
        Jn = n @ Jl
        A = float(Jn @ np.linalg.solve(M, Jn))
        a_unc = float(Jn @ qs + n @ out["acc_ee"])
        f = contact_force(prm, A, a_unc, float(Jn @ v), dist)
        qc = Jn * f
    return dict(M=M, fs=fs, bias=bias, qc=qc, f=f, active=active, Jl=Jl, R_ee=R_ee, p_ee=p_ee, n_mj=np.asarray(n_mj))


def step(prm, q, v, tau, n_mj, p0_mj, integrate=True):
    """One control step; returns (q, v, obs dict) in the plant record's terms."""
    q = np.array(q, float)
    v = np.array(v, float)
    nsub = prm["n_substeps"] if integrate else 1
    h = prm["timestep"]
    fw = None
    for _ in range(nsub):
        fw = forward(prm, q, v, tau, n_mj, p0_mj)
        if not integrate:
            break
        qa = np.linalg.solve(fw["M"] + h * np.diag(prm["damping"]), fw["fs"] + fw["qc"])
        v = v + h * qa
        q = q + h * v
    J_mj = R_MJ @ fw["Jl"]
    obs = dict(q=q, dq=v, bias=fw["bias"], tau_c=fw["qc"], ee_pos=R_MJ @ fw["p_ee"], ee_vel=J_mj @ v,
               ee_R=R_MJ @ fw["R_ee"] @ R_SITE, f_world=fw["n_mj"] * fw["f"], fn=fw["f"],
               ncon=1.0 if fw["active"] else 0.0, J=J_mj)
    return q, v, obs
