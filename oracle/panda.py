"""ORACLE — test infrastructure only.  Never imported by the product path.

CPU (numpy, fp64) restatement of the rigid-body algorithms that the reference
reaches through Pinocchio for the Franka Panda 7-DoF arm.  Only `tests/`,
`__graft_entry__.smoke()` and `bench.py`'s `cpu_baseline` leg may import this
package, and only as the checker.

Parity status: Pinocchio is not vendored in /root/reference and is not
installed here, so these routines cannot be run against the
real library.  They are pinned instead by
  * finite differences / complex-step identities (tests/test_oracle_*.py),
  * physical identities (M symmetric positive definite, RNEA(q,v,ABA(q,v,tau))
    == tau, power balance, KKT residuals),
  * the MJCF kinematics of assets/scenes/panda_robot.xml (test parses the XML
    when /root/reference is present and compares every parameter).
Parity against real Pinocchio/Crocoddyl: UNPINNED.

Model: link placements, masses, COMs and inertias
transcribed from /root/reference/assets/scenes/panda_robot.xml:98-199, armature
0, no hand payload.  The Pinocchio world is the MJCF link0 frame (the MJCF
applies a 180 deg yaw to link0, panda_robot.xml:98, which is exactly the
R_mj_from_pin = diag(-1,-1,1) map of src/mpc/crocoddyl_classical.py:151).
The EE frame "panda_link8" is link7 translated by (0, 0, 0.107)
(franka URDF joint8; the MJCF tool body sits at the same origin,
panda_robot.xml:189).

All functions are vectorised over arbitrary leading batch dimensions and are
complex-safe (only +, *, sin, cos, matmul) so that complex-step
differentiation can be used for the derivatives Pinocchio computes
analytically (computeRNEADerivatives, getFrameAccelerationDerivatives,
getFrameVelocityDerivatives).

Spatial algebra convention (Pinocchio): motion = (linear v, angular w),
force = (linear f, angular n), all expressed in the WORLD frame at the world
origin ("oMi / ov / oa / of" quantities of Pinocchio's derivative algorithms).
"""
from __future__ import annotations

import numpy as np

NQ = 7
GRAVITY = np.array([0.0, 0.0, -9.81])

_SQ = np.sqrt(0.5)


def _rx(deg: float) -> np.ndarray:
    if deg == 90.0:
        return np.array([[1.0, 0, 0], [0, 0, -1.0], [0, 1.0, 0]])
    if deg == -90.0:
        return np.array([[1.0, 0, 0], [0, 0, 1.0], [0, -1.0, 0]])
    if deg == 0.0:
        return np.eye(3)
    raise ValueError(deg)


def _fullinertia(ixx, iyy, izz, ixy, ixz, iyz) -> np.ndarray:
    # MuJoCo fullinertia order: (Ixx, Iyy, Izz, Ixy, Ixz, Iyz)
    return np.array([[ixx, ixy, ixz], [ixy, iyy, iyz], [ixz, iyz, izz]], dtype=float)


# --- panda_robot.xml:113-187 (body pos / quat / inertial of link1..link7) ----
# quat="1 -1 0 0" is -90 deg about x, quat="1 1 0 0" is +90 deg about x.
JOINT_PLACEMENT_P = np.array(
    [
        [0.0, 0.0, 0.333],      # link1  pos="0 0 0.333"            (:113)
        [0.0, 0.0, 0.0],        # link2  quat="1 -1 0 0"            (:119)
        [0.0, -0.316, 0.0],     # link3  pos="0 -0.316 0" quat="1 1 0 0" (:125)
        [0.0825, 0.0, 0.0],     # link4  pos="0.0825 0 0" quat="1 1 0 0" (:134)
        [-0.0825, 0.384, 0.0],  # link5  pos="-0.0825 0.384 0" quat="1 -1 0 0" (:143)
        [0.0, 0.0, 0.0],        # link6  quat="1 1 0 0"             (:153)
        [0.088, 0.0, 0.0],      # link7  pos="0.088 0 0" quat="1 1 0 0" (:175)
    ]
)
JOINT_PLACEMENT_R = np.stack([_rx(0.0), _rx(-90.0), _rx(90.0), _rx(90.0), _rx(-90.0), _rx(90.0), _rx(90.0)])

LINK_MASS = np.array([4.970684, 0.646926, 3.228604, 3.587895, 1.225946, 1.666555, 7.35522e-01])
LINK_COM = np.array(
    [
        [0.003875, 0.002081, -0.04762],
        [-0.003141, -0.02872, 0.003495],
        [2.7518e-2, 3.9252e-2, -6.6502e-2],
        [-5.317e-2, 1.04419e-1, 2.7454e-2],
        [-1.1953e-2, 4.1065e-2, -3.8437e-2],
        [6.0149e-2, -1.4117e-2, -1.0517e-2],
        [1.0517e-2, -4.252e-3, 6.1597e-2],
    ]
)
LINK_INERTIA = np.stack(
    [
        _fullinertia(0.70337, 0.70661, 0.0091170, -0.00013900, 0.0067720, 0.019169),
        _fullinertia(0.0079620, 2.8110e-2, 2.5995e-2, -3.925e-3, 1.0254e-2, 7.04e-4),
        _fullinertia(3.7242e-2, 3.6155e-2, 1.083e-2, -4.761e-3, -1.1396e-2, -1.2805e-2),
        _fullinertia(2.5853e-2, 1.9552e-2, 2.8323e-2, 7.796e-3, -1.332e-3, 8.641e-3),
        _fullinertia(3.5549e-2, 2.9474e-2, 8.627e-3, -2.117e-3, -4.037e-3, 2.29e-4),
        _fullinertia(1.964e-3, 4.354e-3, 5.433e-3, 1.09e-4, -1.158e-3, 3.41e-4),
        _fullinertia(1.2516e-2, 1.0027e-2, 4.815e-3, -4.28e-4, -1.196e-3, -7.41e-4),
    ]
)
EE_OFFSET = np.array([0.0, 0.0, 0.107])  # panda_link8 in link7 (tool body, :189)

# joint ranges: class default (:9) overridden for joints 2, 4, 6 (:122, :137, :156)
Q_LOWER = np.array([-2.8973, -1.7628, -2.8973, -3.0718, -2.8973, -0.0175, -2.8973])
Q_UPPER = np.array([2.8973, 1.7628, 2.8973, -0.0698, 2.8973, 3.7525, 2.8973])
Q_NEUTRAL = np.array([0.0, -0.758, 0.0, -2.22, 0.0, 1.43, 0.0])  # keyframe "neutral" (:233)

# site frame: tool body quat="0.3826834 0 0 0.9238795" = 135 deg about z (:189)
_C135, _S135 = np.cos(np.deg2rad(135.0)), np.sin(np.deg2rad(135.0))
R_SITE_FROM_EE = np.array([[_C135, -_S135, 0.0], [_S135, _C135, 0.0], [0.0, 0.0, 1.0]])
R_MJ_FROM_PIN = np.diag([-1.0, -1.0, 1.0])  # crocoddyl_classical.py:151


# ---------------------------------------------------------------------------
# small helpers (complex-safe, batched)
# ---------------------------------------------------------------------------
def cross(a, b):
    return np.stack(
        [
            a[..., 1] * b[..., 2] - a[..., 2] * b[..., 1],
            a[..., 2] * b[..., 0] - a[..., 0] * b[..., 2],
            a[..., 0] * b[..., 1] - a[..., 1] * b[..., 0],
        ],
        axis=-1,
    )


def mv(M, v):
    return np.einsum("...ij,...j->...i", M, v)


def mm(A, B):
    return np.einsum("...ij,...jk->...ik", A, B)


def skew(v):
    z = np.zeros(v.shape[:-1], dtype=v.dtype)
    return np.stack(
        [
            np.stack([z, -v[..., 2], v[..., 1]], -1),
            np.stack([v[..., 2], z, -v[..., 0]], -1),
            np.stack([-v[..., 1], v[..., 0], z], -1),
        ],
        -2,
    )


def rotz(q):
    c, s = np.cos(q), np.sin(q)
    o, z = np.ones_like(q), np.zeros_like(q)
    return np.stack([np.stack([c, -s, z], -1), np.stack([s, c, z], -1), np.stack([z, z, o], -1)], -2)


def motion_cross(v1, w1, v2, w2):
    """(v1,w1) x (v2,w2) for spatial motions."""
    return cross(w1, v2) + cross(v1, w2), cross(w1, w2)


def force_cross(v, w, f, n):
    """(v,w) x* (f,n) for a motion acting on a force."""
    return cross(w, f), cross(w, n) + cross(v, f)


# ---------------------------------------------------------------------------
# kinematics
# ---------------------------------------------------------------------------
def forward_kinematics(q):
    """Joint frames in world: oR (...,7,3,3), op (...,7,3); EE frame (R,p).

    Restates pinocchio::forwardKinematics + updateFramePlacements
    (called at crocoddyl_classical.py:201-202)."""
    Rs, ps = [], []
    R = np.broadcast_to(np.eye(3), q.shape[:-1] + (3, 3)).astype(q.dtype)
    p = np.zeros(q.shape[:-1] + (3,), dtype=q.dtype)
    for i in range(NQ):
        p = p + mv(R, JOINT_PLACEMENT_P[i].astype(q.dtype))
        R = mm(mm(R, JOINT_PLACEMENT_R[i].astype(q.dtype)), rotz(q[..., i]))
        Rs.append(R)
        ps.append(p)
    oR = np.stack(Rs, -3)
    op = np.stack(ps, -2)
    R_ee = oR[..., 6, :, :]
    p_ee = op[..., 6, :] + mv(R_ee, EE_OFFSET.astype(q.dtype))
    return oR, op, R_ee, p_ee


def motion_subspace(oR, op):
    """World-frame motion subspace of each revolute-z joint: S_i = (o_i x z_i, z_i)."""
    z = oR[..., :, 2]
    return cross(op, z), z


def link_inertia_world(oR, op):
    """Per-link spatial inertia in the world frame as 6x6 (v,w)->(f,n)."""
    m = LINK_MASS
    c = op + mv(oR, LINK_COM.astype(oR.dtype))  # world COM (...,7,3)
    Ic = mm(mm(oR, LINK_INERTIA.astype(oR.dtype)), np.swapaxes(oR, -1, -2))
    cx = skew(c)
    mI = m[:, None, None] * np.eye(3)
    top = np.concatenate([np.broadcast_to(mI, cx.shape).astype(oR.dtype), -m[:, None, None] * cx], -1)
    bot = np.concatenate([m[:, None, None] * cx, Ic - m[:, None, None] * mm(cx, cx)], -1)
    return np.concatenate([top, bot], -2)


def rnea_full(q, v, a, f_ee=None, gravity=True):
    """Recursive Newton-Euler in the world frame.

    Returns tau and the kinematic quantities the contact/cost models need:
    EE pose, EE LWA velocity (v_p, w) and EE classical acceleration (gravity
    free), evaluated at joint acceleration `a`.

    f_ee: external LINEAR force (world-aligned) applied ON the robot at the EE
    origin (the contact force lambda of the KKT system), i.e. pinocchio's fext.
    Restates pinocchio::rnea (crocoddyl_classical.py:451) with fext as used by
    computeRNEADerivatives inside DifferentialActionModelContactFwdDynamics.
    """
    dt = np.result_type(q, v, a) if f_ee is None else np.result_type(q, v, a, f_ee)
    q = q.astype(dt)
    v = v.astype(dt)
    a = a.astype(dt)
    oR, op, R_ee, p_ee = forward_kinematics(q)
    Sv, Sw = motion_subspace(oR, op)
    I6 = link_inertia_world(oR, op)
    batch = q.shape[:-1]
    vv = np.zeros(batch + (3,), dtype=dt)
    vw = np.zeros(batch + (3,), dtype=dt)
    av = np.zeros(batch + (3,), dtype=dt)
    aw = np.zeros(batch + (3,), dtype=dt)
    g_lin = GRAVITY.astype(dt) if gravity else np.zeros(3, dtype=dt)
    fs = []
    for i in range(NQ):
        sv, sw = Sv[..., i, :], Sw[..., i, :]
        vv = vv + sv * v[..., i : i + 1]
        vw = vw + sw * v[..., i : i + 1]
        cv, cw = motion_cross(vv, vw, sv * v[..., i : i + 1], sw * v[..., i : i + 1])
        av = av + sv * a[..., i : i + 1] + cv
        aw = aw + sw * a[..., i : i + 1] + cw
        Ii = I6[..., i, :, :]
        h = mv(Ii, np.concatenate([vv, vw], -1))
        ia = mv(Ii, np.concatenate([av - g_lin, aw], -1))
        fxv, fxw = force_cross(vv, vw, h[..., :3], h[..., 3:])
        fs.append((ia[..., :3] + fxv, ia[..., 3:] + fxw))
        if i == NQ - 1:
            vv7, vw7, av7, aw7 = vv, vw, av, aw
    if f_ee is not None:
        f_ee = f_ee.astype(dt)
        fl, fa = fs[-1]
        fs[-1] = (fl - f_ee, fa - cross(p_ee, f_ee))
    tau = []
    Fl = np.zeros(batch + (3,), dtype=dt)
    Fa = np.zeros(batch + (3,), dtype=dt)
    for i in reversed(range(NQ)):
        Fl = Fl + fs[i][0]
        Fa = Fa + fs[i][1]
        tau.append(np.sum(Sv[..., i, :] * Fl, -1) + np.sum(Sw[..., i, :] * Fa, -1))
    tau = np.stack(tau[::-1], -1)
    # EE (LOCAL_WORLD_ALIGNED) velocity and classical acceleration of its origin
    v_p = vv7 + cross(vw7, p_ee)
    a_p = av7 + cross(aw7, p_ee) + cross(vw7, v_p)
    return dict(tau=tau, R_ee=R_ee, p_ee=p_ee, v_ee=v_p, w_ee=vw7, acc_ee=a_p, oR=oR, op=op, Sv=Sv, Sw=Sw)


def rnea(q, v, a, f_ee=None):
    return rnea_full(q, v, a, f_ee)["tau"]


def gravity_torque(q):
    """tau_ref = rnea(q0, 0, 0) (crocoddyl_classical.py:447-451)."""
    z = np.zeros_like(q)
    return rnea(q, z, z)


def crba(q):
    """Joint-space inertia M(q) by the composite-rigid-body algorithm (world frame)."""
    oR, op, _, _ = forward_kinematics(q)
    Sv, Sw = motion_subspace(oR, op)
    I6 = link_inertia_world(oR, op)
    Icomp = np.cumsum(I6[..., ::-1, :, :], axis=-3)[..., ::-1, :, :]  # Ic_i = sum_{k>=i} I_k
    S = np.concatenate([Sv, Sw], -1)  # (...,7,6)
    M = np.zeros(q.shape[:-1] + (NQ, NQ), dtype=q.dtype)
    for j in range(NQ):
        F = mv(Icomp[..., j, :, :], S[..., j, :])
        for i in range(j + 1):
            M[..., i, j] = np.sum(S[..., i, :] * F, -1)
            M[..., j, i] = M[..., i, j]
    return M


def frame_jacobian_lwa(q):
    """6x7 LOCAL_WORLD_ALIGNED Jacobian of the EE frame (linear rows first).

    Restates pinocchio::getFrameJacobian(..., LOCAL_WORLD_ALIGNED).
    Column i = (z_i x (p_ee - o_i), z_i)."""
    oR, op, R_ee, p_ee = forward_kinematics(q)
    z = oR[..., :, 2]
    lin = cross(z, p_ee[..., None, :] - op)
    J = np.concatenate([lin, z], -1)  # (...,7,6)
    return np.swapaxes(J, -1, -2), R_ee, p_ee


def ee_site_pose_mj(q):
    """MuJoCo-world pose of ee_site for the MJCF model (used for the calibration
    constants the reference computes in _calibrate_site_*, crocoddyl_classical.py:199-225)."""
    _, _, R_ee, p_ee = forward_kinematics(q)
    return R_MJ_FROM_PIN @ p_ee, R_MJ_FROM_PIN @ R_ee @ R_SITE_FROM_EE


# ---------------------------------------------------------------------------
# SO(3) log and its Jacobian (pinocchio::log3 / Jlog3)
# ---------------------------------------------------------------------------
_TAYLOR3 = np.finfo(float).eps ** (1.0 / 3.0)


def log3(R):
    """pinocchio::log3 for the regime theta < pi - 1e-2 used here."""
    tr = R[..., 0, 0] + R[..., 1, 1] + R[..., 2, 2]
    c = np.clip((tr - 1.0) / 2.0, -1.0, 1.0)
    th = np.arccos(c)
    t = np.where(th > _TAYLOR3, th / np.sin(np.where(th > _TAYLOR3, th, 1.0)), 1.0) / 2.0
    w = np.stack([R[..., 2, 1] - R[..., 1, 2], R[..., 0, 2] - R[..., 2, 0], R[..., 1, 0] - R[..., 0, 1]], -1)
    return t[..., None] * w, th


def jlog3(r, th):
    """pinocchio::Jlog3 : alpha*I + beta*r r^T + 0.5*[r]x."""
    big = th >= _TAYLOR3
    ths = np.where(big, th, 1.0)
    st, ct = np.sin(ths), np.cos(ths)
    st_1mct = st / (1.0 - ct)
    alpha = np.where(big, ths * st_1mct / 2.0, 1.0)
    beta = np.where(big, 1.0 / (ths * ths) - st_1mct / (2.0 * ths), 1.0 / 12.0)
    J = beta[..., None, None] * (r[..., :, None] * r[..., None, :])
    J = J + alpha[..., None, None] * np.eye(3) + 0.5 * skew(r)
    return J


def complex_step_jacobian(f, x, h=1e-30):
    """d f / d x by complex step.  f maps (...,n)->(...,m); returns (...,m,n)."""
    n = x.shape[-1]
    E = np.eye(n)
    X = x[None, ...].astype(np.result_type(x.dtype, np.complex128)) + 1j * h * E.reshape((n,) + (1,) * (x.ndim - 1) + (n,))
    F = f(X)
    J = np.imag(F) / h  # (n, ..., m)
    return np.moveaxis(J, 0, -1)
