"""Franka Panda 7-DoF model data (product side).

Transcribed from /root/reference/assets/scenes/panda_robot.xml:98-199 (link
placements, masses, COMs, full inertias, joint ranges, neutral keyframe
:233).  This replaces example_robot_data.load("panda") +
pin.buildReducedModel (crocoddyl_classical.py:137-145, 189-197), which are not
available offline: armature 0, no hand payload.
The Pinocchio world is the MJCF link0 frame; R_MJ_FROM_PIN = diag(-1,-1,1)
(crocoddyl_classical.py:151).
"""
from __future__ import annotations

import numpy as np

# rotations of the MJCF body quats "1 -1 0 0" (-90 deg about x) and "1 1 0 0" (+90 deg about x)
_RX_M90 = np.array([[1.0, 0.0, 0.0], [0.0, 0.0, 1.0], [0.0, -1.0, 0.0]])
_RX_P90 = np.array([[1.0, 0.0, 0.0], [0.0, 0.0, -1.0], [0.0, 1.0, 0.0]])
_I3 = np.eye(3)

JOINT_R = np.stack([_I3, _RX_M90, _RX_P90, _RX_P90, _RX_M90, _RX_P90, _RX_P90])
JOINT_P = np.array(
    [
        [0.0, 0.0, 0.333],
        [0.0, 0.0, 0.0],
        [0.0, -0.316, 0.0],
        [0.0825, 0.0, 0.0],
        [-0.0825, 0.384, 0.0],
        [0.0, 0.0, 0.0],
        [0.088, 0.0, 0.0],
    ]
)
MASS = np.array([4.970684, 0.646926, 3.228604, 3.587895, 1.225946, 1.666555, 0.735522])
COM = np.array(
    [
        [0.003875, 0.002081, -0.04762],
        [-0.003141, -0.02872, 0.003495],
        [0.027518, 0.039252, -0.066502],
        [-0.05317, 0.104419, 0.027454],
        [-0.011953, 0.041065, -0.038437],
        [0.060149, -0.014117, -0.010517],
        [0.010517, -0.004252, 0.061597],
    ]
)
# MJCF fullinertia = (Ixx, Iyy, Izz, Ixy, Ixz, Iyz), about the COM, link frame
_FULL = np.array(
    [
        [0.70337, 0.70661, 0.0091170, -0.00013900, 0.0067720, 0.019169],
        [0.0079620, 0.028110, 0.025995, -0.003925, 0.010254, 0.000704],
        [0.037242, 0.036155, 0.01083, -0.004761, -0.011396, -0.012805],
        [0.025853, 0.019552, 0.028323, 0.007796, -0.001332, 0.008641],
        [0.035549, 0.029474, 0.008627, -0.002117, -0.004037, 0.000229],
        [0.001964, 0.004354, 0.005433, 0.000109, -0.001158, 0.000341],
        [0.012516, 0.010027, 0.004815, -0.000428, -0.001196, -0.000741],
    ]
)
INERTIA = np.stack(
    [np.array([[a, d, e], [d, b, f], [e, f, c]]) for (a, b, c, d, e, f) in _FULL]
)
EE_P = np.array([0.0, 0.0, 0.107])  # panda_link8 / tool body (:189)
EE_R = np.eye(3)
GRAVITY = np.array([0.0, 0.0, -9.81])

Q_LOWER = np.array([-2.8973, -1.7628, -2.8973, -3.0718, -2.8973, -0.0175, -2.8973])
Q_UPPER = np.array([2.8973, 1.7628, 2.8973, -0.0698, 2.8973, 3.7525, 2.8973])
Q_NEUTRAL = np.array([0.0, -0.758, 0.0, -2.22, 0.0, 1.43, 0.0])
TAU_LIMITS = np.array([87.0, 87.0, 87.0, 87.0, 12.0, 12.0, 12.0])  # crocoddyl_classical.py:87

R_MJ_FROM_PIN = np.diag([-1.0, -1.0, 1.0])
_c, _s = np.cos(np.deg2rad(135.0)), np.sin(np.deg2rad(135.0))
R_SITE_FROM_EE = np.array([[_c, -_s, 0.0], [_s, _c, 0.0], [0.0, 0.0, 1.0]])  # tool quat (:189)


def vertical_down_rotation_mj() -> np.ndarray:
    """_make_vertical_down_rotation_mj (crocoddyl_classical.py:241-248)."""
    z = np.array([0.0, 0.0, -1.0])
    x = np.array([1.0, 0.0, 0.0])
    y = np.cross(z, x)
    y /= np.linalg.norm(y) + 1e-12
    x = np.cross(y, z)
    x /= np.linalg.norm(x) + 1e-12
    return np.column_stack([x, y, z])


def rot_mj_to_pin(R_mj_site, R_site_from_pin_ee=R_SITE_FROM_EE) -> np.ndarray:
    """_rot_mj_to_pin (crocoddyl_classical.py:257-258)."""
    return R_MJ_FROM_PIN.T @ np.asarray(R_mj_site, float) @ np.asarray(R_site_from_pin_ee).T


def default_R_des() -> np.ndarray:
    """R_des = _rot_mj_to_pin(vertical down) (crocoddyl_classical.py:157)."""
    return rot_mj_to_pin(vertical_down_rotation_mj())
