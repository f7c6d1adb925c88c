"""ctypes binding of include/ffddp.h (the drop-in C-ABI).

The library is built in-tree (franka-force-feedback-mpc_amd/lib/libffddp.so)
by __graft_entry__.build() / `make -C franka-force-feedback-mpc_amd/csrc`.
There is no CPU fallback: if the library is missing, import fails loudly.
"""
from __future__ import annotations

import ctypes as C
import os
import weakref
from pathlib import Path

import numpy as np

from . import robot as R

LIB_PATH = Path(__file__).resolve().parents[1] / "lib" / "libffddp.so"

FFDDP_CLASSICAL = 0
FFDDP_FORCE_FEEDBACK = 1

SYMBOLS = (
    "ffddp_create",
    "ffddp_destroy",
    "ffddp_last_error",
    "ffddp_solve_batch",
    "ffddp_solve_batch_dev",
    "ffddp_calc_diff",
    "ffddp_frame_placement",
    "ffddp_gravity_torque",
    "ffddp_gravity_torque_dev",
    "ffddp_build_problem_dev",
    "ffddp_profile_enable",
    "ffddp_profile_read",
    "ffddp_plant_create",
    "ffddp_plant_destroy",
    "ffddp_plant_step",
    "ffddp_plant_step_dev",
    "ffddp_get_solver_params",
    "ffddp_set_solver_params",
    "ffddp_trace_enable",
    "ffddp_trace_read",
    "ffddp_host_alloc",
    "ffddp_host_free",
    "ffddp_plan_create",
    "ffddp_plan_run",
    "ffddp_plan_destroy",
)
PLANT_OBS = 69
NSTATS = 10
TRACE_W = 10
TRACE_FIELDS = ("iter", "cost", "stop", "grad", "preg", "dreg", "step", "ffeas", "dV", "dV_exp")
NEGSTEP_CROCODDYL = 0
NEGSTEP_BOUNDED_RISE = 1
KERNEL_CLASSES = ("init", "node", "backward", "forward", "accept", "commit", "finalize", "forward2")


class Robot(C.Structure):
    _fields_ = [
        ("joint_R", C.c_double * 9 * 7),
        ("joint_p", C.c_double * 3 * 7),
        ("mass", C.c_double * 7),
        ("com", C.c_double * 3 * 7),
        ("inertia", C.c_double * 9 * 7),
        ("ee_R", C.c_double * 9),
        ("ee_p", C.c_double * 3),
        ("gravity", C.c_double * 3),
    ]


class OcpConfig(C.Structure):
    _fields_ = [
        ("variant", C.c_int32),
        ("horizon", C.c_int32),
        ("nc", C.c_int32),
        ("use_box", C.c_int32),
        ("dt", C.c_double),
        ("z_press", C.c_double),
        ("w_ee_pos", C.c_double),
        ("w_ee_ori", C.c_double),
        ("ori_weights", C.c_double * 3),
        ("w_posture", C.c_double),
        ("w_v", C.c_double),
        ("v_damp_weights", C.c_double * 7),
        ("w_tau", C.c_double),
        ("w_tau_soft_limits", C.c_double),
        ("tau_soft_limit_margin", C.c_double),
        ("w_q_soft_limits", C.c_double),
        ("q_soft_limit_margin", C.c_double),
        ("q_lower", C.c_double * 7),
        ("q_upper", C.c_double * 7),
        ("w_tangent_pos", C.c_double),
        ("w_tangent_vel", C.c_double),
        ("w_plane_z", C.c_double),
        ("w_vz", C.c_double),
        ("w_unilateral", C.c_double),
        ("friction_margin", C.c_double),
        ("w_fn", C.c_double),
        ("fn_des", C.c_double),
        ("w_wdamp", C.c_double),
        ("w_wdamp_weights", C.c_double * 3),
        ("contact_gains", C.c_double * 2),
        ("contact_inv_damping", C.c_double),
        ("tau_limits", C.c_double * 7),
        ("R_des", C.c_double * 9),
        ("ff_alpha", C.c_double),
        ("w_w", C.c_double),
        ("w_w_soft_limits", C.c_double),
        ("w_y", C.c_double),
        ("y_weights", C.c_double * 21),
        ("use_inner_state_reg", C.c_int32),
        ("use_inner_tau_reg", C.c_int32),
        ("w_friction_cone", C.c_double),
        ("mu", C.c_double),
    ]


class PlanIO(C.Structure):
    """ffddp_plan_io (include/ffddp.h): the plan's page-locked inputs / outputs."""

    _fields_ = [(n, C.c_void_p) for n in ("x0", "node_ref", "inst_ref", "surface", "xs_init", "us_init", "xs", "us",
                                          "K", "cost", "iters", "ok", "fn_pred", "stats")]


class SolverParams(C.Structure):
    """ffddp_solver_params: crocoddyl.SolverBoxFDDP / SolverFDDP properties."""

    _fields_ = [
        ("th_stop", C.c_double),
        ("th_grad", C.c_double),
        ("th_acceptstep", C.c_double),
        ("th_acceptnegstep", C.c_double),
        ("th_stepdec", C.c_double),
        ("th_stepinc", C.c_double),
        ("reg_min", C.c_double),
        ("reg_max", C.c_double),
        ("reg_incfactor", C.c_double),
        ("reg_decfactor", C.c_double),
        ("neg_step_rule", C.c_int32),
        ("reserved", C.c_int32),
    ]


def solver_params(use_box: bool = True, **overrides) -> SolverParams:
    """SolverParams with the SolverBoxFDDP (use_box) / SolverFDDP defaults the
    library's handles start from (ffddp_consts.hpp fill_consts), then `overrides`."""
    p = SolverParams()
    vals = dict(th_stop=5e-5 if use_box else 1e-9, th_grad=1e-12, th_acceptstep=0.1, th_acceptnegstep=2.0,
                th_stepdec=0.5, th_stepinc=0.01, reg_min=1e-9, reg_max=1e9, reg_incfactor=10.0, reg_decfactor=10.0,
                neg_step_rule=NEGSTEP_CROCODDYL)
    vals.update(overrides)
    for k, v in vals.items():
        setattr(p, k, v)
    return p


class Task(C.Structure):
    """ffddp_task: the device problem builder's task (trajectories.py:8-93,
    run_classical.py:221-264, crocoddyl_classical.py:250-258, 447-466)."""

    _fields_ = [
        ("center", C.c_double * 3),
        ("radius", C.c_double),
        ("omega", C.c_double),
        ("z_contact", C.c_double),
        ("t_approach", C.c_double),
        ("t_pre", C.c_double),
        ("z_pre", C.c_double),
        ("t_hold", C.c_double),
        ("ee_start", C.c_double * 3),
        ("has_ee_start", C.c_int32),
        ("has_z_pre", C.c_int32),
        ("p_site_minus_frame", C.c_double * 3),
        ("q_nom", C.c_double * 7),
        ("posture_mode", C.c_int32),
        ("torque_mode", C.c_int32),
    ]


class PlantParams(C.Structure):
    """ffddp_plant_params: the closed-loop plant stand-in (ffddp_plant.hpp)."""

    _fields_ = [
        ("timestep", C.c_double),
        ("n_substeps", C.c_int32),
        ("armature", C.c_double * 7),
        ("damping", C.c_double * 7),
        ("r_tool", C.c_double),
        ("margin", C.c_double),
        ("solref", C.c_double * 2),
        ("solimp", C.c_double * 5),
        ("site_R", C.c_double * 2),
    ]


POSTURE_MODES = {"x0": 0, "q_nom": 1}
TORQUE_MODES = {"gravity_x0": 0, "gravity_q_nom": 1, "zero": 2}


def make_task(
    center,
    radius: float,
    omega: float,
    z_contact: float,
    t_approach: float = 2.0,
    ee_start=None,
    z_pre=None,
    t_pre: float = 0.0,
    t_hold: float = 0.0,
    p_site_minus_frame=(0.0, 0.0, 0.0),
    q_nom=None,
    posture_ref_mode: str = "q_nom",
    torque_ref_mode: str = "gravity_x0",
) -> Task:
    """Task with make_approach_then_circle's arguments (trajectories.py:8-17),
    the benchmark hold t_hold (run_classical.py:256-264: 0.2 s) and the
    controller's reference modes (crocoddyl_classical.py:447-466)."""
    t = Task()
    _fill(t.center, center)
    t.radius, t.omega, t.z_contact = float(radius), float(omega), float(z_contact)
    t.t_approach, t.t_pre, t.t_hold = float(t_approach), float(t_pre), float(t_hold)
    t.has_ee_start = int(ee_start is not None)
    if ee_start is not None:
        _fill(t.ee_start, ee_start)
    t.has_z_pre = int(z_pre is not None)
    t.z_pre = float(z_pre) if z_pre is not None else 0.0
    _fill(t.p_site_minus_frame, p_site_minus_frame)
    _fill(t.q_nom, R.Q_NEUTRAL if q_nom is None else q_nom)
    if posture_ref_mode not in POSTURE_MODES or torque_ref_mode not in TORQUE_MODES:
        raise ValueError(f"unknown reference mode {posture_ref_mode!r} / {torque_ref_mode!r}")
    t.posture_mode = POSTURE_MODES[posture_ref_mode]
    t.torque_mode = TORQUE_MODES[torque_ref_mode]
    return t


def _fill(arr, values):
    flat = np.asarray(values, dtype=float).reshape(-1)
    buf = (C.c_double * flat.size).from_buffer(arr)
    for i, v in enumerate(flat):
        buf[i] = float(v)


def make_robot() -> Robot:
    rb = Robot()
    _fill(rb.joint_R, R.JOINT_R)
    _fill(rb.joint_p, R.JOINT_P)
    _fill(rb.mass, R.MASS)
    _fill(rb.com, R.COM)
    _fill(rb.inertia, R.INERTIA)
    _fill(rb.ee_R, R.EE_R)
    _fill(rb.ee_p, R.EE_P)
    _fill(rb.gravity, R.GRAVITY)
    return rb


_lib = None


def load() -> C.CDLL:
    """Load libffddp.so.  Raises (never falls back) when it is missing."""
    global _lib
    if _lib is not None:
        return _lib
    # One HIP runtime per process: torch wheels ship their own libamdhip64.so.7
    # and load it by path; if ours (/opt/rocm) were loaded first, torch would
    # bring a second runtime and fail to initialise.  Importing torch first makes
    # the dynamic loader bind our NEEDED libamdhip64.so.7 to the torch copy.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    path = Path(os.environ.get("FFDDP_LIB", str(LIB_PATH)))
    if not path.exists():
        raise ImportError(
            f"ffddp: HIP library not found at {path}; build it with "
            "`python -c 'import __graft_entry__ as g; g.build()'` (no CPU fallback exists)"
        )
    lib = C.CDLL(str(path))
    dp, ip, up, vp = C.POINTER(C.c_double), C.POINTER(C.c_int32), C.POINTER(C.c_uint8), C.c_void_p
    lib.ffddp_create.argtypes = [C.POINTER(Robot), C.POINTER(OcpConfig), C.c_int, C.c_int, C.POINTER(C.c_void_p)]
    lib.ffddp_create.restype = C.c_int
    lib.ffddp_destroy.argtypes = [C.c_void_p]
    lib.ffddp_destroy.restype = None
    lib.ffddp_last_error.argtypes = [C.c_void_p]
    lib.ffddp_last_error.restype = C.c_char_p
    solve_args = [C.c_void_p, C.c_int, dp, dp, dp, up, dp, dp, C.c_int, C.c_int, dp, dp, dp, dp, ip, up, dp, ip]
    lib.ffddp_solve_batch.argtypes = solve_args
    lib.ffddp_solve_batch.restype = C.c_int
    dev_args = [C.c_void_p, C.c_int] + [vp] * 6 + [C.c_int, C.c_int] + [vp] * 8 + [vp]
    lib.ffddp_solve_batch_dev.argtypes = dev_args
    lib.ffddp_solve_batch_dev.restype = C.c_int
    lib.ffddp_calc_diff.argtypes = [C.c_void_p, C.c_int, dp, dp, dp, up, dp, dp] + [dp] * 10
    lib.ffddp_calc_diff.restype = C.c_int
    lib.ffddp_frame_placement.argtypes = [C.POINTER(Robot), dp, dp, dp]
    lib.ffddp_frame_placement.restype = C.c_int
    lib.ffddp_gravity_torque.argtypes = [C.POINTER(Robot), C.c_int, dp, dp]
    lib.ffddp_gravity_torque.restype = C.c_int
    lib.ffddp_gravity_torque_dev.argtypes = [C.c_void_p, C.c_int, vp, vp, vp]
    lib.ffddp_gravity_torque_dev.restype = C.c_int
    lib.ffddp_build_problem_dev.argtypes = [C.c_void_p, C.c_int, C.POINTER(Task)] + [vp] * 6
    lib.ffddp_build_problem_dev.restype = C.c_int
    lib.ffddp_profile_enable.argtypes = [C.c_void_p, C.c_int]
    lib.ffddp_profile_enable.restype = C.c_int
    lib.ffddp_profile_read.argtypes = [C.c_void_p, dp, C.POINTER(C.c_int64), C.c_int]
    lib.ffddp_profile_read.restype = C.c_int
    lib.ffddp_plant_create.argtypes = [C.POINTER(Robot), C.POINTER(PlantParams), C.c_int, C.c_int,
                                       C.POINTER(C.c_void_p)]
    lib.ffddp_plant_create.restype = C.c_int
    lib.ffddp_plant_destroy.argtypes = [C.c_void_p]
    lib.ffddp_plant_destroy.restype = None
    lib.ffddp_plant_step.argtypes = [C.c_void_p, C.c_int, dp, dp, dp, dp, C.c_int, dp]
    lib.ffddp_plant_step.restype = C.c_int
    lib.ffddp_plant_step_dev.argtypes = [C.c_void_p, C.c_int] + [vp] * 4 + [C.c_int, vp, vp, vp]
    lib.ffddp_plant_step_dev.restype = C.c_int
    lib.ffddp_get_solver_params.argtypes = [C.c_void_p, C.POINTER(SolverParams)]
    lib.ffddp_get_solver_params.restype = C.c_int
    lib.ffddp_set_solver_params.argtypes = [C.c_void_p, C.POINTER(SolverParams)]
    lib.ffddp_set_solver_params.restype = C.c_int
    lib.ffddp_trace_enable.argtypes = [C.c_void_p, C.c_int]
    lib.ffddp_trace_enable.restype = C.c_int
    lib.ffddp_trace_read.argtypes = [C.c_void_p, C.c_int, dp]
    lib.ffddp_trace_read.restype = C.c_int
    lib.ffddp_host_alloc.argtypes = [C.c_size_t, C.POINTER(C.c_void_p)]
    lib.ffddp_host_alloc.restype = C.c_int
    lib.ffddp_host_free.argtypes = [C.c_void_p]
    lib.ffddp_host_free.restype = C.c_int
    lib.ffddp_plan_create.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_int, C.POINTER(C.c_void_p), C.POINTER(PlanIO)]
    lib.ffddp_plan_create.restype = C.c_int
    lib.ffddp_plan_run.argtypes = [C.c_void_p]
    lib.ffddp_plan_run.restype = C.c_int
    lib.ffddp_plan_destroy.argtypes = [C.c_void_p]
    lib.ffddp_plan_destroy.restype = None
    _lib = lib
    return lib


def dptr(a: np.ndarray):
    assert a.dtype == np.float64 and a.flags["C_CONTIGUOUS"]
    return a.ctypes.data_as(C.POINTER(C.c_double))


def iptr(a: np.ndarray):
    assert a.dtype == np.int32 and a.flags["C_CONTIGUOUS"]
    return a.ctypes.data_as(C.POINTER(C.c_int32))


def _pinned_buffer(nbytes: int):
    """One ffddp_host_alloc allocation as a ctypes buffer, freed (weakref
    finalizer, no reference cycle) as soon as the buffer -- and so the last
    numpy array viewing it -- is gone."""
    lib = load()
    n = max(int(nbytes), 1)
    p = C.c_void_p()
    rc = lib.ffddp_host_alloc(n, C.byref(p))
    if rc != 0:
        raise MemoryError(f"ffddp_host_alloc({nbytes}) failed ({rc})")
    buf = (C.c_char * n).from_address(p.value)
    weakref.finalize(buf, lib.ffddp_host_free, C.c_void_p(p.value))
    return buf


def pinned_arrays(specs) -> dict:
    """numpy arrays in one page-locked host allocation (ffddp_host_alloc):
    ffddp_solve_batch copies such arrays by DMA on the slice streams instead
    of through its staging buffer.  specs: {name: (shape, dtype)}."""
    offs, tot = {}, 0
    for k, (shape, dt) in specs.items():
        offs[k] = tot
        tot += (int(np.prod(shape)) * np.dtype(dt).itemsize + 255) // 256 * 256
    buf = _pinned_buffer(tot)
    return {k: np.frombuffer(buf, dtype=dt, count=int(np.prod(shape)), offset=offs[k]).reshape(shape)
            for k, (shape, dt) in specs.items()}


def uptr(a: np.ndarray):
    assert a.dtype == np.uint8 and a.flags["C_CONTIGUOUS"]
    return a.ctypes.data_as(C.POINTER(C.c_uint8))


_ROBOT = None


def robot_struct() -> Robot:
    global _ROBOT
    if _ROBOT is None:
        _ROBOT = make_robot()
    return _ROBOT


def frame_placement(q) -> tuple[np.ndarray, np.ndarray]:
    """EE placement (R, p) on the host via the library's model code."""
    lib = load()
    q = np.ascontiguousarray(q, dtype=np.float64).reshape(7)
    Rm = np.zeros(9)
    p = np.zeros(3)
    rc = lib.ffddp_frame_placement(C.byref(robot_struct()), dptr(q), dptr(Rm), dptr(p))
    if rc:
        raise RuntimeError(f"ffddp_frame_placement failed ({rc})")
    return Rm.reshape(3, 3), p


def gravity_torque(q) -> np.ndarray:
    """rnea(q, 0, 0) for a batch (B,7) on the host via the library's model code."""
    lib = load()
    q = np.ascontiguousarray(np.atleast_2d(q), dtype=np.float64)
    out = np.zeros_like(q)
    rc = lib.ffddp_gravity_torque(C.byref(robot_struct()), q.shape[0], dptr(q), dptr(out))
    if rc:
        raise RuntimeError(f"ffddp_gravity_torque failed ({rc})")
    return out
