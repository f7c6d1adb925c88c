"""ORACLE-SIDE CPU BASELINE — test / benchmark infrastructure only.

ctypes binding of oracle/cpu/libffddp_cpu.so (oracle/cpu/ffddp_cpu.cpp): a
scalar C++ BoxFDDP over the same OCP, OpenMP over instances on the host
cores — the CPU path the reference runs (crocoddyl.SolverBoxFDDP.solve at
src/mpc/crocoddyl_classical.py:367, 442-445), restated because Crocoddyl is
absent (SURVEY.md §8(c), §8(d) "CPU baseline" item 1).  Same arguments and
outputs as ffddp_solve_batch (include/ffddp.h).  Checked against the numpy
oracle by tests/test_cpu_baseline.py; timed by bench.py's cpu_baseline leg.
"""
from __future__ import annotations

import ctypes as C
from pathlib import Path

import numpy as np

LIB = Path(__file__).resolve().parent / "cpu" / "libffddp_cpu.so"
NSTATS = 10
_lib = None


def load():
    global _lib
    if _lib is None:
        if not LIB.exists():
            raise ImportError(f"{LIB} missing: build it with `make -C oracle/cpu` (or __graft_entry__.build())")
        lib = C.CDLL(str(LIB))
        dp, ip, up, vp = C.POINTER(C.c_double), C.POINTER(C.c_int32), C.POINTER(C.c_uint8), C.c_void_p
        lib.ffddp_cpu_solve_batch.argtypes = [vp, vp, C.c_int, dp, dp, dp, up, dp, dp, C.c_int, C.c_int,
                                              dp, dp, dp, dp, ip, up, ip, vp, C.c_int]
        lib.ffddp_cpu_solve_batch.restype = C.c_int
        lib.ffddp_cpu_max_threads.restype = C.c_int
        _lib = lib
    return _lib


def solve_batch(robot_struct, cfg_struct, batch, maxiter=10, is_feasible=False, nthreads=0, xs_init=None,
                us_init=None, solver_params=None):
    """robot_struct / cfg_struct: ctypes ffddp_robot / ffddp_ocp_config
    (ffddp._abi.Robot / OcpConfig); batch: workload.Batch; solver_params: an
    _abi.SolverParams (None = the defaults).  Returns a dict with xs, us, K,
    cost, iter, ok, stats (numpy)."""
    lib = load()
    B = int(batch.x0.shape[0])
    N = int(cfg_struct.horizon)
    nx = 21 if cfg_struct.variant == 1 else 14
    f = lambda a, shape: np.ascontiguousarray(np.asarray(a, np.float64).reshape(shape))
    x0 = f(batch.x0, (B, nx))
    nref = f(batch.node_ref, (B, N + 1, 6))
    iref = f(batch.inst_ref, (B, 21))
    surf = np.ascontiguousarray(np.asarray(batch.surface, np.uint8).reshape(B))
    xsi = f(batch.xs_init if xs_init is None else xs_init, (B, N + 1, nx))
    usi = f(batch.us_init if us_init is None else us_init, (B, N, 7))
    out = dict(xs=np.zeros((B, N + 1, nx)), us=np.zeros((B, N, 7)), K=np.zeros((B, N, 7, nx)), cost=np.zeros(B),
               iter=np.zeros(B, np.int32), ok=np.zeros(B, np.uint8), stats=np.zeros((B, NSTATS), np.int32))
    d = lambda a: a.ctypes.data_as(C.POINTER(C.c_double))
    i32 = lambda a: a.ctypes.data_as(C.POINTER(C.c_int32))
    u8 = lambda a: a.ctypes.data_as(C.POINTER(C.c_uint8))
    rc = lib.ffddp_cpu_solve_batch(C.byref(robot_struct), C.byref(cfg_struct), B, d(x0), d(nref), d(iref), u8(surf),
                                   d(xsi), d(usi), int(maxiter), int(bool(is_feasible)), d(out["xs"]), d(out["us"]),
                                   d(out["K"]), d(out["cost"]), i32(out["iter"]), u8(out["ok"]), i32(out["stats"]),
                                   C.byref(solver_params) if solver_params is not None else None, int(nthreads))
    if rc != 0:
        raise RuntimeError(f"ffddp_cpu_solve_batch failed ({rc})")
    out["ok"] = out["ok"].astype(bool)
    return out


def max_threads() -> int:
    return int(load().ffddp_cpu_max_threads())
