"""The pybind11 module over the C ABI.

`ffddp.native.Solver(cfg, max_batch, device)` is crocoddyl.SolverBoxFDDP for a
batch (crocoddyl_classical.py:442-445), built as a C++ extension
(`csrc/ffddp_pybind.cpp` -> `lib/_ffddp_native*.so`, linking lib/libffddp.so).
`solve(batch, maxiter, is_feasible)` has BatchedBoxFDDP.solve's semantics on
host arrays and sets the same read-backs (xs, us, K, cost, iter, ok, fn_pred,
stats); the extension releases the GIL while the device solves.  The ctypes
class (ffddp.solver.BatchedBoxFDDP) remains the full surface (device-resident
solves, tracing, solver properties, profiling); both drive the same library.
"""
from __future__ import annotations

import importlib.machinery
import importlib.util
import sysconfig
from pathlib import Path

import numpy as np

from . import _abi
from .config import OcpConfig

NATIVE_PATH = _abi.LIB_PATH.parent / ("_ffddp_native" + sysconfig.get_config_var("EXT_SUFFIX"))
_mod = None


def load():
    """Import the extension (raises when it is not built; no fallback)."""
    global _mod
    if _mod is not None:
        return _mod
    _abi.load()  # torch first, then the one libffddp.so the extension links
    if not Path(NATIVE_PATH).exists():
        raise ImportError(f"ffddp: pybind11 module not found at {NATIVE_PATH}; run __graft_entry__.build()")
    loader = importlib.machinery.ExtensionFileLoader("_ffddp_native", str(NATIVE_PATH))
    spec = importlib.util.spec_from_file_location("_ffddp_native", str(NATIVE_PATH), loader=loader)
    mod = importlib.util.module_from_spec(spec)
    loader.exec_module(mod)
    _mod = mod
    return mod


class Solver:
    """Batched SolverBoxFDDP through the pybind11 module."""

    def __init__(self, cfg: OcpConfig, max_batch: int, device: int = 0):
        m = load()
        self.cfg = cfg
        self._s = m.Solver(bytes(_abi.robot_struct()), bytes(cfg.to_struct()), int(device), int(max_batch))
        self.N, self.nx, self.max_batch = self._s.N, self._s.nx, self._s.max_batch
        self.xs = self.us = self.K = self.cost = self.iter = self.ok = self.fn_pred = self.stats = None

    def solve(self, batch, maxiter: int = 10, is_feasible: bool = False, xs_init=None, us_init=None):
        """batch: workload.Batch (x0, node_ref, inst_ref, surface, xs_init,
        us_init).  Returns ok (B,) bool."""
        out = self._s.solve(
            np.asarray(batch.x0, np.float64), np.asarray(batch.node_ref, np.float64),
            np.asarray(batch.inst_ref, np.float64), np.asarray(batch.surface, np.uint8),
            np.asarray(batch.xs_init if xs_init is None else xs_init, np.float64),
            np.asarray(batch.us_init if us_init is None else us_init, np.float64), int(maxiter), bool(is_feasible))
        self.xs, self.us, self.K, self.cost = out["xs"], out["us"], out["K"], out["cost"]
        self.iter, self.fn_pred, self.stats = out["iter"], out["fn_pred"], out["stats"]
        self.ok = out["ok"].astype(bool)
        return self.ok

    def close(self):
        if getattr(self, "_s", None) is not None:
            self._s.close()
            self._s = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
