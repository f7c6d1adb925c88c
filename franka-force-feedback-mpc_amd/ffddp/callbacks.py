"""Solver callbacks: the crocoddyl.CallbackVerbose the reference installs with
`solver.setCallbacks([crocoddyl.CallbackVerbose()])` when cfg.verbose is set
(src/mpc/crocoddyl_classical.py:352-353, 360-361; crocoddyl_force_feedback.py
588-599).

The batched solver runs every iteration on the device, so the per-iteration
values Crocoddyl's callback reads from the solver object (iter, cost, stop,
d[1], preg, dreg, steplength, ffeas) are recorded there (include/ffddp.h,
ffddp_trace_*) and the callback is replayed after the solve, one line per
iteration of the selected instance, in CallbackVerbose's column layout
(Crocoddyl 2.x, level _1: header every 10 iterations, scientific values with
a sign column, step length fixed to 4 decimals; gfeas / hfeas are 0 for the
unconstrained FDDP problem).  The exact spacing of the real callback is not
checkable here (Crocoddyl is absent): only the fields are the contract.
"""
from __future__ import annotations

import math
import sys

import numpy as np

from . import _abi

_F = {k: i for i, k in enumerate(_abi.TRACE_FIELDS)}


def _center(s: str, width: int) -> str:
    pad = max(width - len(s), 0)
    return " " * (pad // 2) + s + " " * (pad - pad // 2)


class CallbackVerbose:
    """crocoddyl.CallbackVerbose(level=1, precision=3) for one instance of the batch."""

    def __init__(self, level: int = 1, precision: int = 3, instance: int = 0, stream=None):
        self.level = int(level)
        self.precision = int(precision)
        self.instance = int(instance)
        self.stream = stream
        self.lines: list[str] = []  # everything printed, for tests / logs

    def header(self) -> str:
        w = self.precision + 7
        cols = ["cost", "stop", "grad", "preg", "dreg"]
        h = "iter " + " ".join(_center(c, w) for c in cols) + " " + _center("step", 6)
        h += " " + " ".join(_center(c, w) for c in ("||ffeas||", "||gfeas||", "||hfeas||"))
        if self.level >= 2:
            h += " " + " ".join(_center(c, w) for c in ("dV-exp", "dV"))
        return h

    def _sci(self, v: float) -> str:
        s = f"{v:.{self.precision}e}" if math.isfinite(v) else f"{v}"
        return s if s.startswith("-") else " " + s

    def format_row(self, row) -> str:
        r = np.asarray(row, float)
        parts = [f"{int(r[_F['iter']]):4d} "]
        for k in ("cost", "stop", "grad", "preg", "dreg"):
            parts.append(self._sci(r[_F[k]]))
        parts.append(f" {r[_F['step']]:.4f}")
        parts.append(self._sci(r[_F["ffeas"]]))
        parts.append(self._sci(0.0))
        parts.append(self._sci(0.0))
        if self.level >= 2:
            parts.append(self._sci(r[_F["dV_exp"]]))
            parts.append(self._sci(r[_F["dV"]]))
        return " ".join(parts)

    def format(self, trace_rows) -> list[str]:
        """Lines for one instance's [max_iters][TRACE_W] records (NaN rows skipped)."""
        out = []
        for row in np.asarray(trace_rows, float):
            if not math.isfinite(row[_F["iter"]]):
                continue
            if int(row[_F["iter"]]) % 10 == 0:
                out.append(self.header())
            out.append(self.format_row(row))
        return out

    def __call__(self, solver, trace: np.ndarray):
        if self.instance >= trace.shape[0]:
            return
        lines = self.format(trace[self.instance])
        self.lines.extend(lines)
        stream = self.stream if self.stream is not None else sys.stdout
        for ln in lines:
            print(ln, file=stream)
