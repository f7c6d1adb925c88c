"""Shared test helpers: identical inputs for the HIP path and the oracle."""
from __future__ import annotations

import numpy as np

from ffddp import _abi, robot as R, workload
from ffddp.config import OcpConfig, classical_preset, ff_preset
from oracle import fddp, ocp


def ee_start_mj():
    return R.R_MJ_FROM_PIN @ _abi.frame_placement(R.Q_NEUTRAL)[1]


def product_cfg(variant: str, horizon: int, contact_model: str = "normal_1d") -> OcpConfig:
    return ff_preset(horizon, contact_model) if variant == "ff" else classical_preset(horizon, contact_model)


def oracle_cfg(c: OcpConfig) -> ocp.OCPConfig:
    """Same parameter values, handed to the independent restatement."""
    o = ocp.OCPConfig()
    for f in o.__dataclass_fields__:
        if f == "ff_alpha":
            o.ff_alpha = c.ff_alpha
        elif f == "use_box_fddp":
            continue
        elif hasattr(c, f):
            setattr(o, f, getattr(c, f))
    o.variant = c.variant
    return o


def make_batch(variant, B, N, seed, surface=None, regime="tracking"):
    return workload.make_batch(
        B, N, variant, _abi.gravity_torque, ee_start_mj(), seed=seed, surface_override=surface,
        regime=regime, fk=_abi.frame_placement,
    )


def oracle_problem(batch, i, N) -> ocp.Problem:
    return ocp.Problem(
        batch.x0[i], batch.node_ref[i, :, :3], batch.node_ref[i, :, 3:], batch.inst_ref[i, :14],
        batch.inst_ref[i, 14:], bool(batch.surface[i]),
    )


def oracle_solve(cfg: OcpConfig, batch, i, maxiter=10, box=True):
    s = fddp.SolverBoxFDDP(oracle_cfg(cfg), oracle_problem(batch, i, cfg.horizon), box=box)
    ok = s.solve(batch.xs_init[i], batch.us_init[i], maxiter, False)
    return ok, s


def rel_err(a, b):
    a, b = np.asarray(a, float), np.asarray(b, float)
    return float(np.max(np.abs(a - b)) / max(1.0, float(np.max(np.abs(b)))))


def log_parity(case: str, **fields):
    """Append one JSON line with the observed errors of a parity case to
    $FFDDP_PARITY_LOG (when set), so the tolerances can be set from data."""
    import json
    import os

    path = os.environ.get("FFDDP_PARITY_LOG")
    if not path:
        return
    rec = {"case": case}
    for k, v in fields.items():
        rec[k] = v.item() if hasattr(v, "item") else v
    with open(path, "a") as f:
        f.write(json.dumps(rec) + "\n")
