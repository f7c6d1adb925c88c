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


def elem_err(a, b):
    """Largest element-wise error |a - b| / (1 + |b|): unlike rel_err, small
    entries of a block with large ones (K: 1e-3 .. 1e3) keep their own scale."""
    a, b = np.asarray(a, float), np.asarray(b, float)
    return float(np.max(np.abs(a - b) / (1.0 + np.abs(b)))) if a.size else 0.0


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


# closed-loop outcome pins (tests/golden/closed_loop_outcome.json): error and
# count metrics within a factor OUTCOME_BAND of the committed value (both
# ways: a change of the closed loop's behaviour is news either way), contact
# loss within OUTCOME_LOSS_PP percentage points, instability fallbacks exact
OUTCOME_BAND = 1.25
OUTCOME_LOSS_PP = 1.0


def closed_loop_pins():
    import json
    from pathlib import Path

    return json.loads((Path(__file__).resolve().parent / "golden" / "closed_loop_outcome.json").read_text())


def check_outcome(got: dict, pin: dict, tag: str):
    for k, ref in pin.items():
        v = float(got[k])
        if k.startswith("contact_loss"):
            assert abs(v - ref) <= OUTCOME_LOSS_PP, (tag, k, v, ref)
        elif k.startswith("unstable"):
            assert v == ref, (tag, k, v, ref)
        elif ref == 0:
            assert v <= 3, (tag, k, v, ref)
        else:
            lo, hi = ref / OUTCOME_BAND, ref * OUTCOME_BAND
            if k.endswith("_ticks") or k.endswith("_ticks_mean"):  # counts: +-3 ticks of slack besides the band
                lo, hi = lo - 3, hi + 3
            assert lo <= v <= hi, (tag, k, v, ref)
