"""CPU baseline (oracle/cpu: the C++ scalar BoxFDDP timed by bench.py's
cpu_baseline leg) against the independent numpy oracle: identical discrete
path (iterations, ok, sequential trials, regularisation retries) and
xs / us / K / cost within 1e-10 (point3d: 1e-7, the KKT-conditioning case of
tests/test_gpu_parity.py).  CPU only."""
from __future__ import annotations

import numpy as np
import pytest

from ffddp import _abi
from helpers import make_batch, product_cfg, rel_err
from oracle import cpu_fddp, fddp
from oracle_pool import solve_many

CASES = [
    ("classical", "normal_1d", 1, "tracking", 1e-10),
    ("classical", "normal_1d", 0, "tracking", 1e-10),
    ("classical", "normal_1d", None, "random", 1e-10),
    ("ff", "normal_1d", 1, "tracking", 1e-10),
    ("classical", "point3d", 1, "tracking", 1e-7),
]


@pytest.mark.parametrize("variant,contact,surf,regime,tol", CASES)
def test_cpu_baseline_matches_oracle(variant, contact, surf, regime, tol):
    N, B = (12 if contact == "normal_1d" else 8), 4
    cfg = product_cfg(variant, N, contact)
    b = make_batch(variant, B, N, seed=3, surface=surf, regime=regime)
    out = cpu_fddp.solve_batch(_abi.robot_struct(), cfg.to_struct(), b, nthreads=2)
    ref = solve_many(cfg, b, range(B))
    for i, r in enumerate(ref):
        assert bool(out["ok"][i]) == r["ok"] and int(out["iter"][i]) == r["iter"]
        assert int(out["stats"][i, 1]) == r["trials"] and int(out["stats"][i, 2]) == r["reg_retries"]
        assert int(out["stats"][i, 8]) == r["neg_branch"] and int(out["stats"][i, 9]) == r["neg_accepted"]
        for k in ("xs", "us", "K"):
            assert rel_err(out[k][i], r[k]) < tol, (k, i, rel_err(out[k][i], r[k]))
        assert rel_err(out["cost"][i], r["cost"]) < tol


def test_cpu_baseline_exceptional_paths():
    """Clamped BoxQP, backward retries and non-finite trials (the GPU parity
    cases) on the CPU baseline vs the oracle."""
    N, B = 10, 2
    for tweak in ("clamp", "retry", "nan"):
        cfg = product_cfg("classical", N)
        b = make_batch("classical", B, N, seed=21, surface=1)
        if tweak == "clamp":
            cfg.tau_limits = np.array([20.0, 20, 20, 20, 3, 3, 3])
        elif tweak == "retry":
            cfg.w_tau = -0.05
        else:
            b.x0 = b.x0.copy()
            b.x0[:, 7:] += 50.0
        # nan: the bounded-rise ascent comparator; Crocoddyl's (dV < 2 dVexp)
        # accepts this start's first gap-closing step at a cost of ~1e24, where
        # two fp64 implementations no longer agree to 1e-9
        rule = _abi.NEGSTEP_BOUNDED_RISE if tweak == "nan" else _abi.NEGSTEP_CROCODDYL
        out = cpu_fddp.solve_batch(_abi.robot_struct(), cfg.to_struct(), b, nthreads=2,
                                   solver_params=_abi.solver_params(neg_step_rule=rule))
        ref = solve_many(cfg, b, range(B), consts=fddp.Consts(neg_step_rule=rule))
        key = {"clamp": "clamped", "retry": "reg_retries", "nan": "forward_errors"}[tweak]
        assert all(r[key] > 0 for r in ref)
        for i, r in enumerate(ref):
            assert bool(out["ok"][i]) == r["ok"] and int(out["iter"][i]) == r["iter"], tweak
            assert int(out["stats"][i, 1]) == r["trials"] and int(out["stats"][i, 2]) == r["reg_retries"], tweak
            assert rel_err(out["xs"][i], r["xs"]) < 1e-9 and rel_err(out["us"][i], r["us"]) < 1e-9, tweak
