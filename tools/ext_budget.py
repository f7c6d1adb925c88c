"""Error budget of the full solves against an extended-precision answer.

For each parity case whose tolerance sits above 1e-9 (point3d contact with
and without the friction cone, the N = 100 point3d long horizon, the
SURVEY-literal random x0), the oracle solve is repeated in x87 extended
precision (np.longdouble: 64-bit significand, ~1e-19), on the same fp64
inputs.  Each fp64 implementation is then measured against it:
  oracle        oracle/ (numpy fp64), feasible-iteration gains K = Hff_inv Qxu^T
                with the explicit inverse, as SolverBoxFDDP::computeGains
  oracle_solve  the same with K by Cholesky solves (oracle.fddp.Consts
                gains_form="solve", the HIP kernel's evaluation order)
  cpu           oracle/cpu (the product's node models compiled for the host)
  gpu           the HIP library (an npz of its outputs, tools/ext_budget_gpu.py)
The extended-precision reference uses the explicit-inverse form (in 64-bit
significands the two forms agree to ~1e-15).
max |impl - ext| / max(1, max |ext|) over xs, us, K, cost; one JSON line per
case.  Oracle / test infrastructure only.

usage: python tools/ext_budget.py OUT.jsonl [GPU.npz[,GPU2.npz,...]] [CASE-NAME-PREFIX]
(several npz: one "gpu:<file stem>" implementation each, e.g. library variants)
"""
from __future__ import annotations

import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))
import ffddp_path  # noqa: E402,F401
import numpy as np  # noqa: E402

# name, variant, contact, cone, N, B, seed, surface, regime (the tests' own inputs)
CASES = [
    ("solve/classical/point3d/surf1/cone0", "classical", "point3d", 0, 12, 4, 22, 1, "tracking"),
    ("solve/classical/point3d/surf1/cone1", "classical", "point3d", 1, 12, 4, 22, 1, "tracking"),
    ("solve/ff/point3d/surf1/cone1", "ff", "point3d", 1, 12, 4, 22, 1, "tracking"),
    ("solve/point3d/N100", "classical", "point3d", 0, 100, 2, 55, 1, "tracking"),
    ("solve/random/N30/B32[:8]", "classical", "normal_1d", 0, 30, 8, 101, None, "random"),
    # tests/test_gpu_batch.py's oracle spread of configs[1] (B = 1024 random x0, seed 77)
    ("batch/classical/random/B1024[spread]", "classical", "normal_1d", 0, 30, 8, 77, None, "random"),
]


def spread_picks(B):
    """The instances tests/test_gpu_batch.py compares with the oracle."""
    rng = np.random.default_rng(1)
    picks = np.unique(np.concatenate([[0, 1, B // 4 - 1, B // 4, B // 2, B - 1], rng.integers(0, B, 10)]))
    return picks[::2]


def case_inputs(case):
    from helpers import make_batch, product_cfg

    name, variant, contact, cone, N, B, seed, surf, regime = case
    cfg = product_cfg(variant, N, contact)
    if cone:
        cfg.w_friction_cone, cfg.mu = 2.0e2, 0.6
    if name.startswith("batch/"):
        full = make_batch(variant, 1024, N, seed=seed, regime=regime)
        idx = spread_picks(1024)[:B]
        for f in ("x0", "node_ref", "inst_ref", "surface", "xs_init", "us_init", "t0"):
            setattr(full, f, np.ascontiguousarray(getattr(full, f)[idx]))
        b = full
    elif name.startswith("solve/random"):
        b = make_batch(variant, 32, N, seed=seed, regime=regime).slice(slice(0, B))
    else:
        b = make_batch(variant, B, N, seed=seed, surface=surf, regime=regime)
    return cfg, b


def _solve(args):
    cfg, b, i, dtype, form = args
    from helpers import oracle_cfg, oracle_problem
    from oracle import fddp

    s = fddp.SolverBoxFDDP(oracle_cfg(cfg), oracle_problem(b, i, cfg.horizon), dtype=dtype,
                           consts=fddp.Consts(gains_form=form))
    ok = s.solve(b.xs_init[i], b.us_init[i], 10, False)
    return dict(ok=bool(ok), iter=int(s.iter), trials=s.stats.trials, xs=np.asarray(s.xs), us=np.asarray(s.us),
                K=np.asarray(s.K), cost=s.cost)


def err(a, ref):
    a = np.asarray(a, np.longdouble)
    ref = np.asarray(ref, np.longdouble)
    return float(np.max(np.abs(a - ref)) / max(1.0, float(np.max(np.abs(ref)))))


def err_elem(a, ref):
    """element-wise |a - ref| / (1 + |ref|) (tests/helpers.py elem_err)"""
    a = np.asarray(a, np.longdouble)
    ref = np.asarray(ref, np.longdouble)
    return float(np.max(np.abs(a - ref) / (1.0 + np.abs(ref))))


def main():
    from concurrent.futures import ProcessPoolExecutor
    from multiprocessing import get_context

    from ffddp import _abi
    from oracle import cpu_fddp

    out_path = Path(sys.argv[1])
    gpus = {}
    if len(sys.argv) > 2 and sys.argv[2]:
        paths = sys.argv[2].split(",")
        for pth in paths:
            gpus["gpu" if len(paths) == 1 else "gpu:" + Path(pth).stem] = dict(np.load(pth))
    lines = []
    with ProcessPoolExecutor(max_workers=8, mp_context=get_context("spawn")) as ex:
        only = sys.argv[3] if len(sys.argv) > 3 else ""
        for case in CASES:
            if not case[0].startswith(only):
                continue
            t0 = time.time()
            cfg, b = case_inputs(case)
            B = b.B
            jobs = [(cfg, b, i, dt, form) for dt, form in ((np.float64, "crocoddyl"), (np.longdouble, "crocoddyl"),
                                                            (np.float64, "solve")) for i in range(B)]
            res = list(ex.map(_solve, jobs))
            f64, ext, f64s = res[:B], res[B:2 * B], res[2 * B:]
            cpu = cpu_fddp.solve_batch(_abi.robot_struct(), cfg.to_struct(), b, nthreads=4)
            rec = {"case": case[0], "B": B, "N": case[4], "same_path": [], "oracle": {}, "oracle_solve": {}, "cpu": {}}
            impls = {"oracle": {k: np.stack([r[k] for r in f64]) for k in ("xs", "us", "K")},
                     "oracle_solve": {k: np.stack([r[k] for r in f64s]) for k in ("xs", "us", "K")},
                     "cpu": {k: cpu[k] for k in ("xs", "us", "K")}}
            impls["oracle"]["cost"] = np.array([r["cost"] for r in f64])
            impls["oracle_solve"]["cost"] = np.array([r["cost"] for r in f64s])
            impls["cpu"]["cost"] = cpu["cost"]
            for gname, gpu in gpus.items():
                if f"{case[0]}/xs" in gpu:
                    impls[gname] = {k: gpu[f"{case[0]}/{k}"] for k in ("xs", "us", "K", "cost")}
            for i in range(B):
                same = (f64[i]["iter"] == ext[i]["iter"] and f64[i]["trials"] == ext[i]["trials"]
                        and f64[i]["ok"] == ext[i]["ok"])
                rec["same_path"].append(bool(same))
            for name, im in impls.items():
                rec.setdefault(name, {})
                for k in ("xs", "us", "K", "cost"):
                    e = max(err(im[k][i], ext[i][k]) for i in range(B) if rec["same_path"][i]) \
                        if any(rec["same_path"]) else None
                    rec[name][k] = e
                rec[name]["K_elem"] = max(err_elem(im["K"][i], ext[i]["K"]) for i in range(B) if rec["same_path"][i]) \
                    if any(rec["same_path"]) else None
            # oracle vs cpu vs gpu pairwise, for reference
            for gname in (g for g in impls if g.startswith("gpu")):
                for ref in ("oracle", "oracle_solve"):
                    rec[f"{gname}_vs_{ref}"] = {k: max(err(impls[gname][k][i], impls[ref][k][i]) for i in range(B))
                                                for k in ("xs", "us", "K", "cost")}
            rec["seconds"] = time.time() - t0
            print(json.dumps(rec), flush=True)
            lines.append(rec)
    out_path.write_text("".join(json.dumps(r) + "\n" for r in lines))


if __name__ == "__main__":
    main()
