"""How often the ascent-direction branch of the acceptance rule decides a
step on the bench workload: numpy oracle (CPU) over the first
`--n` instances of bench.py's seeded batch, under both comparators
(include/ffddp.h FFDDP_NEGSTEP_*).  Writes one JSON object.

    python tools/neg_branch_stats.py --n 256 > profiles/r03_neg_branch.json
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "franka-force-feedback-mpc_amd")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=256)
    ap.add_argument("--regime", default="tracking")
    a = ap.parse_args()
    import bench
    from helpers import make_batch, product_cfg
    from oracle import fddp
    from oracle_pool import solve_many

    cfg = product_cfg("classical", 30)
    batch = make_batch("classical", a.n, 30, seed=bench.SEED, regime=a.regime)
    out = {"workload": f"bench.py batch (seed {bench.SEED}, {a.regime} regime), first {a.n} instances, maxiter 10",
           "solver": "numpy oracle (oracle/fddp.py), BoxFDDP"}
    res = {}
    for name, rule in (("crocoddyl", 0), ("bounded_rise", 1)):
        r = solve_many(cfg, batch, range(a.n), consts=fddp.Consts(neg_step_rule=rule))
        res[name] = r
        out[name] = {
            "ok_frac": float(np.mean([x["ok"] for x in r])),
            "mean_iter": float(np.mean([x["iter"] for x in r])),
            "mean_trials": float(np.mean([x["trials"] for x in r])),
            "neg_branch_per_solve": float(np.mean([x["neg_branch"] for x in r])),
            "neg_accepted_per_solve": float(np.mean([x["neg_accepted"] for x in r])),
            "solves_with_neg_branch": int(sum(x["neg_branch"] > 0 for x in r)),
            "solves_with_neg_accept": int(sum(x["neg_accepted"] > 0 for x in r)),
        }
    c, b = res["crocoddyl"], res["bounded_rise"]
    out["solves_that_differ"] = int(sum(x["iter"] != y["iter"] or not np.array_equal(x["xs"], y["xs"])
                                        for x, y in zip(c, b)))
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
