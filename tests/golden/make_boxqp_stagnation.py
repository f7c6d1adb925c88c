#!/usr/bin/env python3
"""Capture a BoxQP whose projected-Newton line search stops accepting steps
(tests/golden/boxqp_stagnation.npz).  Test input, not a reference vector: the
QP comes from the numpy oracle's own BoxFDDP solve of the random-x0 batch the
GPU parity test uses (tests/test_gpu_parity.py::test_solve_random_regime_horizon30,
seed 101: instance 14 has one, ~1 QP in 3700).  The kernel's BoxQP stops at the first
iteration that accepts no step length; crocoddyl::BoxQP::solve runs on to
maxiter with x unchanged.  tests/test_oracle.py::test_boxqp_stagnation_exit
checks on this QP that both return the same solution.

Run:  python tests/golden/make_boxqp_stagnation.py   (needs the built library
for the batch generator's FK; takes ~1 min)"""
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT / "tests"))
sys.path.insert(0, str(ROOT))
import ffddp_path  # noqa: E402,F401
from oracle import fddp  # noqa: E402
from helpers import make_batch, oracle_solve, product_cfg  # noqa: E402

found = []
_boxqp = fddp.boxqp


calls = [0]


def _probe(H, q, lb, ub, xinit, c):
    info = {}
    out = _boxqp(H, q, lb, ub, xinit, c, info=info)
    calls[0] += 1
    if info["stalled"] and not found:
        found.append(dict(H=H, q=q, lb=lb, ub=ub, xinit=xinit, stall_iter=np.int64(info["stall_iter"]),
                          iters=np.int64(info["iters"])))
    return out


fddp.boxqp = _probe
cfg = product_cfg("classical", 30)
b = make_batch("classical", 32, 30, seed=101, regime="random")
for i in range(32):
    oracle_solve(cfg, b, i)
    if found:
        break
assert found, "no stagnating QP in the 32 instances"
np.savez(Path(__file__).with_name("boxqp_stagnation.npz"), **found[0])
print("instance", i, "QP call", calls[0], "stalls from iteration", int(found[0]["stall_iter"]), "of", int(found[0]["iters"]))
