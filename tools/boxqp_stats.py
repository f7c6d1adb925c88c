#!/usr/bin/env python3
"""BoxQP work per backward node (numpy oracle, CPU): projected-Newton
iterations per QP (the last one is the convergence test), factorisations per
QP (the clamped set changed) and line-search trials per iteration, for the
tracking and random-x0 regimes.  Explains the two-wave backward's phase D
split (profiles/r06_phase_prof.txt).  usage: python tools/boxqp_stats.py [B]"""
import collections
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))
import ffddp_path  # noqa: E402,F401
import numpy as np  # noqa: E402
from oracle import fddp  # noqa: E402
from helpers import make_batch, oracle_solve, product_cfg  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 6
N = 30
trials, iters, facts = collections.Counter(), collections.Counter(), collections.Counter()
orig = fddp.boxqp


def counted(H, q, lb, ub, xinit, c, stall_exit=False, info=None):
    """Replays oracle.fddp.boxqp's discrete path (clamped sets, trials) and
    counts it, then returns the oracle's own result."""
    n = q.shape[0]
    x = np.maximum(np.minimum(xinit, ub), lb)
    prev, its, nf = None, 0, 0
    for _ in range(c.qp_maxiter):
        its += 1
        g = q + H @ x
        cl = tuple(j for j in range(n) if (x[j] == lb[j] and g[j] > 0) or (x[j] == ub[j] and g[j] < 0))
        nf += cl != prev
        prev = cl
        free = [j for j in range(n) if j not in cl]
        Hff = H[np.ix_(free, free)].copy()
        Hff[np.diag_indices(len(free))] += c.qp_reg
        dxf = -q[free]
        if cl:
            dxf = dxf - H[np.ix_(free, list(cl))] @ x[list(cl)]
        dx = np.zeros(n)
        if free:
            dx[free] = np.linalg.solve(Hff, dxf) - x[free]
        if np.max(np.abs(dx)) < c.qp_th_grad:
            break
        fold = 0.5 * x @ (H @ x) + q @ x
        k, ok = 0, False
        for a in c.alphas:
            k += 1
            xn = np.maximum(np.minimum(x + a * dx, ub), lb)
            if fold - (0.5 * xn @ (H @ xn) + q @ xn) > c.qp_th_acceptstep * (g @ (x - xn)):
                x, ok = xn, True
                break
        trials[k] += 1
        if not ok:
            break
    iters[its] += 1
    facts[nf] += 1
    return orig(H, q, lb, ub, xinit, c, stall_exit, info)


fddp.boxqp = counted
for regime in ("tracking", "random"):
    trials.clear(), iters.clear(), facts.clear()
    cfg = product_cfg("classical", N)
    b = make_batch("classical", B, N, seed=31, regime=regime)
    for i in range(B):
        oracle_solve(cfg, b, i, maxiter=10)
    n = sum(iters.values())
    print(f"{regime}: {n} QPs, {sum(k * v for k, v in iters.items()) / max(n, 1):.2f} iterations per QP, "
          f"{sum(k * v for k, v in facts.items()) / max(n, 1):.2f} factorisations per QP, "
          f"line-search trials per stepping iteration {dict(sorted(trials.items()))}, "
          f"iterations per QP {dict(sorted(iters.items()))}")
