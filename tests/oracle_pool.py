"""Oracle solves of many instances in worker processes (test infrastructure).

The numpy oracle takes ~1 s per horizon-30 solve on one core, so the GPU
parity tests that compare dozens of instances fan the oracle out over the
host cores.  Workers are spawned (fresh interpreters: they never touch the
GPU and inherit nothing of the parent's HIP state) and run only oracle/.
"""
from __future__ import annotations

import os
from concurrent.futures import ProcessPoolExecutor
from multiprocessing import get_context

import numpy as np


def _workers(n_jobs: int) -> int:
    try:
        cores = len(os.sched_getaffinity(0))
    except AttributeError:
        cores = os.cpu_count() or 1
    # the GPU box grants 16 CPUs per GPU whatever the machine shows
    return max(1, min(16, cores, n_jobs))


def _solve_one(args):
    ocfg, prob, xs_init, us_init, maxiter, is_feasible, box, consts = args
    from oracle import fddp

    s = fddp.SolverBoxFDDP(ocfg, prob, box=box, consts=consts)
    ok = s.solve(xs_init, us_init, maxiter, is_feasible)
    st = s.stats
    return dict(ok=bool(ok), iter=int(s.iter), xs=s.xs, us=s.us, K=s.K, cost=float(s.cost),
                iters_run=st.iters_run, trials=st.trials, reg_retries=st.reg_retries,
                forward_errors=st.forward_errors, neg_branch=st.neg_branch, neg_accepted=st.neg_accepted,
                clamped=st.clamped,
                preg=float(s.preg), trace=np.array(s.trace, float).reshape(-1, 10))


def solve_many(cfg, batch, idx, maxiter=10, box=True, is_feasible=False, xs_init=None, us_init=None, consts=None):
    """Oracle solves of instances `idx` of `batch` (product OcpConfig `cfg`,
    oracle.fddp.Consts `consts`); returns one dict per instance (ok, iter, xs,
    us, K, cost, counters, per-iteration trace)."""
    from helpers import oracle_cfg, oracle_problem

    ocfg = oracle_cfg(cfg)
    xs0 = batch.xs_init if xs_init is None else xs_init
    us0 = batch.us_init if us_init is None else us_init
    jobs = [(ocfg, oracle_problem(batch, int(i), cfg.horizon), np.array(xs0[i]), np.array(us0[i]), maxiter,
             is_feasible, box, consts) for i in idx]
    n = _workers(len(jobs))
    if n == 1:
        return [_solve_one(j) for j in jobs]
    with ProcessPoolExecutor(max_workers=n, mp_context=get_context("spawn")) as ex:
        return list(ex.map(_solve_one, jobs))
