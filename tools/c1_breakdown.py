"""Where a configs[0] closed-loop tick goes (flat scenario, one robot, HIP
solver + HIP plant): per tick, the controller's wall time, the solve() call
inside it (the solve plan's graph launch and wait, or with --no-plan the host
entry point: staging, copies, launches, wait), and the
solve's kernels (per-class HIP-event sums, ffddp_profile_read).  Prints one
JSON line.

    python tools/c1_breakdown.py [--time 4] [--neg-step-rule 0] [--no-plan | --profile] [--cpu]
"""
from __future__ import annotations

import argparse
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import ffddp_path  # noqa: E402,F401
import numpy as np  # noqa: E402

from ffddp import closed_loop, controller as CT, solver as SV  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--time", type=float, default=4.0)
    ap.add_argument("--neg-step-rule", type=int, default=0)
    ap.add_argument("--profile", action="store_true", help="per-kernel HIP events (adds event overhead; host-array"
                    " solve only: a plan captures no timing events)")
    ap.add_argument("--no-plan", action="store_true", help="plain host-array solve instead of the solve plan")
    ap.add_argument("--cpu", action="store_true", help="also time the C++ scalar BoxFDDP (oracle/cpu, one thread) "
                    "on every tick's problem, beside the GPU solve (the loop keeps the GPU results)")
    a = ap.parse_args()
    solve_s, iters, ctrl_s = [], [], []
    orig_solve = SV.BatchedBoxFDDP.solve
    orig_run = SV.SolvePlan.run
    orig_cc = CT.ClassicalCrocoddylMPC.compute_control
    prof = {}

    def solve(self, *args, **kw):
        if a.profile and not getattr(self, "_prof_on", False):
            self.profile(True)
            self._prof_on = True
        t0 = time.perf_counter()
        r = orig_solve(self, *args, **kw)
        solve_s.append(time.perf_counter() - t0)
        iters.append(int(self.iter[0]))
        if a.profile:
            for k, (ms, n) in self.profile_read(reset=True).items():
                p = prof.setdefault(k, [0.0, 0])
                p[0] += ms
                p[1] += n
        return r

    cpu_s, cpu_same = [], []

    def run(self):
        t0 = time.perf_counter()
        r = orig_run(self)
        solve_s.append(time.perf_counter() - t0)
        iters.append(int(self.iter[0]))
        if a.cpu:  # the same problem on one host core (checker leg: oracle/cpu)
            import types

            from ffddp import _abi
            from oracle import cpu_fddp

            b = types.SimpleNamespace(x0=self.x0, node_ref=self.node_ref, inst_ref=self.inst_ref,
                                      surface=self.surface, xs_init=self.xs_init, us_init=self.us_init)
            sp = self.solver.solver_params
            t1 = time.perf_counter()
            out = cpu_fddp.solve_batch(_abi.robot_struct(), self.solver._cfg_struct, b, self.maxiter, False, 1,
                                       solver_params=sp)
            cpu_s.append(time.perf_counter() - t1)
            cpu_same.append(int(out["iter"][0]) == int(self.iter[0]) and bool(out["ok"][0]) == bool(self.ok[0]))
        return r

    def cc(self, obs, t):
        t0 = time.perf_counter()
        r = orig_cc(self, obs, t)
        ctrl_s.append(time.perf_counter() - t0)
        return r

    SV.BatchedBoxFDDP.solve = solve
    SV.SolvePlan.run = run
    CT.ClassicalCrocoddylMPC.compute_control = cc
    if a.no_plan or a.profile:
        init = CT.ClassicalCrocoddylMPC.__init__
        CT.ClassicalCrocoddylMPC.__init__ = lambda self, *args, **kw: init(self, *args, **{**kw, "use_plan": False})
    s = closed_loop.run_single("flat", a.time, verbose=False, log=False, neg_step_rule=a.neg_step_rule)
    n = len(solve_s)
    skip = min(20, n // 4)  # first ticks: allocation, staging buffers
    sl = slice(skip, None)
    out = {"ticks": s["ticks"], "neg_step_rule": a.neg_step_rule, "plan": not (a.no_plan or a.profile),
           "wall_ms_per_tick": 1e3 * s["wall_s"] / s["ticks"],
           "controller_ms": 1e3 * float(np.mean(ctrl_s[sl])), "solve_call_ms": 1e3 * float(np.mean(solve_s[sl])),
           "solve_call_ms_p50": 1e3 * float(np.median(solve_s[sl])), "mean_iters": float(np.mean(iters[sl])),
           "host_controller_ms": 1e3 * float(np.mean(np.array(ctrl_s[sl]) - np.array(solve_s[sl])))}
    if a.cpu:
        out["cpu_solve_ms"] = 1e3 * float(np.mean(cpu_s[sl]))
        out["cpu_solve_ms_p50"] = 1e3 * float(np.median(cpu_s[sl]))
        out["cpu_same_iters_ok_frac"] = float(np.mean(cpu_same))
    if a.profile:
        out["kernels_ms_per_solve"] = {k: v[0] / n for k, v in prof.items() if v[1]}
        out["launches_per_solve"] = {k: v[1] / n for k, v in prof.items() if v[1]}
        out["kernel_ms_per_solve"] = sum(v[0] for v in prof.values()) / n
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
