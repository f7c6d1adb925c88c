"""Closed loop on the CPU (diagnostic; test infrastructure, imports oracle/).

Runs ffddp.closed_loop.run_single with the HIP pieces swapped for their
checkers: the solver is the C++ scalar BoxFDDP of oracle/cpu (same OCP and
solver algorithm, same solver properties) and the plant is oracle/plant.py
(the numpy restatement of k_plant).  The controller, trajectory, uncertainty
injector and summary metrics are the product's own host code.  Used to
compare the two ascent-direction comparators (include/ffddp.h
FFDDP_NEGSTEP_*) on the closed loop without a GPU; the GPU runs of the same
comparison are `python -m ffddp.closed_loop --neg-step-rule R` and
`tools/sweep_c4.py --neg-step-rule R`.

    python tools/closed_loop_cpu.py --scenario flat --time 20 --rule 0
"""
from __future__ import annotations

import argparse
import json
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import ffddp_path  # noqa: E402,F401
from ffddp import _abi, closed_loop, controller as CT, plant as PL  # noqa: E402
from oracle import cpu_fddp, plant as OP  # noqa: E402


class CpuBatchedPlant:
    """ffddp.plant.BatchedPlant over oracle/plant.py (one record layout)."""

    def __init__(self, B, timestep=PL.DEFAULT_TIMESTEP, n_substeps=1, device=0):
        self.B = int(B)
        self.params = PL.plant_params(timestep, n_substeps)
        self.prm = OP.default_params(timestep, n_substeps)
        self.q = np.tile(PL.R.Q_NEUTRAL, (self.B, 1))
        self.v = np.zeros((self.B, 7))
        self.plane = np.tile(np.concatenate(PL.table_plane(0.0)), (self.B, 1))
        self.obs = np.zeros((self.B, _abi.PLANT_OBS))

    @property
    def dt(self):
        return float(self.params.timestep * self.params.n_substeps)

    def set_tilt(self, tilt_deg):
        tilt = np.broadcast_to(np.asarray(tilt_deg, dtype=float), (self.B,))
        self.plane = np.stack([np.concatenate(PL.table_plane(t)) for t in tilt])

    def step(self, tau, integrate=True):
        tau = np.broadcast_to(np.asarray(tau, dtype=float), (self.B, 7))
        for b in range(self.B):
            q, v, o = OP.step(self.prm, self.q[b], self.v[b], tau[b], self.plane[b, :3], self.plane[b, 3:], integrate)
            self.q[b], self.v[b] = q, v
            r = self.obs[b]
            r[0:7], r[7:14], r[14:21], r[21:28] = o["q"], o["dq"], o["bias"], o["tau_c"]
            r[28:31], r[31:34], r[34:43] = o["ee_pos"], o["ee_vel"], o["ee_R"].reshape(9)
            r[43:46], r[46], r[47], r[48:69] = o["f_world"], o["fn"], o["ncon"], o["J"].reshape(21)
        return self.obs

    def close(self):
        pass


class CpuSolver:
    """ffddp.BatchedBoxFDDP surface over the C++ CPU BoxFDDP (fn_pred NaN)."""

    def __init__(self, cfg, max_batch, device=0):
        self.cfg = cfg
        self.N = int(cfg.horizon)
        self._cfg_struct = cfg.to_struct()
        self.neg_step_rule = 0

    def setCallbacks(self, callbacks, max_iters=64):
        pass

    def solve(self, batch, maxiter=10, is_feasible=False, xs_init=None, us_init=None):
        params = _abi.solver_params(use_box=bool(self.cfg.use_box_fddp), neg_step_rule=int(self.neg_step_rule))
        out = cpu_fddp.solve_batch(_abi.robot_struct(), self._cfg_struct, batch, maxiter, is_feasible, 1,
                                   xs_init=xs_init, us_init=us_init, solver_params=params)
        self.xs, self.us, self.K, self.cost, self.iter = out["xs"], out["us"], out["K"], out["cost"], out["iter"]
        self.ok, self.stats = out["ok"], out["stats"]
        self.fn_pred = np.full((self.xs.shape[0], 2), np.nan)
        return self.ok

    def close(self):
        pass


def run_cpu(scenario="flat", total_time=20.0, rule=0, variant="classical"):
    """closed_loop.run_single on the CPU checkers; returns its summary."""
    saved = PL.BatchedPlant, CT.BatchedBoxFDDP
    PL.BatchedPlant, CT.BatchedBoxFDDP = CpuBatchedPlant, CpuSolver
    try:
        return closed_loop.run_single(scenario, total_time, variant=variant, log=False, verbose=False,
                                      neg_step_rule=rule)
    finally:
        PL.BatchedPlant, CT.BatchedBoxFDDP = saved


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--scenario", default="flat")
    ap.add_argument("--time", type=float, default=20.0)
    ap.add_argument("--rule", type=int, default=0, help="FFDDP_NEGSTEP_*: 0 Crocoddyl, 1 bounded rise")
    args = ap.parse_args(argv)
    s = run_cpu(args.scenario, args.time, args.rule)
    keys = ("rms_tangential_error", "rms_tangential_error_contact_phase", "avg_abs_force_err",
            "contact_loss_contact_phase_pct", "unstable_ticks", "neg_accepted_ticks", "neg_accepted_total", "solve_not_ok_ticks")
    print(json.dumps({"scenario": args.scenario, "time": args.time, "rule": args.rule, "solver": "cpu",
                      **{k: s.get(k) for k in keys}}))


if __name__ == "__main__":
    main()
