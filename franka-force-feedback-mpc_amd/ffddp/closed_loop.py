"""Closed-loop benchmark runner over the HIP solver and the HIP plant stand-in
(BASELINE.json configs[0]: ``ClassicalCrocoddylMPC --scenario flat --time 20
--no-viewer``).

Mirrors ``_run_single`` of src/run/run_classical.py:183-579 and
src/run/run_force_feedback.py in benchmark mode: 1 kHz physics with 5
substeps per control step (dt = 5 ms), plant reset to the neutral keyframe,
approach-then-circle reference from the initial EE position with the
contact-onset hold, controller built on the flat table, hidden table tilt /
actuation mismatch applied afterwards, per-tick RunLogger rows, summary
statistics in meta.json.  The plant is ffddp.plant (MuJoCo is not available;
its parity is unpinned).

usage:  python -m ffddp.closed_loop --scenario flat --time 20 [--variant ff]
"""
from __future__ import annotations

import argparse
import time
from pathlib import Path
from typing import Optional

import numpy as np

from . import controller as CT
from .plant import PandaTablePlant
from .runlog import RunLogger, summary_metrics
from .trajectory import TABLE_CENTER, TABLE_HALF_Z, TOOL_RADIUS, make_approach_then_circle, with_contact_hold
from .uncertainty import ScenarioUncertaintyInjector, config_for_scenario

SCENARIOS = ("flat", "tilted_5", "tilted_10", "tilted_15", "actuation_uncertainty")
_SEEDS = {"flat": 11, "tilted_5": 12, "tilted_10": 13, "tilted_15": 14, "actuation_uncertainty": 15, "tilted": 16}
_TILT = {"flat": 0.0, "tilted_5": 5.0, "tilted_10": 10.0, "tilted_15": 15.0, "actuation_uncertainty": 0.0,
         "tilted": 8.0}
_LABEL = {"flat": "Flat table", "tilted_5": "Tilted table (5deg)", "tilted_10": "Tilted table (10deg)",
          "tilted_15": "Tilted table (15deg)", "actuation_uncertainty": "Actuation gain mismatch",
          "tilted": "Tilted table (8deg)"}
ACTUATION_SCALE = np.array([0.90, 1.08, 0.92, 1.05, 0.88, 1.10, 0.86])


def scenario_seed(name: str) -> int:
    """_scenario_seed (run_classical.py:30-39)."""
    return int(_SEEDS.get(name, 99))


def scenario_settings(name: str) -> dict:
    """_scenario_settings (run_classical.py:53-91)."""
    if name not in _TILT:
        raise ValueError(f"Unknown scenario '{name}'")
    scale = ACTUATION_SCALE.copy() if name == "actuation_uncertainty" else np.ones(7)
    return {"tilt_deg": _TILT[name], "torque_scale": scale, "label": _LABEL[name]}


def run_single(scenario: str = "flat", total_time: float = 20.0, variant: str = "classical",
               results_dir: Path | str = "results/classical_eval", contact_model: str = "normal_1d",
               mpc_iters: Optional[int] = None, circle_radius: float = 0.10, circle_omega: float = 1.5,
               horizon: Optional[int] = None, device: int = 0, verbose: bool = True, log: bool = True,
               neg_step_rule: int = 0) -> dict:
    """One closed-loop run; returns the summary dict (and writes the run log).
    neg_step_rule: the solver's ascent-direction comparator (include/ffddp.h
    FFDDP_NEGSTEP_*; 0 = Crocoddyl's, the reference's behaviour)."""
    settings = scenario_settings(scenario)
    plant = PandaTablePlant(n_substeps=5, timestep=0.001, device=device)
    obs = plant.reset("neutral")
    obs = plant.get_observation(with_ee=True, with_jacobian=True)
    z_top = float(TABLE_CENTER[2] + TABLE_HALF_Z)
    z_contact = z_top + TOOL_RADIUS - 8.0e-3
    z_pre = z_contact + 0.05
    center = np.array([TABLE_CENTER[0], TABLE_CENTER[1], z_contact])
    t_approach, t_pre, t_stab = 0.55, 0.25, 0.2
    base = make_approach_then_circle(center=center, radius=float(circle_radius), omega=float(circle_omega),
                                     z_pre=z_pre, z_contact=z_contact, t_approach=t_approach,
                                     ee_start=obs.ee_pos.copy(), t_pre=t_pre)
    t_contact_phase = float(t_pre + t_approach)

    traj = with_contact_hold(base, t_contact_phase, t_stab)

    max_iters = int(mpc_iters) if mpc_iters is not None else 10
    if variant == "ff":
        cfg = CT.ff_benchmark_config(plant.dt, z_contact, max_iters=max_iters, contact_model=contact_model,
                                     neg_step_rule=neg_step_rule,
                                     **({"horizon": horizon} if horizon else {}))
        mpc = CT.ForceFeedbackCrocoddylMPC(sim=plant, traj_fn=traj, config=cfg, device=device)
    else:
        cfg = CT.classical_benchmark_config(plant.dt, z_contact, max_iters=max_iters, contact_model=contact_model,
                                            neg_step_rule=neg_step_rule,
                                            **({"horizon": horizon} if horizon else {}))
        mpc = CT.ClassicalCrocoddylMPC(sim=plant, traj_fn=traj, config=cfg, device=device)
    if abs(settings["tilt_deg"]) > 1e-12:
        plant.set_table_tilt(settings["tilt_deg"])  # hidden from the controller
        obs = plant.get_observation(with_ee=True, with_jacobian=True)
    unc = None
    unc_meta = None
    ucfg = config_for_scenario(scenario, seed=scenario_seed(scenario))
    if ucfg is not None:
        unc = ScenarioUncertaintyInjector(dt=plant.dt, nu=7, config=ucfg, tau_lpf_alpha=plant.tau_meas_lpf_alpha)
        unc_meta = unc.meta()
    logger = RunLogger(f"{variant}_{scenario}", results_dir=results_dir,
                       notes={"scenario": scenario, "scene": "panda_table_scene (ffddp plant stand-in)"}) if log \
        else None
    steps = int(total_time / plant.dt)
    series = {k: [] for k in ("t", "err_tan", "err_3d", "fn_meas", "fn_pred", "contact", "unstable", "neg_acc",
                                "not_ok")}
    t = 0.0
    wall0 = time.perf_counter()
    solve_s = 0.0
    for k in range(steps):
        ctrl_obs = unc.observation_for_controller(obs) if unc is not None else obs
        ts = time.perf_counter()
        tau_cmd = mpc.compute_control(ctrl_obs, t)
        solve_s += time.perf_counter() - ts
        tau_applied = unc.command_for_plant(tau_cmd) if unc is not None else tau_cmd * settings["torque_scale"]
        obs = plant.step(tau_applied)
        t = t + plant.dt
        p_ref, v_ref, surf_ref = traj(t)
        err = np.asarray(obs.ee_pos, float) - np.asarray(p_ref, float)
        err_tan, err_3d = float(np.linalg.norm(err[:2])), float(np.linalg.norm(err))
        fn_meas = float(obs.f_contact_normal)
        info = dict(mpc.last_info)
        fn_pred = float(info.get("fn_pred", np.nan))
        in_contact = fn_meas > 0.5
        for key, val in (("t", t), ("err_tan", err_tan), ("err_3d", err_3d), ("fn_meas", fn_meas),
                         ("fn_pred", fn_pred), ("contact", 1.0 if in_contact else 0.0),
                         ("unstable", float(bool(info.get("unstable", False)))),
                         ("neg_acc", float(info.get("neg_accepted", 0))),
                         ("not_ok", float(bool(info.get("solved_now", False)) and not bool(info.get("ok", False))))):
            series[key].append(val)
        if logger is not None:
            logger.log(
                t=t, ee_pos=np.asarray(obs.ee_pos, float).copy(), ee_ref=np.asarray(p_ref, float).copy(),
                ee_vel=np.asarray(obs.ee_vel, float).copy(), ee_vel_ref=np.asarray(v_ref, float).copy(),
                err_tan=err_tan, err_3d=err_3d, fn_meas=fn_meas, fn_pred=fn_pred, fn_des=float(cfg.fn_des),
                tau_cmd=np.asarray(tau_cmd, float).copy(), tau_meas=obs.tau_meas.copy(),
                tau_meas_filt=obs.tau_meas_filt.copy(), tau_cmd_sim=obs.tau_cmd.copy(), tau_act=obs.tau_act.copy(),
                tau_constraint=obs.tau_constraint.copy(), tau_total=obs.tau_total.copy(),
                tau_applied=np.asarray(tau_applied, float).copy(), contact=int(in_contact),
                surface_ref=int(surf_ref), solver_iters=int(info.get("iters", -1)),
                solver_cost=float(info.get("cost", np.nan)), solver_success=int(bool(info.get("ok", False))),
                solver_unstable=int(bool(info.get("unstable", False))),
                solver_solved_now=int(bool(info.get("solved_now", False))),
                solver_policy_idx=int(info.get("policy_idx", -1)),
                tau_raw_inf=float(info.get("tau_raw_inf", np.nan)), tau_cmd_inf=float(info.get("tau_cmd_inf", np.nan)),
            )
        if verbose and k % 100 == 0:
            print(f"k={k:4d} t={t:6.3f}s | EE=[{obs.ee_pos[0]:.3f}, {obs.ee_pos[1]:.3f}, {obs.ee_pos[2]:.4f}] | "
                  f"|p-p_ref|={err_3d:.4f}m | err_tan={err_tan:.4f}m | Fn_meas={fn_meas:.2f}N "
                  f"Fn_pred={fn_pred:.2f}N | contact={int(in_contact)}", flush=True)
    wall = time.perf_counter() - wall0
    summ = summary_metrics(series["t"], series["err_tan"], series["err_3d"], series["fn_meas"], series["contact"],
                           float(cfg.fn_des), t_contact_phase)
    # solver health over the run: ticks whose command fell back to the
    # instability guard (crocoddyl_classical.py:392-404, logged as
    # solver_unstable at run_classical.py:480) and solves that accepted a step
    # through the ascent-direction branch (include/ffddp.h neg_step_rule)
    neg = np.asarray(series["neg_acc"])
    summ.update(unstable_ticks=int(np.sum(series["unstable"])), neg_accepted_ticks=int(np.sum(neg > 0)),
                neg_accepted_total=int(np.sum(neg)), solve_not_ok_ticks=int(np.sum(series["not_ok"])))
    summ.update(total_time=float(total_time), dt=float(plant.dt), scenario_label=settings["label"],
                scenario_tilt_deg=float(settings["tilt_deg"]), uncertainty_profile=unc_meta,
                torque_scale=settings["torque_scale"].tolist(), fn_des=float(cfg.fn_des),
                wall_s=wall, controller_s=solve_s, ticks=steps,
                cfg_summary={"horizon": int(cfg.horizon), "dt": float(cfg.dt), "dt_ocp": float(cfg.dt_ocp),
                             "z_contact": float(cfg.z_contact), "z_press": float(cfg.z_press),
                             "max_iters": int(cfg.max_iters), "contact_model": str(cfg.contact_model),
                             "variant": variant})
    if logger is not None:
        logger.set_meta(benchmark_mode=True, plant="ffddp.plant (HIP stand-in for MuJoCo)", **summ)
        logger.save()
        summ["run_dir"] = str(logger.run_dir)
    mpc.close()
    plant.close()
    if verbose:
        print(f"RMS tangential error: {summ['rms_tangential_error']:.4f} m | contact-phase RMS "
              f"{summ['rms_tangential_error_contact_phase']:.4f} m | avg |Fn-Fdes| {summ['avg_abs_force_err']:.2f} N"
              f" | contact loss {summ['contact_loss_contact_phase_pct']:.1f} % | {steps} ticks in {wall:.1f} s "
              f"({1e3 * solve_s / max(1, steps):.2f} ms/tick controller)", flush=True)
    return summ


def main(argv=None):
    ap = argparse.ArgumentParser(description="closed-loop MPC on the ffddp plant stand-in")
    ap.add_argument("--scenario", choices=SCENARIOS + ("tilted", "all"), default="flat")
    ap.add_argument("--variant", choices=("classical", "ff"), default="classical")
    ap.add_argument("--time", type=float, default=12.0)
    ap.add_argument("--no-viewer", action="store_true", help="accepted for CLI parity (there is no viewer)")
    ap.add_argument("--results-dir", type=Path, default=Path("results/classical_eval"))
    ap.add_argument("--contact-model", choices=("normal_1d", "point3d"), default="normal_1d")
    ap.add_argument("--mpc-iters", type=int, default=None)
    ap.add_argument("--horizon", type=int, default=None)
    ap.add_argument("--circle-radius", type=float, default=0.10)
    ap.add_argument("--circle-omega", type=float, default=1.5)
    ap.add_argument("--neg-step-rule", type=int, choices=(0, 1), default=0,
                    help="ascent-direction comparator: 0 Crocoddyl's (default), 1 bounded rise")
    args = ap.parse_args(argv)
    names = SCENARIOS if args.scenario == "all" else (args.scenario,)
    out = {}
    for name in names:
        out[name] = run_single(name, args.time, args.variant, args.results_dir, args.contact_model, args.mpc_iters,
                               args.circle_radius, args.circle_omega, args.horizon,
                               neg_step_rule=args.neg_step_rule)
    return out


if __name__ == "__main__":
    main()
