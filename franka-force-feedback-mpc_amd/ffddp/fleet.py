"""Fleet closed loop: B independent classical MPC controllers stepped together
(BASELINE.json configs[3]: "All 5 scenarios x 256 seeds = 1280-instance sweep
sharded over 8 MI355X, RCCL all-gather of costs").

``FleetClassicalMPC`` keeps, per instance, exactly the state and the per-tick
logic of ``ClassicalCrocoddylMPC.compute_control`` (crocoddyl_classical.py:
305-440, our B = 1 mirror in controller.py) in arrays, and runs ONE batched
device solve per control tick for all B instances (warm starts, problem
references and results stay in HBM; only x0, the shared node references and
the first knot of the solution cross PCIe).  Supported configuration: the
benchmark one (solve every tick, ``mpc_update_steps = 1``; no command filter).

``run_sweep`` closes B loops around ``BatchedPlant`` (one launch per tick for
all plants): per instance a scenario (table tilt / actuation mismatch /
uncertainty injector, run_classical.py:53-91 and uncertainty_profiles.py) and
a seed.  The seed perturbs the start posture (q0 = neutral + N(0, 0.02^2),
seeded) and seeds the actuation-uncertainty injector; the reference runs one
scenario from the keyframe with a fixed seed, so this is a sweep around its
configuration rather than a replay of it.  Ranks (torch.distributed) take
contiguous shards of the instances; the per-instance summary metrics are
all-gathered at the end (RCCL on the GPU box).
"""
from __future__ import annotations

import time
from typing import Callable, Optional, Sequence, Tuple

import numpy as np

from . import _abi
from . import robot as R
from .config import OcpConfig
from .controller import _OCP_FIELDS, _quat_wxyz_to_R, classical_benchmark_config
from .plant import BatchedPlant, PandaTablePlant
from .runlog import summary_metrics
from .solver import BatchedBoxFDDP
from .trajectory import TABLE_CENTER, TABLE_HALF_Z, TOOL_RADIUS, make_approach_then_circle, with_contact_hold
from .uncertainty import BatchedUncertaintyInjector, config_for_scenario

Traj = Callable[[float], Tuple[np.ndarray, np.ndarray, bool]]


class FleetClassicalMPC:
    """B classical controllers, one batched solve per tick.

    q_nom (B, 7): each instance's initial posture (the scalar controller's
    ``q_nom = obs0.q``); tau0 (B, 7): its initial command (``obs0.tau_bias``);
    R_site_from_pin_ee / p_site_minus_frame_pin: the site calibration
    (crocoddyl_classical.py:199-226; one robot model, so shared).
    """

    def __init__(self, B: int, traj_fn: Traj, config, q_nom, tau0, R_site_from_pin_ee, p_site_minus_frame_pin,
                 device: int = 0):
        import torch

        cfg = config
        if int(cfg.mpc_update_steps) != 1 or bool(cfg.apply_command_filter):
            raise NotImplementedError("FleetClassicalMPC supports the benchmark setup: mpc_update_steps=1, no filter")
        self.torch = torch
        self.B, self.cfg, self.traj_fn = int(B), cfg, traj_fn
        self.N = int(cfg.horizon)
        self.dev = torch.device("cuda", device)
        self.R_mj_from_pin = R.R_MJ_FROM_PIN.copy()
        self.R_site_from_pin_ee = np.asarray(R_site_from_pin_ee, float)
        self.p_site_minus_frame_pin = np.asarray(p_site_minus_frame_pin, float)
        self.R_des = self.R_mj_from_pin.T @ R.vertical_down_rotation_mj() @ self.R_site_from_pin_ee.T
        self.q_nom = np.asarray(q_nom, float).reshape(self.B, 7).copy()
        self.tau_prev = np.asarray(tau0, float).reshape(self.B, 7).copy()
        self.dt_ocp = float(cfg.dt_ocp) if cfg.dt_ocp is not None else float(cfg.dt)
        ocp = OcpConfig(variant="classical", horizon=self.N, dt=self.dt_ocp, R_des=self.R_des)
        for f in _OCP_FIELDS:
            setattr(ocp, f, getattr(cfg, f))
        ocp.tau_limits = np.asarray(cfg.tau_limits, float).copy()
        self.solver = BatchedBoxFDDP(ocp, max_batch=self.B, device=device)
        self.solver.neg_step_rule = int(getattr(cfg, "neg_step_rule", 0))
        f64 = dict(dtype=torch.float64, device=self.dev)
        B, N = self.B, self.N
        self.T = dict(
            x0=torch.zeros((B, 14), **f64), node_ref=torch.zeros((B, N + 1, 6), **f64),
            inst_ref=torch.zeros((B, 21), **f64), surface=torch.zeros(B, dtype=torch.uint8, device=self.dev),
            xs_init=torch.zeros((B, N + 1, 14), **f64), us_init=torch.zeros((B, N, 7), **f64),
            xs=torch.zeros((B, N + 1, 14), **f64), us=torch.zeros((B, N, 7), **f64),
            K=torch.zeros((B, N, 7, 14), **f64), cost=torch.zeros(B, **f64),
            iters=torch.zeros(B, dtype=torch.int32, device=self.dev), ok=torch.zeros(B, dtype=torch.uint8, device=self.dev),
            fn_pred=torch.zeros((B, 2), **f64), stats=torch.zeros((B, _abi.NSTATS), dtype=torch.int32, device=self.dev),
        )
        # the kept solution (solver.xs/us/K of the last solve whose us[0] was finite)
        self.keep_xs = torch.zeros((B, N + 1, 14), **f64)
        self.keep_us = torch.zeros((B, N, 7), **f64)
        self.keep_K = torch.zeros((B, N, 7, 14), **f64)
        self.valid = np.zeros(B, bool)
        self.latched = np.zeros(B, bool)
        self.loss_count = np.zeros(B, np.int64)
        self.prev_mode = np.full(B, -1, np.int8)
        self._stream = torch.cuda.current_stream(self.dev).cuda_stream
        self.last_info = {}

    def close(self):
        self.solver.close()

    # -- per-tick pieces (crocoddyl_classical.py line refs as in controller.py) -------
    def _surface(self, fn_meas, ee_z, hint: bool) -> np.ndarray:
        """_surface_mode / _detect_surface (:286-303), vectorised."""
        if str(self.cfg.phase_source).strip().lower() != "force_latch":
            return np.full(self.B, bool(hint))
        near = np.isfinite(ee_z) & (ee_z <= float(self.cfg.z_contact) + float(self.cfg.z_contact_band))
        lost = fn_meas < self.cfg.fn_contact_off
        cnt = np.where(self.latched, np.where(lost, self.loss_count + 1, 0), 0)
        release = self.latched & (cnt >= int(self.cfg.contact_release_steps))
        engage = (~self.latched) & ((fn_meas > self.cfg.fn_contact_on) | (bool(hint) & near))
        self.latched = (self.latched & ~release) | engage
        self.loss_count = np.where(release | engage, 0, cnt)
        return self.latched.copy()

    def _node_ref(self, t0: float) -> np.ndarray:
        out = np.zeros((self.N + 1, 6))
        sample = getattr(self.traj_fn, "sample", None)
        if sample is not None:  # same bits as the loop below (R_MJ_FROM_PIN is a signed permutation)
            P, V, _ = sample(np.array([t0 + k * self.dt_ocp for k in range(self.N + 1)]))
            out[:, :3] = P @ self.R_mj_from_pin - self.p_site_minus_frame_pin
            out[:, 3:] = V @ self.R_mj_from_pin
            return out
        for k in range(self.N + 1):
            p, v, _ = self.traj_fn(t0 + k * self.dt_ocp)
            out[k, :3] = self.R_mj_from_pin.T @ np.asarray(p, float) - self.p_site_minus_frame_pin
            out[k, 3:] = self.R_mj_from_pin.T @ np.asarray(v, float)
        return out

    def compute_control(self, q, v, tau_bias, fn_meas, ee_z, t: float) -> np.ndarray:
        torch = self.torch
        cfg, B, N, T = self.cfg, self.B, self.N, self.T
        q = np.asarray(q, float).reshape(B, 7)
        v = np.asarray(v, float).reshape(B, 7)
        x0 = np.concatenate([q, v], 1)
        _, _, hint = self.traj_fn(t)
        surface_now = self._surface(np.asarray(fn_meas, float), np.asarray(ee_z, float), hint)
        # _track_mode: a mode switch drops the warm start
        changed = (self.prev_mode >= 0) & (surface_now != (self.prev_mode == 1))
        self.valid &= ~changed
        self.prev_mode = surface_now.astype(np.int8)
        # problem references (_problem_arrays, crocoddyl_classical.py:521-556)
        mode = str(cfg.posture_ref_mode).strip().lower()
        xreg = np.concatenate([self.q_nom, np.zeros((B, 7))], 1) if mode == "q_nom" else x0.copy()
        tmode = str(cfg.torque_ref_mode).strip().lower()
        if tmode == "zero":
            tref = np.zeros((B, 7))
        elif tmode == "gravity_qnom":
            tref = _abi.gravity_torque(self.q_nom)
        else:
            tref = _abi.gravity_torque(q)
        # the tick's inputs go up as ONE copy (packed float64: x0, inst_ref,
        # tau_prev, surface, warm-start mask per instance, then the shared
        # node references), its outputs come down as one (below)
        pk = np.concatenate([x0, xreg, tref, self.tau_prev, surface_now[:, None].astype(np.float64),
                             self.valid[:, None].astype(np.float64)], 1)
        up = torch.from_numpy(np.concatenate([pk.ravel(), self._node_ref(t).ravel()])).to(self.dev)
        pk_d = up[: B * 44].view(B, 44)
        x0_d = pk_d[:, 0:14]
        T["x0"].copy_(x0_d)
        T["node_ref"].copy_(up[B * 44:].view(1, N + 1, 6).expand(B, N + 1, 6))
        T["inst_ref"].copy_(pk_d[:, 14:35])
        T["surface"].copy_(pk_d[:, 42].to(torch.uint8))
        # warm start (_shift_guess, :733-757): [x0] + xs[1:], us[1:] + [us[-1]]; cold: [x0]*(N+1), [tau_prev]*N
        vmask = pk_d[:, 43] != 0
        xs_i = x0_d[:, None, :].expand(B, N + 1, 14).clone()
        xs_i[:, 1:] = torch.where(vmask[:, None, None], self.keep_xs[:, 1:], xs_i[:, 1:])
        tp = pk_d[:, 35:42][:, None, :].expand(B, N, 7)
        us_sh = torch.cat([self.keep_us[:, 1:], self.keep_us[:, -1:]], 1)
        T["xs_init"].copy_(xs_i)
        T["us_init"].copy_(torch.where(vmask[:, None, None], us_sh, tp))
        self.solver.solve_dev(T, maxiter=int(cfg.max_iters), is_feasible=False, stream=self._stream)
        us0_new = T["us"][:, 0]
        fin = torch.isfinite(us0_new).all(1)
        f3 = fin[:, None, None]
        self.keep_xs.copy_(torch.where(f3, T["xs"], self.keep_xs))
        self.keep_us.copy_(torch.where(f3, T["us"], self.keep_us))
        self.keep_K.copy_(torch.where(fin[:, None, None, None], T["K"], self.keep_K))
        f64 = torch.float64
        down = torch.cat([fin.to(f64)[:, None], self.keep_us[:, 0], self.keep_xs[:, 0], self.keep_K[:, 0].reshape(B, 98),
                          T["cost"][:, None], T["iters"].to(f64)[:, None], T["ok"].to(f64)[:, None],
                          T["stats"][:, 9].to(f64)[:, None], T["fn_pred"][:, 0:1]], 1).cpu().numpy()
        self.valid |= down[:, 0] != 0
        us0, xs0, K0 = down[:, 1:8], down[:, 8:22], down[:, 22:120].reshape(B, 7, 14)
        cost = down[:, 120].copy()
        iters = down[:, 121].astype(np.int32)
        ok = down[:, 122] != 0
        neg_acc = down[:, 123].astype(np.int32)  # ascent-direction acceptances of this solve
        fn_pred = np.where(surface_now, down[:, 124], np.nan)
        # _policy_control (:759-779): u = us[0] + s K[0] (x - xs[0])
        tau_raw = np.where(self.valid[:, None], us0, self.tau_prev)
        if cfg.use_feedback_policy:
            # stacked matmul: per instance the same gemv as the scalar
            # controller's K[0] @ dx (np.einsum sums in another order and
            # differs in the last bit for about half the entries)
            fb = float(cfg.feedback_gain_scale) * np.matmul(K0, (x0 - xs0)[:, :, None])[:, :, 0]
            tau_raw = np.where(self.valid[:, None], tau_raw + fb, tau_raw)
        policy_idx = np.where(self.valid, 0, -1)
        tau_raw_inf = np.max(np.abs(tau_raw), 1)
        unstable = (~np.isfinite(cost)) | (cost > float(cfg.max_solver_cost)) | (tau_raw_inf > float(cfg.max_tau_raw_inf))
        fallback = np.asarray(tau_bias, float).reshape(B, 7) - float(cfg.fallback_dq_damping) * v
        tau_raw = np.where(unstable[:, None], fallback, tau_raw)
        self.valid &= ~unstable
        # _safe_tau (:260-284) without the command filter
        lim = np.asarray(cfg.tau_limits, float)
        bad = ~np.all(np.isfinite(tau_raw), 1)
        tau_cmd = np.clip(np.where(bad[:, None], self.tau_prev, tau_raw), -lim, lim)
        self.tau_prev = tau_cmd.copy()
        self.last_info = dict(ok=ok, cost=cost, iters=iters, tau_raw_inf=tau_raw_inf,
                              tau_cmd_inf=np.max(np.abs(tau_cmd), 1), surface_mode=surface_now, unstable=unstable,
                              fn_pred=fn_pred, solved_now=np.ones(B, bool), policy_idx=policy_idx,
                              neg_accepted=neg_acc)
        return tau_cmd


def site_calibration(obs0):
    """_calibrate_site_rotation / _calibrate_site_position_offset
    (crocoddyl_classical.py:199-226; controller._MPCBase) from one observation."""
    R_pin_ee, p_pin_ee = _abi.frame_placement(np.asarray(obs0.q, float))
    R_site = R_pin_ee.T @ R.R_MJ_FROM_PIN.T @ _quat_wxyz_to_R(obs0.ee_quat)
    p_off = R.R_MJ_FROM_PIN.T @ np.asarray(obs0.ee_pos, float).reshape(3) - p_pin_ee
    return R_site, p_off


def _sweep_instances(scenarios: Sequence[str], seeds: int):
    from .closed_loop import scenario_seed, scenario_settings

    names, tilt, scale, seed = [], [], [], []
    for s in scenarios:
        st = scenario_settings(s)
        for k in range(seeds):
            names.append(s)
            tilt.append(st["tilt_deg"])
            scale.append(st["torque_scale"])
            seed.append(scenario_seed(s) * 100003 + k)
    return np.array(names), np.array(tilt), np.array(scale), np.array(seed)


def run_sweep(scenarios: Sequence[str] = ("flat", "tilted_5", "tilted_10", "tilted_15", "actuation_uncertainty"),
              seeds: int = 256, total_time: float = 4.0, rank: int = 0, world: int = 1, device: int = 0,
              q_sigma: float = 0.02, verbose: bool = True, record: Sequence[int] = (),
              neg_step_rule: int = 0) -> dict:
    """Closed-loop sweep of len(scenarios) * seeds instances; this rank runs
    its contiguous shard.  Returns per-instance summary arrays (this shard).
    record: shard-local instance indices whose controller inputs (the plant
    record as the controller sees it, after any measurement noise) and
    commanded torques are kept per tick, with what a scalar controller needs
    to replay them (the task, the config, the start states).
    neg_step_rule: the solver's ascent-direction comparator (include/ffddp.h
    FFDDP_NEGSTEP_*; 0 = Crocoddyl's, the reference's behaviour)."""
    names, tilt, scale, seed = _sweep_instances(scenarios, seeds)
    n_all = len(names)
    per = (n_all + world - 1) // world
    lo, hi = rank * per, min(n_all, (rank + 1) * per)
    names, tilt, scale, seed = names[lo:hi], tilt[lo:hi], scale[lo:hi], seed[lo:hi]
    B = len(names)
    # nominal geometry and trajectory: planned from the keyframe's EE (run_classical.py:209-264)
    nominal = PandaTablePlant(n_substeps=5, timestep=0.001, device=device)
    obs0 = nominal.reset("neutral")
    z_top = float(TABLE_CENTER[2] + TABLE_HALF_Z)
    z_contact = z_top + TOOL_RADIUS - 8.0e-3
    center = np.array([TABLE_CENTER[0], TABLE_CENTER[1], z_contact])
    base = make_approach_then_circle(center=center, radius=0.10, omega=1.5, z_pre=z_contact + 0.05,
                                     z_contact=z_contact, t_approach=0.55, ee_start=obs0.ee_pos.copy(), t_pre=0.25)
    t_cp = 0.8

    traj = with_contact_hold(base, t_cp, 0.2)

    R_site_from_pin_ee, p_off = site_calibration(obs0)
    nominal.close()
    plant = BatchedPlant(B, timestep=0.001, n_substeps=5, device=device)
    q0 = np.stack([R.Q_NEUTRAL + np.random.default_rng(int(s)).normal(0.0, q_sigma, 7) for s in seed])
    plant.q = q0.copy()
    plant.v = np.zeros((B, 7))
    plant.set_tilt(0.0)
    plant.step(np.zeros((B, 7)), integrate=False)  # mj_forward at the start state
    tau0 = plant.obs[:, 14:21].copy()
    cfg = classical_benchmark_config(plant.dt, z_contact, neg_step_rule=neg_step_rule)
    mpc = FleetClassicalMPC(B, traj, cfg, q_nom=q0, tau0=tau0, R_site_from_pin_ee=R_site_from_pin_ee,
                            p_site_minus_frame_pin=p_off, device=device)
    plant.set_tilt(tilt)  # hidden from the controllers
    plant.step(tau0 * 0.0, integrate=False)
    # the scenarios' uncertainty injectors, batched (BatchedUncertaintyInjector:
    # draw for draw the per-instance ScenarioUncertaintyInjector)
    ucfg = {b: config_for_scenario(str(names[b]), seed=int(seed[b])) for b in range(B)}
    inj_idx = np.array([b for b in range(B) if ucfg[b] is not None], dtype=np.int64)
    inj = BatchedUncertaintyInjector(dt=plant.dt, nu=7, configs=[ucfg[b] for b in inj_idx]) if inj_idx.size else None
    steps = int(total_time / plant.dt)
    series = {k: np.zeros((steps, B)) for k in ("t", "err_tan", "err_3d", "fn_meas", "contact")}
    # solver health per instance: ticks on the instability fallback
    # (crocoddyl_classical.py:392-404; solver_unstable, run_classical.py:480)
    # ticks whose solve accepted an ascent-direction step and ticks whose
    # solve returned ok = False
    unstable_ticks = np.zeros(B)
    neg_ticks = np.zeros(B)
    not_ok_ticks = np.zeros(B)
    rec_idx = [int(i) for i in record]
    rec_obs = np.zeros((steps, len(rec_idx), plant.obs.shape[1]))
    rec_tau = np.zeros((steps, len(rec_idx), 7))
    rec_t = np.zeros(steps)
    obs = plant.obs.copy()
    t = 0.0
    wall0 = time.perf_counter()
    ctrl_s = 0.0
    for k in range(steps):
        q, v, bias = obs[:, 0:7], obs[:, 7:14], obs[:, 14:21]
        fn, ee = obs[:, 46] * (obs[:, 47] > 0.5), obs[:, 28:31]
        if inj is not None:
            q, v = q.copy(), v.copy()
            q[inj_idx], v[inj_idx] = inj.observation_for_controller(q[inj_idx], v[inj_idx])
        tc = time.perf_counter()
        tau = mpc.compute_control(q, v, bias, fn, ee[:, 2], t)
        ctrl_s += time.perf_counter() - tc
        unstable_ticks += mpc.last_info["unstable"]
        neg_ticks += mpc.last_info["neg_accepted"] > 0
        not_ok_ticks += ~mpc.last_info["ok"]
        if rec_idx:
            rec_t[k] = t
            rec_obs[k] = obs[rec_idx]
            rec_obs[k][:, 0:7], rec_obs[k][:, 7:14] = q[rec_idx], v[rec_idx]
            rec_tau[k] = tau[rec_idx]
        tau_app = tau * scale
        if inj is not None:
            tau_app[inj_idx] = inj.command_for_plant(tau[inj_idx])
        obs = plant.step(tau_app).copy()
        t += plant.dt
        p_ref, _, _ = traj(t)
        err = obs[:, 28:31] - np.asarray(p_ref, float)[None]
        fnm = obs[:, 46] * (obs[:, 47] > 0.5)
        series["t"][k] = t
        series["err_tan"][k] = np.linalg.norm(err[:, :2], axis=1)
        series["err_3d"][k] = np.linalg.norm(err, axis=1)
        series["fn_meas"][k] = fnm
        series["contact"][k] = (fnm > 0.5).astype(float)
        if verbose and k % 100 == 0:
            print(f"k={k:4d} t={t:6.3f}s | B={B} | median |p-p_ref|={np.median(series['err_3d'][k]):.4f} m | "
                  f"median Fn={np.median(fnm):.2f} N | ok={np.mean(mpc.last_info['ok']):.3f}", flush=True)
    wall = time.perf_counter() - wall0
    mpc.close()
    plant.close()
    keys = SUMMARY_KEYS[:-3]
    per_inst = {k: np.zeros(B) for k in SUMMARY_KEYS}
    for b in range(B):
        s = summary_metrics(series["t"][:, b], series["err_tan"][:, b], series["err_3d"][:, b],
                            series["fn_meas"][:, b], series["contact"][:, b], float(cfg.fn_des), t_cp)
        for k_ in keys:
            per_inst[k_][b] = s[k_]
    per_inst["unstable_ticks"] = unstable_ticks
    per_inst["neg_accepted_ticks"] = neg_ticks
    per_inst["solve_not_ok_ticks"] = not_ok_ticks
    out = dict(names=names, seed=seed, per_instance=per_inst, ticks=steps, wall_s=wall, controller_s=ctrl_s,
               instances=B, shard=(lo, hi), n_all=n_all)
    if rec_idx:
        out["record"] = dict(index=np.array(rec_idx), t=rec_t, obs=rec_obs, tau=rec_tau, q0=q0[rec_idx], traj=traj,
                             config=cfg, dt=plant.dt, calibration_obs=obs0)
    return out


SUMMARY_KEYS = ("rms_tangential_error", "rms_tangential_error_contact_phase", "rms_3d_error", "avg_abs_force_err",
                "max_fn", "contact_loss_contact_phase_pct", "fn_mean_contact_phase", "unstable_ticks",
                "neg_accepted_ticks", "solve_not_ok_ticks")


def gather_summaries(res: dict, n_all: int, device=None):
    """All-gather every rank's per-instance summaries into (n_all, len(SUMMARY_KEYS))
    in instance order (the sweep's one exchange; RCCL when the tensors live on
    a GPU, gloo on the CPU)."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size() if dist.is_initialized() else 1
    per = (n_all + world - 1) // world
    local = np.full((per, len(SUMMARY_KEYS)), np.nan)
    m = np.stack([res["per_instance"][k] for k in SUMMARY_KEYS], 1)
    local[: m.shape[0]] = m
    t = torch.from_numpy(local)
    if device is not None:
        t = t.to(device)
    if world == 1:
        return local[:n_all]
    out = [torch.empty_like(t) for _ in range(world)]
    dist.all_gather(out, t)
    return torch.cat(out, 0).cpu().numpy()[:n_all]


def scenario_table(names, metrics: np.ndarray) -> dict:
    """Per-scenario mean / median / p95 of each summary metric."""
    out = {}
    for s in dict.fromkeys(names):
        sel = metrics[np.asarray(names) == s]
        out[str(s)] = {k: {"mean": float(np.nanmean(sel[:, i])), "median": float(np.nanmedian(sel[:, i])),
                           "p95": float(np.nanpercentile(sel[:, i], 95))} for i, k in enumerate(SUMMARY_KEYS)}
        out[str(s)]["instances"] = int(sel.shape[0])
    return out
