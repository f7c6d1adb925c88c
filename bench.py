#!/usr/bin/env python3
"""Benchmark: batched Franka 7-DoF horizon-30 (Box)FDDP solves/s on MI355X.

BASELINE.json metric: "FDDP solves/sec, Franka 7-DoF horizon-30 batch=4096,
at 1/2/4/8 MI355X".  One step = one solver.solve(xs_init, us_init, 10, False)
(crocoddyl_classical.py:367) for a batch of B synthetic OCP instances per GPU
(classical nx=14 nu=7, contact model normal_1d, cold warm start), inputs
already resident in HBM.  N GPUs = N independent shards (one process per GPU,
weak scaling); the only collective is the final all-gather of per-instance
costs and first controls (RCCL, the exchange the north star names).

Prints ONE JSON line (rank 0).  Extra objects:
  roofline      dominant kernel's algorithmic bytes per launch / its average
                HIP-event-timed launch duration, vs 8 TB/s.
  cpu_baseline  the numpy oracle (oracle/, the CPU restatement) timed on a
                bounded sample of the same workload on the host cores (one
                worker process per core, up to 16), in a child process.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))
import ffddp_path  # noqa: E402,F401

import numpy as np  # noqa: E402

METRIC = "FDDP solves/sec, Franka 7-DoF horizon-30 batch=4096, at 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s spec
HBM_MEASURED_GBS = 6290.0  # float4 copy, same table
FP64_VALU_PEAK_TFLOPS = 78.6  # AMD public MI355X vector fp64 spec


def algorithmic_words(nx: int, nu: int, N: int):
    """Per-node fp64 words of the staged calcDiff -> backward -> forward design
    (SURVEY.md §8(d)): A = calcDiff (running node), B = backward, C = one
    forward trial; *_T the terminal node; IO per solve."""
    a_r = 2 * nx + nu + 6
    a_w = 2 * nx * nx + 2 * nx * nu + nu * nu + 2 * nx + nu + 1
    A = a_r + a_w
    Bw = (a_w - 1) + nu * nx + nu + nx
    Cf = 3 * nx + 2 * nu + nu * nx + 6 + nx + nu
    A_T = (nx + 6) + (nx * nx + nx + 1)
    B_T = nx * nx + 2 * nx
    C_T = 4 * nx + 6
    io = nx + (N + 1) * nx + N * nu + (N + 1) * 6 + 21 + (N + 1) * nx + N * nu + N * nu * nx + 1
    return dict(A=A, B=Bw, C=Cf, A_T=A_T, B_T=B_T, C_T=C_T, IO=io)


def kernel_bytes(stats: np.ndarray, nx: int, nu: int, N: int) -> dict:
    """Algorithmic bytes of one solve of the whole batch, per kernel class
    (one kernel per class): node = the calcDiff record (A words per running
    node), primal = the calc's reads (x_t, u_t, x_t+1, refs) and writes (gap,
    cost), backward = B words per node, forward / forward2 = C words per node
    for every step length the first / second line-search pass evaluated."""
    w = algorithmic_words(nx, nu, N)
    n_calc = stats[:, 4].astype(np.float64)
    n_bw = stats[:, 0].astype(np.float64)
    ev1 = stats[:, 6].astype(np.float64)
    ev2 = stats[:, 7].astype(np.float64)
    primal_words = 2 * nx + nu + 6 + nx + 1
    per_trial = N * w["C"] + w["C_T"]
    return {
        "node": 8.0 * float(np.sum(n_calc)) * (N * w["A"] + w["A_T"]),
        "primal": 8.0 * float(np.sum(n_calc)) * (N + 1) * primal_words,
        "backward": 8.0 * float(np.sum(n_bw)) * (N * w["B"] + w["B_T"]),
        "forward": 8.0 * float(np.sum(ev1)) * per_trial,
        "forward2": 8.0 * float(np.sum(ev2)) * per_trial,
        "io": 8.0 * stats.shape[0] * w["IO"],
    }


def _oracle_solve_one(args):
    """Worker: one oracle solve of instance i (CPU restatement, maxiter=10)."""
    cfg_kw, i = args
    from oracle import fddp, ocp  # noqa: WPS433 (checker import, baseline leg only)

    batch = _CPU_STATE["batch"]
    prob = ocp.Problem(batch.x0[i], batch.node_ref[i, :, :3], batch.node_ref[i, :, 3:], batch.inst_ref[i, :14],
                       batch.inst_ref[i, 14:], bool(batch.surface[i]))
    s = fddp.SolverBoxFDDP(_CPU_STATE["ocfg"], prob)
    s.solve(batch.xs_init[i], batch.us_init[i], 10, False)
    return i


_CPU_STATE: dict = {}


def _cpu_worker(argv) -> None:
    """Child process of the cpu_baseline leg (never touches the GPU): rebuilds
    the same seeded batch, times the oracle over a bounded sample on all the
    host cores this process may use, prints one JSON object."""
    import multiprocessing as mp

    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int)
    ap.add_argument("--horizon", type=int)
    ap.add_argument("--variant")
    ap.add_argument("--contact")
    ap.add_argument("--regime")
    ap.add_argument("--seed", type=int)
    ap.add_argument("--budget", type=float)
    a = ap.parse_args(argv)
    from ffddp import _abi, robot as R, workload
    from ffddp.config import classical_preset, ff_preset

    sys.path.insert(0, str(ROOT / "tests"))
    from helpers import oracle_cfg  # noqa: E402

    cfg = ff_preset(a.horizon, a.contact) if a.variant == "ff" else classical_preset(a.horizon, a.contact)
    ee = R.R_MJ_FROM_PIN @ _abi.frame_placement(R.Q_NEUTRAL)[1]
    batch = workload.make_batch(a.batch, a.horizon, a.variant, _abi.gravity_torque, ee, seed=a.seed,
                                regime=a.regime, fk=_abi.frame_placement)
    _CPU_STATE["batch"] = batch
    _CPU_STATE["ocfg"] = oracle_cfg(cfg)
    try:
        cores = len(os.sched_getaffinity(0))
    except AttributeError:
        cores = os.cpu_count() or 1
    workers = max(1, min(16, cores))  # the GPU box grants 16 CPUs per GPU
    t0 = time.perf_counter()
    _oracle_solve_one((None, 0))
    t1 = time.perf_counter() - t0
    n = int(min(batch.B, max(workers, workers * max(1, int(a.budget / max(t1, 1e-3))))))
    ctx = mp.get_context("fork")
    t0 = time.perf_counter()
    with ctx.Pool(workers) as pool:
        pool.map(_oracle_solve_one, [(None, i) for i in range(n)], chunksize=1)
    dt = time.perf_counter() - t0
    print(json.dumps({
        "value": n / dt, "unit": "solves/s", "cores": workers, "kind": "port",
        "sample": f"first {n} instances of the rank-0 batch (same seed/workload), numpy oracle (oracle/fddp.py), "
                  f"maxiter=10, {workers} worker processes, {dt:.1f} s wall ({t1:.2f} s for one solve on one core)",
    }))


def cpu_baseline(args, seed: int) -> dict:
    """The oracle timed on the host cores in a child process (the GPU is
    initialised in this one); bounded to about args.cpu_budget seconds."""
    import subprocess

    cmd = [sys.executable, str(Path(__file__).resolve()), "--_cpu_worker", "--batch", str(args.batch), "--horizon",
           str(args.horizon), "--variant", args.variant, "--contact", args.contact, "--regime", args.regime, "--seed",
           str(seed), "--budget", str(args.cpu_budget)]
    # one BLAS thread per worker process: the oracle's matrices are tiny and
    # the workers already cover the cores
    env = dict(os.environ, OMP_NUM_THREADS="1", OPENBLAS_NUM_THREADS="1", MKL_NUM_THREADS="1")
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=max(120.0, 10 * args.cpu_budget), env=env)
    lines = [x for x in r.stdout.splitlines() if x.startswith("{")]
    if r.returncode != 0 or not lines:
        return {"value": None, "error": (r.stderr or r.stdout)[-400:]}
    return json.loads(lines[-1])


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "--_cpu_worker":
        return _cpu_worker(sys.argv[2:])
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--batch", type=int, default=4096, help="instances per GPU")
    ap.add_argument("--horizon", type=int, default=30)
    ap.add_argument("--variant", choices=("classical", "ff"), default="classical")
    ap.add_argument("--contact", choices=("normal_1d", "point3d"), default="normal_1d")
    ap.add_argument("--maxiter", type=int, default=10)
    ap.add_argument("--regime", choices=("tracking", "random"), default="tracking")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-budget", type=float, default=12.0)
    ap.add_argument("--no-profile", action="store_true", help="disable per-kernel HIP-event timing")
    ap.add_argument("--no-host-io", action="store_true", help="skip the PCIe-inclusive host-array rate")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    from ffddp import BatchedBoxFDDP, _abi, robot as R, shard, workload
    from ffddp.config import classical_preset, ff_preset

    rank, world, local_rank = shard.env_ranks()
    shard.init("nccl", local_rank, world)
    dev = torch.device("cuda", local_rank)
    torch.cuda.set_device(dev)

    B, N = args.batch, args.horizon
    cfg = ff_preset(N, args.contact) if args.variant == "ff" else classical_preset(N, args.contact)
    nx, nu = cfg.nx, 7
    ee = R.R_MJ_FROM_PIN @ _abi.frame_placement(R.Q_NEUTRAL)[1]
    batch = workload.make_batch(
        B, N, args.variant, _abi.gravity_torque, ee, seed=shard.shard_seed(1234, rank), regime=args.regime,
        fk=_abi.frame_placement,
    )
    f64 = dict(dtype=torch.float64, device=dev)
    T = dict(
        x0=torch.tensor(batch.x0, **f64),
        node_ref=torch.tensor(batch.node_ref, **f64),
        inst_ref=torch.tensor(batch.inst_ref, **f64),
        surface=torch.tensor(batch.surface, dtype=torch.uint8, device=dev),
        xs_init=torch.tensor(batch.xs_init, **f64),
        us_init=torch.tensor(batch.us_init, **f64),
        xs=torch.zeros((B, N + 1, nx), **f64),
        us=torch.zeros((B, N, nu), **f64),
        K=torch.zeros((B, N, nu, nx), **f64),
        cost=torch.zeros(B, **f64),
        iters=torch.zeros(B, dtype=torch.int32, device=dev),
        ok=torch.zeros(B, dtype=torch.uint8, device=dev),
        fn_pred=torch.zeros((B, 2), **f64),
        stats=torch.zeros((B, _abi.NSTATS), dtype=torch.int32, device=dev),
    )
    solver = BatchedBoxFDDP(cfg, max_batch=B, device=local_rank)
    stream = torch.cuda.current_stream(dev).cuda_stream
    gathered = torch.zeros((world, B, 1 + nu), **f64) if world > 1 else None

    def step():
        solver.solve_dev(T, maxiter=args.maxiter, is_feasible=False, stream=stream)
        if world > 1:  # final exchange: per-instance cost + first control to every rank
            shard.gather_results(T["cost"], T["us"][:, 0, :], gathered)

    # warmup; the last warmup step times every kernel class once to find the
    # dominant kernel, and only that kernel is event-timed inside the timed
    # region (events around every launch of 3 streams would perturb it)
    warm_prof = None
    for w in range(args.warmup):
        if not args.no_profile and w == args.warmup - 1:
            solver.profile(True)
            solver.profile_read(reset=True)
        step()
    torch.cuda.synchronize(dev)
    dom = None
    if not args.no_profile:
        warm_prof = solver.profile_read(reset=True)
        dom = max(("primal", "node", "backward", "forward"), key=lambda k: warm_prof[k][0])
        solver.profile([dom])
        solver.profile_read(reset=True)
    elapsed = shard.timed_steps(step, args.steps, lambda: torch.cuda.synchronize(dev))
    prof = solver.profile_read(reset=True) if not args.no_profile else None

    stats = T["stats"].cpu().numpy()
    ok = T["ok"].cpu().numpy()
    iters = T["iters"].cpu().numpy()
    cost = T["cost"].cpu().numpy()
    total = B * world * args.steps
    value = total / elapsed

    roofline = None
    kernels = None
    if prof is not None:
        kb = kernel_bytes(stats, nx, nu, N)
        # per-class times of the (untimed) profiling warmup step, for reference
        kernels = {k: {"ms_per_solve": v[0], "launches_per_solve": v[1]} for k, v in warm_prof.items() if v[1] > 0}
        ms, launches = prof[dom]
        avg_launch_s = ms / 1e3 / max(1, launches)
        bytes_per_launch = kb[dom] * args.steps / max(1, launches)
        achieved = bytes_per_launch / avg_launch_s / 1e9
        traffic = None
        tf = ROOT / "profiles" / "traffic_latest.json"
        if tf.exists():
            try:
                tj = json.loads(tf.read_text())
                if tj.get("config") == f"{args.variant}/{args.contact}/B{B}/N{N}":
                    per_solve = tj.get("kernels", {}).get(dom, {}).get("hbm_bytes_per_solve")
                    if per_solve is not None:
                        traffic = per_solve * args.steps / max(1, launches)
            except Exception:
                traffic = None
        roofline = {
            "bound": "hbm",
            "kernel": dom,
            "achieved": achieved,
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS,
            "traffic": traffic,
            "bytes_per_launch": bytes_per_launch,
            "avg_launch_ms": avg_launch_s * 1e3,
            "frac_of_measured_copy": achieved / HBM_MEASURED_GBS,
        }

    host_io = None
    if not args.no_host_io:
        # PCIe-inclusive rate of the host-array entry point (ffddp_solve_batch):
        # H2D of the inputs + solve + D2H of xs/us/K/cost/...; reported beside
        # `value`, never as `value`.
        solver.profile(False)
        solver.solve(batch, maxiter=args.maxiter)
        th0 = time.perf_counter()
        reps = 3
        for _ in range(reps):
            solver.solve(batch, maxiter=args.maxiter)
        th = (time.perf_counter() - th0) / reps
        host_io = {"value": B / th, "unit": "solves/s", "ms_per_step": th * 1e3, "per_gpu": True}

    if rank == 0:
        base = None
        if not args.no_cpu_baseline and world == 1:
            base = cpu_baseline(args, shard.shard_seed(1234, rank))
        line = {
            "metric": METRIC,
            "value": value,
            "unit": "solves/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (seeded workload.make_batch, tracking regime: x0 near IK of the benchmark "
            "trajectory at t0~U(0,20)s; cold warm start)",
            "config": {
                "workload": f"{args.variant} BoxFDDP solve, nx={nx} nu={nu}, horizon={N}, batch={B}/GPU, "
                f"maxiter={args.maxiter}, contact={args.contact}",
                "variant": args.variant,
                "horizon": N,
                "batch_per_gpu": B,
                "global_batch": B * world,
                "maxiter": args.maxiter,
                "contact_model": args.contact,
                "parallelism": f"shard{world}",
            },
            "roofline": roofline,
            "cpu_baseline": base,
            "solver": {
                "ok_frac": float(np.mean(ok)),
                "mean_iter": float(np.mean(iters)),
                "mean_iters_run": float(np.mean(stats[:, 0])),
                "mean_trials": float(np.mean(stats[:, 1])),
                "mean_trials_evaluated": float(np.mean(stats[:, 6] + stats[:, 7])),
                "cost_finite_frac": float(np.mean(np.isfinite(cost))),
            },
            "kernels": kernels,
            "host_io": host_io,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
