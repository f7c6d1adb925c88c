#!/usr/bin/env python3
"""Benchmark: batched Franka 7-DoF horizon-30 (Box)FDDP solves/s on MI355X.

BASELINE.json metric: "FDDP solves/sec, Franka 7-DoF horizon-30 batch=4096,
at 1/2/4/8 MI355X".  One step = one solver.solve(xs_init, us_init, 10, False)
(crocoddyl_classical.py:367) of every instance of a batch of B = 4096
synthetic OCP instances per GPU (classical nx=14 nu=7, contact model
normal_1d, cold warm start), inputs already resident in HBM.  The instances
are independent (north_star: the batch "shards embarrassingly across the 8
GPUs"), so each of G processes solves its own B-instance shard with no
collective in the data path: weak scaling, value = G * B solves per step over
the max-over-ranks time.  The one exchange is the final all-gather of the
per-instance results over RCCL ("costs": cost, iters, ok, u0 by default;
"full": xs, us, K, cost), inside every timed step.

Prints ONE JSON line (rank 0).  Extra objects:
  roofline      SURVEY §8(d): algorithmic HBM bytes of the whole solve (every
                kernel, from the device-counted iterations / line-search
                trials) / wall time of the timed region, vs 8 TB/s; plus the
                per-kernel fractions from a separate single-stream profiling
                step (HIP events around every launch, no overlap) and the
                PMC-measured traffic when profiles/ holds it for this config.
  cpu_baseline  the C++ scalar BoxFDDP (oracle/cpu, the same OCP and solver
                algorithm) on the host cores, OpenMP over the same instances.
  strong        (G > 1) the other reading of the metric, with the same fields
                as the headline (value, ms_per_step, scaling "strong",
                roofline): one 4096-instance batch split into G contiguous
                slices (B / G instances per GPU: the per-GPU latency end).
  random_regime the SURVEY-literal x0 draw (q_neutral + U(+-0.15)), same B,
                with its own roofline.
  ff            the force-feedback variant (nx = 21) at the metric's batch
                and horizon, with its own roofline.
  host_io       PCIe-inclusive rate of the host-array entry point.
roofline.fp64 prices the same run against the measured fp64 VALU peak
(tools/micro/fp64_peak.hip -> profiles/r05_fp64_peak.json) with the USEFUL
flops: the operation count of the scalar C++ implementation per node stage /
backward node / trial node (tools/flop_count.py -> profiles/
r06_useful_flops.json) x the device-counted units of this run.  Its
issue_rate field is the issued fp64 lane-flops of a PMC pass of this
configuration (tools/pmc_fp64.sh -> profiles/fp64_latest.json: every lane of
every issued wave instruction, idle lanes included) on the same roof.
roofline.bound names the roof the run is closer to by the useful figure;
roofline.frac stays SURVEY §8(d)'s HBM fraction.
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
SEED = 1234


def algorithmic_words(nx: int, nu: int, N: int):
    """Per-node fp64 words of the staged calcDiff -> backward -> forward design
    (SURVEY.md §8(d)): A = calcDiff (running node), B = backward, C = one
    forward trial (SURVEY's per-trial count); *_T the terminal node; IO per
    solve.  The line search reads (xs, us, K, k, fs, w, refs) once per
    instance per launch however many step lengths it evaluates concurrently
    (C_shared) and writes one trial per step length (C_trial)."""
    a_r = 2 * nx + nu + 6
    a_w = 2 * nx * nx + 2 * nx * nu + nu * nu + 2 * nx + nu + 1
    A = a_r + a_w
    Bw = (a_w - 1) + nu * nx + nu + nx
    Cf = 3 * nx + 2 * nu + nu * nx + 6 + nx + nu
    A_T = (nx + 6) + (nx * nx + nx + 1)
    B_T = nx * nx + 2 * nx
    C_T = 4 * nx + 6
    io = nx + (N + 1) * nx + N * nu + (N + 1) * 6 + 21 + (N + 1) * nx + N * nu + N * nu * nx + 1
    C_shared = N * (3 * nx + 2 * nu + nu * nx + 6) + (3 * nx + 6)
    C_trial = N * (nx + nu) + nx
    return dict(A=A, B=Bw, C=Cf, A_T=A_T, B_T=B_T, C_T=C_T, IO=io, C_shared=C_shared, C_trial=C_trial)


def solve_bytes(stats: np.ndarray, nx: int, nu: int, N: int) -> dict:
    """Algorithmic bytes of one batched solve, per kernel class and in total,
    from the per-instance device counters (include/ffddp.h stats):
    [0] successful backward passes (= first-pass line-search launches),
    [4] calcDiffs, [5] line-search launches (both passes), [6]/[7] step
    lengths evaluated by the first / second pass."""
    w = algorithmic_words(nx, nu, N)
    s = stats.astype(np.float64)
    n_calc, n_bw, n_fw, ev1, ev2 = s[:, 4].sum(), s[:, 0].sum(), s[:, 5].sum(), s[:, 6].sum(), s[:, 7].sum()
    calc = 8.0 * n_calc * (N * w["A"] + w["A_T"])  # k_node: calc + calcDiff, fused
    out = {
        "node": calc,
        "backward": 8.0 * n_bw * (N * w["B"] + w["B_T"]),
        "forward": 8.0 * (n_bw * w["C_shared"] + ev1 * w["C_trial"]),
        "forward2": 8.0 * ((n_fw - n_bw) * w["C_shared"] + ev2 * w["C_trial"]),
        "io": 8.0 * stats.shape[0] * w["IO"],
    }
    out["total"] = out["node"] + out["backward"] + out["forward"] + out["forward2"] + out["io"]
    # SURVEY §8(d) literal: every evaluated step length reads its inputs again
    out["total_survey_formula"] = 8.0 * (n_calc * (N * w["A"] + w["A_T"]) + n_bw * (N * w["B"] + w["B_T"]) +
                                         (ev1 + ev2) * (N * w["C"] + w["C_T"]) + stats.shape[0] * w["IO"])
    return out


def pmc_traffic(variant, contact, B, N):
    """Per-solve HBM bytes per kernel class measured by rocprofv3 PMC passes
    (tools/pmc_traffic.py -> profiles/traffic_latest.json), if they are for
    this configuration."""
    tf = ROOT / "profiles" / "traffic_latest.json"
    if not tf.exists():
        return None
    try:
        tj = json.loads(tf.read_text())
    except ValueError:
        return None
    if tj.get("config") != f"{variant}/{contact}/B{B}/N{N}":
        return None
    return {k: v.get("hbm_bytes_per_solve") for k, v in tj.get("kernels", {}).items()}


def sq_limiter(variant, contact, B, N):
    """What the SQ counters of the same configuration show limits the kernels
    (tools/pmc_sq2.sh -> tools/pmc_summary.py --json -> profiles/sq_latest.json),
    if they are for this configuration: per kernel, the FMA share of VALU
    instructions and the fractions of wave time VALU-active, LDS-active,
    parked on s_waitcnt / barriers, and issue-stalled."""
    f = ROOT / "profiles" / "sq_latest.json"
    if not f.exists():
        return None
    try:
        j = json.loads(f.read_text())
    except ValueError:
        return None
    if j.get("config") != f"{variant}/{contact}/B{B}/N{N}":
        return None
    out = {"source": j.get("source"), "summary": j.get("summary"), "kernels": j.get("kernels")}
    # VALU lane utilisation per kernel (tools/pmc_lanes.sh -> profiles/lanes_latest.json: the mean fraction of
    # a wave's 64 lanes enabled while it issues VALU instructions, SQ_THREAD_CYCLES_VALU / SQ_ACTIVE_INST_VALU
    # normalised by a 64-lane calibration kernel)
    lj = _profile_json("lanes_latest.json", variant, contact, B, N)
    if lj:
        out["lane_utilisation"] = {k: v.get("lane_util") for k, v in lj.get("kernels", {}).items()
                                   if v.get("lane_util") is not None}
        out["lane_source"] = lj.get("source")
    return out


def _profile_json(name, variant, contact, B, N):
    f = ROOT / "profiles" / name
    if not f.exists():
        return None
    try:
        j = json.loads(f.read_text())
    except ValueError:
        return None
    return j if j.get("config") == f"{variant}/{contact}/B{B}/N{N}" else None


def fp64_peak_tflops():
    """Measured fp64 FMA throughput of one MI355X (tools/micro/fp64_peak.hip)."""
    f = ROOT / "profiles" / "r05_fp64_peak.json"
    try:
        return float(json.loads(f.read_text())["peak_fp64_fma_tflops"])
    except (OSError, ValueError, KeyError):
        return None


def solve_units(stats: np.ndarray, N: int) -> dict:
    """Device-counted work units of one batched solve: node stages (calcDiffs
    x (N + 1)), backward nodes (backward passes x N), line-search trial nodes
    (evaluated step lengths x (N + 1))."""
    s = stats.astype(np.float64)
    return {"node": float(s[:, 4].sum()) * (N + 1), "backward": float(s[:, 0].sum()) * N,
            "forward": float((s[:, 6] + s[:, 7]).sum()) * (N + 1)}


def solve_counts(stats: np.ndarray) -> dict:
    s = stats.astype(np.float64)
    return {"calcdiff": float(s[:, 4].sum()), "backward": float(s[:, 0].sum()),
            "trials": float((s[:, 6] + s[:, 7]).sum()), "forward_launches": float(s[:, 5].sum())}


def useful_per_unit(variant, contact, N):
    """Useful (algorithmic) fp64 flops per node stage / backward node / trial
    node of this OCP: the scalar C++ CPU baseline executed with a counting
    fp64 type (tools/flop_count.py -> profiles/r06_useful_flops.json; no SIMD
    lanes, so no idle or duplicate lanes), if the file holds this config."""
    f = ROOT / "profiles" / "r06_useful_flops.json"
    try:
        c = json.loads(f.read_text())["configs"][f"{variant}/{contact}/N{N}"]
        return {k: c["phases"][k]["flops_per_unit"] for k in ("node", "backward", "forward")}
    except (OSError, ValueError, KeyError):
        return None


def useful_flops(stats, N, per) -> float | None:
    """Useful fp64 flops of one batched solve: useful_per_unit x this solve's
    device-counted units."""
    if not per:
        return None
    u = solve_units(stats, N)
    return sum(per[c] * u[c] for c in ("node", "backward", "forward"))


def fp64_flops(stats, N, per_unit) -> float | None:
    """Issued fp64 lane-flops of one batched solve: the PMC per-unit figures
    (tools/pmc_fp64.py) x this solve's device-counted units."""
    if not per_unit:
        return None
    u = solve_units(stats, N)
    k = per_unit.get("kernels", {})
    tot = 0.0
    for c in ("node", "backward", "forward"):
        if c not in k or "lane_flops_per_unit" not in k[c]:
            return None
        tot += k[c]["lane_flops_per_unit"] * u[c]
    # the per-solve kernels (init, accept, commit, finalize): as profiled
    tot += sum(v.get("lane_flops_per_solve", 0.0) for c, v in k.items() if c not in ("node", "backward", "forward"))
    return tot


def rooflines(bytes_per_step, flops_per_step, sec_per_step, world):
    """HBM and fp64-VALU fractions of one timed configuration (all ranks)."""
    hbm = {"achieved": bytes_per_step / sec_per_step / 1e9, "peak": HBM_PEAK_GBS * world, "unit": "GB/s"}
    hbm["frac"] = hbm["achieved"] / hbm["peak"]
    pk = fp64_peak_tflops()
    fp = None
    if flops_per_step is not None and pk:
        fp = {"achieved": flops_per_step / sec_per_step / 1e12, "peak": pk * world, "unit": "TFLOP/s"}
        fp["frac"] = fp["achieved"] / fp["peak"]
    return hbm, fp


def fp64_block(fp, useful_flops_step, per_unit, fpi, issued_flops_step):
    """roofline.fp64: the useful-work fraction (frac; algorithmic flops of the
    scalar implementation per unit x device-counted units / time / measured
    fp64 FMA peak) and, beside it, the issue-rate utilisation (issued fp64
    lane-flops from the PMC: every lane of every issued wave instruction,
    idle and duplicate lanes included)."""
    if fp is None and fpi is None:
        return None
    out = {} if fp is None else dict(fp, useful=True, flops_per_step=useful_flops_step, flops_per_unit=per_unit,
                                     basis="useful fp64 flops per node stage / backward node / trial node of the "
                                           "scalar C++ implementation (oracle/cpu/ffddp_cpu.cpp run with a counting "
                                           "fp64 type, tools/flop_count.py -> profiles/r06_useful_flops.json) x this "
                                           "run's device-counted units, over the measured fp64 FMA peak "
                                           "(tools/micro/fp64_peak.hip, profiles/r05_fp64_peak.json)")
    if fpi is not None:
        out["issue_rate"] = dict(fpi, flops_per_step=issued_flops_step, basis=(
            "issue-rate utilisation: issued fp64 lane-flops (64 x (2 FMA + MUL + ADD) per wave instruction, every "
            "lane, masked ones included; tools/pmc_fp64.sh, profiles/fp64_latest.json) x device-counted units"))
        if fp is not None and fpi["achieved"] > 0:
            out["useful_share_of_issued"] = fp["achieved"] / fpi["achieved"]
    return out


def cpu_baseline(cfg, batch, maxiter: int, budget_s: float) -> dict:
    """The C++ scalar BoxFDDP (oracle/cpu) on the host cores: OpenMP over the
    same instances, one per thread at a time; warm-up, then the median of 5
    timed runs over the sample (median of >= 5; the sample
    is sized so the 5 runs take about budget_s of CPU time)."""
    from ffddp import _abi
    from oracle import cpu_fddp  # checker / baseline leg only

    try:
        cores = len(os.sched_getaffinity(0))
    except AttributeError:
        cores = os.cpu_count() or 1
    threads = max(1, min(16, cores))  # the GPU box grants 16 CPUs per GPU
    rb, cs = _abi.robot_struct(), cfg.to_struct()
    warm = batch.slice(slice(0, min(batch.B, 2 * threads)))
    t0 = time.perf_counter()
    cpu_fddp.solve_batch(rb, cs, warm, maxiter=maxiter, nthreads=threads)
    per_solve = (time.perf_counter() - t0) / warm.B * threads
    runs = 5
    n = int(min(batch.B, max(2 * threads, budget_s / runs / max(per_solve, 1e-6) * threads)))
    sample = batch.slice(slice(0, n))
    times = []
    for _ in range(runs):
        t0 = time.perf_counter()
        out = cpu_fddp.solve_batch(rb, cs, sample, maxiter=maxiter, nthreads=threads)
        times.append(time.perf_counter() - t0)
    med = float(np.median(times))
    return {
        "value": n / med, "unit": "solves/s", "cores": threads, "kind": "port",
        "sample": f"first {n} of the {batch.B} instances of the same seeded workload; C++ scalar BoxFDDP "
                  f"(oracle/cpu/ffddp_cpu.cpp: the product's node models compiled for the host + a sequential "
                  f"Crocoddyl-style solver), OpenMP {threads} threads, maxiter={maxiter}, median of {runs} runs "
                  f"({med:.2f} s each; ok {float(np.mean(out['ok'])):.2f}, mean iter {float(np.mean(out['iter'])):.2f})",
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--batch", type=int, default=4096, help="instances per GPU (the metric's batch)")
    ap.add_argument("--horizon", type=int, default=30)
    ap.add_argument("--variant", choices=("classical", "ff"), default="classical")
    ap.add_argument("--contact", choices=("normal_1d", "point3d"), default="normal_1d")
    ap.add_argument("--maxiter", type=int, default=10)
    ap.add_argument("--regime", choices=("tracking", "random"), default="tracking")
    ap.add_argument("--gather", choices=("costs", "full", "none"), default="costs")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-budget", type=float, default=12.0)
    ap.add_argument("--no-profile", action="store_true", help="skip the single-stream per-kernel profiling step")
    ap.add_argument("--profile-only", action="store_true",
                    help="run only the single-stream profiling step (for rocprofv3 of the per-kernel numbers)")
    ap.add_argument("--no-host-io", action="store_true")
    ap.add_argument("--no-extras", action="store_true", help="skip the strong-scaling, random-regime and ff extras")
    ap.add_argument("--no-ff", action="store_true", help="skip the force-feedback extra")
    ap.add_argument("--force-collective", action="store_true",
                    help="RCCL process group and all-gather even at one process (rehearses RCCL's stream beside "
                         "the solver's 4 slice streams; DESIGN.md §8)")
    args = ap.parse_args()
    if args.profile_only and args.no_profile:
        ap.error("--profile-only runs only the profiling step: it cannot be combined with --no-profile")

    import torch
    import torch.distributed as dist

    from ffddp import BatchedBoxFDDP, _abi, robot as R, shard, workload
    from ffddp.config import classical_preset, ff_preset

    rank, world, local_rank = shard.env_ranks()
    # FFDDP_BENCH_ONE_GPU=1: every rank on cuda:0 with gloo collectives, a
    # one-GPU rehearsal of the N > 1 path (slices, max-over-ranks timing,
    # gather); never how the metric is measured
    one_gpu = os.environ.get("FFDDP_BENCH_ONE_GPU") == "1"
    dev_rank = local_rank
    if one_gpu:
        local_rank = 0
    dev = torch.device("cuda", local_rank)
    torch.cuda.set_device(dev)
    # The device, the null stream and the solver's slice streams come first,
    # the process group after them (the solver is tuned to one hardware
    # queue per slice, 4 per process; shard.prepare_device)
    torch.zeros(1, device=dev)

    B, N, nu = args.batch, args.horizon, 7
    cfg = ff_preset(N, args.contact) if args.variant == "ff" else classical_preset(N, args.contact)
    nx = cfg.nx
    ee = R.R_MJ_FROM_PIN @ _abi.frame_placement(R.Q_NEUTRAL)[1]

    def make(Bg, seed, regime):
        return workload.make_batch(Bg, N, args.variant, _abi.gravity_torque, ee, seed=seed, regime=regime,
                                   fk=_abi.frame_placement)

    f64 = dict(dtype=torch.float64, device=dev)

    def tensors(b):
        Bl = b.B
        return dict(
            x0=torch.tensor(b.x0, **f64), node_ref=torch.tensor(b.node_ref, **f64),
            inst_ref=torch.tensor(b.inst_ref, **f64),
            surface=torch.tensor(b.surface, dtype=torch.uint8, device=dev),
            xs_init=torch.tensor(b.xs_init, **f64), us_init=torch.tensor(b.us_init, **f64),
            xs=torch.zeros((Bl, N + 1, nx), **f64), us=torch.zeros((Bl, N, nu), **f64),
            K=torch.zeros((Bl, N, nu, nx), **f64), cost=torch.zeros(Bl, **f64),
            iters=torch.zeros(Bl, dtype=torch.int32, device=dev), ok=torch.zeros(Bl, dtype=torch.uint8, device=dev),
            fn_pred=torch.zeros((Bl, 2), **f64),
            stats=torch.zeros((Bl, _abi.NSTATS), dtype=torch.int32, device=dev),
        )

    stream = torch.cuda.current_stream(dev).cuda_stream
    sync = lambda: torch.cuda.synchronize(dev)  # noqa: E731

    # ---- the metric: every rank solves its own B-instance shard (weak
    # scaling; rank 0's shard is the one-GPU workload) ----
    glob = make(B, SEED + rank, args.regime)
    mine = glob
    T = tensors(mine)
    counts = [B] * world
    solver = BatchedBoxFDDP(cfg, max_batch=B, device=local_rank)  # creates the slice streams
    if one_gpu:
        shard.init("gloo", dev_rank, world)
    else:
        shard.init("nccl", local_rank, world, force=args.force_collective)
    gather = None
    if (world > 1 or args.force_collective) and args.gather != "none":
        width = shard.pack_results(T, args.gather).shape[1]
        gather = shard.Gatherer(counts, width, dev)

    def step():
        solver.solve_dev(T, maxiter=args.maxiter, is_feasible=False, stream=stream)
        if gather is not None:
            gather(shard.pack_results(T, args.gather))

    elapsed = None
    if not args.profile_only:
        for _ in range(args.warmup):
            step()
        sync()
        elapsed = shard.timed_steps(step, args.steps, sync)

    stats = T["stats"].cpu().numpy()
    ok = T["ok"].cpu().numpy()
    iters = T["iters"].cpu().numpy()
    cost = T["cost"].cpu().numpy()
    sb = solve_bytes(stats, nx, nu, N)
    fp_unit = _profile_json("fp64_latest.json", args.variant, args.contact, B, N)
    fl = fp64_flops(stats, N, fp_unit)
    uf_unit = useful_per_unit(args.variant, args.contact, N)
    ufl = useful_flops(stats, N, uf_unit)
    # whole-job sums over ranks: algorithmic bytes per step, ok count, iterations, fp64 flops (issued, useful)
    tot = shard.sum_over_ranks(torch.tensor([sb["total"], sb["total_survey_formula"], float(ok.sum()),
                                             float(iters.sum()), fl if fl is not None else -1.0,
                                             ufl if ufl is not None else -1.0], **f64)).cpu().numpy()
    tot_bytes, tot_survey, tot_ok, tot_it, tot_fl, tot_ufl = (float(v) for v in tot)
    tot_fl = tot_fl if fl is not None else None
    tot_ufl = tot_ufl if ufl is not None else None
    unit_counts = {k: float(v) for k, v in zip(("calcdiff", "backward", "trials", "forward_launches"),
                                           shard.sum_over_ranks(torch.tensor(list(solve_counts(stats).values()),
                                                                             **f64)).cpu().numpy())}

    # ---- per-kernel profiling: the same slice on ONE stream, HIP events
    # around every launch (no overlap between launches) ----
    kernels = dominant = None
    if not args.no_profile:
        old = os.environ.get("FFDDP_STREAMS")
        os.environ["FFDDP_STREAMS"] = "1"
        psolver = BatchedBoxFDDP(cfg, max_batch=max(counts), device=local_rank)
        if old is None:
            del os.environ["FFDDP_STREAMS"]
        else:
            os.environ["FFDDP_STREAMS"] = old
        psolver.solve_dev(T, maxiter=args.maxiter, stream=stream)  # warm-up
        sync()
        psolver.profile(True)
        psolver.profile_read(reset=True)
        n_prof = 2
        t0 = time.perf_counter()
        for _ in range(n_prof):
            psolver.solve_dev(T, maxiter=args.maxiter, stream=stream)
        sync()
        t_single = (time.perf_counter() - t0) / n_prof
        prof = psolver.profile_read(reset=True)
        psolver.profile(False)
        pstats = T["stats"].cpu().numpy()
        pb = solve_bytes(pstats, nx, nu, N)
        pun = solve_units(pstats, N)
        # the profile times the two line-search passes as two classes; the
        # PMC per-unit figure is one (k_forward_g8 runs both)
        pun["forward"] = float(pstats[:, 6].sum()) * (N + 1)
        pun["forward2"] = float(pstats[:, 7].sum()) * (N + 1)
        pk64 = fp64_peak_tflops()
        total_ms = sum(v[0] for v in prof.values())
        kernels = {}
        for k, (ms, n) in prof.items():
            if n == 0:
                continue
            e = {"ms_per_solve": ms / n_prof, "launches_per_solve": n / n_prof, "avg_launch_ms": ms / n,
                 "share_of_kernel_time": ms / total_ms if total_ms > 0 else None}
            if k in pb:
                bpl = pb[k] * n_prof / n
                ach = bpl / (ms / n / 1e3) / 1e9
                e.update({"bytes_per_launch": bpl, "achieved_gbs": ach, "frac": ach / HBM_PEAK_GBS})
            pu = (fp_unit or {}).get("kernels", {}).get("forward" if k == "forward2" else k, {})
            if pk64 and "lane_flops_per_unit" in pu and k in pun:
                fpl = pu["lane_flops_per_unit"] * pun[k] * n_prof / n
                e.update({"fp64_issued_flops_per_launch": fpl,
                          "fp64_issue_frac": fpl / (ms / n / 1e3) / 1e12 / pk64})
            uk = "forward" if k == "forward2" else k
            if pk64 and uf_unit and uk in uf_unit and k in pun:
                ufl_k = uf_unit[uk] * pun[k] * n_prof / n
                e.update({"fp64_useful_flops_per_launch": ufl_k,
                          "fp64_useful_frac": ufl_k / (ms / n / 1e3) / 1e12 / pk64})
            kernels[k] = e
        dom = max((k for k in kernels if "achieved_gbs" in kernels[k]), key=lambda k: kernels[k]["ms_per_solve"])
        dominant = dict(name=dom, **kernels[dom])
        dominant["single_stream_ms_per_solve"] = t_single * 1e3
        psolver.close()
        if args.profile_only:
            if rank == 0:
                print(json.dumps({"profile_only": True, "kernels": kernels, "dominant": dominant}), flush=True)
            shard.shutdown()
            return

    value = B * world * args.steps / elapsed
    traffic = pmc_traffic(args.variant, args.contact, B, N) if world == 1 else None
    hbm, fp = rooflines(tot_bytes, tot_ufl, elapsed / args.steps, world)
    _, fpi = rooflines(tot_bytes, tot_fl, elapsed / args.steps, world)
    roofline = {
        # the roof this run is closer to: SURVEY §8(d)'s HBM roof, or the
        # measured fp64 VALU roof priced with the USEFUL flops (the scalar
        # algorithm's operation count; the issued lane-flops, idle lanes
        # included, are reported as issue-rate utilisation beside it)
        "bound": "fp64_valu" if fp is not None and fp["frac"] > hbm["frac"] else "hbm",
        "scope": "whole solve: algorithmic bytes of every kernel (SURVEY.md §8(d) per-node words x device-counted "
                 "calcDiffs / backward passes / line-search launches and step lengths, all ranks) / wall time "
                 "of the timed region",
        "achieved": hbm["achieved"],
        "peak": hbm["peak"],
        "unit": "GB/s",
        "frac": hbm["frac"],
        "traffic": (sum(v for v in traffic.values() if v) if traffic else None),
        "bytes_per_step": tot_bytes,
        "frac_survey_formula": tot_survey * args.steps / elapsed / 1e9 / (HBM_PEAK_GBS * world),
        "frac_of_measured_copy": tot_bytes * args.steps / elapsed / 1e9 / (HBM_MEASURED_GBS * world),
        "fp64": fp64_block(fp, tot_ufl, uf_unit, fpi, tot_fl),
        "dominant_kernel": dominant,
        # what the SQ counters of this configuration show limits the kernels
        # (profiles/sq_latest.json, when it is for this configuration)
        "limiter": sq_limiter(args.variant, args.contact, B, N) if world == 1 else None,
    }
    if dominant is not None and traffic and traffic.get(dominant["name"]) is not None:
        dominant["traffic_per_launch"] = traffic[dominant["name"]] / dominant["launches_per_solve"]

    extras = {}
    if not args.no_extras:
        # SURVEY-literal random x0 regime, a B-instance shard per rank
        rb = make(B, SEED + 1 + rank, "random")
        TR = tensors(rb)
        rsolver = solver
        rsolver.solve_dev(TR, maxiter=args.maxiter, stream=stream)
        sync()
        rs = 3
        el = shard.timed_steps(lambda: rsolver.solve_dev(TR, maxiter=args.maxiter, stream=stream), rs, sync)
        rok = float(shard.sum_over_ranks(torch.tensor([float(TR["ok"].sum().item())], **f64)).cpu()[0])
        rit = float(shard.sum_over_ranks(torch.tensor([float(TR["iters"].sum().item())], **f64)).cpu()[0])
        rstats = TR["stats"].cpu().numpy()
        rby = float(shard.sum_over_ranks(torch.tensor([solve_bytes(rstats, nx, nu, N)["total"]], **f64)).cpu()[0])
        rufl = useful_flops(rstats, N, uf_unit)
        if rufl is not None:
            rufl = float(shard.sum_over_ranks(torch.tensor([rufl], **f64)).cpu()[0])
        rh, rfp = rooflines(rby, rufl, el / rs, world)
        extras["random_regime"] = {"value": B * world * rs / el, "unit": "solves/s", "ms_per_step": el / rs * 1e3,
                                   "scaling": "weak", "ok_frac": rok / (B * world), "mean_iter": rit / (B * world),
                                   "roofline": dict(rh, bound="fp64_valu" if rfp and rfp["frac"] > rh["frac"] else "hbm",
                                                    bytes_per_step=rby,
                                                    fp64=fp64_block(rfp, rufl, uf_unit, None, None))}
        del TR
        if world > 1:
            # strong scaling: rank 0's B-instance batch split into contiguous
            # slices, one per rank (B / G instances per GPU: the latency end)
            b0, b1 = shard.slice_bounds(B, world, rank)
            sb = make(B, SEED, args.regime).slice(slice(b0, b1))
            TS = tensors(sb)
            scounts = shard.slice_counts(B, world)
            ssolver = BatchedBoxFDDP(cfg, max_batch=max(scounts), device=local_rank)
            sgather = shard.Gatherer(scounts, shard.pack_results(TS, args.gather).shape[1], dev) \
                if args.gather != "none" else None

            def sstep():
                ssolver.solve_dev(TS, maxiter=args.maxiter, stream=stream)
                if sgather is not None:
                    sgather(shard.pack_results(TS, args.gather))

            sstep()
            sync()
            ss = 3
            el = shard.timed_steps(sstep, ss, sync)
            sst = TS["stats"].cpu().numpy()
            sby = float(shard.sum_over_ranks(torch.tensor([solve_bytes(sst, nx, nu, N)["total"]], **f64)).cpu()[0])
            sh, _ = rooflines(sby, None, el / ss, world)
            extras["strong"] = {"metric": METRIC, "value": B * ss / el, "unit": "solves/s", "n_gpus": world,
                                "steps": ss, "ms_per_step": el / ss * 1e3, "higher_is_better": True,
                                "scaling": "strong", "global_batch": B, "batch_per_gpu": scounts,
                                "roofline": dict(sh, bound="hbm", bytes_per_step=sby),
                                "note": "one B-instance batch split into contiguous B/G slices (SURVEY §8(e)); "
                                        "the headline gives every GPU its own B-instance shard (weak)"}
            ssolver.close()
            del TS
        if not args.no_ff and args.variant == "classical":
            # the force-feedback variant (configs[2]'s model, nx = 21) at the
            # metric's batch and horizon: every rank its own B-instance shard
            fcfg = ff_preset(N, args.contact)
            fb = workload.make_batch(B, N, "ff", _abi.gravity_torque, ee, seed=SEED + 2 + rank, regime=args.regime,
                                     fk=_abi.frame_placement)
            TF = tensors(fb)
            for k, shp in (("xs", (B, N + 1, 21)), ("K", (B, N, nu, 21))):
                TF[k] = torch.zeros(shp, **f64)
            fsolver = BatchedBoxFDDP(fcfg, max_batch=B, device=local_rank)
            fsolver.solve_dev(TF, maxiter=args.maxiter, stream=stream)
            sync()
            fs_ = 3
            el = shard.timed_steps(lambda: fsolver.solve_dev(TF, maxiter=args.maxiter, stream=stream), fs_, sync)
            fst = TF["stats"].cpu().numpy()
            fok = float(shard.sum_over_ranks(torch.tensor([float(TF["ok"].sum().item())], **f64)).cpu()[0])
            fit = float(shard.sum_over_ranks(torch.tensor([float(TF["iters"].sum().item())], **f64)).cpu()[0])
            fby = float(shard.sum_over_ranks(torch.tensor([solve_bytes(fst, 21, nu, N)["total"]], **f64)).cpu()[0])
            ffl = fp64_flops(fst, N, _profile_json("fp64_latest_ff.json", "ff", args.contact, B, N))
            if ffl is not None:
                ffl = float(shard.sum_over_ranks(torch.tensor([ffl], **f64)).cpu()[0])
            fuf_unit = useful_per_unit("ff", args.contact, N)
            fufl = useful_flops(fst, N, fuf_unit)
            if fufl is not None:
                fufl = float(shard.sum_over_ranks(torch.tensor([fufl], **f64)).cpu()[0])
            fh, ffpu = rooflines(fby, fufl, el / fs_, world)
            _, ffpi = rooflines(fby, ffl, el / fs_, world)
            ffp = fp64_block(ffpu, fufl, fuf_unit, ffpi, ffl)
            extras["ff"] = {"value": B * world * fs_ / el, "unit": "solves/s", "ms_per_step": el / fs_ * 1e3,
                            "scaling": "weak", "workload": f"ForceFeedback (q,v,tau_hat)/w nx=21 nu=7, horizon={N}, "
                                                          f"batch={B} per GPU, maxiter={args.maxiter}, "
                                                          f"contact={args.contact}",
                            "ok_frac": fok / (B * world), "mean_iter": fit / (B * world),
                            "roofline": dict(fh, bound="fp64_valu" if ffp and ffp.get("frac", 0) > fh["frac"] else "hbm",
                                             bytes_per_step=fby, fp64=ffp)}
            fsolver.close()
            del TF

    host_io = None
    if not args.no_host_io and world == 1:
        # PCIe-inclusive rate of the host-array entry point (ffddp_solve_batch):
        # H2D of the inputs + solve + D2H of xs/us/K/cost/... per slice on the
        # slice streams; reported beside `value`, never as `value` (DESIGN.md
        # §7).  Always pageable numpy inputs (the workload's arrays, staged by
        # the library slice by slice while earlier slices run) except "pinned":
        #   default   BatchedBoxFDDP.solve() as a caller runs it: fresh output
        #             arrays per call, in page-locked memory recycled from
        #             earlier calls' arrays (outputs="recycled"), filled by DMA
        #   fresh     fresh pageable np.zeros output arrays per call (staged,
        #             first-touched while the device solves; rounds 1-5's value)
        #   pinned_outputs / pinned   solver-owned page-locked outputs (and
        #             page-locked inputs: a serving loop refilling its arrays)
        host_io = {"unit": "solves/s"}
        pinned = BatchedBoxFDDP(cfg, max_batch=max(counts), device=local_rank, outputs="pinned")
        fresh = BatchedBoxFDDP(cfg, max_batch=max(counts), device=local_rank, outputs="fresh")
        hsolver = BatchedBoxFDDP(cfg, max_batch=max(counts), device=local_rank)  # default outputs
        pin_in = pinned.pinned_batch(mine)
        for key, hs, inp in (("default", hsolver, mine), ("fresh", fresh, mine), ("pinned_outputs", pinned, mine),
                             ("pinned", pinned, pin_in)):
            hs.solve(inp, maxiter=args.maxiter)
            # median of 9 timed calls (single calls vary with host-side jitter)
            ts = []
            for _ in range(9):
                th0 = time.perf_counter()
                hs.solve(inp, maxiter=args.maxiter)
                ts.append(time.perf_counter() - th0)
            th = float(np.median(ts))
            host_io[key] = {"value": mine.B / th, "ms_per_step": th * 1e3, "reps": len(ts)}
        assert np.array_equal(pinned.xs, hsolver.xs) and np.array_equal(pinned.K, hsolver.K)
        assert np.array_equal(fresh.xs, hsolver.xs) and np.array_equal(fresh.K, hsolver.K)
        for hs in (pinned, fresh, hsolver):
            hs.close()
        del pin_in
        # value: the default solve() (pageable numpy inputs, fresh numpy
        # outputs); value_pinned: page-locked inputs and outputs
        host_io["value"] = host_io["default"]["value"]
        host_io["value_pinned"] = host_io["pinned"]["value"]

    if rank == 0:
        base = None
        if not args.no_cpu_baseline and world == 1:
            base = cpu_baseline(cfg, glob, args.maxiter, args.cpu_budget)
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
            "vs_baseline": None,  # BASELINE.md publishes no number for this metric
            "dtype": "f64",
            "data": f"synthetic (seeded workload.make_batch, {args.regime} regime"
                    + (": x0 near IK of the benchmark trajectory at t0~U(0,20)s" if args.regime == "tracking" else "")
                    + "; cold warm start)",
            "config": {
                "workload": f"{args.variant} BoxFDDP solve, nx={nx} nu={nu}, horizon={N}, batch={B} per GPU on "
                            f"{world} GPU(s) (global {B * world}), maxiter={args.maxiter}, contact={args.contact}",
                "variant": args.variant,
                "horizon": N,
                "global_batch": B * world,
                "batch_per_gpu": B,
                "maxiter": args.maxiter,
                "contact_model": args.contact,
                "parallelism": f"batch-shard{world}",
                "gather": args.gather if world > 1 else "none",
            },
            "roofline": roofline,
            "cpu_baseline": base,
            "counts_per_step": unit_counts,
            "solver": {
                "ok_frac": tot_ok / (B * world),
                "mean_iter": tot_it / (B * world),
                "rank0_mean_iters_run": float(np.mean(stats[:, 0])),
                "rank0_mean_trials": float(np.mean(stats[:, 1])),
                "rank0_mean_trials_evaluated": float(np.mean(stats[:, 6] + stats[:, 7])),
                "rank0_cost_finite_frac": float(np.mean(np.isfinite(cost))),
            },
            "kernels": kernels,
            "host_io": host_io,
            **extras,
        }
        print(json.dumps(line), flush=True)
    shard.shutdown()  # the reserved handle, then the process group


if __name__ == "__main__":
    main()
