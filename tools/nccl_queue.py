#!/usr/bin/env python3
"""One GPU: does an RCCL communicator in the process slow the solver's four
slice streams (4 hardware queues per process, GPU_MAX_HW_QUEUES)?  Runs one
configuration per process (--mode):
  none         no process group (the one-GPU bench)
  rccl_raw     one-process nccl group created first by init_process_group
               itself (no shard.prepare_device), then the solver: the
               order without the fix
  rccl_first   one-process nccl group through shard.init (which creates the
               solver's slice streams first), then the solver
  solver_first the solver's slice streams created (one warm-up solve) before
               the nccl group
and prints solves/s of B instances for --gather none / costs / full.
usage: python tools/nccl_queue.py --mode rccl_first --batch 4096 --gather none"""
import argparse
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import ffddp_path  # noqa: E402,F401


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mode", choices=("none", "rccl_raw", "rccl_first", "solver_first", "bench_order", "bench_touch",
                                       "bench_solver"), required=True)
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--gather", choices=("none", "costs", "full"), default="none")
    ap.add_argument("--steps", type=int, default=20)
    a = ap.parse_args()
    import torch
    import torch.distributed as dist

    from ffddp import BatchedBoxFDDP, _abi, robot as R, shard, workload
    from ffddp.config import classical_preset

    import os
    aff0 = len(os.sched_getaffinity(0))
    # bench_order: the process group before anything else (bench.py up to
    # round 5); bench_touch: one device tensor first (the null stream in
    # use); bench_solver: the solver handle first (its slice streams)
    if a.mode == "bench_touch":
        torch.cuda.set_device(0)
        torch.zeros(1, device="cuda:0")
    if a.mode == "bench_solver":
        cfg0 = classical_preset(30, "normal_1d")
        solver0 = BatchedBoxFDDP(cfg0, max_batch=a.batch, device=0)
    if a.mode in ("bench_order", "bench_touch", "bench_solver"):
        shard.init("nccl", 0, 1, force=True)
    aff1 = len(os.sched_getaffinity(0))
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    B, N = a.batch, 30
    cfg = classical_preset(N, "normal_1d")
    ee = R.R_MJ_FROM_PIN @ _abi.frame_placement(R.Q_NEUTRAL)[1]
    b = workload.make_batch(B, N, "classical", _abi.gravity_torque, ee, seed=1234, regime="tracking",
                            fk=_abi.frame_placement)
    f64 = dict(dtype=torch.float64, device=dev)
    T = dict(x0=torch.tensor(b.x0, **f64), node_ref=torch.tensor(b.node_ref, **f64),
             inst_ref=torch.tensor(b.inst_ref, **f64), surface=torch.tensor(b.surface, dtype=torch.uint8, device=dev),
             xs_init=torch.tensor(b.xs_init, **f64), us_init=torch.tensor(b.us_init, **f64),
             xs=torch.zeros((B, N + 1, 14), **f64), us=torch.zeros((B, N, 7), **f64),
             K=torch.zeros((B, N, 7, 14), **f64), cost=torch.zeros(B, **f64),
             iters=torch.zeros(B, dtype=torch.int32, device=dev), ok=torch.zeros(B, dtype=torch.uint8, device=dev),
             fn_pred=torch.zeros((B, 2), **f64), stats=torch.zeros((B, _abi.NSTATS), dtype=torch.int32, device=dev))
    stream = torch.cuda.current_stream(dev).cuda_stream
    solver = None
    if a.mode == "solver_first":
        solver = BatchedBoxFDDP(cfg, max_batch=B, device=0)
        solver.solve_dev(T, stream=stream)
        torch.cuda.synchronize(dev)
    if a.mode in ("rccl_first", "solver_first"):
        shard.init("nccl", 0, 1, force=True)
    if a.mode == "rccl_raw":
        dist.init_process_group("nccl", device_id=dev, store=dist.HashStore(), rank=0, world_size=1)
    aff2 = len(os.sched_getaffinity(0))
    if a.mode == "bench_solver":
        solver = solver0
    if solver is None:
        solver = BatchedBoxFDDP(cfg, max_batch=B, device=0)
    gather = None
    if a.mode != "none" and a.gather != "none":
        gather = shard.Gatherer([B], shard.pack_results(T, a.gather).shape[1], dev)

    def step():
        solver.solve_dev(T, stream=stream)
        if gather is not None:
            gather(shard.pack_results(T, a.gather))

    for _ in range(3):
        step()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    enq = 0.0
    for _ in range(a.steps):
        te = time.perf_counter()
        step()
        enq += time.perf_counter() - te
    torch.cuda.synchronize(dev)
    el = time.perf_counter() - t0
    print(json.dumps({"mode": a.mode, "batch": B, "gather": a.gather, "value": B * a.steps / el,
                      "ms_per_step": el / a.steps * 1e3, "host_enqueue_ms_per_step": enq / a.steps * 1e3,
                      "affinity_cpus": [aff0, aff1, aff2]}))
    if dist.is_initialized():
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
