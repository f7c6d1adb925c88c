#!/usr/bin/env python3
"""BASELINE configs[3]: all 5 scenarios x 256 seeds = 1280 closed-loop runs,
sharded over the ranks (one process per GPU, torchrun), each rank stepping its
shard as one fleet (FleetClassicalMPC + BatchedPlant); RCCL all-gather of the
per-instance summaries; rank 0 prints one JSON line (per-scenario statistics,
wall time, closed-loop ticks/s).

  python tools/sweep_c4.py [--seeds 256] [--time 4]            # 1 GPU
  torchrun --nproc-per-node 8 --master-addr 127.0.0.1 tools/sweep_c4.py
"""
import argparse
import json
import os
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import ffddp_path  # noqa: E402,F401


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seeds", type=int, default=256)
    ap.add_argument("--time", type=float, default=4.0)
    ap.add_argument("--out", type=str, default="")
    ap.add_argument("--neg-step-rule", type=int, choices=(0, 1), default=0,
                    help="ascent-direction comparator: 0 Crocoddyl's (default), 1 bounded rise")
    a = ap.parse_args()
    import torch
    import torch.distributed as dist
    from ffddp import fleet, shard

    rank, world, local = shard.env_ranks()
    shard.init("nccl", local, world)
    torch.cuda.set_device(local)
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    res = fleet.run_sweep(seeds=a.seeds, total_time=a.time, rank=rank, world=world, device=local, verbose=(rank == 0),
                           neg_step_rule=a.neg_step_rule)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    wall = time.perf_counter() - t0
    m = fleet.gather_summaries(res, res["n_all"], device=torch.device("cuda", local))
    names, _, _, _ = fleet._sweep_instances(("flat", "tilted_5", "tilted_10", "tilted_15", "actuation_uncertainty"),
                                            a.seeds)
    if rank == 0:
        line = {"config": "5 scenarios x %d seeds closed loop, %.1f s each" % (a.seeds, a.time), "ranks": world,
                "neg_step_rule": a.neg_step_rule,
                "instances": int(res["n_all"]), "ticks": res["ticks"], "wall_s": wall,
                "closed_loop_ticks_per_s": res["n_all"] * res["ticks"] / wall,
                "rank0_controller_s": res["controller_s"], "scenarios": fleet.scenario_table(names, m)}
        print(json.dumps(line), flush=True)
        if a.out:
            Path(a.out).write_text(json.dumps(line, indent=1))
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
