"""Multi-GPU sharding of the batched solve.

The OCP instances of a batch are independent, so N GPUs run N disjoint shards
(one process per GPU, instance ids rank*B .. rank*B+B-1) with no collective in
the data path.  The one exchange is the final all-gather of each instance's
(cost, u0) — what a fleet-level MPC server returns to its callers — over RCCL
(backend "nccl") on the GPU box, over gloo in the CPU tests.  Timing follows
the bench contract: barrier + device sync on both sides of the timed region,
elapsed = max over ranks.
"""
from __future__ import annotations

import os
import time
from typing import Callable, Optional

import torch
import torch.distributed as dist


def env_ranks():
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", "0")))


def init(backend: str, local_rank: int, world: int):
    """Process group for world > 1 (MASTER_ADDR defaults to 127.0.0.1)."""
    if world <= 1:
        return
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    if backend == "nccl":
        torch.cuda.set_device(local_rank)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
    else:
        dist.init_process_group(backend)


def shard_seed(base: int, rank: int) -> int:
    return base + rank


def shard_range(rank: int, per_rank: int):
    return rank * per_rank, (rank + 1) * per_rank


def gather_results(cost: torch.Tensor, u0: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """All-gather [cost | u0] of every shard -> (world, B, 1 + nu), rank order."""
    local = torch.cat([cost[:, None], u0], 1).contiguous()
    world = dist.get_world_size() if dist.is_initialized() else 1
    if world == 1:
        return local[None]
    if out is None:
        out = torch.empty((world,) + tuple(local.shape), dtype=local.dtype, device=local.device)
    if dist.get_backend() == "nccl":
        dist.all_gather_into_tensor(out, local)
    else:
        parts = list(out.unbind(0))
        dist.all_gather(parts, local)
    return out


def timed_steps(step: Callable[[], None], steps: int, sync: Callable[[], None]) -> float:
    """Run `steps` calls of step() between barrier+sync fences; max elapsed over ranks (s)."""
    multi = dist.is_initialized() and dist.get_world_size() > 1
    if multi:
        dist.barrier()
    sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    sync()
    if multi:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if multi:
        dev = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend() == "nccl" else torch.device("cpu")
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    return elapsed
