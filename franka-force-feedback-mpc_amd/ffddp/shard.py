"""Multi-GPU partition of the batched solve.

The OCP instances of a batch are independent, so G GPUs (one process each)
solve shards of instances with no collective in the data path.  bench.py's
metric gives every rank its own B-instance shard (weak scaling: the task's
partitioned-path rule; BASELINE.json "batch=4096 at 1/2/4/8 MI355X" per
GPU); its "strong" extra field splits one B-instance batch into contiguous
slices (slice_bounds: the remainder goes to the last ranks).  The one
exchange is the final all-gather of the per-instance results over RCCL
(backend "nccl") on the GPU box, gloo in the CPU tests:
  * "costs" (default): cost, iterations, ok and the first control u0 of every
    instance — what a fleet-level MPC server returns to its callers;
  * "full": the whole solution, xs, us, K and cost (117 MB at B = 4096,
    N = 30), i.e. the reference solver's read-backs for every instance.
Slices are padded to the largest slice for all_gather_into_tensor and
unpadded in rank order.  Timing follows the bench contract: barrier + device
sync on both sides of the timed region, elapsed = max over ranks.
Replaces the single-process solve call at src/mpc/crocoddyl_classical.py:367.
"""
from __future__ import annotations

import os
import time
from typing import Callable, Dict, Sequence

import torch
import torch.distributed as dist


def env_ranks():
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", "0")))


_RESERVED = []  # keeps the slice streams' reference alive for the process


def prepare_device(local_rank: int):
    """The device, its null stream and the solver library's slice streams,
    created before the RCCL communicator: a process gets 4 hardware queues
    (GPU_MAX_HW_QUEUES) and the solver is tuned to one per slice, so its
    streams are claimed before RCCL creates its own.  On the round-5 head no
    creation order measured slower on one GPU (tools/nccl_queue.py,
    profiles/r05_nccl_queue.txt); the order is kept because
    it does not depend on how the runtime maps streams to queues.  A
    one-instance handle holds the library's per-device stream pool for the
    life of the process."""
    torch.cuda.set_device(local_rank)
    torch.zeros(1, device=torch.device("cuda", local_rank))
    if not _RESERVED:
        from .config import classical_preset
        from .solver import BatchedBoxFDDP

        _RESERVED.append(BatchedBoxFDDP(classical_preset(2, "normal_1d"), max_batch=1, device=local_rank))


def shutdown():
    """Close the handle prepare_device reserved (and with it the slice
    streams' last reference) and then the process group, so neither outlives
    the HIP runtime or RCCL at interpreter teardown.  Idempotent."""
    while _RESERVED:
        _RESERVED.pop().close()
    if dist.is_initialized():
        dist.destroy_process_group()


def init(backend: str, local_rank: int, world: int, force: bool = False):
    """Process group for world > 1 (MASTER_ADDR defaults to 127.0.0.1).
    force: a one-process group as well (an in-memory store), so that one GPU
    can rehearse the RCCL all-gather and its stream beside the solver's.
    nccl: prepare_device first (the solver's streams before RCCL's)."""
    if world <= 1 and not force:
        return
    if backend == "nccl":
        prepare_device(local_rank)
    if world <= 1:
        kw = dict(store=dist.HashStore(), rank=0, world_size=1)
        if backend == "nccl":
            torch.cuda.set_device(local_rank)
            dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank), **kw)
        else:
            dist.init_process_group(backend, **kw)
        return
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    if backend == "nccl":
        torch.cuda.set_device(local_rank)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
    else:
        dist.init_process_group(backend)


def slice_bounds(B: int, world: int, rank: int):
    """Contiguous slice [b0, b1) of a global batch of B instances for `rank`
    of `world`: floor(B / world) each, the remainder to the last ranks."""
    base, rem = divmod(int(B), int(world))
    extra_from = world - rem  # ranks >= extra_from get one more instance
    b0 = rank * base + max(0, rank - extra_from)
    return b0, b0 + base + (1 if rank >= extra_from else 0)


def slice_counts(B: int, world: int):
    return [slice_bounds(B, world, r)[1] - slice_bounds(B, world, r)[0] for r in range(world)]


def pack_results(res: Dict[str, torch.Tensor], mode: str) -> torch.Tensor:
    """Per-instance results -> one (B_local, W) float64 block.
    costs: [cost, iters, ok, u0(7)];  full: [cost, xs, us, K]."""
    B = res["cost"].shape[0]
    cost = res["cost"].reshape(B, 1).to(torch.float64)
    if mode == "costs":
        parts = [cost, res["iters"].reshape(B, 1).to(torch.float64), res["ok"].reshape(B, 1).to(torch.float64),
                 res["us"][:, 0, :].to(torch.float64)]
    elif mode == "full":
        parts = [cost] + [res[k].reshape(B, -1) for k in ("xs", "us", "K")]
    else:
        raise ValueError(mode)
    return torch.cat(parts, 1).contiguous()


def unpack_full(block: torch.Tensor, N: int, nx: int, nu: int = 7):
    """Inverse of pack_results(..., "full") on a gathered (B, W) block."""
    B = block.shape[0]
    o = 1
    xs = block[:, o:o + (N + 1) * nx].reshape(B, N + 1, nx)
    o += (N + 1) * nx
    us = block[:, o:o + N * nu].reshape(B, N, nu)
    o += N * nu
    K = block[:, o:o + N * nu * nx].reshape(B, N, nu, nx)
    return dict(cost=block[:, 0], xs=xs, us=us, K=K)


class Gatherer:
    """All-gather of the packed per-instance results of every rank's slice
    into the global batch order; buffers allocated once (bench reuses it
    every step)."""

    def __init__(self, counts: Sequence[int], width: int, device, dtype=torch.float64):
        self.counts = list(counts)
        self.world = len(self.counts)
        self.maxB = max(self.counts)
        self.send = torch.zeros((self.maxB, width), dtype=dtype, device=device)
        self.recv = torch.zeros((self.world, self.maxB, width), dtype=dtype, device=device)

    def __call__(self, local: torch.Tensor) -> torch.Tensor:
        n = local.shape[0]
        if self.world == 1 and not dist.is_initialized():
            return local
        self.send[:n].copy_(local)
        if dist.get_backend() == "nccl":
            dist.all_gather_into_tensor(self.recv, self.send)
        else:
            dist.all_gather(list(self.recv.unbind(0)), self.send)
        return torch.cat([self.recv[r, :c] for r, c in enumerate(self.counts)], 0)


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


def sum_over_ranks(x: torch.Tensor) -> torch.Tensor:
    """Element-wise sum over ranks (identity on one process)."""
    if dist.is_initialized() and dist.get_world_size() > 1:
        x = x.clone()
        dist.all_reduce(x, op=dist.ReduceOp.SUM)
    return x
