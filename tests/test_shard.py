"""world_size-2 gloo run of the sharded solve path (ffddp.shard) on CPU.

Each rank builds its own seeded shard, solves it (the numpy oracle stands in
for the HIP kernel here — there is no GPU in this test), all-gathers
(cost, u0) and times its steps with the bench fences.  Rank 0 checks that the
gathered block of every rank equals an independent recomputation of that
rank's shard, and that the timed elapsed is the max over ranks."""
from __future__ import annotations

import os
import socket
import sys
from pathlib import Path

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = Path(__file__).resolve().parents[1]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _solve_shard(rank, B, N):
    from helpers import make_batch, oracle_solve, product_cfg
    from ffddp import shard, workload  # noqa: F401

    cfg = product_cfg("classical", N)
    b = make_batch("classical", B, N, seed=shard.shard_seed(1234, rank))
    cost, u0 = np.zeros(B), np.zeros((B, 7))
    for i in range(B):
        _, s = oracle_solve(cfg, b, i, maxiter=2)
        cost[i], u0[i] = s.cost, s.us[0]
    return cost, u0


def _worker(rank, world, port, B, N, q):
    sys.path.insert(0, str(ROOT))
    sys.path.insert(0, str(ROOT / "tests"))
    import ffddp_path  # noqa: F401
    from ffddp import shard

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    r, w, lr = shard.env_ranks()
    shard.init("gloo", lr, w)
    try:
        cost, u0 = _solve_shard(r, B, N)
        out = shard.gather_results(torch.tensor(cost), torch.tensor(u0))
        slow = 0.3 if r == 1 else 0.0
        import time

        elapsed = shard.timed_steps(lambda: time.sleep(slow), 1, lambda: None)
        q.put((r, out.numpy(), elapsed))
    finally:
        dist.destroy_process_group()


def test_two_rank_gather_and_timing():
    world, B, N = 2, 2, 4
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, B, N, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        r, out, el = q.get(timeout=300)
        res[r] = (out, el)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    out0, el0 = res[0]
    out1, el1 = res[1]
    assert out0.shape == (world, B, 8)
    np.testing.assert_array_equal(out0, out1)
    for r in range(world):
        cost, u0 = _solve_shard(r, B, N)
        np.testing.assert_array_equal(out0[r, :, 0], cost)
        np.testing.assert_array_equal(out0[r, :, 1:], u0)
    # shards differ (distinct seeds) and the timing is the max over ranks
    assert not np.array_equal(out0[0], out0[1])
    assert el0 == el1 and el0 >= 0.3


def test_single_rank_passthrough():
    import ffddp_path  # noqa: F401
    from ffddp import shard

    out = shard.gather_results(torch.arange(3.0), torch.ones(3, 7))
    assert out.shape == (1, 3, 8)
    assert shard.shard_range(2, 4096) == (8192, 12288)
