"""world_size-2 gloo run of the partitioned solve path (ffddp.shard) on CPU.

One global batch of B instances is split into contiguous slices (remainder to
the last ranks); each rank solves its slice (the numpy oracle stands in for
the HIP kernel here — there is no GPU in this test), all-gathers the packed
results in both modes ("costs": cost, iters, ok, u0; "full": cost, xs, us,
K) and times its steps with the bench fences.  Rank 0 checks the gathered
global arrays against an independent single-process solve of the whole
batch, and that the timed elapsed is the max over ranks."""
from __future__ import annotations

import os
import socket
import sys
from pathlib import Path

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = Path(__file__).resolve().parents[1]
B_GLOBAL, N = 5, 4


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _solve(idx):
    """Oracle solves of global instances idx -> result tensors (the solver outputs bench gathers)."""
    from helpers import make_batch, oracle_solve, product_cfg

    cfg = product_cfg("classical", N)
    b = make_batch("classical", B_GLOBAL, N, seed=1234)
    res = dict(cost=[], iters=[], ok=[], xs=[], us=[], K=[])
    for i in idx:
        ok, s = oracle_solve(cfg, b, int(i), maxiter=2)
        for k, v in (("cost", s.cost), ("iters", s.iter), ("ok", ok), ("xs", s.xs), ("us", s.us), ("K", s.K)):
            res[k].append(v)
    return {k: torch.tensor(np.array(v, dtype=np.float64)) for k, v in res.items()}


def _worker(rank, world, port, q):
    sys.path.insert(0, str(ROOT))
    sys.path.insert(0, str(ROOT / "tests"))
    import ffddp_path  # noqa: F401
    from ffddp import shard

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    r, w, lr = shard.env_ranks()
    shard.init("gloo", lr, w)
    try:
        b0, b1 = shard.slice_bounds(B_GLOBAL, w, r)
        res = _solve(range(b0, b1))
        counts = shard.slice_counts(B_GLOBAL, w)
        out = {}
        for mode in ("costs", "full"):
            local = shard.pack_results(res, mode)
            out[mode] = shard.Gatherer(counts, local.shape[1], "cpu")(local).numpy()
        slow = 0.3 if r == 1 else 0.0
        import time

        elapsed = shard.timed_steps(lambda: time.sleep(slow), 1, lambda: None)
        tot = shard.sum_over_ranks(torch.tensor([float(b1 - b0)])).item()
        q.put((r, (b0, b1), out, elapsed, tot))
    finally:
        shard.shutdown()


def test_two_rank_strong_split_and_gathers():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        r, bounds, out, el, tot = q.get(timeout=300)
        res[r] = (bounds, out, el, tot)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    # contiguous slices covering the global batch, remainder on the last rank
    assert res[0][0] == (0, 2) and res[1][0] == (2, 5)
    assert res[0][3] == res[1][3] == B_GLOBAL
    from ffddp import shard

    ref = _solve(range(B_GLOBAL))
    for r in range(world):
        out = res[r][1]
        assert out["costs"].shape == (B_GLOBAL, 10)
        assert out["full"].shape == (B_GLOBAL, 1 + (N + 1) * 14 + N * 7 + N * 7 * 14)
        np.testing.assert_array_equal(out["costs"][:, 0], ref["cost"].numpy())
        np.testing.assert_array_equal(out["costs"][:, 1], ref["iters"].numpy())
        np.testing.assert_array_equal(out["costs"][:, 3:], ref["us"].numpy()[:, 0])
        full = shard.unpack_full(torch.tensor(out["full"]), N, 14)
        for k in ("cost", "xs", "us", "K"):
            np.testing.assert_array_equal(full[k].numpy(), ref[k].numpy())
    # the timing is the max over ranks
    assert res[0][2] == res[1][2] and res[0][2] >= 0.3


def test_slice_bounds_partition():
    from ffddp import shard

    for B in (1, 7, 512, 4096, 4097):
        for world in (1, 2, 3, 4, 8):
            b = [shard.slice_bounds(B, world, r) for r in range(world)]
            assert b[0][0] == 0 and b[-1][1] == B
            assert all(b[r][1] == b[r + 1][0] for r in range(world - 1))
            c = shard.slice_counts(B, world)
            assert max(c) - min(c) <= 1 and c == sorted(c)  # remainder on the last ranks
    assert shard.slice_bounds(4096, 8, 3) == (1536, 2048)


def test_single_rank_passthrough():
    from ffddp import shard

    res = dict(cost=torch.arange(3.0), iters=torch.ones(3), ok=torch.ones(3), us=torch.ones(3, 4, 7))
    local = shard.pack_results(res, "costs")
    assert local.shape == (3, 10)
    assert torch.equal(shard.Gatherer([3], 10, "cpu")(local), local)


def _forced_worker(q):
    sys.path.insert(0, str(ROOT))
    import ffddp_path  # noqa: F401
    from ffddp import shard

    shard.init("gloo", 0, 1, force=True)  # bench --force-collective at one process
    try:
        assert dist.is_initialized() and dist.get_world_size() == 1
        local = torch.arange(12, dtype=torch.float64).reshape(3, 4)
        g = shard.Gatherer([3], 4, torch.device("cpu"))
        out = g(local)
        # the collective ran (the gather went through the process group's
        # buffers, not the one-process shortcut) and kept the rows
        res = (bool(torch.equal(out, local)), bool(torch.equal(g.recv[0], local)))
    finally:
        shard.shutdown()  # bench's exit path: the process group goes (idempotent)
    shard.shutdown()
    q.put(res + (not dist.is_initialized(),))


def test_forced_one_process_group():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_forced_worker, args=(q,))
    p.start()
    p.join(120)
    assert p.exitcode == 0
    assert q.get(timeout=5) == (True, True, True)
