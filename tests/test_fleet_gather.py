"""world_size-2 gloo run of the fleet sweep's exchange (ffddp.fleet.gather_summaries)
and of its instance sharding / per-scenario table, on CPU.  Each rank fakes its
shard's per-instance summaries as a known function of the global instance id;
rank 0 checks the gathered matrix is in instance order and the table's
statistics."""
from __future__ import annotations

import os
import socket
import sys
from pathlib import Path

import numpy as np
import torch.multiprocessing as mp

ROOT = Path(__file__).resolve().parents[1]
SCEN = ("flat", "tilted_5", "tilted_10", "tilted_15", "actuation_uncertainty")


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, seeds, q):
    sys.path.insert(0, str(ROOT))
    import ffddp_path  # noqa: F401
    import torch.distributed as dist
    from ffddp import fleet, shard

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    shard.init("gloo", rank, world)
    try:
        names, _, _, seed = fleet._sweep_instances(SCEN, seeds)
        n_all = len(names)
        per = (n_all + world - 1) // world
        lo, hi = rank * per, min(n_all, (rank + 1) * per)
        ids = np.arange(lo, hi, dtype=float)
        res = {"per_instance": {k: ids * 10 + j for j, k in enumerate(fleet.SUMMARY_KEYS)}}
        m = fleet.gather_summaries(res, n_all)
        if rank == 0:
            q.put((m, list(names), fleet.scenario_table(names, m)))
    finally:
        dist.destroy_process_group()


def test_gather_summaries_two_ranks():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    seeds = 5  # 25 instances: uneven shards (13 + 12)
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, seeds, q)) for r in range(2)]
    for p in procs:
        p.start()
    m, names, table = q.get(timeout=120)
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    n = len(names)
    from ffddp import fleet

    nk = len(fleet.SUMMARY_KEYS)
    assert m.shape == (n, nk)
    ids = np.arange(n, dtype=float)
    for j in range(nk):
        np.testing.assert_array_equal(m[:, j], ids * 10 + j)
    assert list(table) == list(SCEN)
    assert table["flat"]["instances"] == seeds
    assert table["tilted_5"]["rms_tangential_error"]["mean"] == np.mean(ids[5:10] * 10)


def test_sweep_instances_layout():
    sys.path.insert(0, str(ROOT))
    from ffddp import fleet

    names, tilt, scale, seed = fleet._sweep_instances(SCEN, 256)
    assert len(names) == 1280 and list(names[:2]) == ["flat", "flat"] and names[-1] == "actuation_uncertainty"
    assert tilt[256] == 5.0 and tilt[3 * 256] == 15.0 and scale[-1][1] == 1.08
    assert len(set(seed.tolist())) == 1280
