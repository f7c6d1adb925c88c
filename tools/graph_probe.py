#!/usr/bin/env python3
"""Does a captured HIP graph keep the 4 slice streams concurrent at large
batches?  Times one B-instance classical solve (N=30, tracking regime) three
ways on one GPU: the host-array entry point with page-locked inputs and
outputs, the solve plan (the same solve captured as one graph: copies up,
every kernel, copies down), and the device entry point (no copies).
Median of --reps calls each; one JSON line.
usage: python tools/graph_probe.py [--batch 4096] [--reps 9]"""
import argparse
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import ffddp_path  # noqa: E402,F401
import numpy as np  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--reps", type=int, default=9)
    a = ap.parse_args()
    import torch

    from ffddp import BatchedBoxFDDP, _abi, robot as R, workload
    from ffddp.config import classical_preset

    B, N = a.batch, 30
    cfg = classical_preset(N, "normal_1d")
    ee = R.R_MJ_FROM_PIN @ _abi.frame_placement(R.Q_NEUTRAL)[1]
    b = workload.make_batch(B, N, "classical", _abi.gravity_torque, ee, seed=1234, regime="tracking",
                            fk=_abi.frame_placement)
    s = BatchedBoxFDDP(cfg, max_batch=B, device=0, pinned_outputs=True)
    pin = s.pinned_batch(b)
    plan = s.plan(B, maxiter=10)
    for k in ("x0", "node_ref", "inst_ref", "surface", "xs_init", "us_init"):
        getattr(plan, k)[...] = getattr(pin, k)

    def med(fn):
        fn()
        ts = []
        for _ in range(a.reps):
            t0 = time.perf_counter()
            fn()
            ts.append(time.perf_counter() - t0)
        return float(np.median(ts)) * 1e3

    out = {"batch": B}
    out["host_pinned_ms"] = med(lambda: s.solve(pin, maxiter=10))
    xs_h = s.xs.copy()
    out["plan_ms"] = med(plan.run)
    out["plan_equal"] = bool(np.array_equal(plan.xs, xs_h))
    dev = torch.device("cuda", 0)
    f64 = dict(dtype=torch.float64, device=dev)
    T = dict(x0=torch.tensor(b.x0, **f64), node_ref=torch.tensor(b.node_ref, **f64),
             inst_ref=torch.tensor(b.inst_ref, **f64), surface=torch.tensor(b.surface, dtype=torch.uint8, device=dev),
             xs_init=torch.tensor(b.xs_init, **f64), us_init=torch.tensor(b.us_init, **f64),
             xs=torch.zeros((B, N + 1, 14), **f64), us=torch.zeros((B, N, 7), **f64),
             K=torch.zeros((B, N, 7, 14), **f64), cost=torch.zeros(B, **f64),
             iters=torch.zeros(B, dtype=torch.int32, device=dev), ok=torch.zeros(B, dtype=torch.uint8, device=dev),
             fn_pred=torch.zeros((B, 2), **f64), stats=torch.zeros((B, _abi.NSTATS), dtype=torch.int32, device=dev))
    stream = torch.cuda.current_stream(dev).cuda_stream

    def dev_solve():
        s.solve_dev(T, maxiter=10, stream=stream)
        torch.cuda.synchronize(dev)

    out["device_ms"] = med(dev_solve)
    plan.close()
    s.close()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
