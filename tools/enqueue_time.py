"""Host enqueue time of one ffddp_solve_batch_dev call vs its GPU time, at
batch B (is the solve launch-bound on the host?).  usage: enqueue_time.py B"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import ffddp_path  # noqa: F401,E402
import numpy as np
import torch

from ffddp import BatchedBoxFDDP, _abi, robot as R, workload
from ffddp.config import classical_preset


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 512
    N = 30
    cfg = classical_preset(N, "normal_1d")
    ee = R.R_MJ_FROM_PIN @ _abi.frame_placement(R.Q_NEUTRAL)[1]
    b = workload.make_batch(B, N, "classical", _abi.gravity_torque, ee, seed=1234, regime="tracking",
                            fk=_abi.frame_placement)
    dev = torch.device("cuda", 0)
    f64 = dict(dtype=torch.float64, device=dev)
    T = dict(x0=torch.tensor(b.x0, **f64), node_ref=torch.tensor(b.node_ref, **f64),
             inst_ref=torch.tensor(b.inst_ref, **f64), surface=torch.tensor(b.surface, dtype=torch.uint8, device=dev),
             xs_init=torch.tensor(b.xs_init, **f64), us_init=torch.tensor(b.us_init, **f64),
             xs=torch.zeros((B, N + 1, 14), **f64), us=torch.zeros((B, N, 7), **f64),
             K=torch.zeros((B, N, 7, 14), **f64), cost=torch.zeros(B, **f64),
             iters=torch.zeros(B, dtype=torch.int32, device=dev), ok=torch.zeros(B, dtype=torch.uint8, device=dev),
             fn_pred=torch.zeros((B, 2), **f64), stats=torch.zeros((B, _abi.NSTATS), dtype=torch.int32, device=dev))
    s = BatchedBoxFDDP(cfg, max_batch=B)
    st = torch.cuda.current_stream(dev).cuda_stream
    for _ in range(3):
        s.solve_dev(T, maxiter=10, stream=st)
    torch.cuda.synchronize()
    enq, tot = [], []
    for _ in range(10):
        t0 = time.perf_counter()
        s.solve_dev(T, maxiter=10, stream=st)
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        enq.append(t1 - t0)
        tot.append(t2 - t0)
    # back-to-back (host may run ahead)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(10):
        s.solve_dev(T, maxiter=10, stream=st)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"B={B}: enqueue {np.median(enq)*1e3:.3f} ms, enqueue+run {np.median(tot)*1e3:.3f} ms per solve; "
          f"10 back-to-back: enqueue {(t1-t0)*1e2:.3f} ms/solve, total {(t2-t0)*1e2:.3f} ms/solve")
    s.close()


if __name__ == "__main__":
    main()
