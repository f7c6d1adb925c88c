"""Per-iteration line-search statistics of the bench batch: for iteration k,
how many step lengths each still-active instance tried (1 = alpha 1 accepted,
..., 10 with none accepted).  Solves with maxiter = 1..10 replay the same
deterministic iterations; the difference of the device-counted trials gives
iteration k's count.  usage: python tools/accept_hist.py [B] [variant] [save.npy]
(REGIME=random for the random-x0 draw)"""
import sys
import pathlib

sys.path.insert(0, str(pathlib.Path(__file__).resolve().parents[1]))
import ffddp_path  # noqa
import numpy as np
import torch  # noqa
from ffddp import BatchedBoxFDDP, _abi, workload, robot as R
from ffddp.config import classical_preset, ff_preset

B = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
variant = sys.argv[2] if len(sys.argv) > 2 else "classical"
N = 30
cfg = ff_preset(N) if variant == "ff" else classical_preset(N)
ee = R.R_MJ_FROM_PIN @ _abi.frame_placement(R.Q_NEUTRAL)[1]
b = workload.make_batch(B, N, variant, _abi.gravity_torque, ee, seed=1234, fk=_abi.frame_placement,
                        regime=__import__("os").environ.get("REGIME", "tracking"))
s = BatchedBoxFDDP(cfg, max_batch=B)
prev_tr = np.zeros(B, np.int64)
hist = np.zeros((10, B), np.int64)  # per-instance tried count per iteration (0: did not run)
prev_fw = np.zeros(B, np.int64)
for k in range(1, 11):
    s.solve(b, maxiter=k)
    st = np.asarray(s.stats).astype(np.int64)
    tr, fw = st[:, 1], st[:, 5]
    ran = fw > prev_fw  # instances that ran the forward pass of iteration k-1
    d = (tr - prev_tr)[ran]
    hist[k - 1][ran] = d
    h = np.bincount(d, minlength=11)[1:11]
    print(f"iter {k - 1}: active {int(ran.sum()):5d}  tried-count hist (1..10) {h.tolist()}  "
          f"need>4: {int((d > 4).sum())}  need>1: {int((d > 1).sum())}")
    prev_tr, prev_fw = tr, fw
if len(sys.argv) > 3:
    np.save(sys.argv[3], hist)
