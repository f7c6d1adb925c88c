"""Solver-work histogram of the bench batch: how many instances are still
active at each FDDP iteration (per sub-batch slice), line-search trials and
backward retries.  usage: python tools/iter_hist.py [B] [variant] [regime]"""
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
regime = sys.argv[3] if len(sys.argv) > 3 else "tracking"
N = 30
cfg = ff_preset(N) if variant == "ff" else classical_preset(N)
ee = R.R_MJ_FROM_PIN @ _abi.frame_placement(R.Q_NEUTRAL)[1]
b = workload.make_batch(B, N, variant, _abi.gravity_torque, ee, seed=1234, regime=regime, fk=_abi.frame_placement)
s = BatchedBoxFDDP(cfg, max_batch=B)
s.solve(b, maxiter=10)
st = np.asarray(s.stats)
it = st[:, 0]
print("iterations run: mean %.2f" % it.mean(), "hist", np.bincount(it, minlength=11).tolist())
print("backward passes: mean %.2f retries: mean %.3f max %d" % (st[:, 3].mean(), st[:, 2].mean(), st[:, 2].max()))
print("trials: mean per instance %.2f, per forward %.2f" % (st[:, 1].mean(), st[:, 1].sum() / max(1, st[:, 5].sum())))
nsl = 3
for sl in range(nsl):
    lo, hi = sl * B // nsl, (sl + 1) * B // nsl
    act = [int(np.sum(it[lo:hi] > k)) for k in range(10)]
    print(f"slice {sl}: active per iteration", act)
print("ok frac %.3f" % np.mean(s.ok))
