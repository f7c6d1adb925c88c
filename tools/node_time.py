"""Time k_node alone: problem.calcDiff of a B-instance batch, 5 calls (run under
rocprofv3 --kernel-trace --stats).  usage: python tools/node_time.py [B]"""
import sys
import pathlib

sys.path.insert(0, str(pathlib.Path(__file__).resolve().parents[1]))
import ffddp_path  # noqa
import numpy as np
import torch  # noqa
from ffddp import BatchedBoxFDDP, _abi, workload, robot as R
from ffddp.config import classical_preset

B = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
N = 30
cfg = classical_preset(N)
ee = R.R_MJ_FROM_PIN @ _abi.frame_placement(R.Q_NEUTRAL)[1]
b = workload.make_batch(B, N, "classical", _abi.gravity_torque, ee, seed=1234, fk=_abi.frame_placement)
s = BatchedBoxFDDP(cfg, max_batch=B)
for _ in range(5):
    s.calc_diff(b, b.xs_init, b.us_init)
print("ok")
