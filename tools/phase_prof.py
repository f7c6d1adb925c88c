"""Per-phase shader-clock breakdown of instance 0 (build with EXTRA=-DFFDDP_PHASE_PROF)."""
import ctypes as C
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
names = sys.argv[3].split(",") if len(sys.argv) > 3 and sys.argv[3] else [f"p{i}" for i in range(8)]
regime = sys.argv[4] if len(sys.argv) > 4 else "tracking"
N = 30
cfg = ff_preset(N) if variant == "ff" else classical_preset(N)
ee = R.R_MJ_FROM_PIN @ _abi.frame_placement(R.Q_NEUTRAL)[1]
b = workload.make_batch(B, N, variant, _abi.gravity_torque, ee, seed=1234, regime=regime, fk=_abi.frame_placement)
s = BatchedBoxFDDP(cfg, max_batch=B)
lib = _abi.load()
f = lib.ffddp_debug_phase_read
f.argtypes = [C.POINTER(C.c_ulonglong), C.c_int, C.c_int]
buf = (C.c_ulonglong * 48)()
s.solve(b, maxiter=10)
f(buf, 48, 1)
s.solve(b, maxiter=10)
f(buf, 48, 1)
st = s.stats[0]
nodes = int(st[3]) * N  # backward passes x nodes
print("instance 0: iters", s.iter[0], "backward passes", st[3], "forward passes", st[5])
bw = ["stage", "A", "B", "C", "D", "E", "F", "G"]
tot = sum(buf[i] for i in range(8))
for i, n in enumerate(bw):
    print(f"  bw {n:8s} {buf[i] / max(1, nodes):10.0f} cycles/node  {100.0 * buf[i] / max(1, tot):5.1f} %")
fw = ["FK", "vel/acc", "EE", "forces", "CRBA", "chol+solve", "contact", "euler+cost", "loop", "tail"]
fnodes = int(st[5]) * (N + 1)
tot = sum(buf[16 + i] for i in range(len(fw)))
for i, n in enumerate(fw):
    print(f"  fw {n:10s} {buf[16 + i] / max(1, fnodes):10.0f} cycles/node  {100.0 * buf[16 + i] / max(1, tot):5.1f} %")
if buf[8]:
    print(f"  bw2 wave 0 staging (in 'stage') {buf[8] / max(1, int(st[3]) * N):10.0f} cycles/node")
if buf[28] or buf[29]:
    bnodes = int(st[3]) * N
    print(f"  bw2 phase D, wave 0 (gains)      {buf[28] / max(1, bnodes):10.0f} cycles/node")
    print(f"  bw2 phase D, wave 1 (stage + spec) {buf[29] / max(1, bnodes):10.0f} cycles/node")
if any(buf[32 + i] for i in range(8)):
    bnodes = int(st[3]) * N
    its, facts = buf[38], buf[39]
    print(f"  BoxQP (two-wave backward, instance 0): {its / max(1, bnodes):.2f} iterations and {facts / max(1, bnodes):.2f} factorisations per node")
    for i, n in enumerate(["gradient+fold+set", "factorisation", "solve", "convergence test", "line search", "early-exit test"]):
        print(f"    {n:20s} {buf[32 + i] / max(1, bnodes):8.0f} cycles/node")
