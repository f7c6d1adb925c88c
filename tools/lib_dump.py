"""Solve fixed seeded batches (classical and FF, tracking and random x0) with
the library FFDDP_LIB points at and save the results, so two library builds
can be compared bit for bit:
  FFDDP_LIB=.../base/libffddp.so python tools/lib_dump.py a.npz
  python tools/lib_dump.py b.npz
  python tools/lib_dump.py --compare a.npz b.npz"""
import sys
import pathlib

sys.path.insert(0, str(pathlib.Path(__file__).resolve().parents[1]))
sys.path.insert(0, str(pathlib.Path(__file__).resolve().parents[1] / "tests"))
import numpy as np

if sys.argv[1] == "--compare":
    a, b = np.load(sys.argv[2]), np.load(sys.argv[3])
    for k in a.files:
        x, y = a[k], b[k]
        same = np.array_equal(x, y, equal_nan=True)
        d = float(np.nanmax(np.abs(x.astype(np.float64) - y.astype(np.float64)))) if x.size else 0.0
        print(f"{k:28s} {'identical' if same else 'DIFFERS'}  max abs diff {d:.3e}")
    sys.exit(0)

import ffddp_path  # noqa
from ffddp import BatchedBoxFDDP
from helpers import make_batch, product_cfg

out = {}
for variant, B, regime in (("classical", 512, "tracking"), ("classical", 1024, "random"), ("ff", 256, "tracking")):
    cfg = product_cfg(variant, 30)
    b = make_batch(variant, B, 30, seed=91, regime=regime)
    s = BatchedBoxFDDP(cfg, max_batch=B)
    s.solve(b, maxiter=10)
    for name in ("xs", "us", "K", "cost", "iter", "ok", "stats"):
        out[f"{variant}_{regime}_{name}"] = np.array(getattr(s, name))
    s.close()
np.savez(sys.argv[1], **out)
print("saved", sys.argv[1])
