"""GPU leg of tools/ext_budget.py: solve the error-budget cases through the
HIP library and save xs / us / K / cost to an npz (run on the GPU box).
usage: python tools/ext_budget_gpu.py OUT.npz"""
from __future__ import annotations

import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tools"))
sys.path.insert(0, str(ROOT / "tests"))
import ffddp_path  # noqa: E402,F401
import numpy as np  # noqa: E402

from ext_budget import CASES, case_inputs  # noqa: E402
from ffddp import BatchedBoxFDDP  # noqa: E402

out = {}
for case in CASES:
    cfg, b = case_inputs(case)
    s = BatchedBoxFDDP(cfg, max_batch=b.B)
    s.solve(b, maxiter=10, is_feasible=False)
    for k in ("xs", "us", "K", "cost"):
        out[f"{case[0]}/{k}"] = np.array(getattr(s, k))
    s.close()
np.savez(sys.argv[1], **out)
print("saved", len(out), "arrays")
