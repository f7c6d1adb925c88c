#!/usr/bin/env python3
"""Golden files for the run-log format, produced by the
REFERENCE's own ``src/utils/logging.py::RunLogger`` (plain import, numpy only)
in this container.  Output: tests/golden/runlog/{a,b}/ with the data.csv,
meta.json (and for run a, data.npz) the reference wrote, plus rows.json
describing the logged rows so the test can replay them through
``ffddp.runlog.RunLogger``.

Run a logs numeric fields only (so its npz holds no object arrays and loads
with allow_pickle=False); run b adds strings, None, a 2-D array and a
long vector (CSV/meta only).

Run:  python tests/golden/make_runlog_golden.py   (needs /root/reference)
"""
from __future__ import annotations

import json
import shutil
import sys
import tempfile
from pathlib import Path

import numpy as np

REF = Path("/root/reference")
OUT = Path(__file__).resolve().parent / "runlog"


def rows_a(n=6):
    rng = np.random.default_rng(7)
    rows = []
    for k in range(n):
        rows.append(dict(
            t=0.005 * (k + 1),
            ee_pos=rng.normal(size=3),
            tau_cmd=rng.normal(size=7) * 10.0,
            err_tan=float(abs(rng.normal())),
            contact=int(k % 2),
            solver_iters=int(3 + k),
            fn_pred=float("nan") if k == 0 else float(rng.normal() * 20.0),
        ))
    return rows


def rows_b(n=4):
    rng = np.random.default_rng(11)
    rows = []
    for k in range(n):
        rows.append(dict(
            t=0.01 * k,
            label="flat" if k % 2 == 0 else "tilted",
            maybe=None,
            xs_block=rng.normal(size=(2, 3)),
            long_vec=rng.normal(size=12),
            q=rng.normal(size=7),
            ok=bool(k % 2),
        ))
    return rows


def to_json_rows(rows):
    out = []
    for r in rows:
        d = {}
        for k, v in r.items():
            if isinstance(v, np.ndarray):
                d[k] = {"ndarray": v.tolist()}
            else:
                d[k] = v
        out.append(d)
    return out


def main():
    sys.path.insert(0, str(REF))
    from src.utils.logging import RunLogger  # the reference implementation

    if OUT.exists():
        shutil.rmtree(OUT)
    notes = {"scenario": "flat", "dt": 0.005, "weights": np.array([1.0, 2.5]), "path": Path("/x/y"), "tup": (1, 2)}
    for name, rows, keep_npz in (("a", rows_a(), True), ("b", rows_b(), False)):
        with tempfile.TemporaryDirectory() as td:
            lg = RunLogger(f"golden_{name}", results_dir=td, notes=notes)
            for r in rows:
                lg.log(**r)
            lg.set_meta(total_time=1.25, torque_scale=np.ones(7), cfg_summary={"horizon": 30, "dt": 0.01})
            lg.save()
            dst = OUT / name
            dst.mkdir(parents=True)
            shutil.copy(lg.path_csv, dst / "data.csv")
            shutil.copy(lg.path_meta, dst / "meta.json")
            if keep_npz:
                shutil.copy(lg.path_npz, dst / "data.npz")
            (dst / "rows.json").write_text(json.dumps(to_json_rows(rows)))
    (OUT / "notes.json").write_text(json.dumps({"notes": {k: (v.tolist() if isinstance(v, np.ndarray) else
                                                              str(v) if isinstance(v, Path) else v)
                                                          for k, v in notes.items()}}))
    print("wrote", OUT)


if __name__ == "__main__":
    main()
