"""Run log and closed-loop summary metrics.

Mirrors the reference's on-disk run format so its plotting/evaluation
scripts read our runs unchanged:

* ``RunLogger``  — reference ``src/utils/logging.py:33-151``: one row per
  control tick via ``log(**fields)``, ``set_meta(**fields)``, and ``save()``
  writing ``<results>/logs/<stamp>_<name>/{data.npz, data.csv, meta.json}``.
    - data.npz: every key (sorted) stacked over rows; ndarray rows are
      stacked along axis 0, anything else becomes a float array, and what
      cannot be a float array an object array of JSON-able values.
    - data.csv: one column per scalar key, ``k[i]`` columns for 1-D arrays of
      at most 10 entries, and a JSON-able cell for anything larger.
    - meta.json: run_name, timestamp, notes + set_meta fields, indent 2.
* ``summary_metrics`` — the end-of-run statistics of
  ``run_classical.py:513-535`` (and the identical block of
  ``run_force_feedback.py``), returned as the dict ``set_meta`` receives.
"""
from __future__ import annotations

import csv
import dataclasses
import json
import time
from pathlib import Path
from typing import Any, Dict, Optional

import numpy as np

__all__ = ["RunLogger", "jsonable", "summary_metrics"]


def jsonable(x: Any) -> Any:
    """JSON-friendly copy of ``x`` (reference ``_to_jsonable``, logging.py:13-30):
    dataclasses -> dict, Path -> str, containers recursively, ndarray -> list,
    JSON scalars unchanged, anything else -> ``str(x)``."""
    if x is None or isinstance(x, (str, bool, int, float)):
        return x
    if dataclasses.is_dataclass(x) and not isinstance(x, type):
        return dataclasses.asdict(x)
    if isinstance(x, Path):
        return str(x)
    if isinstance(x, dict):
        return {str(k): jsonable(v) for k, v in x.items()}
    if isinstance(x, (list, tuple)):
        return [jsonable(v) for v in x]
    if isinstance(x, np.ndarray):
        return x.tolist()
    return str(x)


def _csv_kind(v: Any) -> int:
    """0: one scalar cell, 1: flattened short vector, 2: one JSON-able cell."""
    if v is None or np.isscalar(v):
        return 0
    if isinstance(v, np.ndarray) and v.ndim == 1 and v.size <= 10:
        return 1
    return 2


class RunLogger:
    """Per-tick run log with the reference's directory layout and file formats.

    ``RunLogger(run_name, results_dir="results", notes=None, overwrite=False)``
    creates ``results_dir/logs/<YYYYmmdd_HHMMSS>_<run_name>/`` immediately and
    raises ``FileExistsError`` if it exists and ``overwrite`` is False
    (logging.py:40-61).
    """

    def __init__(self, run_name: str, results_dir: Path | str = "results", notes: Optional[Dict[str, Any]] = None,
                 overwrite: bool = False):
        self.results_dir = Path(results_dir)
        self.logs_dir = self.results_dir / "logs"
        self.logs_dir.mkdir(parents=True, exist_ok=True)
        stamp = time.strftime("%Y%m%d_%H%M%S")
        self.run_dir = self.logs_dir / f"{stamp}_{run_name}"
        if self.run_dir.exists() and not overwrite:
            raise FileExistsError(f"Run dir exists: {self.run_dir}")
        self.run_dir.mkdir(parents=True, exist_ok=True)
        self._rows: list = []
        self.meta: Dict[str, Any] = {"run_name": run_name, "timestamp": stamp, "notes": jsonable(notes or {})}

    @property
    def path_npz(self) -> Path:
        return self.run_dir / "data.npz"

    @property
    def path_csv(self) -> Path:
        return self.run_dir / "data.csv"

    @property
    def path_meta(self) -> Path:
        return self.run_dir / "meta.json"

    def __len__(self) -> int:
        return len(self._rows)

    def log(self, **fields: Any) -> None:
        """Append one control tick (arrays are kept as given)."""
        self._rows.append(fields)

    def set_meta(self, **fields: Any) -> None:
        self.meta.update(jsonable(fields))

    # -- file writers ---------------------------------------------------------
    def _column(self, key: str):
        vals = [row.get(key) for row in self._rows]
        if isinstance(vals[0], np.ndarray):
            try:
                return np.stack(vals, axis=0)
            except (ValueError, TypeError):
                pass
        try:
            return np.array(vals, dtype=float)
        except (ValueError, TypeError):
            return np.array([jsonable(v) for v in vals], dtype=object)

    def save(self) -> None:
        """Write data.npz, data.csv and meta.json (no-op for an empty log)."""
        if not self._rows:
            return
        keys = sorted(self._rows[0].keys())
        np.savez_compressed(self.path_npz, **{k: self._column(k) for k in keys})

        first = self._rows[0]
        kinds = [_csv_kind(first.get(k)) for k in keys]
        header = []
        for k, kind in zip(keys, kinds):
            header.extend([f"{k}[{i}]" for i in range(first[k].size)] if kind == 1 else [k])
        with open(self.path_csv, "w", newline="") as fh:
            w = csv.writer(fh)
            w.writerow(header)
            for row in self._rows:
                cells = []
                for k in keys:
                    v = row.get(k)
                    kind = _csv_kind(v)
                    if kind == 0:
                        cells.append(v)
                    elif kind == 1:
                        cells.extend(v.tolist())
                    else:
                        cells.append(jsonable(v))
                w.writerow(cells)

        with open(self.path_meta, "w") as fh:
            json.dump(self.meta, fh, indent=2)


def _rms(a: np.ndarray) -> float:
    return float(np.sqrt(np.mean(a ** 2))) if a.size else float("nan")


def summary_metrics(t, err_tan, err_3d, fn_meas, contact, fn_des: float, t_contact_phase: float) -> Dict[str, float]:
    """End-of-run statistics of the closed loop (run_classical.py:513-535).

    Inputs are the per-tick series the runner collects (``summary`` dict,
    run_classical.py:452-457); ``contact`` is 1.0 where fn_meas > 0.5 N.
    The contact phase is t >= t_contact_phase.
    """
    t = np.asarray(t, dtype=float)
    err_tan = np.asarray(err_tan, dtype=float)
    err_3d = np.asarray(err_3d, dtype=float)
    fn_meas = np.asarray(fn_meas, dtype=float)
    contact = np.asarray(contact, dtype=float)
    phase = t >= float(t_contact_phase)
    nan = float("nan")
    c_phase, fn_phase, et_phase = contact[phase], fn_meas[phase], err_tan[phase]
    return {
        "avg_abs_position_err": float(np.mean(np.abs(err_tan))) if err_tan.size else nan,
        "avg_abs_force_err": float(np.mean(np.abs(fn_meas - float(fn_des)))) if fn_meas.size else nan,
        "rms_tangential_error": _rms(err_tan),
        "rms_tangential_error_contact_phase": _rms(et_phase),
        "rms_3d_error": _rms(err_3d),
        "max_fn": float(np.max(fn_meas)) if fn_meas.size else nan,
        "contact_loss_pct": float((1.0 - np.mean(contact)) * 100.0) if contact.size else nan,
        "contact_loss_contact_phase_pct": float((1.0 - np.mean(c_phase)) * 100.0) if c_phase.size else nan,
        "fn_mean_contact_phase": float(np.mean(fn_phase)) if fn_phase.size else nan,
        "contact_phase_start_s": float(t_contact_phase),
    }
