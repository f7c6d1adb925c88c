"""Run-log format: ffddp.runlog.RunLogger replays the rows
the reference's RunLogger logged (tests/golden/make_runlog_golden.py) and must
write byte-identical data.csv, equal data.npz arrays and the same meta.json
(timestamp aside).  summary_metrics is checked against a direct restatement of
run_classical.py:513-535 on synthetic series (parity unpinned: the reference
computes it inline in run(), which needs MuJoCo)."""
from __future__ import annotations

import json
from pathlib import Path

import numpy as np
import pytest

from ffddp.runlog import RunLogger, jsonable, summary_metrics

GOLD = Path(__file__).resolve().parent / "golden" / "runlog"


def _rows(name):
    rows = json.loads((GOLD / name / "rows.json").read_text())
    out = []
    for r in rows:
        out.append({k: (np.asarray(v["ndarray"], dtype=float) if isinstance(v, dict) and "ndarray" in v else v)
                    for k, v in r.items()})
    return out


def _notes():
    n = json.loads((GOLD / "notes.json").read_text())["notes"]
    n["weights"] = np.asarray(n["weights"])
    n["path"] = Path(n["path"])
    n["tup"] = tuple(n["tup"])
    return n


@pytest.mark.parametrize("name", ["a", "b"])
def test_runlogger_matches_reference_files(tmp_path, name):
    lg = RunLogger(f"golden_{name}", results_dir=tmp_path, notes=_notes())
    for r in _rows(name):
        lg.log(**r)
    lg.set_meta(total_time=1.25, torque_scale=np.ones(7), cfg_summary={"horizon": 30, "dt": 0.01})
    lg.save()
    assert lg.run_dir.parent == tmp_path / "logs" and lg.run_dir.name.endswith(f"_golden_{name}")
    assert lg.path_csv.read_bytes() == (GOLD / name / "data.csv").read_bytes()
    got, want = json.loads(lg.path_meta.read_text()), json.loads((GOLD / name / "meta.json").read_text())
    got.pop("timestamp"), want.pop("timestamp")
    assert got == want
    if (GOLD / name / "data.npz").exists():
        a, b = np.load(lg.path_npz), np.load(GOLD / name / "data.npz")
        assert sorted(a.files) == sorted(b.files)
        for k in a.files:
            assert a[k].dtype == b[k].dtype and a[k].shape == b[k].shape, k
            np.testing.assert_array_equal(a[k], b[k])


def test_runlogger_empty_and_exists(tmp_path, monkeypatch):
    import ffddp.runlog as RL

    monkeypatch.setattr(RL.time, "strftime", lambda fmt: "20260101_000000")
    lg = RunLogger("x", results_dir=tmp_path)
    lg.save()
    assert not lg.path_npz.exists() and not lg.path_csv.exists()
    with pytest.raises(FileExistsError):
        RunLogger("x", results_dir=tmp_path)
    assert RunLogger("x", results_dir=tmp_path, overwrite=True).run_dir == lg.run_dir


def test_jsonable():
    assert jsonable({1: (np.arange(2), Path("/a"))}) == {"1": [[0, 1], "/a"]}
    assert jsonable(np.float32(1.5)) == "1.5"


def test_summary_metrics_restatement():
    rng = np.random.default_rng(3)
    n = 400
    t = np.arange(1, n + 1) * 0.005
    err_tan = np.abs(rng.normal(size=n)) * 0.01
    err_3d = err_tan + 0.002
    fn = np.clip(rng.normal(20.0, 5.0, n), 0, None)
    fn[:50] = 0.0
    contact = (fn > 0.5).astype(float)
    s = summary_metrics(t, err_tan, err_3d, fn, contact, fn_des=22.0, t_contact_phase=0.8)
    ph = t >= 0.8
    assert s["rms_tangential_error"] == pytest.approx(np.sqrt(np.mean(err_tan ** 2)), rel=1e-15)
    assert s["rms_tangential_error_contact_phase"] == pytest.approx(np.sqrt(np.mean(err_tan[ph] ** 2)), rel=1e-15)
    assert s["rms_3d_error"] == pytest.approx(np.sqrt(np.mean(err_3d ** 2)), rel=1e-15)
    assert s["avg_abs_position_err"] == pytest.approx(np.mean(err_tan), rel=1e-15)
    assert s["avg_abs_force_err"] == pytest.approx(np.mean(np.abs(fn - 22.0)), rel=1e-15)
    assert s["max_fn"] == fn.max()
    assert s["contact_loss_pct"] == pytest.approx(100.0 * (1 - contact.mean()), rel=1e-15)
    assert s["contact_loss_contact_phase_pct"] == pytest.approx(100.0 * (1 - contact[ph].mean()), rel=1e-15, abs=1e-12)
    assert s["fn_mean_contact_phase"] == pytest.approx(fn[ph].mean(), rel=1e-15)
    e = summary_metrics([], [], [], [], [], 22.0, 0.8)
    assert np.isnan(e["rms_tangential_error"]) and np.isnan(e["max_fn"])
