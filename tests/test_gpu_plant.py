"""GPU: the plant stand-in kernel (ffddp_plant_step, C-ABI) against the numpy
restatement oracle/plant.py, and a short closed loop (HIP solver + HIP plant)
for both controller variants.  Plant parity with MuJoCo: unpinned."""
from __future__ import annotations

import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

from ffddp import plant as PL  # noqa: E402
from oracle import plant as OP  # noqa: E402
from test_closed_loop import _contact_pose  # noqa: E402


def _states(B, rng):
    q0 = _contact_pose()
    qs, vs, taus, tilts = [], [], [], []
    for b in range(B):
        if b % 2 == 0:  # in contact (with some penetration / approach velocity)
            q = q0 + rng.normal(scale=0.004, size=7)
        else:
            q = np.array([0.0, -0.758, 0.0, -2.22, 0.0, 1.43, 0.0]) + rng.uniform(-0.3, 0.3, 7)
        qs.append(q)
        vs.append(rng.normal(scale=0.2, size=7))
        taus.append(rng.normal(scale=5.0, size=7))
        tilts.append([0.0, 5.0, 10.0, 15.0][b % 4])
    return np.array(qs), np.array(vs), np.array(taus), np.array(tilts)


@pytest.mark.parametrize("integrate", [False, True])
def test_plant_kernel_matches_oracle(integrate):
    rng = np.random.default_rng(3)
    B = 12
    q, v, tau, tilt = _states(B, rng)
    bp = PL.BatchedPlant(B, timestep=0.001, n_substeps=5)
    bp.q, bp.v = q.copy(), v.copy()
    bp.set_tilt(tilt)
    obs = bp.step(tau, integrate=integrate).copy()
    prm = OP.default_params(0.001, 5)
    ncon = 0
    for b in range(B):
        n, p0 = PL.table_plane(tilt[b])
        qo, vo, o = OP.step(prm, q[b], v[b], tau[b], n, p0, integrate=integrate)
        ncon += int(o["ncon"])
        np.testing.assert_allclose(bp.q[b], qo, rtol=1e-12, atol=1e-12)
        np.testing.assert_allclose(bp.v[b], vo, rtol=1e-10, atol=1e-10)
        r = obs[b]
        np.testing.assert_allclose(r[0:7], qo, rtol=1e-12, atol=1e-12)
        np.testing.assert_allclose(r[14:21], o["bias"], rtol=1e-10, atol=1e-10)
        np.testing.assert_allclose(r[21:28], o["tau_c"], rtol=1e-9, atol=1e-9)
        np.testing.assert_allclose(r[28:31], o["ee_pos"], rtol=1e-12, atol=1e-12)
        np.testing.assert_allclose(r[31:34], o["ee_vel"], rtol=1e-10, atol=1e-10)
        np.testing.assert_allclose(r[34:43].reshape(3, 3), o["ee_R"], rtol=1e-12, atol=1e-12)
        np.testing.assert_allclose(r[43:46], o["f_world"], rtol=1e-9, atol=1e-9)
        assert r[46] == pytest.approx(o["fn"], rel=1e-9, abs=1e-9)
        assert r[47] == o["ncon"]
        np.testing.assert_allclose(r[48:69].reshape(3, 7), o["J"], rtol=1e-12, atol=1e-12)
    assert ncon >= 2  # the contact branch was exercised
    bp.close()


def test_plant_interface_reset_step():
    sim = PL.PandaTablePlant(n_substeps=5, timestep=0.001)
    obs = sim.reset("neutral")
    np.testing.assert_allclose(obs.q, [0.0, -0.758, 0.0, -2.22, 0.0, 1.43, 0.0])
    assert obs.f_contact_normal == 0.0 and obs.ee_pos.shape == (3,) and obs.ee_quat.shape == (4,)
    assert sim.dt == pytest.approx(0.005)
    obs2 = sim.step(obs.tau_bias)  # gravity compensation holds the arm
    assert np.max(np.abs(obs2.q - obs.q)) < 1e-5
    with pytest.raises(ValueError):
        sim.step(np.zeros(6))
    sim.close()


@pytest.mark.parametrize("variant", ["classical", "ff"])
def test_closed_loop_short_run(tmp_path, variant):
    from ffddp import closed_loop as CL

    s = CL.run_single("flat", total_time=1.2, variant=variant, results_dir=tmp_path, verbose=False)
    assert s["ticks"] == 240
    run = next((tmp_path / "logs").iterdir())
    for f in ("data.npz", "data.csv", "meta.json"):
        assert (run / f).exists()
    d = np.load(run / "data.npz")
    assert d["ee_pos"].shape == (240, 3) and np.all(np.isfinite(d["tau_cmd"]))
    assert np.all(np.isfinite(d["err_3d"])) and s["rms_3d_error"] < 0.2
