"""GPU: the fleet controller (B instances, one batched device solve per tick)
against B copies of the B = 1 controller mirror (ffddp.controller, itself
pinned to the reference's numpy code) fed the same observations, plus a short
5-scenario sweep through run_sweep."""
from __future__ import annotations

import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

from ffddp import controller as CT  # noqa: E402
from ffddp import fleet as FL  # noqa: E402
from ffddp import plant as PL  # noqa: E402
from ffddp import robot as R  # noqa: E402
from ffddp.trajectory import benchmark_traj  # noqa: E402


@pytest.mark.parametrize("phase_source", ["trajectory", "force_latch"])
def test_fleet_matches_scalar_controllers(phase_source):
    B, ticks = 3, 40
    rng = np.random.default_rng(4)
    q0 = R.Q_NEUTRAL + rng.normal(0.0, 0.02, (B, 7))
    nominal = PL.PandaTablePlant(n_substeps=5, timestep=0.001)
    obs_n = nominal.reset("neutral")
    traj, meta = benchmark_traj(obs_n.ee_pos)
    t_start = 0.7  # just before contact onset: exercises the mode switch and the contact model
    plant = PL.BatchedPlant(B, timestep=0.001, n_substeps=5)
    plant.q, plant.v = q0.copy(), np.zeros((B, 7))
    plant.step(np.zeros((B, 7)), integrate=False)
    cfg = CT.classical_benchmark_config(plant.dt, meta["z_contact"], phase_source=phase_source)
    # the fleet calibrates the site once, from instance 0's start observation;
    # the scalar controllers take that same calibration (calibration_obs) and
    # everything else from their own start state, so both paths build the
    # same problem bit for bit and every tick must agree exactly
    obs_cal = PL.observation_from_record(plant.obs[0])
    scal = []
    for b in range(B):
        sim = PL.PandaTablePlant(n_substeps=5, timestep=0.001)
        sim.set_state(q0[b])
        scal.append((sim, CT.ClassicalCrocoddylMPC(sim=sim, traj_fn=traj, config=cfg, calibration_obs=obs_cal)))
    Rs, p_off = FL.site_calibration(obs_cal)
    fleet = FL.FleetClassicalMPC(B, traj, cfg, q_nom=q0, tau0=plant.obs[:, 14:21], R_site_from_pin_ee=Rs,
                                 p_site_minus_frame_pin=p_off)
    assert np.array_equal(fleet.R_des, scal[1][1].R_des)
    t = t_start
    for tick in range(ticks):
        rec = plant.obs.copy()
        fn = rec[:, 46] * (rec[:, 47] > 0.5)
        tau_f = fleet.compute_control(rec[:, 0:7], rec[:, 7:14], rec[:, 14:21], fn, rec[:, 30], t)
        for b in range(B):
            tau_s = scal[b][1].compute_control(PL.observation_from_record(rec[b]), t)
            info, fi = scal[b][1].last_info, fleet.last_info
            tag = (phase_source, tick, b)
            # one batched device solve vs B one-instance plans: the solver is
            # batch-independent bit for bit (tests/test_gpu_batch.py), so
            # converged or not (ok = False after maxiter) the ticks agree exactly
            assert bool(fi["ok"][b]) == bool(info["ok"]), tag
            assert int(fi["iters"][b]) == int(info["iters"]), tag
            assert bool(fi["surface_mode"][b]) == bool(info["surface_mode"]), tag
            assert bool(fi["unstable"][b]) == bool(info["unstable"]), tag
            assert np.array_equal(fi["cost"][b], info["cost"], equal_nan=True), tag
            assert np.array_equal(tau_f[b], tau_s), (tag, tau_f[b] - tau_s)
        plant.step(tau_f)
        t += plant.dt
    for sim, c in scal:
        c.close()
        sim.close()
    fleet.close()
    plant.close()
    nominal.close()


def test_sweep_short():
    out = FL.run_sweep(seeds=4, total_time=1.2, verbose=False)
    assert out["instances"] == 20 and out["ticks"] == 240
    pi = out["per_instance"]
    assert np.all(np.isfinite(pi["rms_3d_error"])) and np.median(pi["rms_3d_error"]) < 0.2
