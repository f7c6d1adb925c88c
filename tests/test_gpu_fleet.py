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
    # scalar controllers, each calibrated from its own start state (as the reference does)
    scal = []
    for b in range(B):
        sim = PL.PandaTablePlant(n_substeps=5, timestep=0.001)
        sim.set_state(q0[b])
        scal.append((sim, CT.ClassicalCrocoddylMPC(sim=sim, traj_fn=traj, config=cfg)))
    Rs, p_off = FL.site_calibration(PL.observation_from_record(plant.obs[0]))
    fleet = FL.FleetClassicalMPC(B, traj, cfg, q_nom=q0, tau0=plant.obs[:, 14:21], R_site_from_pin_ee=Rs,
                                 p_site_minus_frame_pin=p_off)
    t = t_start
    worst = 0.0
    for _ in range(ticks):
        rec = plant.obs.copy()
        fn = rec[:, 46] * (rec[:, 47] > 0.5)
        tau_f = fleet.compute_control(rec[:, 0:7], rec[:, 7:14], rec[:, 14:21], fn, rec[:, 30], t)
        for b in range(B):
            tau_s = scal[b][1].compute_control(PL.observation_from_record(rec[b]), t)
            info = scal[b][1].last_info
            assert bool(fleet.last_info["ok"][b]) == bool(info["ok"])
            assert int(fleet.last_info["iters"][b]) == int(info["iters"])
            # The two paths build the same problem to rounding level (the
            # device builder vs the host code: sin / cos / pose algebra in
            # different operation orders), and the solve amplifies those
            # roundings near the torque limits: converged solves agree to
            # ~1e-6 N m (1.6e-6 observed on the round-5 head, < 1e-7 on the
            # round-4 one; the solver's own rounding changed), a solve that
            # returns ok = False (maxiter on an infeasible iterate) to ~5e-3 N m
            tol = 1e-7 if info["ok"] else 1e-2
            np.testing.assert_allclose(tau_f[b], tau_s, rtol=tol, atol=tol)
            if info["ok"]:
                worst = max(worst, float(np.max(np.abs(tau_f[b] - tau_s))))
            assert bool(fleet.last_info["surface_mode"][b]) == bool(info["surface_mode"])
        plant.step(tau_f)
        t += plant.dt
    for sim, c in scal:
        c.close()
        sim.close()
    fleet.close()
    plant.close()
    nominal.close()
    assert worst < 1e-5, worst


def test_sweep_short():
    out = FL.run_sweep(seeds=4, total_time=1.2, verbose=False)
    assert out["instances"] == 20 and out["ticks"] == 240
    pi = out["per_instance"]
    assert np.all(np.isfinite(pi["rms_3d_error"])) and np.median(pi["rms_3d_error"]) < 0.2
