"""Closed-loop pieces on the CPU.

* ffddp.uncertainty mirrors src/run/uncertainty_profiles.py draw for draw:
  pinned by vectors the reference's injector produced
  (tests/golden/make_closed_loop_golden.py).
* ffddp.plant.mat_to_quat_wxyz pinned by the reference's
  FrankaMujocoSim._mat_to_quat_wxyz outputs.
* The plant restatement (oracle/plant.py) against physical identities: a
  gravity-compensated arm stays put, an arm pressing on the table settles to
  the commanded normal force, tilt moves the plane normal.  (MuJoCo itself is
  absent: parity of the plant with MuJoCo is unpinned.)
"""
from __future__ import annotations

from pathlib import Path

import numpy as np
import pytest

from ffddp import closed_loop as CL
from ffddp import plant as PL
from ffddp import uncertainty as U
from oracle import panda as P
from oracle import plant as OP

G = np.load(Path(__file__).resolve().parent / "golden" / "closed_loop_vectors.npz")


def _synthetic_obs(k, rng):
    f = lambda n: rng.normal(size=n)  # noqa: E731
    return PL.Observation(q=f(7), dq=f(7), tau_meas=f(7), tau_meas_filt=f(7), tau_meas_act=f(7),
                          tau_meas_act_filt=f(7), tau_cmd=f(7), tau_act=f(7), tau_constraint=f(7), tau_total=f(7),
                          tau_bias=f(7), f_contact_world=f(3), f_contact_normal=float(k), f_contact_normal_world_z=0.0,
                          f_contact_tangent=0.0, contact_count_ee=0, contact_count_table=0,
                          table_normal_world=np.array([0.0, 0.0, 1.0]), ee_pos=f(3), ee_quat=f(4), J_pos=None,
                          J_rot=None, ee_vel=f(3))


@pytest.mark.parametrize("tag,dt", [("dt5", 0.005), ("dt1", 0.001)])
def test_uncertainty_injector_matches_reference(tag, dt):
    assert U.config_for_scenario("flat", seed=11) is None
    inj = U.ScenarioUncertaintyInjector(dt=dt, nu=7, config=U.config_for_scenario("actuation_uncertainty", seed=15),
                                        tau_lpf_alpha=0.2)
    m = inj.meta()
    np.testing.assert_array_equal([m["a"], m["b"], m["delta_obs_steps"], m["delta_cmd_steps"]], G[f"{tag}_meta"])
    rng = np.random.default_rng(5)
    for k in range(12):
        o = _synthetic_obs(k, rng)
        c = rng.normal(size=7) * 5.0
        np.testing.assert_array_equal(np.concatenate([o.q, o.dq]), G[f"{tag}_obs_in"][k])
        np.testing.assert_array_equal(c, G[f"{tag}_cmd_in"][k])
        d = inj.observation_for_controller(o)
        a = inj.command_for_plant(c)
        np.testing.assert_array_equal(d.q, G[f"{tag}_q_out"][k])
        np.testing.assert_array_equal(d.dq, G[f"{tag}_dq_out"][k])
        np.testing.assert_array_equal(d.tau_meas, G[f"{tag}_tau_meas_out"][k])
        np.testing.assert_array_equal(d.tau_meas_filt, G[f"{tag}_tau_filt_out"][k])
        np.testing.assert_array_equal(a, G[f"{tag}_cmd_out"][k])


def test_quaternion_matches_reference():
    for Rm, q in zip(G["quat_R"], G["quat_q"]):
        np.testing.assert_allclose(PL.mat_to_quat_wxyz(Rm), q, rtol=0, atol=1e-15)


def test_scenarios():
    assert CL.SCENARIOS == ("flat", "tilted_5", "tilted_10", "tilted_15", "actuation_uncertainty")
    assert [CL.scenario_seed(s) for s in CL.SCENARIOS] == [11, 12, 13, 14, 15]
    s = CL.scenario_settings("tilted_10")
    assert s["tilt_deg"] == 10.0 and np.all(s["torque_scale"] == 1.0)
    assert CL.scenario_settings("actuation_uncertainty")["torque_scale"][1] == 1.08
    with pytest.raises(ValueError):
        CL.scenario_settings("nope")
    n, p0 = PL.table_plane(0.0)
    np.testing.assert_allclose(n, [0, 0, 1])
    np.testing.assert_allclose(p0, [-0.5, 0.0, 0.32])
    n, p0 = PL.table_plane(10.0)
    np.testing.assert_allclose(n, [np.sin(np.deg2rad(10)), 0, np.cos(np.deg2rad(10))], atol=1e-15)


def _contact_pose():
    """A q with the tool sphere 1 mm into the flat table (IK by Gauss-Newton)."""
    q = np.array([0.0, 0.35, 0.0, -2.0, 0.0, 2.35, 0.785])
    target_z = 0.32 + 0.03 - 0.001
    for _ in range(50):
        J6, _, p = P.frame_jacobian_lwa(q)
        p_mj = OP.R_MJ @ p
        e = np.array([0.0, 0.0, target_z - p_mj[2]])
        Jm = OP.R_MJ @ J6[:3]
        q = q + np.linalg.lstsq(Jm, e, rcond=None)[0]
    return q


def test_plant_gravity_compensated_rest():
    prm = OP.default_params()
    q0 = np.array([0.0, -0.758, 0.0, -2.22, 0.0, 1.43, 0.0])
    n, p0 = PL.table_plane(0.0)
    tau = P.gravity_torque(q0)
    q, v, obs = OP.step(prm, q0, np.zeros(7), tau, n, p0)
    assert obs["ncon"] == 0.0 and obs["fn"] == 0.0
    np.testing.assert_allclose(q, q0, atol=1e-12)
    np.testing.assert_allclose(v, 0.0, atol=1e-10)
    np.testing.assert_allclose(obs["bias"], tau, rtol=1e-13)


def test_plant_press_settles_to_commanded_force():
    prm = OP.default_params()
    q = _contact_pose()
    v = np.zeros(7)
    n, p0 = PL.table_plane(0.0)
    F = 20.0
    for _ in range(400):  # 2 s of control steps
        J6, _, _ = P.frame_jacobian_lwa(q)
        Jn = (OP.R_MJ @ J6[:3])[2]
        tau = P.gravity_torque(q) - Jn * F - 30.0 * v  # push down with F, damp the joints
        q, v, obs = OP.step(prm, q, v, tau, n, p0)
    assert obs["ncon"] == 1.0
    assert obs["fn"] == pytest.approx(F, rel=2e-3)
    np.testing.assert_allclose(obs["f_world"], [0, 0, obs["fn"]], atol=1e-12)
    # the table holds the sphere near the surface (soft constraint: sub-mm penetration)
    assert abs(obs["ee_pos"][2] - (0.32 + 0.03)) < 2e-3


@pytest.mark.parametrize("dt", [0.005, 0.001])
def test_batched_injector_matches_scalar(dt):
    """The fleet's BatchedUncertaintyInjector gives every instance exactly the
    scalar injector's perturbed (q, dq) and applied command, tick for tick
    (600 ticks: across the pre-draw chunk boundary; dt = 1 ms: delay lines)."""
    seeds = [15, 1500003, 7, 42, 99]
    cfgs = [U.config_for_scenario("actuation_uncertainty", seed=s) for s in seeds]
    bat = U.BatchedUncertaintyInjector(dt=dt, nu=7, configs=cfgs)
    sc = [U.ScenarioUncertaintyInjector(dt=dt, nu=7, config=c) for c in cfgs]
    assert bat.obs_delay_steps == sc[0].obs_delay_steps and bat.cmd_delay_steps == sc[0].cmd_delay_steps
    rng = np.random.default_rng(3)
    for k in range(600):
        q, dq, tau = rng.normal(size=(5, 7)), rng.normal(size=(5, 7)), rng.normal(size=(5, 7)) * 10
        qb, dqb = bat.observation_for_controller(q, dq)
        ab = bat.command_for_plant(tau)
        for b, j in enumerate(sc):
            o = _synthetic_obs(k, rng)
            o.q, o.dq = q[b].copy(), dq[b].copy()
            d = j.observation_for_controller(o)
            np.testing.assert_array_equal(qb[b], d.q)
            np.testing.assert_array_equal(dqb[b], d.dq)
            np.testing.assert_array_equal(ab[b], j.command_for_plant(tau[b]))
