"""Synthetic workload generator (bench inputs) — determinism, shapes, regimes."""
import numpy as np

from ffddp import _abi, robot as R
from ffddp.workload import ik_pose, pos_mj_to_pin

from helpers import make_batch


def test_batch_shapes_and_determinism():
    a = make_batch("classical", 16, 30, seed=1)
    b = make_batch("classical", 16, 30, seed=1)
    assert a.x0.shape == (16, 14) and a.node_ref.shape == (16, 31, 6) and a.inst_ref.shape == (16, 21)
    assert a.xs_init.shape == (16, 31, 14) and a.us_init.shape == (16, 30, 7)
    for f in ("x0", "node_ref", "inst_ref", "surface", "xs_init", "us_init"):
        assert np.array_equal(getattr(a, f), getattr(b, f))
    f = make_batch("ff", 8, 10, seed=2)
    assert f.x0.shape == (8, 21) and np.allclose(f.us_init[:, 0], f.x0[:, 14:])


def test_cold_start_and_references():
    a = make_batch("classical", 8, 20, seed=3)
    assert np.allclose(a.xs_init, a.x0[:, None, :])
    assert np.allclose(a.inst_ref[:, 14:], _abi.gravity_torque(a.x0[:, :7]))
    assert np.allclose(a.inst_ref[:, :7], R.Q_NEUTRAL)
    assert a.surface.mean() > 0.8  # t0 ~ U(0, 20) s, contact after ~0.8 s


def test_ik_reaches_reference():
    R_des = R.default_R_des()
    p = pos_mj_to_pin(np.array([-0.4, 0.05, 0.342]))
    q = ik_pose(_abi.frame_placement, p, R_des, R.Q_NEUTRAL)
    Rq, pq = _abi.frame_placement(q)
    assert np.linalg.norm(pq - p) < 1e-6 and np.abs(Rq - R_des).max() < 1e-5
