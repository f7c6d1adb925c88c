"""Device-side problem builder (ffddp_build_problem_dev)
against the reference's own trajectory samples (tests/golden, produced by
src/tasks/trajectories.py itself), the host workload mapping
(crocoddyl_classical.py:250-258, 447-466) and the oracle's gravity.

Tolerances: EE references are affine maps of sin/cos/smoothstep values —
atol 1e-13 (device sincos vs numpy, a few ulp); surface flags exact; gravity
torques 1e-12 relative to the oracle's RNEA; solves from a device-built
problem vs the host-built one within the parity suite's 1e-6.
"""
from pathlib import Path

import numpy as np
import pytest

from ffddp import BatchedBoxFDDP, _abi, robot as R
from ffddp.trajectory import TABLE_CENTER, TABLE_HALF_Z, TOOL_RADIUS
from ffddp.workload import pos_mj_to_pin, vel_mj_to_pin
from oracle import panda as P

from helpers import ee_start_mj, make_batch, product_cfg, rel_err

pytestmark = pytest.mark.gpu

G = np.load(Path(__file__).resolve().parent / "golden" / "reference_vectors.npz")
TOL_REF = 1e-13


def _torch():
    import torch

    assert torch.cuda.is_available()
    return torch


def _build(solver, task, t0, x0):
    torch = _torch()
    B, N = len(t0), solver.N
    t = {
        "t0": torch.tensor(np.asarray(t0, float), device="cuda"),
        "x0": torch.tensor(np.ascontiguousarray(x0, float), device="cuda"),
        "node_ref": torch.full((B, N + 1, 6), np.nan, dtype=torch.float64, device="cuda"),
        "inst_ref": torch.full((B, 21), np.nan, dtype=torch.float64, device="cuda"),
        "surface": torch.full((B,), 7, dtype=torch.uint8, device="cuda"),
    }
    solver.build_problem_dev(task, t)
    torch.cuda.synchronize()
    return {k: t[k].cpu().numpy() for k in ("node_ref", "inst_ref", "surface")}


def _bench_task(t_hold=0.2, **kw):
    z_contact = TABLE_CENTER[2] + TABLE_HALF_Z + TOOL_RADIUS - 8.0e-3
    return _abi.make_task(
        center=[TABLE_CENTER[0], TABLE_CENTER[1], z_contact], radius=0.10, omega=1.5, z_contact=z_contact,
        t_approach=0.55, ee_start=ee_start_mj(), z_pre=z_contact + 0.05, t_pre=0.25, t_hold=t_hold, **kw,
    )


def _golden_check(name, task, horizon=3):
    ts = G[f"{name}_t"]
    solver = BatchedBoxFDDP(product_cfg("classical", horizon), max_batch=len(ts))
    x0 = np.zeros((len(ts), 14))
    x0[:, :7] = R.Q_NEUTRAL
    out = _build(solver, task, ts, x0)
    p_pin = np.array([pos_mj_to_pin(p) for p in G[f"{name}_p"]])
    v_pin = np.array([vel_mj_to_pin(v) for v in G[f"{name}_v"]])
    np.testing.assert_allclose(out["node_ref"][:, 0, :3], p_pin, rtol=0, atol=TOL_REF)
    np.testing.assert_allclose(out["node_ref"][:, 0, 3:], v_pin, rtol=0, atol=TOL_REF)
    np.testing.assert_array_equal(out["surface"], G[f"{name}_surf"].astype(np.uint8))
    # knot k samples t0 + k dt: knot 2 of instance i is knot 0 of instance i + 4 (dt 0.01, grid 0.005);
    # positions only (the reference velocity jumps at the circle start, t = t_pre + t_approach)
    # (on the leading uniform part of the fixture's time grid)
    m = int(np.argmax(~np.isclose(np.diff(ts), 0.005))) + 1
    assert m > 100
    np.testing.assert_allclose(out["node_ref"][: m - 4, 2, :3], out["node_ref"][4:m, 0, :3], rtol=0, atol=1e-12)


def test_build_matches_reference_trajectory_benchmark_args():
    a = G["traj_bench_args"]
    task = _abi.make_task(center=a[0:3], radius=a[3], omega=a[4], z_pre=a[5], z_contact=a[6], t_approach=a[7],
                          ee_start=a[9:12], t_pre=a[8])
    _golden_check("traj_bench", task)


def test_build_matches_reference_trajectory_defaults():
    # no ee_start / z_pre, t_pre = 0: trajectories.py's derived start and pre-contact height
    task = _abi.make_task(center=[-0.5, 0.0, 0.342], radius=0.07, omega=2.0, z_contact=0.35, t_approach=1.0)
    _golden_check("traj_raw", task)


@pytest.mark.parametrize("variant", ["classical", "ff"])
def test_build_matches_host_workload(variant):
    """Same t0 / x0 as workload.make_batch (benchmark trajectory with the 0.2 s
    hold, q_nom posture, gravity(x0) torque reference)."""
    N, B = 30, 256
    b = make_batch(variant, B, N, seed=5)
    solver = BatchedBoxFDDP(product_cfg(variant, N), max_batch=B)
    out = _build(solver, _bench_task(), b.t0, b.x0)
    assert np.max(np.abs(out["node_ref"] - b.node_ref)) < TOL_REF
    np.testing.assert_array_equal(out["surface"], b.surface)
    g = np.array([P.gravity_torque(q) for q in b.x0[:, :7]])
    assert rel_err(out["inst_ref"][:, 14:], g) < 1e-12
    np.testing.assert_array_equal(out["inst_ref"][:, :14], b.inst_ref[:, :14])
    assert 0 < int(out["surface"].sum()) < B  # both phases present


def test_build_hold_window_and_reference_modes():
    N, B = 10, 64
    solver = BatchedBoxFDDP(product_cfg("classical", N), max_batch=B)
    tc = 0.25 + 0.55
    t0 = np.linspace(tc - 0.05, tc + 0.3, B)
    rng = np.random.default_rng(3)
    x0 = np.concatenate([R.Q_NEUTRAL + rng.uniform(-0.2, 0.2, (B, 7)), rng.normal(0, 0.1, (B, 7))], 1)
    q_nom = R.Q_NEUTRAL + 0.1
    held = _build(solver, _bench_task(posture_ref_mode="x0", torque_ref_mode="gravity_q_nom", q_nom=q_nom), t0, x0)
    free = _build(solver, _bench_task(t_hold=0.0, torque_ref_mode="zero"), t0, x0)
    z_contact = TABLE_CENTER[2] + TABLE_HALF_Z + TOOL_RADIUS - 8.0e-3
    p_hold = pos_mj_to_pin([TABLE_CENTER[0] + 0.10, TABLE_CENTER[1], z_contact])
    n_held = 0
    for i in range(B):
        for k in range(N + 1):
            t = t0[i] + k * 0.01
            h = held["node_ref"][i, k]
            if tc <= t < tc + 0.2:  # hold: contact-start point, zero velocity (run_classical.py:256-264)
                n_held += 1
                np.testing.assert_allclose(h[:3], p_hold, rtol=0, atol=TOL_REF)
                np.testing.assert_array_equal(h[3:], 0.0)
            else:
                np.testing.assert_allclose(h, free["node_ref"][i, k], rtol=0, atol=TOL_REF)
    assert n_held > 0
    np.testing.assert_array_equal(held["inst_ref"][:, :14], x0)
    g_nom = P.gravity_torque(q_nom)
    assert rel_err(held["inst_ref"][:, 14:], np.broadcast_to(g_nom, (B, 7))) < 1e-12
    np.testing.assert_array_equal(free["inst_ref"][:, 14:], 0.0)
    np.testing.assert_array_equal(free["inst_ref"][:, :7], np.broadcast_to(R.Q_NEUTRAL, (B, 7)))
    np.testing.assert_array_equal(free["inst_ref"][:, 7:14], 0.0)
    np.testing.assert_array_equal(held["surface"], free["surface"])
    np.testing.assert_array_equal(held["surface"], (t0 >= tc).astype(np.uint8))


def test_solve_from_device_built_problem():
    """build_problem_dev -> solve_dev entirely in HBM equals the host-built solve."""
    torch = _torch()
    N, B = 30, 128
    b = make_batch("classical", B, N, seed=9)
    cfg = product_cfg("classical", N)
    s_host = BatchedBoxFDDP(cfg, max_batch=B)
    s_host.solve(b)
    s_dev = BatchedBoxFDDP(cfg, max_batch=B)
    dev = lambda a, dt=torch.float64: torch.tensor(np.ascontiguousarray(a), dtype=dt, device="cuda")
    t = {
        "t0": dev(b.t0), "x0": dev(b.x0),
        "node_ref": torch.empty((B, N + 1, 6), dtype=torch.float64, device="cuda"),
        "inst_ref": torch.empty((B, 21), dtype=torch.float64, device="cuda"),
        "surface": torch.empty((B,), dtype=torch.uint8, device="cuda"),
        "xs_init": dev(b.xs_init), "us_init": dev(b.us_init),
        "xs": torch.empty((B, N + 1, 14), dtype=torch.float64, device="cuda"),
        "us": torch.empty((B, N, 7), dtype=torch.float64, device="cuda"),
        "K": torch.empty((B, N, 7, 14), dtype=torch.float64, device="cuda"),
        "cost": torch.empty(B, dtype=torch.float64, device="cuda"),
        "iters": torch.empty(B, dtype=torch.int32, device="cuda"),
        "ok": torch.empty(B, dtype=torch.uint8, device="cuda"),
        "fn_pred": torch.empty((B, 2), dtype=torch.float64, device="cuda"),
        "stats": torch.empty((B, _abi.NSTATS), dtype=torch.int32, device="cuda"),
    }
    s_dev.build_problem_dev(_bench_task(), t)
    s_dev.solve_dev(t, maxiter=10)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(t["iters"].cpu().numpy(), s_host.iter)
    np.testing.assert_array_equal(t["ok"].cpu().numpy().astype(bool), s_host.ok)
    assert rel_err(t["xs"].cpu().numpy(), s_host.xs) < 1e-6
    assert rel_err(t["us"].cpu().numpy(), s_host.us) < 1e-6
    assert rel_err(t["cost"].cpu().numpy(), s_host.cost) < 1e-6


def test_solve_dev_matches_host_entry_and_in_place():
    """The device entry point iterates in the caller's xs / us / K (no copy
    after the last kernel): bit-identical to the host entry point at B = 520
    (4 slices), also with the warm start in place (xs_init is xs, us_init is us)."""
    torch = _torch()
    N, B = 30, 520
    b = make_batch("classical", B, N, seed=17)
    cfg = product_cfg("classical", N)
    s_host = BatchedBoxFDDP(cfg, max_batch=B)
    s_host.solve(b)
    dev = lambda a, dt=torch.float64: torch.tensor(np.ascontiguousarray(a), dtype=dt, device="cuda")
    for in_place in (False, True):
        s_dev = BatchedBoxFDDP(cfg, max_batch=B)
        t = {
            "x0": dev(b.x0), "node_ref": dev(b.node_ref), "inst_ref": dev(b.inst_ref),
            "surface": dev(b.surface, torch.uint8),
            "xs_init": dev(b.xs_init), "us_init": dev(b.us_init),
            "K": torch.full((B, N, 7, 14), float("nan"), dtype=torch.float64, device="cuda"),
            "cost": torch.empty(B, dtype=torch.float64, device="cuda"),
            "iters": torch.empty(B, dtype=torch.int32, device="cuda"),
            "ok": torch.empty(B, dtype=torch.uint8, device="cuda"),
            "fn_pred": torch.empty((B, 2), dtype=torch.float64, device="cuda"),
            "stats": torch.empty((B, _abi.NSTATS), dtype=torch.int32, device="cuda"),
        }
        if in_place:
            t["xs"], t["us"] = t["xs_init"], t["us_init"]
        else:
            t["xs"] = torch.full((B, N + 1, 14), float("nan"), dtype=torch.float64, device="cuda")
            t["us"] = torch.full((B, N, 7), float("nan"), dtype=torch.float64, device="cuda")
        s_dev.solve_dev(t, maxiter=10)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(t["xs"].cpu().numpy(), s_host.xs)
        np.testing.assert_array_equal(t["us"].cpu().numpy(), s_host.us)
        np.testing.assert_array_equal(t["K"].cpu().numpy(), s_host.K)
        np.testing.assert_array_equal(t["cost"].cpu().numpy(), s_host.cost)
        np.testing.assert_array_equal(t["iters"].cpu().numpy(), s_host.iter)
        np.testing.assert_array_equal(t["ok"].cpu().numpy().astype(bool), s_host.ok)
        s_dev.close()
    s_host.close()
