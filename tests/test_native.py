"""The pybind11 module (ffddp.native, csrc/ffddp_pybind.cpp): loads, its
struct sizes agree with the header / ctypes layouts, and it rejects bad
input before touching a device.  GPU: bit-for-bit the ctypes path's solve."""
from __future__ import annotations

import ctypes
import threading

import numpy as np
import pytest

from ffddp import _abi, native
from ffddp.config import classical_preset, ff_preset


def test_module_loads_and_matches_abi():
    m = native.load()
    assert m.NSTATS == _abi.NSTATS
    assert m.ROBOT_BYTES == ctypes.sizeof(_abi.Robot)
    assert m.CFG_BYTES == ctypes.sizeof(_abi.OcpConfig)
    assert "GIL" in m.Solver.solve.__doc__


def test_rejects_bad_structs_and_config():
    m = native.load()
    with pytest.raises(ValueError):
        m.Solver(b"\0" * 8, bytes(classical_preset(30).to_struct()), 0, 4)
    c = classical_preset(30).to_struct()
    c.nc = 2  # neither ContactModel1D nor 3D: refused before any device call
    with pytest.raises(RuntimeError, match="ffddp_create"):
        m.Solver(bytes(_abi.robot_struct()), bytes(c), 0, 4)


@pytest.mark.gpu
@pytest.mark.parametrize("variant,B", [("classical", 70), ("ff", 16)])
def test_native_solve_bit_identical_to_ctypes(variant, B):
    from ffddp import BatchedBoxFDDP
    from helpers import make_batch

    cfg = ff_preset(30) if variant == "ff" else classical_preset(30)
    b = make_batch(variant, B, 30, seed=61)
    ref = BatchedBoxFDDP(cfg, max_batch=B)
    ref.solve(b, maxiter=10)
    s = native.Solver(cfg, max_batch=B)
    ok = s.solve(b, maxiter=10)
    for name in ("xs", "us", "K", "cost", "iter", "fn_pred", "stats"):
        assert np.array_equal(getattr(s, name), getattr(ref, name), equal_nan=True), name
    assert np.array_equal(ok, ref.ok)
    with pytest.raises(ValueError):
        s._s.solve(b.x0[:, :5], b.node_ref, b.inst_ref, b.surface, b.xs_init, b.us_init, 10, False)
    # two Python threads on two handles: the extension releases the GIL
    s2 = native.Solver(cfg, max_batch=B)
    res = {}

    def run(key, solver):
        solver.solve(b, maxiter=10)
        res[key] = solver.xs.copy()

    th = [threading.Thread(target=run, args=(k, sv)) for k, sv in (("a", s), ("b", s2))]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert np.array_equal(res["a"], ref.xs) and np.array_equal(res["b"], ref.xs)
    for x in (s, s2, ref):
        x.close()
