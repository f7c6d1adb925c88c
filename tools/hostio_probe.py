"""Where the host entry point's wall time goes outside the library call
(ffddp_solve_batch with pageable numpy arrays, as BatchedBoxFDDP.solve makes
them): np.zeros of the outputs, the call itself, and the release of the
previous call's outputs (munmap of ~118 MB of faulted pages at B = 4096).
usage: python tools/hostio_probe.py [B] [reps]"""
import sys
import pathlib
import time

sys.path.insert(0, str(pathlib.Path(__file__).resolve().parents[1]))
import ffddp_path  # noqa: F401,E402
import numpy as np  # noqa: E402
from ffddp import BatchedBoxFDDP, _abi, robot as R, workload  # noqa: E402
from ffddp.config import classical_preset  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 6
N, nx = 30, 14
cfg = classical_preset(N)
ee = R.R_MJ_FROM_PIN @ _abi.frame_placement(R.Q_NEUTRAL)[1]
b = workload.make_batch(B, N, "classical", _abi.gravity_torque, ee, seed=1234, fk=_abi.frame_placement)
s = BatchedBoxFDDP(cfg, max_batch=B)
lib, h = s._lib, s._h
f = lambda a, shape: np.ascontiguousarray(np.asarray(a, np.float64).reshape(shape))
x0, nref, iref = f(b.x0, (B, nx)), f(b.node_ref, (B, N + 1, 6)), f(b.inst_ref, (B, 21))
surf = np.ascontiguousarray(np.asarray(b.surface, np.uint8).reshape(B))
xsi, usi = f(b.xs_init, (B, N + 1, nx)), f(b.us_init, (B, N, 7))
specs = dict(xs=((B, N + 1, nx), np.float64), us=((B, N, 7), np.float64), K=((B, N, 7, nx), np.float64),
             cost=((B,), np.float64), iters=((B,), np.int32), ok=((B,), np.uint8), fn=((B, 2), np.float64),
             stats=((B, _abi.NSTATS), np.int32))
d, i, u = _abi.dptr, _abi.iptr, _abi.uptr
prev = None
for r in range(reps):
    t0 = time.perf_counter()
    o = {k: np.zeros(shape, dt) for k, (shape, dt) in specs.items()}
    t1 = time.perf_counter()
    rc = lib.ffddp_solve_batch(h, B, d(x0), d(nref), d(iref), u(surf), d(xsi), d(usi), 10, 0, d(o["xs"]), d(o["us"]),
                               d(o["K"]), d(o["cost"]), i(o["iters"]), u(o["ok"]), d(o["fn"]), i(o["stats"]))
    assert rc == 0
    t2 = time.perf_counter()
    prev = o  # releases the previous call's arrays
    t3 = time.perf_counter()
    print(f"rep {r}: zeros {1e3 * (t1 - t0):.2f} ms  call {1e3 * (t2 - t1):.2f} ms  release previous {1e3 * (t3 - t2):.2f} ms"
          f"  total {1e3 * (t3 - t0):.2f} ms", flush=True)
s.close()
