"""Host entry point timing (ffddp_solve_batch) next to the device-resident
entry point (ffddp_solve_batch_dev) on the same handle, at the metric's
B = 4096: recycled page-locked output arrays (the default), fresh pageable
ones (names "fresh*" / "pageable*"), solver-owned page-locked ones ("pinned*").  FFDDP_HOSTIO_TIMING=1
makes the library print stage-in / enqueue / per-slice done and copied times
to stderr.  usage: python tools/hostio.py [B] [reps]"""
import os
import sys
import time
import pathlib

sys.path.insert(0, str(pathlib.Path(__file__).resolve().parents[1]))
import ffddp_path  # noqa: F401,E402
import numpy as np  # noqa: E402
import torch  # noqa: E402
from ffddp import BatchedBoxFDDP, _abi, robot as R, workload  # noqa: E402
from ffddp.config import classical_preset  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
N, nx = 30, 14
cfg = classical_preset(N)
ee = R.R_MJ_FROM_PIN @ _abi.frame_placement(R.Q_NEUTRAL)[1]
b = workload.make_batch(B, N, "classical", _abi.gravity_torque, ee, seed=1234, fk=_abi.frame_placement)
f64 = dict(dtype=torch.float64, device="cuda")
T = dict(x0=torch.tensor(b.x0, **f64), node_ref=torch.tensor(b.node_ref, **f64), inst_ref=torch.tensor(b.inst_ref, **f64),
         surface=torch.tensor(b.surface, dtype=torch.uint8, device="cuda"), xs_init=torch.tensor(b.xs_init, **f64),
         us_init=torch.tensor(b.us_init, **f64), xs=torch.zeros((B, N + 1, nx), **f64), us=torch.zeros((B, N, 7), **f64),
         K=torch.zeros((B, N, 7, nx), **f64), cost=torch.zeros(B, **f64),
         iters=torch.zeros(B, dtype=torch.int32, device="cuda"), ok=torch.zeros(B, dtype=torch.uint8, device="cuda"),
         fn_pred=torch.zeros((B, 2), **f64), stats=torch.zeros((B, _abi.NSTATS), dtype=torch.int32, device="cuda"))
stream = torch.cuda.current_stream().cuda_stream
# name:dbg[:ENV=VAL...]  (e.g. pageable_reg:0:FFDDP_HOSTIO_REGISTER=1)
configs = [c.split(":") for c in (os.environ.get("HOSTIO_CONFIGS") or "pageable:0,pinned:0").split(",")]
for name, dbg, *envs in configs:
    os.environ["FFDDP_HOSTIO_DBG"] = dbg
    for k in ("FFDDP_HOSTIO_REGISTER", "FFDDP_COPY_THREADS"):
        os.environ.pop(k, None)
    for e in envs:
        k, v = e.split("=", 1)
        os.environ[k] = v
    outputs = "pinned" if name.startswith("pinned") else ("fresh" if name.startswith(("fresh", "pageable")) else "recycled")
    s = BatchedBoxFDDP(cfg, max_batch=B, outputs=outputs)
    s.solve(b)
    s.solve_dev(T, stream=stream)
    torch.cuda.synchronize()
    th, td = [], []
    for _ in range(reps):
        t0 = time.perf_counter()
        s.solve_dev(T, stream=stream)
        torch.cuda.synchronize()
        td.append(time.perf_counter() - t0)
        os.environ["FFDDP_HOSTIO_TIMING"] = "1"
        t0 = time.perf_counter()
        s.solve(b)
        th.append(time.perf_counter() - t0)
        del os.environ["FFDDP_HOSTIO_TIMING"]
    print(f"{name}/dbg{dbg}: host ms", " ".join("%.2f" % (t * 1e3) for t in th),
          "| dev ms", " ".join("%.2f" % (t * 1e3) for t in td),
          "-> host %.0f dev %.0f solves/s" % (B / np.median(th), B / np.median(td)), flush=True)
    s.close()
