"""Quick device-resident timing of the batched solve (development tool)."""
import sys, time, pathlib
sys.path.insert(0, str(pathlib.Path(__file__).resolve().parents[1]))
import ffddp_path  # noqa
import numpy as np, torch
from ffddp import BatchedBoxFDDP, _abi, workload, robot as R
from ffddp.config import classical_preset, ff_preset

B = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
variant = sys.argv[2] if len(sys.argv) > 2 else "classical"
N = 30
cfg = ff_preset(N) if variant == "ff" else classical_preset(N)
ee = R.R_MJ_FROM_PIN @ _abi.frame_placement(R.Q_NEUTRAL)[1]
t = time.time()
b = workload.make_batch(B, N, variant, _abi.gravity_torque, ee, seed=0, fk=_abi.frame_placement)
print("batch gen %.1fs" % (time.time() - t), flush=True)
nx = cfg.nx
dev = "cuda"
T = dict(
    x0=torch.tensor(b.x0, device=dev), node_ref=torch.tensor(b.node_ref, device=dev),
    inst_ref=torch.tensor(b.inst_ref, device=dev), surface=torch.tensor(b.surface, device=dev),
    xs_init=torch.tensor(b.xs_init, device=dev), us_init=torch.tensor(b.us_init, device=dev),
    xs=torch.zeros((B, N + 1, nx), dtype=torch.float64, device=dev), us=torch.zeros((B, N, 7), dtype=torch.float64, device=dev),
    K=torch.zeros((B, N, 7, nx), dtype=torch.float64, device=dev), cost=torch.zeros(B, dtype=torch.float64, device=dev),
    iters=torch.zeros(B, dtype=torch.int32, device=dev), ok=torch.zeros(B, dtype=torch.uint8, device=dev),
    fn_pred=torch.zeros((B, 2), dtype=torch.float64, device=dev), stats=torch.zeros((B, 4), dtype=torch.int32, device=dev),
)
s = BatchedBoxFDDP(cfg, max_batch=B)
for rep in range(4):
    torch.cuda.synchronize(); t = time.time()
    s.solve_dev(T, maxiter=10)
    torch.cuda.synchronize(); dt = time.time() - t
    print("rep %d: %.2f ms  -> %.0f solves/s" % (rep, dt * 1e3, B / dt), flush=True)
ok = T["ok"].cpu().numpy(); it = T["iters"].cpu().numpy(); st = T["stats"].cpu().numpy()
print("ok frac", ok.mean(), "iters mean", it.mean(), "stats mean", st.mean(0), "cost finite", np.isfinite(T["cost"].cpu().numpy()).mean())
