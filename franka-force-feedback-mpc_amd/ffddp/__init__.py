"""ffddp — MI355X-native batched (Box)FDDP for the Franka force-feedback MPC.

Drop-in for the reference's `solver.solve(xs_init, us_init, max_iters, False)`
(src/mpc/crocoddyl_classical.py:367, src/mpc/crocoddyl_force_feedback.py:605).
Host Python -> ctypes -> C-ABI (include/ffddp.h) -> hand-written HIP kernels.
"""
from .config import OcpConfig, classical_preset, ff_preset  # noqa: F401
from .solver import BatchedBoxFDDP, FfddpError  # noqa: F401
from .callbacks import CallbackVerbose  # noqa: F401
