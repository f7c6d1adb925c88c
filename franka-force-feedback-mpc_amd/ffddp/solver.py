"""Crocoddyl-like solver surface over the batched HIP (Box)FDDP.

Mirrors what the reference uses of crocoddyl.SolverBoxFDDP
(crocoddyl_classical.py:350-388, 442-445; crocoddyl_force_feedback.py:588-628):

    solver = BatchedBoxFDDP(cfg, max_batch)            # SolverBoxFDDP(problem)
    ok = solver.solve(batch, maxiter=10, is_feasible=False)   # solver.solve(...)
    solver.xs, solver.us, solver.K, solver.cost, solver.iter  # read-backs

with a leading batch axis.  Numerical failure never raises (ok[b] = False,
like Crocoddyl); API / device errors raise RuntimeError.

Solver properties (th_stop, th_acceptnegstep, reg_min, ...) are attributes as
on crocoddyl.SolverBoxFDDP; setCallbacks([CallbackVerbose()]) prints the
per-iteration record of instance 0 after each solve (ffddp.callbacks).
"""
from __future__ import annotations

import ctypes as C
import threading
import weakref

import numpy as np

from . import _abi
from .config import OcpConfig


class FfddpError(RuntimeError):
    pass


_PARAMS = ("th_stop", "th_grad", "th_acceptstep", "th_acceptnegstep", "th_stepdec", "th_stepinc", "reg_min",
           "reg_max", "reg_incfactor", "reg_decfactor", "neg_step_rule")


class _RecycledPinned:
    """Page-locked host blocks (ffddp_host_alloc) for solve()'s output arrays,
    recycled instead of freed: every solve() returns fresh arrays (no other
    live array shares their memory), and when the last array viewing a block
    is gone (weakref finalizer) the block goes back to the free list rather
    than to the allocator.  In steady state a solve then neither faults in
    nor unmaps ~118 MB of output pages (B = 4096), and ffddp_solve_batch
    copies into them by DMA as each slice finishes (no staging copy).  At
    most `cap` bytes are page-locked; past that solve() falls back to plain
    numpy arrays."""

    def __init__(self, cap: int):
        self.cap = int(cap)
        self.total = 0
        self.free = {}  # nbytes -> [addresses]
        self.closed = False
        self.lock = threading.Lock()

    def arrays(self, specs):
        offs, tot = {}, 0
        for k, (shape, dt) in specs.items():
            offs[k] = tot
            tot += (int(np.prod(shape)) * np.dtype(dt).itemsize + 255) // 256 * 256
        tot = max(tot, 1)
        with self.lock:
            lst = self.free.get(tot)
            p = lst.pop() if lst else None
            if p is None and self.total + tot <= self.cap:
                self.total += tot
                p = -1
        if p is None:
            return None
        if p == -1:
            q = C.c_void_p()
            if _abi.load().ffddp_host_alloc(tot, C.byref(q)) != 0:
                with self.lock:
                    self.total -= tot
                return None
            p = q.value
        buf = (C.c_char * tot).from_address(p)
        weakref.finalize(buf, self._give_back, tot, p)
        return {k: np.frombuffer(buf, dtype=dt, count=int(np.prod(shape)), offset=offs[k]).reshape(shape)
                for k, (shape, dt) in specs.items()}

    def _give_back(self, tot, p):
        with self.lock:
            if not self.closed:
                self.free.setdefault(tot, []).append(p)
                return
            self.total -= tot
        _abi.load().ffddp_host_free(C.c_void_p(p))

    def close(self):
        with self.lock:
            self.closed = True
            blocks = [(t, p) for t, lst in self.free.items() for p in lst]
            self.free = {}
            self.total -= sum(t for t, _ in blocks)
        lib = _abi.load()
        for _, p in blocks:
            lib.ffddp_host_free(C.c_void_p(p))


class BatchedBoxFDDP:
    def __init__(self, cfg: OcpConfig, max_batch: int, device: int = 0, pinned_outputs: bool = False,
                 outputs: str | None = None):
        """outputs: how solve() returns xs / us / K / cost / ...:
          "recycled" (default): fresh numpy arrays per solve() in page-locked
              memory recycled from earlier solves whose arrays are gone
              (_RecycledPinned; up to 4 solves' worth at max_batch), filled by
              DMA as each slice finishes;
          "fresh": fresh pageable numpy arrays per solve() (np.zeros, filled
              through the library's staging buffer);
          "pinned" (or pinned_outputs=True): page-locked arrays owned by the
              solver and overwritten by the next solve() -- copy what must
              outlive it, as the reference does (crocoddyl_classical.py:
              382-385)."""
        self.cfg = cfg
        if outputs is None:
            outputs = "pinned" if pinned_outputs else "recycled"
        if outputs not in ("recycled", "fresh", "pinned"):
            raise ValueError(f"outputs={outputs!r}")
        self.outputs = outputs
        self.pinned_outputs = outputs == "pinned"
        self._pin = {}
        self._pool = None
        self._callbacks = []
        self._trace_it = 0
        self._plans = weakref.WeakSet()  # live SolvePlans: closed before the handle
        self.N = int(cfg.horizon)
        self.nx = cfg.nx
        self.nu = 7
        self.max_batch = int(max_batch)
        self._lib = _abi.load()
        self._cfg_struct = cfg.to_struct()
        h = C.c_void_p()
        rc = self._lib.ffddp_create(
            C.byref(_abi.robot_struct()), C.byref(self._cfg_struct), int(device), self.max_batch, C.byref(h)
        )
        if rc != 0:
            raise FfddpError(f"ffddp_create failed with code {rc}")
        self._h = h
        self.xs = self.us = self.K = self.cost = self.iter = self.ok = self.fn_pred = self.stats = None
        if outputs == "recycled":
            N, nx, Bm = self.N, self.nx, self.max_batch
            one = 8 * Bm * ((N + 1) * nx + N * 7 + N * 7 * nx + 1 + 2) + 4 * Bm * (1 + _abi.NSTATS) + Bm + 8 * 256
            self._pool = _RecycledPinned(4 * one)

    # -- solver properties (crocoddyl SolverFDDP / SolverBoxFDDP attributes) ----------
    @property
    def solver_params(self) -> _abi.SolverParams:
        p = _abi.SolverParams()
        self._check(self._lib.ffddp_get_solver_params(self._h, C.byref(p)), "ffddp_get_solver_params")
        return p

    @solver_params.setter
    def solver_params(self, p: _abi.SolverParams):
        self._check(self._lib.ffddp_set_solver_params(self._h, C.byref(p)), "ffddp_set_solver_params")

    def __getattr__(self, name):
        if name in _PARAMS:
            return getattr(self.solver_params, name)
        raise AttributeError(name)

    def __setattr__(self, name, value):
        if name in _PARAMS:
            p = self.solver_params
            setattr(p, name, value)
            self.solver_params = p
        else:
            object.__setattr__(self, name, value)

    # -- callbacks / per-iteration trace ------------------------------------------------
    def setCallbacks(self, callbacks, max_iters: int = 64):
        """crocoddyl solver.setCallbacks (crocoddyl_classical.py:353): the device
        keeps a per-iteration record (include/ffddp.h ffddp_trace_*); every
        callback is called with (solver, trace) after each solve."""
        callbacks = list(callbacks)
        self.trace_enable(max_iters if callbacks else 0)  # raises while a SolvePlan is open
        self._callbacks = callbacks

    def getCallbacks(self):
        return list(self._callbacks)

    def trace_enable(self, max_iters: int):
        """Fails (FfddpError) while a SolvePlan of this solver is open: a
        plan's graph keeps the trace buffer it was captured with."""
        self._check(self._lib.ffddp_trace_enable(self._h, int(max_iters)), "ffddp_trace_enable")
        self._trace_it = int(max_iters)

    def trace(self, B: int | None = None) -> np.ndarray:
        """[B][max_iters][TRACE_W] records of the last solve (NaN rows for
        iterations an instance did not run); fields _abi.TRACE_FIELDS."""
        if self._trace_it == 0:
            raise FfddpError("trace not enabled (trace_enable / setCallbacks)")
        B = int(self.cost.shape[0]) if B is None else int(B)
        out = np.zeros((B, self._trace_it, _abi.TRACE_W))
        self._check(self._lib.ffddp_trace_read(self._h, B, _abi.dptr(out)), "ffddp_trace_read")
        return out

    def _run_callbacks(self, B):
        if self._callbacks:
            tr = self.trace(B)
            for cb in self._callbacks:
                cb(self, tr)

    # -- lifecycle ------------------------------------------------------------------
    def close(self):
        for plan in list(getattr(self, "_plans", ())):
            plan.close()
        if getattr(self, "_pool", None) is not None:
            self._pool.close()
        if getattr(self, "_h", None) is not None and self._h.value:
            self._lib.ffddp_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, rc: int, what: str):
        if rc != 0:
            msg = self._lib.ffddp_last_error(self._h)
            raise FfddpError(f"{what} failed ({rc}): {msg.decode() if msg else ''}")

    # -- solve (host arrays) ----------------------------------------------------------
    def pinned_batch(self, batch):
        """A copy of `batch`'s solve inputs in page-locked host memory
        (ffddp_host_alloc): solve() then copies them by DMA per slice on the
        slice streams, overlapping the other slices' kernels, instead of
        staging them.  For callers that refill the same input arrays every
        tick."""
        import types

        B, N, nx = int(batch.x0.shape[0]), self.N, self.nx
        specs = dict(x0=((B, nx), np.float64), node_ref=((B, N + 1, 6), np.float64),
                     inst_ref=((B, 21), np.float64), surface=((B,), np.uint8),
                     xs_init=((B, N + 1, nx), np.float64), us_init=((B, N, 7), np.float64))
        o = _abi.pinned_arrays(specs)
        for k, (shape, dt) in specs.items():
            o[k][...] = np.asarray(getattr(batch, k), dt).reshape(shape)
        return types.SimpleNamespace(**o)

    def solve(self, batch, maxiter: int = 10, is_feasible: bool = False, xs_init=None, us_init=None):
        """batch: workload.Batch (or any object with x0, node_ref, inst_ref, surface,
        xs_init, us_init).  Returns ok (B,) bool."""
        B = int(batch.x0.shape[0])
        N, nx = self.N, self.nx
        f = lambda a, shape: np.ascontiguousarray(np.asarray(a, np.float64).reshape(shape))
        x0 = f(batch.x0, (B, nx))
        nref = f(batch.node_ref, (B, N + 1, 6))
        iref = f(batch.inst_ref, (B, 21))
        surf = np.ascontiguousarray(np.asarray(batch.surface, np.uint8).reshape(B))
        xsi = f(batch.xs_init if xs_init is None else xs_init, (B, N + 1, nx))
        usi = f(batch.us_init if us_init is None else us_init, (B, N, 7))
        specs = dict(xs=((B, N + 1, nx), np.float64), us=((B, N, 7), np.float64), K=((B, N, 7, nx), np.float64),
                     cost=((B,), np.float64), iters=((B,), np.int32), ok=((B,), np.uint8), fn=((B, 2), np.float64),
                     stats=((B, _abi.NSTATS), np.int32))
        o = None
        if self.outputs == "pinned":
            if B not in self._pin:
                self._pin = {B: _abi.pinned_arrays(specs)}
            o = self._pin[B]
        elif self.outputs == "recycled":
            o = self._pool.arrays(specs)
        if o is None:
            o = {k: np.zeros(shape, dt) for k, (shape, dt) in specs.items()}
        xs, us, K, cost, iters, ok, fn, stats = (o[k] for k in ("xs", "us", "K", "cost", "iters", "ok", "fn", "stats"))
        d, i, u = _abi.dptr, _abi.iptr, _abi.uptr
        rc = self._lib.ffddp_solve_batch(
            self._h, B, d(x0), d(nref), d(iref), u(surf), d(xsi), d(usi), int(maxiter), int(bool(is_feasible)),
            d(xs), d(us), d(K), d(cost), i(iters), u(ok), d(fn), i(stats),
        )
        self._check(rc, "ffddp_solve_batch")
        self.xs, self.us, self.K, self.cost, self.iter = xs, us, K, cost, iters
        self.ok, self.fn_pred, self.stats = ok.astype(bool), fn, stats
        self._run_callbacks(B)
        return self.ok

    # -- solve plan (receding-horizon loop: one graph launch per tick) -----------------
    def plan(self, B: int, maxiter: int = 10, is_feasible: bool = False) -> "SolvePlan":
        """ffddp_plan_create: the host-array solve of B instances captured as one
        HIP graph; see SolvePlan."""
        plan = SolvePlan(self, B, maxiter, is_feasible)
        self._plans.add(plan)
        return plan

    # -- solve (device-resident torch tensors; bench path) ---------------------------
    def solve_dev(self, t, maxiter: int = 10, is_feasible: bool = False, stream=None):
        """t: dict of contiguous torch.cuda tensors with keys x0, node_ref, inst_ref,
        surface (uint8), xs_init, us_init and outputs xs, us, K, cost, iters (int32),
        ok (uint8), fn_pred, stats (int32).  Asynchronous on `stream` (hipStream_t int)."""
        B = int(t["x0"].shape[0])
        p = lambda k: C.c_void_p(int(t[k].data_ptr()))
        rc = self._lib.ffddp_solve_batch_dev(
            self._h, B, p("x0"), p("node_ref"), p("inst_ref"), p("surface"), p("xs_init"), p("us_init"),
            int(maxiter), int(bool(is_feasible)), p("xs"), p("us"), p("K"), p("cost"), p("iters"), p("ok"),
            p("fn_pred"), p("stats"), C.c_void_p(stream if stream else 0),
        )
        self._check(rc, "ffddp_solve_batch_dev")

    # -- device-side problem builder ----------------------------------------------
    def build_problem_dev(self, task, t, stream=None):
        """Fill t["node_ref"], t["inst_ref"], t["surface"] on the device from
        t["t0"] (B,) and t["x0"] (B, nx) for `task` (_abi.Task / make_task):
        _build_problem's references (crocoddyl_classical.py:521-556) for B
        instances in one launch.  Asynchronous on `stream`."""
        B = int(t["x0"].shape[0])
        p = lambda k: C.c_void_p(int(t[k].data_ptr()))
        rc = self._lib.ffddp_build_problem_dev(
            self._h, B, C.byref(task), p("t0"), p("x0"), p("node_ref"), p("inst_ref"), p("surface"),
            C.c_void_p(stream if stream else 0),
        )
        self._check(rc, "ffddp_build_problem_dev")

    # -- per-kernel device timing ----------------------------------------------------
    def profile(self, on=True):
        """on: True (every kernel class), False, or an iterable of class names
        from _abi.KERNEL_CLASSES to time only those."""
        if on is True:
            mask = (1 << len(_abi.KERNEL_CLASSES)) - 1
        elif not on:
            mask = 0
        else:
            mask = 0
            for name in on:
                mask |= 1 << _abi.KERNEL_CLASSES.index(name)
        self._check(self._lib.ffddp_profile_enable(self._h, int(mask)), "ffddp_profile_enable")

    def profile_read(self, reset: bool = True) -> dict:
        ms = np.zeros(len(_abi.KERNEL_CLASSES))
        n = np.zeros(len(_abi.KERNEL_CLASSES), np.int64)
        self._check(
            self._lib.ffddp_profile_read(self._h, _abi.dptr(ms), n.ctypes.data_as(C.POINTER(C.c_int64)), int(reset)),
            "ffddp_profile_read",
        )
        return {k: (float(ms[i]), int(n[i])) for i, k in enumerate(_abi.KERNEL_CLASSES)}

    # -- problem.calcDiff(xs, us) -------------------------------------------------------
    def calc_diff(self, batch, xs, us):
        B = int(batch.x0.shape[0])
        N, nx = self.N, self.nx
        f = lambda a, shape: np.ascontiguousarray(np.asarray(a, np.float64).reshape(shape))
        out = dict(
            Fx=np.zeros((B, N, nx, nx)), Fu=np.zeros((B, N, nx, 7)), Lx=np.zeros((B, N + 1, nx)),
            Lu=np.zeros((B, N, 7)), Lxx=np.zeros((B, N + 1, nx, nx)), Lxu=np.zeros((B, N, nx, 7)),
            Luu=np.zeros((B, N, 7, 7)), cost=np.zeros((B, N + 1)), xnext=np.zeros((B, N, nx)),
            lam=np.zeros((B, N + 1, 3)),
        )
        d = _abi.dptr
        rc = self._lib.ffddp_calc_diff(
            self._h, B, d(f(batch.x0, (B, nx))), d(f(batch.node_ref, (B, N + 1, 6))), d(f(batch.inst_ref, (B, 21))),
            _abi.uptr(np.ascontiguousarray(np.asarray(batch.surface, np.uint8))), d(f(xs, (B, N + 1, nx))),
            d(f(us, (B, N, 7))), d(out["Fx"]), d(out["Fu"]), d(out["Lx"]), d(out["Lu"]), d(out["Lxx"]),
            d(out["Lxu"]), d(out["Luu"]), d(out["cost"]), d(out["xnext"]), d(out["lam"]),
        )
        self._check(rc, "ffddp_calc_diff")
        return out


class SolvePlan:
    """A captured solve of a fixed batch (include/ffddp.h ffddp_plan_*): the
    per-tick solve of a receding-horizon loop (crocoddyl_classical.py:367,
    run_classical.py:412) as one graph launch -- inputs up, every kernel,
    outputs down.  Fill the input views (x0, node_ref, inst_ref, surface,
    xs_init, us_init: page-locked numpy arrays owned by the plan) in place,
    call run(); the output views (xs, us, K, cost, iter, ok, fn_pred, stats)
    hold the last run's solution and are overwritten by the next run, so copy
    what must outlive it.  Same results as BatchedBoxFDDP.solve, bit for bit."""

    def __init__(self, solver: BatchedBoxFDDP, B: int, maxiter: int, is_feasible: bool):
        self.solver, self.B, self.maxiter = solver, int(B), int(maxiter)
        lib = solver._lib
        io = _abi.PlanIO()
        h = C.c_void_p()
        solver._check(lib.ffddp_plan_create(solver._h, self.B, self.maxiter, int(bool(is_feasible)), C.byref(h),
                                            C.byref(io)), "ffddp_plan_create")
        self._h, self._lib = h, lib
        B, N, nx = self.B, solver.N, solver.nx

        def view(ptr, shape, ct, dt):
            return np.ctypeslib.as_array(C.cast(ptr, C.POINTER(ct)), shape=shape).view(dt)

        f, i32, u8 = C.c_double, C.c_int32, C.c_uint8
        self.x0 = view(io.x0, (B, nx), f, np.float64)
        self.node_ref = view(io.node_ref, (B, N + 1, 6), f, np.float64)
        self.inst_ref = view(io.inst_ref, (B, 21), f, np.float64)
        self.surface = view(io.surface, (B,), u8, np.uint8)
        self.xs_init = view(io.xs_init, (B, N + 1, nx), f, np.float64)
        self.us_init = view(io.us_init, (B, N, 7), f, np.float64)
        self.xs = view(io.xs, (B, N + 1, nx), f, np.float64)
        self.us = view(io.us, (B, N, 7), f, np.float64)
        self.K = view(io.K, (B, N, 7, nx), f, np.float64)
        self.cost = view(io.cost, (B,), f, np.float64)
        self.iter = view(io.iters, (B,), i32, np.int32)
        self._ok = view(io.ok, (B,), u8, np.uint8)
        self.fn_pred = view(io.fn_pred, (B, 2), f, np.float64)
        self.stats = view(io.stats, (B, _abi.NSTATS), i32, np.int32)

    @property
    def ok(self) -> np.ndarray:
        return self._ok.astype(bool)

    def fill(self, batch, xs_init=None, us_init=None):
        """Copy a workload.Batch (and optional warm start) into the input views."""
        self.x0[...] = np.asarray(batch.x0, np.float64).reshape(self.x0.shape)
        self.node_ref[...] = np.asarray(batch.node_ref, np.float64).reshape(self.node_ref.shape)
        self.inst_ref[...] = np.asarray(batch.inst_ref, np.float64).reshape(self.inst_ref.shape)
        self.surface[...] = np.asarray(batch.surface, np.uint8).reshape(self.surface.shape)
        self.xs_init[...] = np.asarray(batch.xs_init if xs_init is None else xs_init, np.float64).reshape(
            self.xs_init.shape)
        self.us_init[...] = np.asarray(batch.us_init if us_init is None else us_init, np.float64).reshape(
            self.us_init.shape)

    def run(self) -> np.ndarray:
        if self._h is None:
            raise FfddpError("plan closed")
        if self.solver._h is None:
            raise FfddpError("the plan's solver is closed")
        self.solver._check(self._lib.ffddp_plan_run(self._h), "ffddp_plan_run")
        self.solver._run_callbacks(self.B)
        return self.ok

    def close(self):
        if getattr(self, "_h", None) is not None and self._h.value:
            self._lib.ffddp_plan_destroy(self._h)
        self._h = None
        plans = getattr(getattr(self, "solver", None), "_plans", None)
        if plans is not None:
            plans.discard(self)

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
