#!/usr/bin/env python3
"""Useful (algorithmic) fp64 flops per unit of work, counted by executing the
scalar C++ CPU baseline with a counting fp64 type (tools/flops/flop_count.cpp;
VERDICT r05 item 5).  The baseline runs the product's node models on one
instance at a time with Crocoddyl's dense backward pass, so its counts are
the work the algorithm needs, with no SIMD lanes idle or duplicated:

  node      calc + calcDiff of one node (per node stage)
  backward  per backward node (dense Fx'VFx, Fx'VFu, Fu'VFu, Cholesky / BoxQP gains,
            Vxx / Vx update, expected-improvement terms; SURVEY a12 prices it at
            ~23.3 kflop classical)
  forward   per line-search trial node (control law + the node's calc)

flops = add/sub + mul + div + 2 fma + sqrt (+ sin / cos counted as 1 each, only
in set-up).  The sample is the bench's own seeded workload (workload.make_batch,
seed 1234, the tracking regime unless --regime), first --sample instances;
bench.py multiplies these per-unit figures by its run's device-counted units
(roofline.fp64.useful).

usage: python tools/flop_count.py [--sample 256] [--out profiles/r06_useful_flops.json]
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import subprocess
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import ffddp_path  # noqa: E402,F401
import numpy as np  # noqa: E402

from ffddp import _abi, robot as R, workload  # noqa: E402
from ffddp.config import classical_preset, ff_preset  # noqa: E402

SRC = ROOT / "tools" / "flops" / "flop_count.cpp"
LIB = ROOT / "tools" / "flops" / "libflopcount.so"
KINDS = ("add", "mul", "div", "fma", "sqrt", "trans")
PHASES = ("other", "node", "backward", "forward")
# the configurations bench.py and the BASELINE configs run
CONFIGS = {
    "classical/normal_1d/N30": dict(variant="classical", contact="normal_1d", N=30),
    "ff/normal_1d/N30": dict(variant="ff", contact="normal_1d", N=30),
    "classical/point3d/N100": dict(variant="classical", contact="point3d", N=100),
}


def build():
    deps = [SRC, ROOT / "oracle" / "cpu" / "ffddp_cpu.cpp"] + list((ROOT / "franka-force-feedback-mpc_amd" / "csrc").glob("*.hpp"))
    if LIB.exists() and all(LIB.stat().st_mtime > d.stat().st_mtime for d in deps):
        return
    subprocess.run(["g++", "-O2", "-std=c++17", "-fPIC", "-shared", "-fopenmp", "-D__HIP_PLATFORM_AMD__",
                    "-I/opt/rocm/include", "-Wno-class-memaccess", "-o", str(LIB), str(SRC)], check=True)


def count(name, variant, contact, N, sample, regime, maxiter=10):
    lib = C.CDLL(str(LIB))
    cfg = ff_preset(N, contact) if variant == "ff" else classical_preset(N, contact)
    nx = cfg.nx
    ee = R.R_MJ_FROM_PIN @ _abi.frame_placement(R.Q_NEUTRAL)[1]
    b = workload.make_batch(sample, N, variant, _abi.gravity_torque, ee, seed=1234, regime=regime,
                            fk=_abi.frame_placement)
    B = sample
    f = lambda a, shape: np.ascontiguousarray(np.asarray(a, np.float64).reshape(shape))
    x0, nref, iref = f(b.x0, (B, nx)), f(b.node_ref, (B, N + 1, 6)), f(b.inst_ref, (B, 21))
    surf = np.ascontiguousarray(np.asarray(b.surface, np.uint8).reshape(B))
    xsi, usi = f(b.xs_init, (B, N + 1, nx)), f(b.us_init, (B, N, 7))
    xs, us, K = np.zeros((B, N + 1, nx)), np.zeros((B, N, 7)), np.zeros((B, N, 7, nx))
    cost, iters, ok = np.zeros(B), np.zeros(B, np.int32), np.zeros(B, np.uint8)
    stats = np.zeros((B, _abi.NSTATS), np.int32)
    cnt = np.zeros((4, 6), np.uint64)
    units = np.zeros(4, np.uint64)
    vp = lambda a: C.c_void_p(a.ctypes.data)
    rs, cs = _abi.robot_struct(), cfg.to_struct()
    t0 = time.perf_counter()
    rc = lib.flop_count_solve(C.byref(rs), C.byref(cs), B, vp(x0), vp(nref), vp(iref), vp(surf), vp(xsi), vp(usi),
                              int(maxiter), vp(xs), vp(us), vp(K), vp(cost), vp(iters), vp(ok), vp(stats), vp(cnt),
                              vp(units))
    if rc != 0:
        raise RuntimeError(f"flop_count_solve failed ({rc})")
    wall = time.perf_counter() - t0
    out = {"config": name, "regime": regime, "sample": B, "maxiter": maxiter, "wall_s": wall,
           "ok_frac": float(ok.mean()), "mean_iter": float(iters.mean()), "phases": {}}
    for p, ph in enumerate(PHASES):
        c = {k: int(cnt[p, i]) for i, k in enumerate(KINDS)}
        flops = c["add"] + c["mul"] + c["div"] + 2 * c["fma"] + c["sqrt"] + c["trans"]
        e = {"counts": c, "flops": flops, "units": int(units[p])}
        if units[p]:
            e["flops_per_unit"] = flops / float(units[p])
        out["phases"][ph] = e
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sample", type=int, default=256)
    ap.add_argument("--regime", default="tracking")
    ap.add_argument("--out", default=str(ROOT / "profiles" / "r06_useful_flops.json"))
    ap.add_argument("--configs", default=",".join(CONFIGS))
    args = ap.parse_args()
    build()
    res = {"source": "tools/flop_count.py (tools/flops/flop_count.cpp: the scalar C++ CPU baseline, oracle/cpu/"
                     "ffddp_cpu.cpp, executed with a counting fp64 type)",
           "flops_rule": "add/sub + mul + div + 2*fma + sqrt (+ sin/cos 1 each)", "configs": {}}
    for name in args.configs.split(","):
        c = CONFIGS[name]
        r = count(name, c["variant"], c["contact"], c["N"], args.sample, args.regime)
        res["configs"][name] = r
        print(name, f"sample {r['sample']} ok {r['ok_frac']:.3f} iters {r['mean_iter']:.2f} ({r['wall_s']:.1f} s):",
              " ".join(f"{ph}={e['flops_per_unit']:.0f}/unit" for ph, e in r["phases"].items() if "flops_per_unit" in e),
              flush=True)
    Path(args.out).write_text(json.dumps(res, indent=1) + "\n")


if __name__ == "__main__":
    main()
