#!/usr/bin/env python3
"""Static instruction mix of the hot kernels from the device assembly.

Builds (or reads) `hipcc --cuda-device-only -S` output of ffddp_kernels.hip
and, for each kernel whose name matches a pattern, counts the instructions of
the whole kernel and of its largest loop (the span from a label to the
backward branch that returns to it: the per-node loop of the rollout, the
backward pass and k_node's tangent loop), by class:
  fma/mul/add f64, other fp64, DPP moves, v_cndmask (selects), other VALU,
  SALU, LDS, VMEM (global/buffer), waitcnt, branches.
usage: tools/isa_mix.py [--asm FILE] [--extra "-DFOO=1"] PATTERN [PATTERN ...]
(DESIGN.md §5 quotes these counts; test/measurement tooling only)"""
from __future__ import annotations

import argparse
import re
import subprocess
import sys
from collections import Counter
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
SRC = ROOT / "franka-force-feedback-mpc_amd" / "csrc" / "ffddp_kernels.hip"


def classify(ins: str) -> str:
    op = ins.split()[0]
    if op.startswith("v_fma_f64") or op.startswith("v_fmac_f64"):
        return "fma_f64"
    if op.startswith("v_mul_f64"):
        return "mul_f64"
    if op.startswith("v_add_f64"):
        return "add_f64"
    if "_dpp" in op or "row_" in ins or "quad_perm" in ins:
        return "dpp"
    if op.endswith("_f64") or "_f64_" in op:
        return "f64_other"
    if op.startswith("v_cndmask"):
        return "cndmask"
    if op.startswith("v_accvgpr"):
        return "accvgpr"
    if op.startswith("v_"):
        return "valu_other"
    if op.startswith("s_waitcnt"):
        return "waitcnt"
    if op.startswith("s_cbranch") or op.startswith("s_branch"):
        return "branch"
    if op.startswith("s_"):
        return "salu"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("global_", "buffer_", "flat_", "scratch_")):
        return "vmem"
    return "other"


VALU = ("fma_f64", "mul_f64", "add_f64", "dpp", "f64_other", "cndmask", "valu_other", "accvgpr")


def kernels(asm: str):
    """{symbol: [lines]} of every kernel body."""
    out = {}
    cur = None
    for ln in asm.splitlines():
        m = re.match(r"^(_Z\w+):", ln)
        if m:
            cur = m.group(1)
            out[cur] = []
            continue
        if cur and ln.startswith("\t.end_amdhsa_kernel"):
            cur = None
        if cur and (ln.startswith(".Lfunc_end")):
            cur = None
        if cur is not None:
            out[cur].append(ln)
    return out


def mix(lines):
    c = Counter()
    for ln in lines:
        s = ln.strip()
        if not s or s.startswith((";", ".", "_")) or s.endswith(":"):
            continue
        c[classify(s)] += 1
    c["VALU"] = sum(c[k] for k in VALU)
    return c


def largest_loop(lines):
    labels = {}
    best = (0, 0, 0)
    for i, ln in enumerate(lines):
        m = re.match(r"^(\.LBB\w+):", ln)
        if m:
            labels[m.group(1)] = i
        m = re.search(r"s_cbranch_\w+\s+(\.LBB\w+)|s_branch\s+(\.LBB\w+)", ln)
        if m:
            tgt = m.group(1) or m.group(2)
            if tgt in labels and i - labels[tgt] > best[0]:
                best = (i - labels[tgt], labels[tgt], i)
    return lines[best[1]:best[2] + 1] if best[0] else []


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--asm")
    ap.add_argument("--extra", default="")
    ap.add_argument("patterns", nargs="+")
    a = ap.parse_args()
    if a.asm:
        asm = Path(a.asm).read_text()
    else:
        out = "/tmp/ffddp_isa_mix.s"
        cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "--cuda-device-only", "-S",
               "-o", out, str(SRC)] + a.extra.split()
        subprocess.run(cmd, check=True, stderr=subprocess.DEVNULL)
        asm = Path(out).read_text()
    ks = kernels(asm)
    cols = ("VALU", "fma_f64", "mul_f64", "add_f64", "f64_other", "dpp", "cndmask", "valu_other", "accvgpr",
            "salu", "lds", "vmem", "waitcnt", "branch")
    print(f"{'kernel / region':60s} " + " ".join(f"{c[:8]:>8s}" for c in cols))
    for sym, lines in ks.items():
        if not any(re.search(p, sym) for p in a.patterns):
            continue
        name = subprocess.run(["c++filt", sym], capture_output=True, text=True).stdout.strip()
        name = re.sub(r"\(anonymous namespace\)::|ffddp::|\(.*", "", name)
        for tag, reg in (("whole", lines), ("loop", largest_loop(lines))):
            c = mix(reg)
            print(f"{(name + ' ' + tag)[:60]:60s} " + " ".join(f"{c[k]:8d}" for k in cols))
    return 0


if __name__ == "__main__":
    sys.exit(main())
