#!/usr/bin/env python3
"""fp64 VALU work per kernel class from a tools/pmc_fp64.sh pass (2 solves),
normalised by the device-counted units of those solves (bench.py's
"counts_per_step"; both solves are identical):
  node      per node stage      (calcDiffs x (N + 1))
  backward  per backward node   (backward passes x N)
  forward   per trial node      (evaluated step lengths x (N + 1))
Figures per unit: issued fp64 wave instructions (FMA, MUL, ADD, TRANS),
issued lane-flops = 64 x (2 FMA + MUL + ADD) (every lane of an issued wave
instruction, the issue-rate view), and SQ_INSTS_VALU_FLOPS_FP64 (the
hardware's flop count).  bench.py multiplies them by its own run's units.

usage: pmc_fp64.py PMC_DIR BENCH_LOG --config=classical/normal_1d/B4096/N30 --json=OUT"""
import csv
import json
import re
import sys
from collections import defaultdict
from pathlib import Path

CLASS_OF = (("k_node", "node"), ("k_backward", "backward"), ("k_forward", "forward"), ("k_accept", "accept"),
            ("k_commit", "commit"), ("k_init", "init"), ("k_finalize", "finalize"))
SOLVES = 2

args = [a for a in sys.argv[1:] if not a.startswith("--")]
opts = dict(a[2:].split("=", 1) for a in sys.argv[1:] if a.startswith("--") and "=" in a)
tot = defaultdict(lambda: defaultdict(float))
for f in Path(args[0]).rglob("*counter_collection.csv"):
    for row in csv.DictReader(f.open()):
        low = {k.lower(): v for k, v in row.items()}
        name = low.get("kernel_name", "")
        c = next((c for k, c in CLASS_OF if k in name), None)
        if c:
            tot[c][low["counter_name"]] += float(low["counter_value"])
line = json.loads([ln for ln in Path(args[1]).read_text().splitlines() if ln.startswith("{")][-1])
cnt = line["counts_per_step"]
N = line["config"]["horizon"]
units = {"node": cnt["calcdiff"] * (N + 1), "backward": cnt["backward"] * N, "forward": cnt["trials"] * (N + 1)}
out = {"config": opts.get("config"), "source": "tools/pmc_fp64.sh", "solves": SOLVES, "counts_per_solve": cnt,
       "kernels": {}}
print(f"{'class':10s} {'units/solve':>12s} {'FMA/u':>8s} {'MUL/u':>8s} {'ADD/u':>8s} {'TRANS/u':>8s} "
      f"{'VALU/u':>8s} {'lane-flop/u':>12s} {'hw-flop/u':>10s} {'FMA share':>9s}")
for c, d in sorted(tot.items()):
    per = {k: v / SOLVES for k, v in d.items()}
    lane = 64.0 * (2 * per.get("SQ_INSTS_VALU_FMA_F64", 0) + per.get("SQ_INSTS_VALU_MUL_F64", 0) +
                   per.get("SQ_INSTS_VALU_ADD_F64", 0))
    e = {"fp64_instr_per_solve": sum(per.get(k, 0.0) for k in ("SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_VALU_MUL_F64",
                                                               "SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_TRANS_F64")),
         "valu_instr_per_solve": per.get("SQ_INSTS_VALU", 0.0),
         "lane_flops_per_solve": lane, "hw_flops_per_solve": per.get("SQ_INSTS_VALU_FLOPS_FP64", 0.0),
         "counters_per_solve": per}
    u = units.get(c)
    if u:
        e.update({"units_per_solve": u, "fp64_instr_per_unit": e["fp64_instr_per_solve"] / u,
                  "valu_instr_per_unit": e["valu_instr_per_solve"] / u,
                  "lane_flops_per_unit": lane / u, "hw_flops_per_unit": e["hw_flops_per_solve"] / u})
        print(f"{c:10s} {u:12.0f} {per.get('SQ_INSTS_VALU_FMA_F64', 0) / u:8.1f} "
              f"{per.get('SQ_INSTS_VALU_MUL_F64', 0) / u:8.1f} {per.get('SQ_INSTS_VALU_ADD_F64', 0) / u:8.1f} "
              f"{per.get('SQ_INSTS_VALU_TRANS_F64', 0) / u:8.1f} {e['valu_instr_per_unit']:8.1f} "
              f"{lane / u:12.0f} {e['hw_flops_per_unit']:10.0f} "
              f"{per.get('SQ_INSTS_VALU_FMA_F64', 0) / max(per.get('SQ_INSTS_VALU', 1), 1):9.1%}")
    out["kernels"][c] = e
if "json" in opts:
    Path(opts["json"]).write_text(json.dumps(out, indent=1) + "\n")
