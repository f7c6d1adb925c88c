#!/usr/bin/env python3
"""Per-kernel-class sums of SQ counters from tools/pmc_sq.sh passes."""
import csv, sys
from collections import defaultdict
from pathlib import Path

CLASSES = ("node", "backward_w", "backward", "forward", "primal", "accept", "commit", "init", "finalize")


def kclass(n):
    for c in CLASSES:
        if f"k_{c}<" in n or f"k_{c}(" in n:
            return c
    return None


tot = defaultdict(lambda: defaultdict(float))
for f in Path(sys.argv[1]).rglob("*counter_collection.csv"):
    for row in csv.DictReader(f.open()):
        low = {k.lower(): v for k, v in row.items()}
        c = kclass(low.get("kernel_name", ""))
        if c:
            tot[c][low["counter_name"]] += float(low["counter_value"])
for c, d in tot.items():
    w = d.get("SQ_WAVES", 0) or 1
    print(f"== {c}: waves {w:.0f}")
    for k in sorted(d):
        print(f"   {k:24s} total {d[k]:.4g}  per-wave {d[k]/w:.4g}")
