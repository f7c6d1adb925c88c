#!/usr/bin/env python3
"""Per-kernel-class sums of SQ counters from tools/pmc_sq2.sh passes."""
import csv, sys
from collections import defaultdict
from pathlib import Path

import re


def kclass(n):
    m = re.search(r"k_[a-z0-9_]+", n)
    return m.group(0)[2:] if m else None


tot = defaultdict(lambda: defaultdict(float))
for f in Path(sys.argv[1]).rglob("*counter_collection.csv"):
    for row in csv.DictReader(f.open()):
        low = {k.lower(): v for k, v in row.items()}
        c = kclass(low.get("kernel_name", ""))
        if c:
            tot[c][low["counter_name"]] += float(low["counter_value"])
busy = 0.0
for c, d in tot.items():
    busy += d.get("SQ_ACTIVE_INST_VALU", 0.0) * 4
print(f"VALU-active cycles (all kernels): {busy:.4g}  = {busy / 1024 / 2.4e9 * 1e3:.3f} ms of all 1024 SIMDs at 2.4 GHz")
for c, d in tot.items():
    w = d.get("SQ_WAVES", 0) or 1
    print(f"== {c}: waves {w:.0f}")
    for k in sorted(d):
        print(f"   {k:24s} total {d[k]:.4g}  per-wave {d[k]/w:.4g}")
