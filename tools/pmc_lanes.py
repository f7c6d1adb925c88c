#!/usr/bin/env python3
"""VALU lane utilisation per kernel class from tools/pmc_lanes.sh:
  lane utilisation = (SQ_THREAD_CYCLES_VALU / SQ_ACTIVE_INST_VALU) of the
                     kernel / the same ratio of the 64-lane calibration kernel
i.e. the mean fraction of a wave's 64 lanes that are enabled while it issues
VALU instructions.  The 8- and 7-lane calibration kernels check the
normalisation (expected 0.125 and 0.109).  Per kernel also: VALU instructions
per wave and the wave count (waves that exit at once included).
usage: pmc_lanes.py CAL_DIR RUN_DIR --config=... --json=OUT"""
import csv
import json
import re
import sys
from collections import defaultdict
from pathlib import Path


def kclass(n):
    m = re.search(r"k_[a-z0-9_]+(<[^>(]*>)?", n)
    return m.group(0)[2:].replace(" ", "") if m else None


def read(d):
    tot = defaultdict(lambda: defaultdict(float))
    for f in Path(d).rglob("*counter_collection.csv"):
        for row in csv.DictReader(f.open()):
            low = {k.lower(): v for k, v in row.items()}
            c = kclass(low.get("kernel_name", ""))
            if c:
                tot[c][low["counter_name"]] += float(low["counter_value"])
    return tot


args = [a for a in sys.argv[1:] if not a.startswith("--")]
opts = dict(a[2:].split("=", 1) for a in sys.argv[1:] if a.startswith("--") and "=" in a)
cal, run = read(args[0]), read(args[1])
ratio = lambda d: d.get("SQ_THREAD_CYCLES_VALU", 0.0) / (d.get("SQ_ACTIVE_INST_VALU", 0.0) or 1.0)  # noqa: E731
full = ratio(cal["lanes<64>"])
out = {"config": opts.get("config"), "source": "tools/pmc_lanes.sh", "full_lane_ratio": full,
       "calibration": {k: ratio(v) / full for k, v in cal.items()}, "kernels": {}}
print("calibration (expected 1, 0.125, 0.109):", {k: round(v, 4) for k, v in out["calibration"].items()})
print(f"{'kernel':34s} {'waves':>9s} {'VALU/wave':>10s} {'lane util':>10s}")
for c, d in sorted(run.items()):
    w = d.get("SQ_WAVES", 0.0) or 1.0
    u = ratio(d) / full if full else None
    out["kernels"][c] = {"waves": d.get("SQ_WAVES", 0.0), "valu_per_wave": d.get("SQ_INSTS_VALU", 0.0) / w,
                         "lane_util": u, "counters": dict(d)}
    print(f"{c:34s} {w:9.0f} {d.get('SQ_INSTS_VALU', 0.0) / w:10.0f} {u:10.3f}")
if "json" in opts:
    Path(opts["json"]).write_text(json.dumps(out, indent=1) + "\n")
