#!/usr/bin/env python3
"""Per-kernel SQ counters from tools/pmc_sq2.sh passes: sums and per-wave
averages per kernel (template variants kept apart, e.g. the two backward
variants), then the derived ratios per kernel.  SQ_WAVE_CYCLES, SQ_WAIT_* and
SQ_ACTIVE_INST_* all count quad-cycles (MI355X_MICROARCH.md, PMC units), and
WAIT_ANY + WAIT_INST_ANY + ACTIVE_INST_ANY ~= WAVE_CYCLES, so:
  FMA share    SQ_INSTS_VALU_FMA_F64 / SQ_INSTS_VALU
  VALU-active  SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES
  LDS-active   SQ_ACTIVE_INST_LDS / SQ_WAVE_CYCLES
  waiting      SQ_WAIT_ANY / SQ_WAVE_CYCLES   (parked on s_waitcnt / barrier)
  issue-stall  SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES
  bank conflicts per wave  SQ_LDS_BANK_CONFLICT / SQ_WAVES
Per-wave averages include waves that exit at once (grid slots past the active
count), so per-wave figures are lower bounds of a working wave's."""
import csv
import re
import sys
from collections import defaultdict
from pathlib import Path


def kclass(n):
    m = re.search(r"k_[a-z0-9_]+(<[^>(]*>)?", n)
    return m.group(0)[2:].replace(" ", "") if m else None


args = [a for a in sys.argv[1:] if not a.startswith("--")]
opts = dict(a[2:].split("=", 1) for a in sys.argv[1:] if a.startswith("--") and "=" in a)
tot = defaultdict(lambda: defaultdict(float))
for f in Path(args[0]).rglob("*counter_collection.csv"):
    for row in csv.DictReader(f.open()):
        low = {k.lower(): v for k, v in row.items()}
        c = kclass(low.get("kernel_name", ""))
        if c:
            tot[c][low["counter_name"]] += float(low["counter_value"])
busy = 0.0
for c, d in tot.items():
    busy += d.get("SQ_ACTIVE_INST_VALU", 0.0) * 4
print(f"VALU-active cycles (all kernels): {busy:.4g}  = {busy / 1024 / 2.4e9 * 1e3:.3f} ms of all 1024 SIMDs at 2.4 GHz")
print()
print(f"{'kernel':34s} {'waves':>8s} {'FMA/VALU':>9s} {'VALU-act':>9s} {'LDS-act':>8s} {'waiting':>8s} "
      f"{'issue-st':>8s} {'bankconf/w':>10s} {'VALU/w':>8s} {'cyc/w':>8s}")
for c, d in sorted(tot.items()):
    w = d.get("SQ_WAVES", 0) or 1
    wc = d.get("SQ_WAVE_CYCLES", 0) or 1
    r = lambda k: d.get(k, 0.0) / wc  # noqa: E731
    fma = d.get("SQ_INSTS_VALU_FMA_F64", 0.0) / (d.get("SQ_INSTS_VALU", 0.0) or 1)
    print(f"{c:34s} {w:8.0f} {fma:9.1%} {r('SQ_ACTIVE_INST_VALU'):9.1%} {r('SQ_ACTIVE_INST_LDS'):8.1%} "
          f"{r('SQ_WAIT_ANY'):8.1%} {r('SQ_WAIT_INST_ANY'):8.1%} {d.get('SQ_LDS_BANK_CONFLICT', 0) / w:10.1f} "
          f"{d.get('SQ_INSTS_VALU', 0) / w:8.0f} {4 * wc / w:8.0f}")
print()
for c, d in sorted(tot.items()):
    w = d.get("SQ_WAVES", 0) or 1
    print(f"== {c}: waves {w:.0f}")
    for k in sorted(d):
        print(f"   {k:24s} total {d[k]:.4g}  per-wave {d[k]/w:.4g}")

if "json" in opts:
    # --json=OUT --config=classical/normal_1d/B4096/N30 --source=profiles/...: the
    # ratios per kernel, for bench.py's roofline.limiter
    import json

    ks = {}
    for c, d in sorted(tot.items()):
        wc = d.get("SQ_WAVE_CYCLES", 0) or 1
        ks[c] = {"waves": d.get("SQ_WAVES", 0),
                 "fma_share_of_valu": d.get("SQ_INSTS_VALU_FMA_F64", 0.0) / (d.get("SQ_INSTS_VALU", 0.0) or 1),
                 "valu_active": d.get("SQ_ACTIVE_INST_VALU", 0.0) / wc,
                 "lds_active": d.get("SQ_ACTIVE_INST_LDS", 0.0) / wc,
                 "waiting": d.get("SQ_WAIT_ANY", 0.0) / wc, "issue_stalled": d.get("SQ_WAIT_INST_ANY", 0.0) / wc,
                 "lds_bank_conflicts_per_wave": d.get("SQ_LDS_BANK_CONFLICT", 0.0) / (d.get("SQ_WAVES", 0) or 1)}
    big = sorted(ks, key=lambda c: -tot[c].get("SQ_WAVE_CYCLES", 0.0))[:4]
    summ = opts.get("summary", "share of wave time VALU-active / waiting, by total wave time: " + "; ".join(
        f"{c} {ks[c]['valu_active']:.0%} / {ks[c]['waiting']:.0%}" for c in big))
    Path(opts["json"]).write_text(json.dumps({"config": opts.get("config"), "source": opts.get("source"),
                                              "summary": summ, "kernels": ks}, indent=1) + "\n")
