"""Per-iteration kernel timeline of one solve from a rocprofv3 kernel trace.

usage: python tools/timeline.py <dir with *kernel_trace.csv> [solve_index]
Prints, for the chosen solve (default: the last one), every dispatch of the
solver kernels as (stream/queue, kernel, start offset us, duration us), then
per queue the sum per kernel class and the time between consecutive kernels
(what a single-launch solve could remove at most).
"""
import csv
import glob
import re
import sys
from collections import defaultdict

d = sys.argv[1]
which = int(sys.argv[2]) if len(sys.argv) > 2 else -1
f = glob.glob(d + "/**/*kernel_trace.csv", recursive=True)[0]
rows = []
for r in csv.DictReader(open(f)):
    name = r["Kernel_Name"]
    m = re.search(r"k_([a-z0-9_]+)", name)
    if not m:
        continue
    rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), m.group(1), r.get("Queue_Id", r.get("Stream_Id", "?"))))
rows.sort()
# a solve starts at each k_init group; group consecutive k_init launches
solves, cur = [], []
for row in rows:
    if row[2] == "init" and cur and cur[-1][2] != "init":
        solves.append(cur)
        cur = []
    cur.append(row)
if cur:
    solves.append(cur)
s = solves[which]
t0 = s[0][0]
print(f"{len(solves)} solves in trace; showing #{which % len(solves)}: span {(s[-1][1] - t0) / 1e3:.1f} us, {len(s)} dispatches")
per_q = defaultdict(list)
for a, b, k, q in s:
    per_q[q].append((a, b, k))
for q, lst in per_q.items():
    print(f"-- queue {q}")
    it = 0
    acc = defaultdict(float)
    for a, b, k in lst:
        print(f"   {k:14s} start {(a - t0) / 1e3:9.1f}  dur {(b - a) / 1e3:8.1f}")
        acc[k] += (b - a) / 1e3
    print("   totals: " + " ".join(f"{k}={v:.0f}" for k, v in acc.items()))
    span = (lst[-1][1] - lst[0][0]) / 1e3
    busy = sum(b - a for a, b, _ in lst) / 1e3
    print(f"   queue span {span:.1f} us, kernels {busy:.1f} us ({busy / max(span, 1e-9):.1%}), gaps {span - busy:.1f} us "
          f"over {len(lst) - 1} launch boundaries ({(span - busy) / max(len(lst) - 1, 1):.2f} us each)")
