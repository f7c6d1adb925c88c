#!/bin/bash
# Instruction-cache counters per kernel over 2 solves of the bench's timed
# configuration (one --pmc pass), plus the list of the box's counters.
# usage: [BENCH_ARGS="--batch 512"] tools/pmc_icache.sh TAG
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/$1
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 --list-avail > $O/avail.txt 2>&1 || true
grep -iE "ICACHE|IFETCH|SQC_" $O/avail.txt > $O/avail_icache.txt || true
CTRS=${CTRS:-"SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE"}
timeout -s KILL 120 rocprofv3 --pmc $CTRS --output-format csv -d $O/ic -o r -- python3 $R/bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-profile --no-host-io --no-extras $BENCH_ARGS > $O/ic.log 2>&1 || { echo "icache pass failed"; tail -5 $O/ic.log; exit 1; }
python3 - $O <<'PY'
import csv, re, sys
from collections import defaultdict
from pathlib import Path
tot = defaultdict(lambda: defaultdict(float))
for f in Path(sys.argv[1], "ic").rglob("*counter_collection.csv"):
    for row in csv.DictReader(f.open()):
        low = {k.lower(): v for k, v in row.items()}
        m = re.search(r"k_[a-z0-9_]+(<[^>(]*>)?", low.get("kernel_name", ""))
        if m:
            tot[m.group(0)][low["counter_name"]] += float(low["counter_value"])
for k, d in sorted(tot.items()):
    print(k, " ".join(f"{c}={v:.4g}" for c, v in sorted(d.items())))
PY
