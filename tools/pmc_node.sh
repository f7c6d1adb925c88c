#!/bin/bash
# PMC passes over k_node alone (tools/node_time.py: 5 calcDiff launches of
# B instances): FETCH_SIZE, WRITE_SIZE, L2 hit/miss + read requests.
# usage: tools/pmc_node.sh TAG [B]
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
TAG=${1:-pmcnode}; B=${2:-4096}
O=$R/gpurun_out/$TAG; rm -rf $O; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/f -o f -- python3 $R/tools/node_time.py $B > $O/f.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/w -o w -- python3 $R/tools/node_time.py $B > $O/w.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum --output-format csv -d $O/h -o h -- python3 $R/tools/node_time.py $B > $O/h.log 2>&1
python3 - <<PY
import csv, glob, collections
for d in ("f", "w", "h"):
    tot = collections.defaultdict(float); n = collections.defaultdict(set)
    for fn in glob.glob("$O/%s/**/*counter_collection.csv" % d, recursive=True):
        for row in csv.DictReader(open(fn)):
            low = {k.lower(): v for k, v in row.items()}
            if "k_node" not in low.get("kernel_name", ""): continue
            tot[low["counter_name"]] += float(low["counter_value"]); n[low["counter_name"]].add(low.get("dispatch_id"))
    for k, v in tot.items():
        print(d, k, "per launch %.4g" % (v / max(1, len(n[k]))), "launches", len(n[k]))
PY
