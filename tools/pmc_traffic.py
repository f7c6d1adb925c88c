#!/usr/bin/env python3
"""Turn rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes into per-solve HBM
bytes for the solver kernels (MI355X_MICROARCH.md §HBM: FETCH_SIZE is reported
in KiB and counts half the bytes of wide streaming reads on gfx950, so it is
doubled; WRITE_SIZE is taken as is).

usage: pmc_traffic.py FETCH_DIR WRITE_DIR CONFIG SOLVES OUT_JSON [SLICE_B]
  CONFIG is bench.py's "<variant>/<contact>/B<B>/N<N>" key; SOLVES the number
  of batched solves each profiled run executed (warmup + steps).  Bytes are
  reported per solve per kernel class (bench.py divides by its own launch
  count of that class).
"""
from __future__ import annotations

import csv
import json
import sys
from collections import defaultdict
from pathlib import Path

# kernel name -> bench/profiler class (ffddp_profile_read classes, one kernel each)
CLASS_OF = (
    ("k_node", "node"), ("k_backward", "backward"), ("k_forward", "forward"),
    ("k_accept", "accept"), ("k_commit", "commit"), ("k_init", "init"), ("k_finalize", "finalize"),
)
SLICE_B = 1024  # instances per sub-batch slice (B / FFDDP_STREAMS)


def kclass(name: str, grid: int = 0):
    for key, c in CLASS_OF:
        if key in name:
            if c == "forward" and grid > 5 * 8 * SLICE_B:
                return "forward2"  # second pass: >= 6 step lengths x 8 lanes per instance
            return c
    return None


def read_counter(d: Path, counter: str):
    """-> {class: (sum of counter over dispatches, n_dispatches)}"""
    files = sorted(d.rglob("*counter_collection.csv"))
    if not files:
        raise SystemExit(f"no counter_collection.csv under {d}")
    tot = defaultdict(float)
    disp = defaultdict(set)
    for f in files:
        with f.open() as fh:
            for row in csv.DictReader(fh):
                low = {k.lower(): v for k, v in row.items()}
                if low.get("counter_name") != counter:
                    continue
                c = kclass(low.get("kernel_name", ""), int(float(low.get("grid_size", 0) or 0)))
                if c is None:
                    continue
                tot[c] += float(low["counter_value"])
                disp[c].add((f, low.get("dispatch_id")))
    return {c: (tot[c], len(disp[c])) for c in tot}


def main():
    global SLICE_B
    fetch_dir, write_dir, config, solves, out = sys.argv[1:6]
    if len(sys.argv) > 6:
        SLICE_B = int(sys.argv[6])
    solves = float(solves)
    fe = read_counter(Path(fetch_dir), "FETCH_SIZE")
    wr = read_counter(Path(write_dir), "WRITE_SIZE")
    kernels = {}
    for c in sorted(set(fe) & set(wr)):
        f_kib, nf = fe[c]
        w_kib, nw = wr[c]
        fetch_b = 2.0 * f_kib * 1024.0 / solves
        write_b = w_kib * 1024.0 / solves
        kernels[c] = {
            "hbm_bytes_per_solve": fetch_b + write_b,
            "fetch_bytes_per_solve": fetch_b,
            "write_bytes_per_solve": write_b,
            "dispatches_fetch_pass": nf,
            "dispatches_write_pass": nw,
        }
    res = {
        "config": config,
        "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes; FETCH_SIZE x2 (gfx950), KiB->B",
        "kernels": kernels,
    }
    Path(out).write_text(json.dumps(res, indent=1))
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
