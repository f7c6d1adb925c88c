"""CPU: the useful-flop count behind bench.py's roofline.fp64 (VERDICT r05
item 5).  tools/flop_count.py runs the scalar C++ CPU baseline with a
counting fp64 type; the committed per-unit figures
(profiles/r06_useful_flops.json) must be reproducible from the committed
tool, and the classical backward node must match SURVEY §8(a) a12's
hand count (~23.3 kflop, FF ~62.2 kflop) to within 10 %."""
from __future__ import annotations

import json
import subprocess
import sys
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parents[1]
PROFILE = ROOT / "profiles" / "r06_useful_flops.json"


def test_committed_counts_match_survey_hand_count():
    cfgs = json.loads(PROFILE.read_text())["configs"]
    bw = cfgs["classical/normal_1d/N30"]["phases"]["backward"]["flops_per_unit"]
    bw_ff = cfgs["ff/normal_1d/N30"]["phases"]["backward"]["flops_per_unit"]
    assert abs(bw / 23.3e3 - 1) < 0.1, bw
    assert abs(bw_ff / 62.2e3 - 1) < 0.1, bw_ff
    for c in cfgs.values():
        for ph in ("node", "backward", "forward"):
            e = c["phases"][ph]
            assert e["units"] > 0 and e["flops_per_unit"] > 1e3


def test_counts_reproduce(tmp_path):
    out = tmp_path / "uf.json"
    subprocess.run([sys.executable, str(ROOT / "tools" / "flop_count.py"), "--sample", "32", "--out", str(out),
                    "--configs", "classical/normal_1d/N30"], check=True, timeout=600)
    got = json.loads(out.read_text())["configs"]["classical/normal_1d/N30"]["phases"]
    ref = json.loads(PROFILE.read_text())["configs"]["classical/normal_1d/N30"]["phases"]
    for ph in ("node", "backward", "forward"):
        # a smaller sample of the same workload: the per-unit mix of free /
        # contact nodes and Cholesky / BoxQP gains moves by a few percent
        assert got[ph]["flops_per_unit"] == pytest.approx(ref[ph]["flops_per_unit"], rel=0.05), ph


def test_bench_useful_roofline_helpers():
    sys.path.insert(0, str(ROOT))
    import bench

    per = bench.useful_per_unit("classical", "normal_1d", 30)
    assert set(per) == {"node", "backward", "forward"}
    assert bench.useful_per_unit("classical", "normal_1d", 17) is None  # no count for that horizon
    stats = np.zeros((2, 10), np.int32)
    stats[:, 4] = 3  # calcDiffs
    stats[:, 0] = 2  # backward passes
    stats[:, 6] = 4  # step lengths, first pass
    stats[:, 7] = 1  # ... second pass
    f = bench.useful_flops(stats, 30, per)
    assert f == pytest.approx(2 * (3 * 31 * per["node"] + 2 * 30 * per["backward"] + 5 * 31 * per["forward"]))
    fp = {"achieved": 2.0, "peak": 10.0, "unit": "TFLOP/s", "frac": 0.2}
    fpi = {"achieved": 4.0, "peak": 10.0, "unit": "TFLOP/s", "frac": 0.4}
    blk = bench.fp64_block(fp, f, per, fpi, 2 * f)
    assert blk["frac"] == 0.2 and blk["issue_rate"]["frac"] == 0.4 and blk["useful_share_of_issued"] == 0.5
