#!/usr/bin/env python3
"""Per-kernel register / scratch / occupancy table of the HIP library
(hipcc -Rpass-analysis=kernel-resource-usage).  usage: tools/resources.py [EXTRA flags...]"""
import re
import subprocess
import sys
from pathlib import Path

CSRC = Path(__file__).resolve().parents[1] / "franka-force-feedback-mpc_amd" / "csrc"
cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "--cuda-device-only", "-c",
       "-Rpass-analysis=kernel-resource-usage", "-o", "/tmp/ffddp_res.o", *sys.argv[1:], "ffddp_kernels.hip"]
out = subprocess.run(cmd, cwd=CSRC, capture_output=True, text=True).stderr
rows, cur = [], None
for line in out.splitlines():
    m = re.search(r"remark: (.*?) \[-Rpass", line)
    if not m:
        continue
    kv = m.group(1)
    if kv.startswith("Function Name:"):
        cur = {"name": kv.split(":", 1)[1].strip()}
        rows.append(cur)
    elif cur is not None and ":" in kv:
        k, v = kv.split(":", 1)
        cur[k.strip()] = v.strip()
for r in rows:
    n = r["name"]
    m = re.search(r"(k_\w+?)I(.*?)EEv", n) or re.search(r"(k_\w+)E", n)
    short = n
    if "_GLOBAL__N_1" in n:
        mm = re.search(r"N_1\d+(k_[a-z0-9_]+)", n)
        short = mm.group(1) if mm else n
        targs = re.findall(r"IL?i?(\d)E?Lb(\d)E?(?:Li(\d)ELb(\d))?", n)
        if targs:
            short += "<" + ",".join(x for x in targs[0] if x) + ">"
    print(f"{short:32s} VGPR {r.get('VGPRs','?'):>4s} AGPR {r.get('AGPRs','?'):>4s} scratch {r.get('ScratchSize [bytes/lane]','?'):>5s} "
          f"occ {r.get('Occupancy [waves/SIMD]','?'):>2s} LDS {r.get('LDS Size [bytes/block]','?'):>6s} SGPR {r.get('TotalSGPRs','?')}")
