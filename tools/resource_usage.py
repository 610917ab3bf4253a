#!/usr/bin/env python3
"""Per-kernel register / scratch / LDS / occupancy table of the gfx950 build (compiler remarks).

usage: python tools/resource_usage.py [source.hip] [extra hipcc flags...]
"""
import re
import subprocess
import sys

src = sys.argv[1] if len(sys.argv) > 1 else "isaacgymenvs-ma_amd/csrc/migym.hip"
cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "-fPIC", "-c", "--cuda-device-only",
       "-Rpass-analysis=kernel-resource-usage", "-o", "/dev/null", src,
       "-Xclang", "-target-feature", "-Xclang", "-packed-fp32-ops"] + sys.argv[2:]   # build.py's flags
if src.endswith("inst.hip"):  # the instance TUs' build flags (build.py)
    cmd += ["-mllvm", "-disable-machine-licm", "-mllvm", "-enable-ipra=false"]
out = subprocess.run(cmd, capture_output=True, text=True).stderr
rows, cur = [], None
for line in out.splitlines():
    m = re.search(r"remark: (.*?) \[-Rpass-analysis", line)
    if not m:
        continue
    k, _, v = m.group(1).strip().partition(": ")
    if k == "Function Name":
        cur = {"name": v}
        rows.append(cur)
    elif cur is not None:
        cur[k] = v
keys = ["VGPRs", "AGPRs", "VGPRs Spill", "ScratchSize [bytes/lane]", "Occupancy [waves/SIMD]", "LDS Size [bytes/block]"]
print(f"{'kernel':70s} " + " ".join(f"{k.split()[0]:>9s}" for k in keys))
for r in rows:
    if not re.search(r"k_(env_step|hand_step|simulate)", r["name"]):
        continue
    m = re.match(r"_Z\d+(k_\w+?)I(.*?)E(?:E|v)", r["name"])
    n = m.group(1) + "<" + ",".join(re.findall(r"L[ib](\d+)E", m.group(2) + "E")) + ">" if m else r["name"]
    print(f"{n[:70]:70s} " + " ".join(f"{r.get(k, '?'):>9s}" for k in keys))
