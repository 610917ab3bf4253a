#!/usr/bin/env python3
"""Where a team kernel spills: compile one instance TU to gfx950 assembly with line tables and attribute every
spill store / reload of one kernel to the source line (and the enclosing Team phase) it belongs to.

usage: python tools/spill_map.py INST KERNEL_REGEX [extra hipcc flags...]
  e.g. python tools/spill_map.py 1 'k_env_step.*Lb0ELb0ELb0E' -DMG_NUM_VGPR=168

Prints the kernel's resource line, then spill / reload counts per source line (top 40) and per function of
team_physics.hpp / step_kernels.hpp (the phase the line sits in).  A register-pressure aid.
"""
import collections
import os
import re
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(ROOT, "isaacgymenvs-ma_amd", "csrc")

inst, kre = sys.argv[1], sys.argv[2]
extra = sys.argv[3:]
out = f"/tmp/spill_map_{inst}.s"
cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "-fPIC", "--cuda-device-only", "-S",
       "-gline-tables-only", "-o", out, os.path.join(CSRC, "inst.hip"), f"-DMG_INST={inst}",
       "-Xclang", "-target-feature", "-Xclang", "-packed-fp32-ops",
       "-mllvm", "-disable-machine-licm", "-mllvm", "-enable-ipra=false"] + extra
subprocess.run(cmd, check=True)
txt = open(out).read().splitlines()
files = {}
for ln in txt:
    m = re.match(r'\s*\.file\s+(\d+)\s+"([^"]*)"(?:\s+"([^"]*)")?', ln)
    if m:
        files[m.group(1)] = os.path.basename(m.group(3) or m.group(2))

# the kernel's body: from its label to .Lfunc_end
start = None
for i, ln in enumerate(txt):
    m = re.match(r"^(_Z\S+):", ln)
    if m and re.search(kre, m.group(1)) and "k_env_step" in m.group(1) or (m and re.search(kre, m.group(1))):
        start, name = i, m.group(1)
        break
if start is None:
    sys.exit("kernel not found")
end = next(i for i in range(start, len(txt)) if txt[i].startswith(".Lfunc_end"))
body = txt[start:end]
loc = ("?", 0)
spill, reload = collections.Counter(), collections.Counter()
ninstr = 0
for ln in body:
    m = re.match(r"\s*\.loc\s+(\d+)\s+(\d+)", ln)
    if m:
        loc = (files.get(m.group(1), m.group(1)), int(m.group(2)))
        continue
    s = ln.strip()
    if not s or s.startswith((".", ";")) or s.endswith(":"):
        continue
    ninstr += 1
    if "Spill" in ln:
        spill[loc] += 1
    elif "Reload" in ln:
        reload[loc] += 1

# resource summary from the metadata
meta = "\n".join(txt[end:end + 60])
def field(k):
    m = re.search(r"\.set\s+" + re.escape(name) + r"\." + k + r",\s*(\d+)", "\n".join(txt))
    return m.group(1) if m else "?"
print(f"{name}\n  instructions {ninstr}  vgpr {field('num_vgpr')}  agpr {field('num_agpr')}  "
      f"private {field('private_seg_size')}  spills {sum(spill.values())}  reloads {sum(reload.values())}")

# enclosing function per source line: the last 'void name(' / 'name(' definition above the line
func_cache = {}
def enclosing(f, line):
    key = (f, line)
    if key in func_cache:
        return func_cache[key]
    path = os.path.join(CSRC, f)
    name = "?"
    if os.path.exists(path):
        src = open(path).read().splitlines()
        for i in range(min(line, len(src)) - 1, -1, -1):
            m = re.search(r"__forceinline__\s+(?:static\s+)?[\w:<>,\s\*&]*?\b(\w+)\s*\(", src[i])
            if m:
                name = m.group(1)
                break
    func_cache[key] = f"{f}:{name}"
    return func_cache[key]

per_func = collections.Counter()
for (f, l), c in list(spill.items()) + list(reload.items()):
    per_func[enclosing(f, l)] += c
print("\nper function (spill + reload instructions):")
for k, c in per_func.most_common(25):
    print(f"  {c:6d}  {k}")
print("\nper line (spill / reload):")
lines = collections.Counter()
for k, c in spill.items():
    lines[k] += c
for k, c in reload.items():
    lines[k] += c
for (f, l), c in lines.most_common(40):
    print(f"  {spill[(f, l)]:5d} / {reload[(f, l)]:5d}  {f}:{l}")
