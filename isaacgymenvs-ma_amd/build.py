"""Build the in-tree HIP library (gfx950) — called by __graft_entry__.build().

    hipcc -O3 --offload-arch=gfx950 -shared -fPIC csrc/migym.hip -> migym/_lib/libmigym.so

``--timing`` builds the phase-timing variant (-DMG_PHASE_TIMING, s_memtime per solver
phase, read back by ``mg_debug_phase_cycles``) into migym/_lib/libmigym_timing.so; it is a
profiling aid (tools/phase_timing.py), never the measured product.
"""
import glob
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(HERE, "csrc", "migym.hip")
OUT = os.path.join(HERE, "migym", "_lib", "libmigym.so")
HEADERS = sorted(glob.glob(os.path.join(HERE, "csrc", "*.hpp"))) + [os.path.join(HERE, "..", "include", "migym.h")]
ARCH = os.environ.get("MIGYM_ARCH", "gfx950")


OUT_TIMING = os.path.join(HERE, "migym", "_lib", "libmigym_timing.so")


def needs_build(out=OUT):
    if not os.path.exists(out):
        return True
    t = os.path.getmtime(out)
    return any(os.path.getmtime(p) > t for p in [SRC] + HEADERS)


def build(force=False, verbose=False, timing=False):
    out = OUT_TIMING if timing else OUT
    if not force and not needs_build(out):
        return out
    os.makedirs(os.path.dirname(out), exist_ok=True)
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    cmd = [hipcc, "-O3", "-std=c++17", f"--offload-arch={ARCH}", "-fPIC", "-shared", "-Wno-unused-result"]
    if timing:
        cmd.append("-DMG_PHASE_TIMING")
    cmd += ["-o", out + ".tmp", SRC]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.check_call(cmd)
    os.replace(out + ".tmp", out)
    return out


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True, timing="--timing" in sys.argv))
