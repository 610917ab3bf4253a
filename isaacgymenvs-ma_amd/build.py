"""Build the in-tree HIP library (gfx950) — called by __graft_entry__.build().

    hipcc -O3 --offload-arch=gfx950 -shared -fPIC csrc/migym.hip -> migym/_lib/libmigym.so
"""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(HERE, "csrc", "migym.hip")
OUT = os.path.join(HERE, "migym", "_lib", "libmigym.so")
HEADERS = [os.path.join(HERE, "csrc", f) for f in ("team_physics.hpp", "hand_task.hpp", "task.hpp", "device_math.hpp")] + [
    os.path.join(HERE, "..", "include", "migym.h")]
ARCH = os.environ.get("MIGYM_ARCH", "gfx950")


def needs_build():
    if not os.path.exists(OUT):
        return True
    t = os.path.getmtime(OUT)
    return any(os.path.getmtime(p) > t for p in [SRC] + HEADERS)


def build(force=False, verbose=False):
    if not force and not needs_build():
        return OUT
    os.makedirs(os.path.dirname(OUT), exist_ok=True)
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    cmd = [hipcc, "-O3", "-std=c++17", f"--offload-arch={ARCH}", "-fPIC", "-shared", "-Wno-unused-result",
           "-o", OUT + ".tmp", SRC]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.check_call(cmd)
    os.replace(OUT + ".tmp", OUT)
    return OUT


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
