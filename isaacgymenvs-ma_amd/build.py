"""Build the in-tree HIP library (gfx950) — called by __graft_entry__.build().

    hipcc -O3 --offload-arch=gfx950 -c csrc/migym.hip            (C ABI + the one-lane-per-env kernels)
    hipcc -O3 --offload-arch=gfx950 -c csrc/inst.hip -DMG_INST=i  (team kernels, one capacity instance
                                                                    per object, i < MG_NUM_INST)
    hipcc -shared *.o -> migym/_lib/libmigym.so

The objects compile in parallel (one process per translation unit, at most MIGYM_JOBS / os.cpu_count()).
``--timing`` builds the phase-timing variant (-DMG_PHASE_TIMING, s_memtime per solver
phase, read back by ``mg_debug_phase_cycles``) into migym/_lib/libmigym_timing.so; it is a
profiling aid (tools/phase_timing.py), never the measured product.
"""
import glob
import os
import re
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
SRC = os.path.join(CSRC, "migym.hip")
INST = os.path.join(CSRC, "inst.hip")
OUT = os.path.join(HERE, "migym", "_lib", "libmigym.so")
OUT_TIMING = os.path.join(HERE, "migym", "_lib", "libmigym_timing.so")
HEADERS = sorted(glob.glob(os.path.join(CSRC, "*.hpp"))) + [os.path.join(HERE, "..", "include", "migym.h")]
ARCH = os.environ.get("MIGYM_ARCH", "gfx950")


def num_instances():
    txt = open(os.path.join(CSRC, "dispatch.hpp")).read()
    return int(re.search(r"#define MG_NUM_INST (\d+)", txt).group(1))


def needs_build(out=OUT):
    if not os.path.exists(out):
        return True
    t = os.path.getmtime(out)
    return any(os.path.getmtime(p) > t for p in [SRC, INST, __file__] + HEADERS)


def _run_parallel(cmds, verbose):
    jobs = int(os.environ.get("MIGYM_JOBS", min(16, os.cpu_count() or 1)))
    pending, running, failed = list(cmds), [], []
    while pending or running:
        while pending and len(running) < jobs:
            c = pending.pop(0)
            if verbose:
                print(" ".join(c), file=sys.stderr)
            running.append((c, subprocess.Popen(c)))
        c, p = running.pop(0)
        if p.wait() != 0:
            failed.append(" ".join(c))
    if failed:
        raise subprocess.CalledProcessError(1, failed[0])


def build(force=False, verbose=False, timing=False, variant=None, defines=(), extra=()):
    """variant: build an A/B variant with extra -D defines into migym/_lib/var/<variant>.so (selected at
    run time through MIGYM_LIB, tools/gpu.sh ab / traffic / pmc)."""
    out = OUT_TIMING if timing else OUT
    if variant:
        out = os.path.join(HERE, "migym", "_lib", "var", variant + ".so")
    if not force and not variant and not needs_build(out):
        return out
    os.makedirs(os.path.dirname(out), exist_ok=True)
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    flags = ["-O3", "-std=c++17", f"--offload-arch={ARCH}", "-fPIC", "-Wno-unused-result"]
    # no packed FP32 (v_pk_fma_f32 / v_pk_mul_f32): the packed forms need their operands in aligned register
    # pairs, and the moves and pair pressure that costs outweigh the halved instruction count in these latency-
    # bound kernels.  Spilled VGPRs: Humanoid 19 -> 2, ShadowHand block 52 -> 33, pen 49 -> 38, egg 57 -> 14;
    # same-box A/B: Ant +3.8 % (16,384 envs +4.5 %), Humanoid +4.7 %, ShadowHand +3.2 % (profiles/r04).
    # (-Xclang reaches the host compile too, where the AMDGPU feature name is ignored)
    flags += ["-Xclang", "-target-feature", "-Xclang", "-packed-fp32-ops"]
    if timing:
        flags.append("-DMG_PHASE_TIMING")
    flags += ["-D" + d for d in defines]
    flags += list(extra)
    objdir = os.path.join(HERE, "build", ("var_" + variant) if variant else ("timing" if timing else "release"))
    os.makedirs(objdir, exist_ok=True)
    objs, cmds = [], []
    for i in range(-1, num_instances()):
        o = os.path.join(objdir, "migym.o" if i < 0 else f"inst{i}.o")
        src = SRC if i < 0 else INST
        # instance TUs: no MachineLICM.  The work-queue kernels' per-item body sits in a loop, and the pass hoists
        # values out of it into registers held across all items (Humanoid: 48 spilled VGPRs vs 25 without it;
        # measured +3 % ShadowHand, +2 % egg, +1 % Humanoid, Ant unchanged)
        # and no interprocedural register allocation (a guard only: a real call in these kernels miscompiled in
        # round 3 with IPRA on -- wrong object states -- and, with the cause not pinned down, with IPRA off too:
        # an illegal address and a 93 % parity build).  Every phase is force-inlined, and
        # codeobj.check_no_calls below fails the build if any call is left in the device code
        inst = [] if i < 0 else [f"-DMG_INST={i}", "-mllvm", "-disable-machine-licm", "-mllvm", "-enable-ipra=false"]
        cmds.append([hipcc] + flags + inst + ["-c", "-o", o, src])
        objs.append(o)
    _run_parallel(cmds, verbose)
    subprocess.check_call([hipcc, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", out + ".tmp"] + objs)
    sys.path.insert(0, HERE)
    import codeobj
    try:
        codeobj.check_no_calls(out + ".tmp", ARCH)
    except Exception:
        os.remove(out + ".tmp")
        raise
    os.replace(out + ".tmp", out)
    return out


if __name__ == "__main__":
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--timing", action="store_true")
    ap.add_argument("--variant", default=None)
    ap.add_argument("-D", dest="defines", action="append", default=[])
    ap.add_argument("--flag", dest="extra", action="append", default=[], help="extra hipcc flag (A/B variants)")
    a = ap.parse_args()
    print(build(force=a.force, verbose=True, timing=a.timing, variant=a.variant, defines=a.defines, extra=a.extra))
