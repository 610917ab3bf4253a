#!/usr/bin/env python3
"""Diagnostic (not a test): k_simulate of ShadowHand objectType egg from the random states of
tests/test_gpu_hand.py::test_hand_physics_step_matches_oracle, run twice on the GPU; prints the
run-to-run difference and the per-env object-pose error against the fp64 oracle."""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "isaacgymenvs-ma_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)
import numpy as np
import torch

import pyoracle as O
from migym import _abi, model as M
from test_gpu_hand import DevHandEnv, PALM_DZ, hand_states, np_, setup, stream

kind = sys.argv[1] if len(sys.argv) > 1 else "egg"
lib = _abi.lib()
print("lib", os.environ.get("MIGYM_LIB", "default"))
spec, sp, tp = setup(kind=kind)
n = 256
outs = []
for rep in range(2):
    rng = np.random.default_rng(5)
    h = hand_states(spec, tp, n, rng, PALM_DZ[kind], pen=kind == "pen")
    h.rb_forces[: n // 2, len(spec.bodies)] = rng.normal(0, 0.3, (n // 2, 3))
    e = DevHandEnv(h)
    mnp = M.pack_model(spec)
    if rep == 0:
        h.simulate(mnp, sp, threads=8)
        ref = h.root.copy()
    sim = C.c_void_p()
    _abi.check(lib.mg_sim_create(mnp.ctypes.data, C.byref(sp), n, 0, C.byref(sim)), lib)
    _abi.check(lib.mg_sim_bind(sim, C.byref(e.views())), lib)
    _abi.check(lib.mg_sim_simulate(sim, stream()), lib)
    torch.cuda.synchronize()
    lib.mg_sim_destroy(sim)
    outs.append(np_(e.root).copy())
a, b = outs
print("finite run0/run1:", np.isfinite(a).all(), np.isfinite(b).all())
print("run-to-run max |diff| object row:", np.nanmax(np.abs(a[:, 1] - b[:, 1])))
err = np.abs(a[:, 1, 0:3] - ref[:, 1, 0:3]).max(1)
print("object position error vs oracle: median %.2e  p90 %.2e  max %.2e  envs>2e-4: %d/%d" % (
    np.nanmedian(err), np.nanpercentile(err, 90), np.nanmax(err), int((err > 2e-4).sum()), n))
bad = np.argsort(-np.nan_to_num(err, nan=1e9))[:6]
for i in bad:
    print(" env", i, "gpu", a[i, 1, 0:3], "oracle", ref[i, 1, 0:3], "ncon", len(O.contacts(mnp, sp, ref[i].ravel() * 0 + h.root[i].ravel(), h.dof[i], 64)) if False else "")
