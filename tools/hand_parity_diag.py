#!/usr/bin/env python3
"""Diagnostic (not a test): the fused ShadowHand step (tests/test_gpu_hand.py::test_hand_fused_env_step_matches_oracle)
stepped one control step at a time on the GPU and in the oracle; for every env whose object row leaves the tolerance
it prints the first step it does, the oracle's contacts at that step's start (deepest gap, count) and which of
parity_stats' discontinuity checks fire there."""
import copy
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "isaacgymenvs-ma_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)
import numpy as np
import torch

import parity_stats as PS
import pyoracle as O
from migym import _abi, model as M
from test_gpu_hand import DevHandEnv, T, np_, setup, stream

kind = sys.argv[1] if len(sys.argv) > 1 else "pen"
lib = _abi.lib()
spec, sp, tp = setup(kind=kind)
n = 192
h = O.HandHostEnv(tp, spec, n)
e = DevHandEnv(h)
mnp = M.pack_model(spec)
sim = C.c_void_p()
_abi.check(lib.mg_sim_create(mnp.ctypes.data, C.byref(sp), n, 0, C.byref(sim)), lib)
_abi.check(lib.mg_sim_bind(sim, C.byref(e.views())), lib)
rng = np.random.default_rng(3)
first = {}
lo, hi = np.array([x.lower for x in spec.nodes[1:]]), np.array([x.upper for x in spec.nodes[1:]])
kp, bd = np.array([x.drive_kp for x in spec.nodes[1:]]), np.array([x.damping for x in spec.nodes[1:]])
eff = np.array([x.effort_limit for x in spec.nodes[1:]])
for t in range(12):
    a = rng.uniform(-1.2, 1.2, (n, tp.num_actions)).astype(np.float32)
    h.actions[:] = a
    e.actions.copy_(T(a))
    pre = copy.deepcopy(h)
    h.env_step(mnp, sp, tp, seed=5, step=t, threads=8)
    _abi.check(lib.mg_env_step(sim, C.byref(tp), C.byref(e.buffers(seed=5, step=t)), stream()), lib)
    torch.cuda.synchronize()
    rg = np_(e.root)
    err = np.abs(rg[:, 1, 0:3] - h.root[:, 1, 0:3]).max(1)
    for i in np.flatnonzero(err > 2e-4):
        if i in first:
            continue
        cs = O.contacts(mnp, sp, pre.root[i].ravel(), pre.dof[i], 64)
        deep = min([c[7] for c in cs], default=0.0)
        why = {"contact_flip": bool(PS.contact_flips(mnp, sp, pre.root[i:i + 1], pre.dof[i:i + 1], 1e-4)[0]),
               "limit_flip": bool(PS.limit_flips(pre.dof[i:i + 1, :, 0], lo, hi, sp.limit_margin)[0]),
               "drive_flip": bool(PS.drive_flips(pre.dof[i:i + 1, :, 0], pre.dof[i:i + 1, :, 1], pre.targets[i:i + 1],
                                                 kp, bd, eff)[0]),
               "deep": bool(PS.deep_contacts(mnp, sp, pre.root[i:i + 1], pre.dof[i:i + 1])[0])}
        first[i] = t
        objc = [c for c in cs if int(c[8]) == -2 or int(c[0]) == -2]
        print(f"env {i}: step {t} err {err[i]:.2e}  contacts {len(cs)} (object {len(objc)}) deepest {deep:.4f}  "
              f"progress {pre.progress[i]} reset {pre.reset[i]}  {why}")
        for c in objc:
            print("     node", int(c[0]), "->", int(c[8]), "gap %.5f" % c[7], "n", np.round(c[4:7], 3))
lib.mg_sim_destroy(sim)
print("diverged envs:", len(first))
