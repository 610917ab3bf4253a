#!/usr/bin/env python3
"""Diagnostic (not a test): which envs of the hand physics-step parity states disagree between the GPU and
the oracle, and which discontinuity (tests/parity_stats.py) each sits at."""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "isaacgymenvs-ma_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)
import copy
import numpy as np
import torch

import pyoracle as O
import parity_stats as PS
from migym import _abi, model as M
from test_gpu_hand import DevHandEnv, PALM_DZ, forearm_top, hand_states, np_, setup, stream

lib = _abi.lib()
for kind in ("block", "egg", "pen"):
    for where in ("palm", "forearm"):
        spec, sp, tp = setup(kind=kind)
        n = 256
        rng = np.random.default_rng(5 if where == "palm" else 11)
        h = hand_states(spec, tp, n, rng, PALM_DZ[kind], pen=kind == "pen")
        if where == "forearm":
            top = forearm_top(spec, h)
            ob = h.root[:, 1]
            reach = {"block": 0.025, "egg": 0.03, "pen": 0.008}[kind]
            ob[:, 0:3] = top + np.c_[rng.normal(0, 0.02, (n, 2)), reach * rng.uniform(0.6, 1.4, n)]
            ob[:, 7:13] = rng.normal(0, 0.1, (n, 6))
            h.dof[:, :, 0] = 0.0
        h.rb_forces[: n // 2, len(spec.bodies)] = rng.normal(0, 0.3, (n // 2, 3))
        e = DevHandEnv(h)
        h0 = copy.deepcopy(h)
        mnp = M.pack_model(spec)
        h.simulate(mnp, sp, threads=8)
        sim = C.c_void_p()
        _abi.check(lib.mg_sim_create(mnp.ctypes.data, C.byref(sp), n, 0, C.byref(sim)), lib)
        _abi.check(lib.mg_sim_bind(sim, C.byref(e.views())), lib)
        _abi.check(lib.mg_sim_simulate(sim, stream()), lib)
        torch.cuda.synchronize()
        lib.mg_sim_destroy(sim)
        rg, dg = np_(e.root), np_(e.dof)
        bad = (PS.env_bad(rg[:, 1, 0:7], h.root[:, 1, 0:7], 2e-4, 0) | PS.env_bad(rg[:, 1, 7:13], h.root[:, 1, 7:13], 2e-3, 2e-3)
               | PS.env_bad(dg[..., 0], h.dof[..., 0], 2e-4, 0) | PS.env_bad(dg[..., 1], h.dof[..., 1], 2e-3, 2e-3))
        lo = np.array([x.lower for x in spec.nodes[1:]]); hi = np.array([x.upper for x in spec.nodes[1:]])
        kp = np.array([x.drive_kp for x in spec.nodes[1:]]); b = np.array([x.damping for x in spec.nodes[1:]])
        eff = np.array([x.effort_limit for x in spec.nodes[1:]])
        lf = PS.limit_flips(h0.dof[..., 0], lo, hi, sp.limit_margin, 1e-3)
        df = PS.drive_flips(h0.dof[..., 0], h0.dof[..., 1], h0.targets, kp, b, eff, 5e-2)
        out = [f"{kind:5s} {where:7s} bad {int(bad.sum()):3d}"]
        for delta in (1e-5, 1e-4, 1e-3):
            cf = PS.contact_flips(mnp, sp, h0.root, h0.dof, delta)
            out.append(f"contact({delta:g}) {int((bad & cf).sum())}")
        cf = PS.contact_flips(mnp, sp, h0.root, h0.dof, 1e-3)
        out.append(f"limit {int((bad & lf).sum())} drive {int((bad & df).sum())} unexplained {int((bad & ~(cf | lf | df)).sum())}")
        st = PS.err_stats(rg[:, 1, 0:3], h.root[:, 1, 0:3])
        out.append(f"obj pos max {st['max']:.2e} p99.9 {st['p999']:.2e}")
        print("  ".join(out), flush=True)
