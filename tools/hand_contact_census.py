#!/usr/bin/env python3
"""Contact census of ShadowHand rollouts (CPU, the oracle's fp32 build as the rollout engine, its fp64 collide as the
counter): per env and substep-start state, how many contacts each (hand geom, object / ground / pair) class emits,
the distribution of the per-env total, and what the heaviest envs are made of.  Input to the contact-reduction
decision (small shards: the slowest wave sets the kernel time).

    python tools/hand_contact_census.py --num-envs 4096 --steps 40 [--object-type block]
"""
import argparse
import collections
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "isaacgymenvs-ma_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--num-envs", type=int, default=4096)
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--object-type", default="block")
    ap.add_argument("--threads", type=int, default=8)
    a = ap.parse_args()
    import pyoracle as O
    from migym import configs, model as M, taskdefs
    n = a.num_envs
    cfg = configs.task_config("ShadowHand", n)
    cfg["env"]["objectType"] = a.object_type
    spec = taskdefs.hand_spec(a.object_type)
    sp = taskdefs.sim_params(cfg, taskdefs.TASK_INFO["ShadowHand"][5], 1)
    tp = taskdefs.task_params("ShadowHand", cfg, spec)
    mnp = M.pack_model(spec)
    h = O.HandHostEnv(tp, spec, n)
    lib = O.lib()
    lib.orc_contacts_full.argtypes = [C.c_void_p, C.POINTER(type(sp)), C.c_void_p, C.c_void_p, C.c_void_p, C.c_int32]
    rng = np.random.default_rng(0)
    gname = [g.name for g in spec.geoms]
    hist = []
    classes = collections.Counter()
    heavy = []
    for t in range(a.steps):
        h.actions[:] = rng.uniform(-1, 1, h.actions.shape).astype(np.float32)
        h.env_step(mnp, sp, tp, seed=0, step=t, threads=a.threads, fp32=True)
        if t < a.steps // 2:
            continue
        for e in range(n):
            out = np.zeros(11 * 128)
            root = np.ascontiguousarray(h.root[e], np.float32)
            dof = np.ascontiguousarray(h.dof[e], np.float32)
            k = lib.orc_contacts_full(mnp.ctypes.data, C.byref(sp), root.ctypes.data, dof.ctypes.data, out.ctypes.data, 128)
            cs = out[:11 * k].reshape(k, 11)
            hist.append(k)
            cls = collections.Counter()
            for c in cs:
                ga, gb = int(c[1]), int(c[3])
                na = gname[ga] if 0 <= ga < len(gname) else f"g{ga}"
                nb = "object" if gb == -2 else ("ground" if gb == -1 else (gname[gb] if 0 <= gb < len(gname) else f"g{gb}"))
                cls[(na, nb)] += 1
            classes.update(cls)
            heavy.append((k, t, e, dict(cls)))
    hist = np.array(hist)
    print(f"ShadowHand {a.object_type}: {n} envs, states of steps {a.steps // 2}..{a.steps - 1}")
    print(f"contacts per env-state: mean {hist.mean():.2f}  p50 {np.median(hist):.0f}  p90 {np.quantile(hist, 0.9):.0f}  "
          f"p99 {np.quantile(hist, 0.99):.0f}  max {hist.max()}")
    print("histogram:", np.bincount(hist).tolist())
    tot = sum(classes.values())
    print("contact classes (share of all contacts):")
    for (na, nb), c in classes.most_common(25):
        print(f"  {na:28s} x {nb:12s} {c / tot:7.2%}  ({c / len(hist):.3f} per env-state)")
    heavy.sort(key=lambda x: -x[0])
    print("heaviest env-states:")
    for k, t, e, cls in heavy[:12]:
        print(f"  {k:3d} contacts (step {t}, env {e}):", sorted(cls.items(), key=lambda x: -x[1])[:8])
    # per (hand geom, object) pair: contacts beyond 4 (what a 4-point manifold per pair would drop)
    beyond = [sum(max(0, v - 4) for v in cls.values()) for _, _, _, cls in heavy]
    print(f"contacts beyond 4 per (geom, other) pair: mean {np.mean(beyond):.3f} per env-state, "
          f"max {max(beyond)}; in the top 1 % of env-states: {np.mean(beyond[:max(1, len(beyond) // 100)]):.2f}")


if __name__ == "__main__":
    main()
