#!/usr/bin/env python3
"""Bit-for-bit comparison of two builds of the library (A/B aid for changes meant to leave every result unchanged,
not a product path).  One process per library (MIGYM_LIB is read at import):

    python tools/bitcmp.py --out a.npz                          # the library in MIGYM_LIB (default: the shipped one)
    MIGYM_LIB=.../var/prev.so python tools/bitcmp.py --out b.npz
    python tools/bitcmp.py --compare a.npz b.npz               # exit status 1 on any differing bit

Each case is a make() rollout with seeded device actions (resets included); the arrays saved are every step's
obs / rew / reset and the final root and DOF state.
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "isaacgymenvs-ma_amd"))

CASES = (("Ant", 4096, "block"), ("Humanoid", 2048, "block"), ("MAAnt", 1024, "block"), ("Cartpole", 256, "block"),
         ("ShadowHand", 1024, "block"), ("ShadowHand", 512, "pen"), ("ShadowHand", 512, "egg"))


def rollout(task, n, obj, steps):
    import torch
    import migym
    from migym import configs
    kw = {}
    if task == "ShadowHand":
        cfg = configs.task_config(task, n, sim_device="cuda:0")
        cfg["env"]["objectType"] = obj
        kw["cfg"] = {"task": cfg}
    env = migym.make(seed=0, task=task, num_envs=n, sim_device="cuda:0", rl_device="cuda:0", headless=True, **kw)
    g = torch.Generator(device="cuda:0").manual_seed(7)
    obs, rew, rst = [], [], []
    for _ in range(steps):
        a = torch.rand((env.num_actors, env.num_actions), device="cuda:0", generator=g) * 2 - 1
        o, r, d, _ = env.step(a)
        obs.append(o["obs"].clone())
        rew.append(r.clone())
        rst.append(d.clone())
    torch.cuda.synchronize()
    out = {"obs": torch.stack(obs).cpu().numpy(), "rew": torch.stack(rew).cpu().numpy(),
           "reset": torch.stack(rst).cpu().numpy(), "root": env.root_states.cpu().numpy(),
           "dof": env.dof_state.cpu().numpy()}
    env.close()
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out")
    ap.add_argument("--steps", type=int, default=24)
    ap.add_argument("--compare", nargs=2)
    ap.add_argument("--tasks", default="", help="comma-separated task names to run (default: every case)")
    a = ap.parse_args()
    import numpy as np
    if a.compare:
        x, y = np.load(a.compare[0]), np.load(a.compare[1])
        bad = 0
        for k in sorted(x.files):
            same = x[k].shape == y[k].shape and np.array_equal(x[k].view(np.uint8), y[k].view(np.uint8))
            if not same:
                bad += 1
                d = np.abs(x[k].astype(np.float64) - y[k].astype(np.float64))
                print(f"DIFF {k}: {np.count_nonzero(d)} elements, max {d.max():.3e}")
        print(f"{len(x.files) - bad} of {len(x.files)} arrays bit-identical")
        sys.exit(1 if bad else 0)
    arrays = {}
    only = set(t for t in a.tasks.split(",") if t)
    for task, n, obj in CASES:
        if only and task not in only:
            continue
        r = rollout(task, n, obj, a.steps)
        for k, v in r.items():
            arrays[f"{task}-{obj}-{n}/{k}"] = v
        print(f"{task} {obj} {n}: done", flush=True)
    np.savez(a.out, **arrays)


if __name__ == "__main__":
    main()
