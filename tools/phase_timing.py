#!/usr/bin/env python3
"""Per-phase shader-cycle breakdown of the fused step (profiling aid, not a product path).

    python isaacgymenvs-ma_amd/build.py --timing     # builds migym/_lib/libmigym_timing.so
    python tools/phase_timing.py --task Ant --num-envs 65536

Loads the phase-timing build (MIGYM_LIB), runs W warm-up + K timed steps and prints the mean
s_memtime cycles per wave per control step for each solver phase (team 0 of every wave).
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "isaacgymenvs-ma_amd"))
os.environ.setdefault("MIGYM_LIB", os.path.join(ROOT, "isaacgymenvs-ma_amd", "migym", "_lib",
                                                "libmigym_timing.so"))

NAMES = {0: "fk", 1: "aba", 2: "collide", 3: "rows", 4: "row_jacobians", 5: "rows_finish", 6: "pgs",
         7: "integrate", 8: "outputs", 9: "task+writeback", 10: "ts_walks", 11: "ts_root", 12: "ts_forward", 13: "rows_count", 14: "load+pre", 15: "substep_entry",
         16: "aba.setup", 17: "aba.backward", 18: "aba.root",   # slot 1 "aba": the forward pass after the marks 16-18
         19: "collide.ground", 20: "collide.pairs", 21: "collide.hull", 22: "hull_stage",
         # inside hull_stage (the wave's slowest team; not added to the total): the narrowphase's parts
         23: "(hull.gjk)", 24: "(hull.mpr)", 25: "(hull.features)", 26: "(hull.bound)",
         27: "(#gjk supports)", 28: "(#mpr supports)", 29: "(gjk.supports)", 30: "(gjk.simplex)",
         31: "collide.staging"}
SUB = (13, 23, 24, 25, 26, 27, 28, 29, 30)   # a count and the sub-phases: not part of the total   # slot 2 "collide": the object candidates
NPHASE = 32


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--task", default="Ant")
    ap.add_argument("--num-envs", type=int, default=65536)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--object-type", default="block", help="ShadowHand objectType")
    ap.add_argument("--per-wave", action="store_true",
                    help="launch by launch: the heaviest 1 %% of items (waves) against the mean item, per phase")
    args = ap.parse_args()
    import ctypes as C
    import numpy as np
    import torch
    import migym
    from migym import _abi
    lib = _abi.lib()
    mk = {}
    if args.task == "ShadowHand" and args.object_type != "block":
        from migym import configs
        tcfg = configs.task_config("ShadowHand", args.num_envs, sim_device="cuda:0")
        tcfg["env"]["objectType"] = args.object_type
        mk["cfg"] = {"task": tcfg}
    env = migym.make(seed=0, task=args.task, num_envs=args.num_envs, sim_device="cuda:0", rl_device="cuda:0",
                     headless=True, **mk)
    g = torch.Generator(device="cuda:0").manual_seed(0)
    acts = [torch.rand((env.num_actors, env.num_actions), device="cuda:0", generator=g) * 2 - 1 for _ in range(4)]
    for i in range(args.warmup):
        env.step(acts[i % 4])
    out = np.zeros(NPHASE, np.uint64)
    timing = lib.mg_debug_phase_cycles(out.ctypes.data, 1) == 0  # production build: wall clock only
    if args.per_wave:
        if not timing:
            sys.exit("--per-wave needs the phase-timing build")
        return per_wave(args, env, lib, acts, out)
    torch.cuda.synchronize()
    import time
    t0 = time.perf_counter()
    for i in range(args.steps):
        env.step(acts[i % 4])
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    if not timing:
        print(json.dumps({"task": args.task, "num_envs": args.num_envs, "ms_per_step": 1e3 * dt / args.steps}))
        return
    _abi.check(lib.mg_debug_phase_cycles(out.ctypes.data, 1), lib)
    from migym import taskdefs
    T = {"Cartpole": 8, "Ant": 16, "MAAnt": 16, "Humanoid": 32, "ShadowHand": 32}[args.task]
    waves = -(-env.num_actors // (64 // T))
    per = out.astype(np.float64) / (waves * args.steps)
    tot = sum(per[i] for i in NAMES if i not in SUB)
    res = {NAMES[i]: round(per[i]) for i in NAMES}
    res["rows_per_substep"] = round(per[13] / env.sim_params.substeps, 2)
    res["total_cycles_per_wave_step"] = round(tot)
    res["ms_per_step"] = round(1e3 * dt / args.steps, 3)
    print(json.dumps({"task": args.task, "num_envs": args.num_envs, "waves": waves, "phases": res}))
    for i in NAMES:
        if i != 13:
            print(f"  {NAMES[i]:16s} {per[i]:12.0f} cycles/wave/step  {100 * per[i] / tot:5.1f} %")


def per_wave(args, env, lib, acts, out):
    """each launch alone: the items' phase rows, the heaviest 1 % of items (by their total cycles) against the mean
    item; phases in cycles per item per control step, averaged over the launches"""
    import numpy as np
    import torch
    from migym import _abi
    T = {"Cartpole": 8, "Ant": 16, "MAAnt": 16, "Humanoid": 32, "ShadowHand": 32}[args.task]
    items = -(-env.num_actors // (64 // T))
    rows = np.zeros((items, NPHASE), np.uint64)
    keys = [i for i in NAMES if i not in SUB]
    heavy, mean, tail, tot_all, sup = [], [], [], [], []
    show = [i for i in NAMES if i != 13]
    for k in range(args.steps):
        _abi.check(lib.mg_debug_phase_cycles(out.ctypes.data, 1), lib)
        env.step(acts[k % 4])
        torch.cuda.synchronize()
        _abi.check(lib.mg_debug_phase_waves(rows.ctypes.data, items), lib)
        r = rows.astype(np.float64)
        tot = r[:, keys].sum(1)
        order = np.argsort(tot)
        top = order[-max(1, items // 100):]
        sup.append(float((rows[:, 23] > 0).mean()))
        heavy.append(r[top].mean(0))
        mean.append(r.mean(0))
        tail.append(r[order[-1]])
        tot_all.append(tot)
    h, m, t = np.mean(heavy, 0), np.mean(mean, 0), np.mean(tail, 0)
    th, tm, tt = h[keys].sum(), m[keys].sum(), t[keys].sum()
    tot_all = np.concatenate(tot_all)
    res = {"task": args.task, "num_envs": args.num_envs, "items": items, "launches": args.steps,
           "item_cycles": {"mean": round(tm), "p50": round(float(np.percentile(tot_all, 50))),
                           "p99": round(float(np.percentile(tot_all, 99))), "heaviest_1pct": round(th),
                           "max": round(tt)},
           "rows_per_substep": {"mean_item": round(m[13] / env.sim_params.substeps, 2),
                                "heaviest_1pct": round(h[13] / env.sim_params.substeps, 2),
                                "max_item": round(t[13] / env.sim_params.substeps, 2)},
           "items_running_the_hull_narrowphase": round(float(np.mean(sup)), 4)}
    print(json.dumps(res))
    print(f"  {'phase':16s} {'mean item':>10s} {'%':>6s} {'heavy 1%':>10s} {'%':>6s} {'heavy/mean':>10s} {'slowest':>10s}")
    for i in show:
        print(f"  {NAMES[i]:16s} {m[i]:10.0f} {100 * m[i] / tm:6.1f} {h[i]:10.0f} {100 * h[i] / th:6.1f} "
              f"{h[i] / max(m[i], 1):10.2f} {t[i]:10.0f}")
    print(f"  {'total':16s} {tm:10.0f} {100.0:6.1f} {th:10.0f} {100.0:6.1f} {th / tm:10.2f} {tt:10.0f}")


if __name__ == "__main__":
    main()
