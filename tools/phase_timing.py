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
         19: "collide.ground", 20: "collide.pairs", 21: "collide.hull"}   # slot 2 "collide": the object candidates
NPHASE = 24


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--task", default="Ant")
    ap.add_argument("--num-envs", type=int, default=65536)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--object-type", default="block", help="ShadowHand objectType")
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
    tot = sum(per[i] for i in NAMES if i not in (13,))
    res = {NAMES[i]: round(per[i]) for i in NAMES}
    res["rows_per_substep"] = round(per[13] / env.sim_params.substeps, 2)
    res["total_cycles_per_wave_step"] = round(tot)
    res["ms_per_step"] = round(1e3 * dt / args.steps, 3)
    print(json.dumps({"task": args.task, "num_envs": args.num_envs, "waves": waves, "phases": res}))
    for i in NAMES:
        if i != 13:
            print(f"  {NAMES[i]:16s} {per[i]:12.0f} cycles/wave/step  {100 * per[i] / tot:5.1f} %")


if __name__ == "__main__":
    main()
