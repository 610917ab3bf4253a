#!/usr/bin/env python3
"""Kernel-duration measurements side by side (one GPU): back-to-back launches timed by wall clock, the device-side
span of each launch (mg_kernel_span_begin) with and without HIP events around the launches, and the events alone.

    python tools/span_diag.py --task Ant --num-envs 65536 --steps 64
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "isaacgymenvs-ma_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--task", default="Ant")
    ap.add_argument("--num-envs", type=int, default=65536)
    ap.add_argument("--steps", type=int, default=64)
    a = ap.parse_args()
    import numpy as np
    import torch
    import migym
    dev = "cuda:0"
    env = migym.make(seed=0, task=a.task, num_envs=a.num_envs, sim_device=dev, rl_device=dev, headless=True)
    g = torch.Generator(device=dev).manual_seed(1)
    pool = [torch.rand((env.num_actors, env.num_actions), device=dev, generator=g) * 2 - 1 for _ in range(8)]
    K = a.steps
    for i in range(20):
        env.step(pool[i % 8])
    torch.cuda.synchronize()

    def timed(spans, events):
        st = [torch.cuda.Event(enable_timing=True) for _ in range(K)]
        en = [torch.cuda.Event(enable_timing=True) for _ in range(K)]
        if spans:
            env.kernel_span_begin(K)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(K):
            env.launch_events = (st[i], en[i]) if events else None
            env.step(pool[i % 8])
        torch.cuda.synchronize()
        wall = (time.perf_counter() - t0) * 1e3 / K
        env.launch_events = None
        sp = env.kernel_span_read(K) if spans else np.zeros(0)
        env.kernel_span_begin(0)
        ev = np.array([st[i].elapsed_time(en[i]) for i in range(K)]) if events else np.zeros(0)
        return wall, sp, ev

    def q(x):
        return "-" if len(x) == 0 else f"min {x.min():.4f} med {np.median(x):.4f} max {x.max():.4f}"

    for name, s, e in (("plain", False, False), ("spans", True, False), ("events", False, True),
                       ("spans+events", True, True), ("plain", False, False), ("spans", True, False)):
        wall, sp, ev = timed(s, e)
        print(f"{name:14s} wall/step {wall:.4f} ms | span {q(sp)} | event {q(ev)}", flush=True)
        if len(sp):
            print("   spans:", " ".join(f"{x:.4f}" for x in sp[:16]), flush=True)
    env.close()


if __name__ == "__main__":
    main()
