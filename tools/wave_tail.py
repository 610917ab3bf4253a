#!/usr/bin/env python3
"""Where a launch's time goes between its waves (profiling aid, not a product path): the raw per-wave start / end
ticks of recorded fused-step launches (mg_kernel_span_waves) -> wave durations, the dispatch ramp (first to last
wave start), the tail (when the last waves finish against the bulk), and the slot utilisation
sum(wave durations) / (span x resident wave slots).

    python tools/wave_tail.py --task Ant --num-envs 65536 --launches 8
"""
import argparse
import ctypes as C
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "isaacgymenvs-ma_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--task", default="Ant")
    ap.add_argument("--num-envs", type=int, default=65536)
    ap.add_argument("--launches", type=int, default=8)
    ap.add_argument("--object-type", default="block")
    ap.add_argument("--slots", type=int, default=2048, help="resident wave slots (256 CUs x 8 for the 2-wave kernels)")
    a = ap.parse_args()
    import numpy as np
    import torch
    import migym
    from migym import _abi, configs
    dev = "cuda:0"
    mk = {}
    if a.task == "ShadowHand":
        cfg = configs.task_config("ShadowHand", a.num_envs, sim_device=dev)
        cfg["env"]["objectType"] = a.object_type
        mk["cfg"] = {"task": cfg}
    env = migym.make(seed=0, task=a.task, num_envs=a.num_envs, sim_device=dev, rl_device=dev, headless=True, **mk)
    g = torch.Generator(device=dev).manual_seed(1)
    pool = [torch.rand((env.num_actors, env.num_actions), device=dev, generator=g) * 2 - 1 for _ in range(8)]
    for i in range(20):
        env.step(pool[i % 8])
    torch.cuda.synchronize()
    K = a.launches
    env.kernel_span_begin(K)
    for i in range(K):
        env.step(pool[i % 8])
    torch.cuda.synchronize()
    lib = env._lib
    out = {"task": a.task, "num_envs": a.num_envs, "launches": []}
    cap = 1 << 22
    buf = np.zeros(2 * cap, np.uint64)
    ms = env.kernel_span_read(K)
    for k in range(K):
        n = C.c_int32(0)
        _abi.check(lib.mg_kernel_span_waves(env.sim, k, buf.ctypes.data, cap, C.byref(n)), lib)
        w = buf[:2 * n.value].reshape(-1, 2).astype(np.float64)
        w = w[(w[:, 0] > 0) & (w[:, 1] >= w[:, 0])]
        t0 = w[:, 0].min()
        st, en = w[:, 0] - t0, w[:, 1] - t0
        span = en.max()
        dur = en - st
        # ticks -> us through the launch's span in ms (mg_kernel_span_read)
        us = 1e3 * ms[k] / span if span > 0 else 0.0
        rec = {"span_us": float(span * us), "waves": int(len(w)),
               "wave_us": {q: float(np.percentile(dur, p) * us) for q, p in (("p10", 10), ("p50", 50), ("p90", 90), ("max", 100))},
               "wave_mean_us": float(dur.mean() * us),
               "start_ramp_us": {q: float(np.percentile(st, p) * us) for q, p in (("p50_of_first_round", 0),)},
               "end_us": {q: float(np.percentile(en, p) * us) for q, p in (("p50", 50), ("p90", 90), ("p99", 99), ("max", 100))},
               "first_round_start_spread_us": float(np.sort(st)[min(a.slots, len(st)) - 1] * us),
               "utilisation": float(dur.sum() / (span * a.slots)) if span > 0 else 0.0}
        out["launches"].append(rec)
    env.kernel_span_begin(0)
    print(json.dumps(out, indent=1))
    L = out["launches"]
    print(f"{a.task} {a.num_envs}: span {np.mean([x['span_us'] for x in L]):.1f} us, waves {L[0]['waves']}, wave mean "
          f"{np.mean([x['wave_mean_us'] for x in L]):.1f} us (p10 {np.mean([x['wave_us']['p10'] for x in L]):.1f}, p90 "
          f"{np.mean([x['wave_us']['p90'] for x in L]):.1f}, max {np.mean([x['wave_us']['max'] for x in L]):.1f}); "
          f"first-round start spread {np.mean([x['first_round_start_spread_us'] for x in L]):.1f} us; end p50 / p90 / max "
          f"{np.mean([x['end_us']['p50'] for x in L]):.1f} / {np.mean([x['end_us']['p90'] for x in L]):.1f} / "
          f"{np.mean([x['end_us']['max'] for x in L]):.1f} us; slot utilisation {np.mean([x['utilisation'] for x in L]):.3f}")
    env.close()


if __name__ == "__main__":
    main()
