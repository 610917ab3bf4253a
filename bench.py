#!/usr/bin/env python3
"""env-steps/s of the fused VecTask.step on MI355X (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--task Ant] [--num-envs 65536]
    torchrun --nproc-per-node N bench.py --gpus N ...

One "step" = one VecTask.step of every env on every rank (controlFrequencyInv=1,
2 physics substeps), random U(-1,1) actions generated on device before the timed
region, inputs resident in HBM.  Envs are independent, so ranks shard them
(weak scaling: --num-envs per GPU, no data-path collective).  Rank 0 prints ONE
JSON line.  See DESIGN.md §Measurement for the roofline accounting.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "isaacgymenvs-ma_amd"))

# algorithmic (compulsory) HBM bytes per env-step: every gym/VecTask-visible tensor
# read and written once per control step; model tables amortised to 0.
ALGO_BYTES = {"Ant": 673, "Humanoid": 1161, "Cartpole": 89, "MAAnt": 4 * 709,
              # ShadowHand: R actions 80, prev targets 96, dof 192, object+goal 104, bufs 28 = 500;
              # W targets 192, dof 192, 3 root rows 156, 27 rigid bodies 1404, dof_force 96, sensors 120,
              # obs 844, scalars 32 = 3036 (full rigid-body tensor materialised)
              "ShadowHand": 3536}
HBM_PEAK = 8.0e12  # B/s, MI355X_MICROARCH.md (spec)


def cpu_baseline(task, seconds=12.0, n=4096):
    """CPU oracle (fp32 task layer + fp64 physics restatement), OpenMP over envs, bounded sample."""
    import numpy as np
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle as O
    from migym import configs, model as M, taskdefs
    cores = min(os.cpu_count() or 1, int(os.environ.get("OMP_NUM_THREADS", "16")), 16)
    cfg = configs.task_config(task, n)
    base = "Ant" if task == "MAAnt" else task
    spec = M.load_builtin(taskdefs.TASK_INFO[base][1])
    A = int(cfg["env"].get("numAgents", 1)) if task == "MAAnt" else 1
    sp = taskdefs.sim_params(cfg, taskdefs.TASK_INFO[base][5], A)
    tp = taskdefs.task_params(task, cfg, spec)
    mnp = M.pack_model(spec)
    if task == "ShadowHand":
        n = min(n, 1024)
    h = O.HandHostEnv(tp, spec, n) if task == "ShadowHand" else O.HostEnv(tp, spec, n * A)
    rng = np.random.default_rng(0)
    acts = rng.uniform(-1, 1, (8,) + h.actions.shape).astype(np.float32)
    h.actions[:] = acts[0]
    h.env_step(mnp, sp, tp, 0, 0, cores)  # warm-up (first step resets every env)
    steps, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < seconds and steps < 5000:
        h.actions[:] = acts[steps % 8]
        h.env_step(mnp, sp, tp, 0, steps + 1, cores)
        steps += 1
    dt = time.perf_counter() - t0
    return {"value": n * steps / dt, "unit": "env-steps/s", "cores": cores, "kind": "port",
            "sample": f"{task} {n} envs x {steps} steps ({dt:.1f} s), oracle/ CPU restatement "
                      f"(fp64 physics, fp32 task layer), not PhysX"}


def pmc_traffic(task, n, kern_ms):
    """Measured HBM traffic of the dominant kernel for this workload, from the committed rocprofv3 --pmc
    passes of the same bench command (tools/gpu_prof.sh -> tools/pmc_summary.py --json): FETCH_SIZE x2
    (gfx950 correction) + WRITE_SIZE per launch, expressed over this run's launch time like `achieved`.
    None when no pass was recorded for this workload."""
    path = os.path.join(ROOT, "profiles", "r01", f"pmc_{task}_{n}.json")
    try:
        with open(path) as f:
            b = json.load(f)["traffic_bytes_per_launch"]
    except (OSError, ValueError, KeyError):
        return {"traffic": None}
    if b is None:
        return {"traffic": None}
    out = {"traffic": b / (kern_ms * 1e-3) / 1e9, "traffic_bytes_per_launch": b,
           "traffic_source": os.path.relpath(path, ROOT)}
    try:
        with open(path) as f:
            issue = json.load(f).get("issue")
        if issue:
            out["pmc_issue"] = issue   # VALU-active / wait fractions of the same launches
    except (OSError, ValueError):
        pass
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--task", default="Ant")
    ap.add_argument("--num-envs", type=int, default=65536, help="envs per GPU")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--gather", nargs="?", const="all", default=None, choices=["all", "root"],
                    help="concatenate obs/rew/reset of every rank each step: 'all' = one RCCL all-gather, "
                         "'root' = point-to-point sends to rank 0 (migym.dist.OutputGather)")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--backend", default="nccl", help="torch.distributed backend (nccl = RCCL)")
    ap.add_argument("--object-type", default="block", choices=["block", "egg", "pen"],
                    help="ShadowHand objectType (shadow_hand.py:86-100)")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    ndev = max(torch.cuda.device_count(), 1)
    dev = f"cuda:{local % ndev}"
    torch.cuda.set_device(dev)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device(dev))
        else:
            dist.init_process_group(args.backend)

    import migym
    n = args.num_envs
    mk = {}
    if args.task == "ShadowHand" and args.object_type != "block":
        from migym import configs
        tcfg = configs.task_config("ShadowHand", n, sim_device=dev)
        tcfg["env"]["objectType"] = args.object_type
        mk["cfg"] = {"task": tcfg}
    env = migym.make(seed=rank, task=args.task, num_envs=n, sim_device=dev, rl_device=dev, headless=True,
                     multi_gpu=world > 1, **mk)
    na = env.num_actions
    g = torch.Generator(device=dev).manual_seed(1234 + rank)
    pool = [torch.rand((env.num_actors, na), device=dev, generator=g) * 2 - 1 for _ in range(8)]
    gather = None
    if args.gather and world > 1 and args.backend == "nccl":
        from migym.dist import OutputGather
        gather = OutputGather(env.num_actors, env.num_obs, dev, mode=args.gather)

    def step(a):
        obs, rew, reset, _ = env.step(a)
        if gather is not None:
            gather(obs["obs"], rew, reset)

    for i in range(args.warmup):
        step(pool[i % 8])
    torch.cuda.synchronize()
    stream = torch.cuda.current_stream()
    starts = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps)]
    ends = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps)]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        starts[i].record(stream)
        step(pool[i % 8])
        ends[i].record(stream)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    kern_ms = sum(s.elapsed_time(e) for s, e in zip(starts, ends)) / args.steps
    if world > 1:
        t = torch.tensor([elapsed, kern_ms], dtype=torch.float64,
                         device=dev if args.backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, kern_ms = float(t[0]), float(t[1])
    value = n * world * args.steps / elapsed
    ms_per_step = 1e3 * elapsed / args.steps
    if rank == 0:
        per_launch = ALGO_BYTES[args.task] * n
        achieved = per_launch / (kern_ms * 1e-3)
        out = {
            "metric": "env-steps/sec (whole node) at num_envs=65536; 1/2/4/8 MI355X scaling",
            "value": value, "unit": "env-steps/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": ms_per_step, "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": "f32", "data": "synthetic (U(-1,1) actions, device-resident)",
            "config": {"workload": f"{args.task} VecTask.step, {n} envs per GPU, {env.sim_params.substeps} substeps, "
                                   f"PGS x{env.sim_params.pos_iters}",
                       "task": args.task, "num_envs_per_gpu": n, "num_envs_total": n * world,
                       "agents_per_env": env.num_agents, "agent_steps_per_s": value * env.num_agents,
                       "obs_gather": args.gather if gather is not None else None,
                       "parallelism": f"env-sharded x{world}",
                       **({"object_type": args.object_type} if args.task == "ShadowHand" else {})},
            "roofline": {"bound": "hbm", "achieved": achieved / 1e9, "peak": HBM_PEAK / 1e9, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK, **pmc_traffic(args.task, n, kern_ms),
                         "kernel": "k_hand_step" if args.task == "ShadowHand" else "k_env_step",
                         "kernel_ms": kern_ms,
                         "algo_bytes_per_env_step": ALGO_BYTES[args.task]},
        }
        if not args.no_cpu_baseline and world == 1:
            try:
                out["cpu_baseline"] = cpu_baseline(args.task, args.cpu_seconds)
            except Exception as ex:  # noqa: BLE001
                out["cpu_baseline"] = {"error": repr(ex)}
        print(json.dumps(out), flush=True)
    env.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
