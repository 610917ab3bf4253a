#!/usr/bin/env python3
"""env-steps/s of the fused VecTask.step on MI355X (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--task Ant] [--num-envs 65536]
    torchrun --nproc-per-node N bench.py --gpus N ...

One "step" = one VecTask.step of every env on every rank (controlFrequencyInv=1,
2 physics substeps), random U(-1,1) actions generated on device before the timed
region, inputs resident in HBM.  Envs are independent, so ranks shard them
(weak scaling: --num-envs per GPU; the only collective is the obs/rew/reset gather to rank 0, timed).  The same
line carries `strong_scaling`: BASELINE.json's fixed-total configs (MA-Ant 65,536 envs, ShadowHand 32,768, and Ant
65,536) split over the ranks, timed the same way.  `roofline.kernel_ms` is the mean device-side span (first wave start
to last wave end, GPU wall clock) of the timed launches themselves.  Rank 0 prints ONE JSON line.  See DESIGN.md §7 for the roofline accounting.
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


def _cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


def usable_cores():
    """(threads to time on, how they were found): the CPUs this process may run on (sched_getaffinity),
    capped by the cgroup CPU quota (cpu.max: quota / period, the box's CPU share) and by OMP_NUM_THREADS
    when the launcher sets it.  nproc alone overstates it on the GPU boxes (the whole machine's CPUs)."""
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    n, how = aff, [f"sched_getaffinity {aff}"]
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
        if q != "max":
            c = max(1, int(int(q) // int(per)))
            how.append(f"cgroup cpu.max {c}")
            n = min(n, c)
    except (OSError, ValueError):
        pass
    omp = os.environ.get("OMP_NUM_THREADS")
    if omp and omp.isdigit() and int(omp) > 0:
        how.append(f"OMP_NUM_THREADS {omp}")
        n = min(n, int(omp))
    return max(1, n), ", ".join(how)


def cpu_baseline(task, seconds=10.0, n=65536, object_type="block", solver="pgs"):
    """The oracle's fp32 restatement of the same step (oracle/build/liboracle_f32.so: fp32 physics, fp32 task
    layer, OpenMP over envs), timed on this box's host cores at the workload's own env count on a bounded
    sample of steps: once with every core this process may use (``usable_cores``: affinity, cgroup quota,
    OMP_NUM_THREADS; nproc and the CPU model are reported beside it) and once on 1 core.  The reference's
    pipeline=cpu PhysX path cannot run anywhere here (no isaacgym), so this is a port, not the reference."""
    import numpy as np
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle as O
    from migym import configs, model as M, taskdefs
    nproc = os.cpu_count() or 1
    threads, usable = usable_cores()
    cfg = configs.task_config(task, n)
    base = "Ant" if task == "MAAnt" else task
    A = int(cfg["env"].get("numAgents", 1)) if task == "MAAnt" else 1
    if task == "ShadowHand":
        cfg["env"]["objectType"] = object_type
    cfg["sim"]["physx"]["solver"] = solver
    spec = taskdefs.hand_spec(object_type) if task == "ShadowHand" else M.load_builtin(taskdefs.TASK_INFO[base][1])
    sp = taskdefs.sim_params(cfg, taskdefs.TASK_INFO[base][5], A)
    tp = taskdefs.task_params(task, cfg, spec)
    mnp = M.pack_model(spec)

    def leg(nthreads, n_envs, secs):
        h = O.HandHostEnv(tp, spec, n_envs) if task == "ShadowHand" else O.HostEnv(tp, spec, n_envs * A)
        rng = np.random.default_rng(0)
        acts = rng.uniform(-1, 1, (4,) + h.actions.shape).astype(np.float32)
        h.actions[:] = acts[0]
        h.env_step(mnp, sp, tp, 0, 0, nthreads, fp32=True)   # warm-up (the first step resets every env)
        steps, t0 = 0, time.perf_counter()
        while time.perf_counter() - t0 < secs and steps < 5000:
            h.actions[:] = acts[steps % 4]
            h.env_step(mnp, sp, tp, 0, steps + 1, nthreads, fp32=True)
            steps += 1
        dt = time.perf_counter() - t0
        return n_envs * steps / dt, f"{task} {n_envs} envs x {steps} steps ({dt:.1f} s)"

    v, smp = leg(threads, n, seconds)
    v1, smp1 = leg(1, min(n, 8192), seconds)
    return {"value": v, "unit": "env-steps/s", "cores": threads, "kind": "port",
            "sample": f"{smp}, {threads} OpenMP threads (every core this process may use: {usable}); oracle/ fp32 "
                      f"CPU restatement of the same step (liboracle_f32.so), not PhysX",
            "usable_cores": usable, "nproc": nproc, "cpu_model": _cpu_model(),
            "single_core": {"value": v1, "unit": "env-steps/s", "cores": 1, "sample": smp1}}


def baseline_config0(dev, steps=1000, n=256):
    """BASELINE.json configs[0]: Cartpole, 256 envs, random actions, 1000 steps.  The reference quotes it
    on pipeline=cpu; here the same rollout runs through the fused HIP step on `dev` (wall clock of the
    1000 VecTask.step calls, each host->device action copy included, since that configuration hands actions
    over from the host) and through the oracle's fp32 CPU restatement on 1 core and on every usable core."""
    import numpy as np
    import torch
    import migym
    env = migym.make(seed=0, task="Cartpole", num_envs=n, sim_device=dev, rl_device=dev, headless=True)
    rng = np.random.default_rng(0)
    host = torch.from_numpy(rng.uniform(-1, 1, (8, n, env.num_actions)).astype(np.float32))
    for i in range(10):
        env.step(host[i % 8].to(dev, non_blocking=True))
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(steps):
        env.step(host[i % 8].to(dev, non_blocking=True))
    torch.cuda.synchronize()
    gpu_s = time.perf_counter() - t0
    env.close()
    # the configuration as BASELINE.json names it: pipeline=cpu, sim_device=cpu, through make() -- the HIP step
    # underneath with host-side views of every task tensor (migym/host_pipeline.py), host actions in, host
    # outputs (rl_device cpu) out, the mirrors' transfers included
    import contextlib
    with contextlib.redirect_stdout(sys.stderr):  # VecTask's "Forcing CPU Pipeline" notice: stdout carries one JSON line
        cenv = migym.make(seed=0, task="Cartpole", num_envs=n, sim_device="cpu", rl_device="cpu", headless=True)
    for i in range(10):
        cenv.step(host[i % 8])
    t0 = time.perf_counter()
    for i in range(steps):
        cenv.step(host[i % 8])
    cpu_pipe_s = time.perf_counter() - t0
    assert cenv.device == "cpu" and cenv.obs_buf.device.type == "cpu"
    cenv.close()
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle as O
    from migym import configs, model as M, taskdefs
    cfg = configs.task_config("Cartpole", n)
    spec = M.load_builtin(taskdefs.TASK_INFO["Cartpole"][1])
    sp = taskdefs.sim_params(cfg, taskdefs.TASK_INFO["Cartpole"][5], 1)
    tp = taskdefs.task_params("Cartpole", cfg, spec)
    mnp = M.pack_model(spec)
    threads, _ = usable_cores()
    cpu = {}
    for nt in sorted({1, threads}):
        h = O.HostEnv(tp, spec, n)
        h.actions[:] = host[0].numpy()
        h.env_step(mnp, sp, tp, 0, 0, nt, fp32=True)
        t0 = time.perf_counter()
        for i in range(steps):
            h.actions[:] = host[i % 8].numpy()
            h.env_step(mnp, sp, tp, 0, i + 1, nt, fp32=True)
        cpu[nt] = time.perf_counter() - t0
    return {"workload": f"Cartpole {n} envs x {steps} random-action steps (BASELINE.json configs[0])",
            "gpu": {"seconds": gpu_s, "env_steps_per_s": n * steps / gpu_s, "device": dev,
                    "note": "fused HIP step, host action copy per step included"},
            "cpu_pipeline": {"seconds": cpu_pipe_s, "env_steps_per_s": n * steps / cpu_pipe_s,
                             "note": "make(sim_device='cpu', rl_device='cpu'): env.device 'cpu', host tensors, the "
                                     "HIP step on the GPU underneath (host_pipeline.py), mirror transfers included"},
            "cpu_port": {f"{nt}_cores": {"seconds": s, "env_steps_per_s": n * steps / s} for nt, s in cpu.items()},
            "cpu_kind": "port (oracle fp32 restatement; the reference's PhysX CPU pipeline is not runnable here)"}


VALU_SIMDS, CLOCK_HZ = 256 * 4, 2.4e9   # MI355X: 256 CUs x 4 SIMD-32, peak engine clock (MI355X_MICROARCH.md)


def pmc_traffic(task, n, kern_ms, object_type="block"):
    """Measured HBM traffic of the dominant kernel for this workload, from the committed rocprofv3 --pmc
    passes of the same bench command (tools/gpu_prof.sh -> tools/pmc_summary.py --json): FETCH_SIZE x2
    (gfx950 correction) + WRITE_SIZE per launch, expressed over this run's launch time like `achieved`.
    None when no pass was recorded for this workload."""
    path = None
    tag = task if (task != "ShadowHand" or object_type == "block") else f"{task}-{object_type}"   # per kernel instance
    for rnd in ("r06", "r05", "r04", "r03", "r02", "r01"):   # the newest round's passes of this workload
        cand = os.path.join(ROOT, "profiles", rnd, f"pmc_{tag}_{n}.json")
        if os.path.exists(cand):
            path = cand
            break
    if path is None:
        return {"traffic": None}
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
            out["pmc_issue"] = dict(issue)   # VALU-active / wait fractions of the same launches
            vi = issue.get("valu_insts_per_launch")
            if vi:
                # the bound that does apply: VALU issue against its peak, one wave64 instruction
                # per 2 cycles on each of the 1,024 SIMD-32s at the 2.4 GHz peak clock
                out["pmc_issue"]["valu_issue_frac_of_peak"] = vi * 2.0 / (VALU_SIMDS * kern_ms * 1e-3 * CLOCK_HZ)
    except (OSError, ValueError):
        pass
    return out


# BASELINE.json's fixed-total configs (split over the ranks), plus the headline Ant total for the strong curve
STRONG_CONFIGS = (("MAAnt", 65536, "BASELINE configs[3]: multi-agent Ant (4 agents/env), 65,536 envs total"),
                  ("ShadowHand", 32768, "BASELINE configs[4]: ShadowHand, 32,768 envs total"),
                  ("Ant", 65536, "Ant, 65,536 envs total (strong-scaling counterpart of the headline)"))


def run_workload(task, n, object_type, args, world, rank, dev, gather_mode, seed, what=None, total=None):
    """One workload: make() `n` envs on this rank, W warm-up steps, K timed steps between barrier + synchronize
    (max over ranks), then a separate kernel-duration pass (HIP events around each of --kernel-samples launches on
    the launch stream, median; the timed region has no events, so its wall time is not diluted by them)."""
    import torch
    import torch.distributed as dist
    import migym
    mk = {}
    if (task == "ShadowHand" and object_type != "block") or args.solver != "pgs":
        from migym import configs
        tcfg = configs.task_config(task, n, sim_device=dev)
        if task == "ShadowHand":
            tcfg["env"]["objectType"] = object_type
        tcfg["sim"]["physx"]["solver"] = args.solver
        mk["cfg"] = {"task": tcfg}
    env = migym.make(seed=seed, task=task, num_envs=n, sim_device=dev, rl_device=dev, headless=True,
                     multi_gpu=world > 1, **mk)
    na = env.num_actions
    g = torch.Generator(device=dev).manual_seed(1234 + rank)
    pool = [torch.rand((env.num_actors, na), device=dev, generator=g) * 2 - 1 for _ in range(8)]
    gather = None
    if gather_mode != "none" and world > 1:
        from migym.dist import PackedGather
        gather = PackedGather(env.num_actors, env.num_obs, dev, mode=gather_mode)
        env.attach_output_gather(gather)
    for i in range(args.warmup):
        env.step(pool[i % 8])
    if gather is not None:
        gather.drain()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    # the device-side span of every timed launch (first wave start -> last wave end on the GPU wall clock,
    # mg_kernel_span_begin: one plain store per wave at its start and end; same-box A/B against a build without the
    # hooks: no difference, profiles/r05/ab_span.txt).  Launches are stream-ordered, so the spans of the timed
    # launches sum to at most the timed wall time: kernel_ms (their mean) <= ms_per_step by construction.
    nspan = min(args.steps, 1024)
    env.kernel_span_begin(nspan)
    t0 = time.perf_counter()
    for i in range(args.steps):
        env.step(pool[i % 8])
    if gather is not None:
        gather.drain()   # the last step's rows have reached the root
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    spans = [float(x) for x in env.kernel_span_read(nspan) if x > 0]
    env.kernel_span_begin(0)
    span_ok = len(spans) == nspan
    # HIP events around each of --kernel-samples further launches (untimed), for comparison: kernel + the event
    # packets' dispatch latency; kernel_ms falls back to their median for a library built without the span hooks
    ks = max(1, args.kernel_samples)
    starts = [torch.cuda.Event(enable_timing=True) for _ in range(ks)]
    ends = [torch.cuda.Event(enable_timing=True) for _ in range(ks)]
    for i in range(ks):
        env.launch_events = (starts[i], ends[i])
        env.step(pool[i % 8])
    env.launch_events = None
    if gather is not None:
        gather.drain()
    torch.cuda.synchronize()
    ev = sorted(starts[i].elapsed_time(ends[i]) for i in range(ks))
    event_ms = ev[ks // 2] if ks % 2 else 0.5 * (ev[ks // 2 - 1] + ev[ks // 2])
    # steady state: a further untimed sample of the same rollout (a short timed run right after the first
    # reset is not steady state -- early-episode rows make the locomotion steps heavier, the hand's lighter)
    steady_ms = None
    if args.steady_steps > 0:
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        for i in range(args.steady_steps):
            env.step(pool[i % 8])
        if gather is not None:
            gather.drain()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        steady_ms = 1e3 * (time.perf_counter() - t1) / args.steady_steps
    if not span_ok:
        print(f"bench.py: the span hooks recorded {len(spans)} of {nspan} launches; kernel_ms from HIP events",
              file=sys.stderr)
    kern_ms = sum(spans) / len(spans) if span_ok else event_ms
    if world > 1:
        t = torch.tensor([elapsed, kern_ms, event_ms, steady_ms or 0.0], dtype=torch.float64,
                         device=dev if args.backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, kern_ms, event_ms = float(t[0]), float(t[1]), float(t[2])
        steady_ms = float(t[3]) if steady_ms is not None else None
    info = {"substeps": env.sim_params.substeps, "pos_iters": env.sim_params.pos_iters, "agents": env.num_agents,
            "solver": "TGS" if env.sim_params.solver_type == 1 else "PGS",
            "vel_sweeps": max(env.sim_params.pos_iters, env.sim_params.vel_iters) if env.sim_params.solver_type == 1
            else 0}
    import ctypes
    tl, cl = ctypes.c_int32(), ctypes.c_int32()
    if env._lib.mg_sim_kernel_layout(env.sim, ctypes.byref(tl), ctypes.byref(cl)) == 0:
        # the step kernel's team layout (MIGYM_LAYOUT): classic 8 / compact 12 waves per CU
        info["team_layout"] = f"T={tl.value} " + ("compact" if cl.value else "classic")
    env.close()
    del env, pool, gather
    value = n * world * args.steps / elapsed
    r = {"value": value, "unit": "env-steps/s", "ms_per_step": 1e3 * elapsed / args.steps, "kernel_ms": kern_ms,
         "kernel_ms_sample": (f"mean over the {nspan} timed launches of each launch's device-side span (first wave "
                              f"start to last wave end, GPU wall clock; max over ranks)") if span_ok else
                             f"median of HIP events around {ks} launches (no span hooks in this library)",
         "event_ms": event_ms,
         "steady_state_ms": steady_ms,
         "steady_state_value": (n * world / (steady_ms * 1e-3)) if steady_ms else None,
         "steady_state_sample": (f"{args.steady_steps} further steps of the same rollout after the timed ones and the "
                                 f"event pass, untimed by the contract (wall clock, barrier + synchronize, max over "
                                 f"ranks): ms_per_step / steady_state_ms - 1 is the timed run's early-episode bias")
                                if steady_ms else None,
         "gathered": gather_mode if (gather_mode != "none" and world > 1) else None, "env_info": info}
    if what is not None:
        r.update({"config": what, "task": task, "num_envs_total": total, "num_envs_per_gpu": n, "n_gpus": world,
                  "agents_per_env": info["agents"], "agent_steps_per_s": value * info["agents"],
                  "scaling": "strong"})
    return r


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--task", default="Ant")
    ap.add_argument("--num-envs", type=int, default=65536, help="envs per GPU")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--gather", default=None, choices=["all", "root", "none"],
                    help="concatenate obs/rew/reset of every rank each step, inside the timed region "
                         "(migym.dist.PackedGather: rows packed by the kernel, double-buffered, overlapped with "
                         "the next step): 'root' = point-to-point sends to rank 0 (default when --gpus > 1), "
                         "'all' = one RCCL all-gather, 'none' = no gather")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--kernel-samples", type=int, default=32,
                    help="launches after the timed region bracketed by HIP events on the launch stream (event_ms, "
                         "their median, reported beside kernel_ms: the timed launches' mean device-side span)")
    ap.add_argument("--no-strong", action="store_true",
                    help="skip the strong-scaling lines (BASELINE configs[3]/[4] and Ant 65,536 as fixed totals "
                         "split over the ranks)")
    ap.add_argument("--steady-steps", type=int, default=200,
                    help="an untimed further sample of the same rollout after the timed steps, reported as "
                         "steady_state_ms beside ms_per_step (0: skip)")
    ap.add_argument("--backend", default="nccl", help="torch.distributed backend (nccl = RCCL)")
    ap.add_argument("--solver", default="pgs", choices=["pgs", "tgs"],
                    help="sim.physx.solver: north_star's PGS (default) or the build-defined TGS (DESIGN.md §4)")
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
    gather_mode = args.gather or ("root" if world > 1 else "none")
    head = run_workload(args.task, n, args.object_type, args, world, rank, dev, gather_mode, seed=rank)
    # strong scaling: BASELINE.json's fixed-total multi-GPU configs, each rank stepping total / world envs of one
    # node-size rollout (global env ids rank * n_rank ..., so the shards are slices of it), same timing rules
    strong = []
    if not args.no_strong:
        for task, total, what in STRONG_CONFIGS:
            if total % world:
                continue
            strong.append(run_workload(task, total // world, "block", args, world, rank, dev, gather_mode, seed=0,
                                       what=what, total=total))
    value = head["value"]
    ms_per_step, kern_ms = head["ms_per_step"], head["kernel_ms"]
    if kern_ms > ms_per_step and rank == 0:   # the device span cannot exceed the steady-state time per step
        print(f"bench.py: kernel_ms {kern_ms:.4f} > ms_per_step {ms_per_step:.4f}", file=sys.stderr)
    if rank == 0:
        per_launch = ALGO_BYTES[args.task] * n
        achieved = per_launch / (kern_ms * 1e-3)
        env = head["env_info"]
        out = {
            "metric": "env-steps/sec (whole node) at num_envs=65536; 1/2/4/8 MI355X scaling",
            "value": value, "unit": "env-steps/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": ms_per_step, "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "steady_state_ms": head["steady_state_ms"], "steady_state_value": head["steady_state_value"],
            "steady_state_sample": head["steady_state_sample"],
            "dtype": "f32", "data": "synthetic (U(-1,1) actions, device-resident)",
            "config": {"workload": f"{args.task} VecTask.step, {n} envs per GPU, {env['substeps']} substeps, "
                                   + (f"PGS x{env['pos_iters']}" if env["solver"] == "PGS" else
                                      f"TGS x{env['pos_iters']} sub-steps + {env['vel_sweeps']} velocity sweeps"),
                       "task": args.task, "num_envs_per_gpu": n, "num_envs_total": n * world,
                       "agents_per_env": env["agents"], "agent_steps_per_s": value * env["agents"],
                       "obs_gather": (f"{gather_mode}: kernel-packed [obs|rew|reset] rows, double-buffered, "
                                      f"overlapped with the next step, inside the timed region")
                                     if head["gathered"] else None,
                       "parallelism": f"env-sharded x{world}", "team_layout": env.get("team_layout"),
                       **({"object_type": args.object_type} if args.task == "ShadowHand" else {})},
            "roofline": {"bound": "hbm", "achieved": achieved / 1e9, "peak": HBM_PEAK / 1e9, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK, **pmc_traffic(args.task, n, kern_ms, args.object_type),
                         "kernel": "k_hand_step" if args.task == "ShadowHand" else "k_env_step",
                         "kernel_ms": kern_ms, "kernel_ms_sample": head["kernel_ms_sample"],
                         "kernel_ms_scope": ("the fused step kernel only: with work ordering on (DESIGN.md §3) the "
                                             "sort's two small launches before it (k_ohist, k_oscatter; rocprof "
                                             "profiles/r06/*kernel_stats.csv) lie outside kernel_ms and inside "
                                             "event_ms and ms_per_step"),
                         "kernel_ms_le_ms_per_step": kern_ms <= ms_per_step,
                         "event_ms": head["event_ms"],
                         "event_ms_note": "HIP events around each launch of the same pass: kernel + the event "
                                          "packets' dispatch latency, so above kernel_ms",
                         "algo_bytes_per_env_step": ALGO_BYTES[args.task]},
        }
        if strong:
            out["strong_scaling"] = [{k: v for k, v in r.items() if k != "env_info"} for r in strong]
        if not args.no_cpu_baseline and world == 1:
            try:
                out["cpu_baseline"] = cpu_baseline(args.task, args.cpu_seconds, n, args.object_type, args.solver)
            except Exception as ex:  # noqa: BLE001
                out["cpu_baseline"] = {"error": repr(ex)}
        if not args.no_cpu_baseline and world == 1:
            try:
                out["baseline_config0"] = baseline_config0(dev)
            except Exception as ex:  # noqa: BLE001
                out["baseline_config0"] = {"error": repr(ex)}
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
