"""Env sharding across ranks (world_size 2, gloo on CPU).

Each rank steps its own contiguous block of envs through the CPU oracle with
env_offset = rank * N (the GPU path takes the same offset through
mg_task_buffers.env_offset), then migym.dist.OutputGather concatenates
obs/rew/reset.  The gathered rollout must equal a single-process rollout of
all envs bit for bit: reset noise is keyed by the global env id.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import pyoracle as O
from migym import configs, model as M, taskdefs
from migym.dist import OutputGather

N_PER_RANK, STEPS = 24, 4


def _setup(task):
    cfg = configs.task_config(task, N_PER_RANK)
    spec = M.load_builtin(taskdefs.TASK_INFO[task][1])
    return spec, taskdefs.sim_params(cfg, taskdefs.TASK_INFO[task][5]), taskdefs.task_params(task, cfg, spec)


def _actions(step, n_total, na):
    return np.random.default_rng(100 + step).uniform(-1, 1, (n_total, na)).astype(np.float32)


def rollout(task, n, offset, n_total, rank_slice):
    spec, sp, tp = _setup(task)
    mnp = M.pack_model(spec)
    h = O.HostEnv(tp, spec, n)
    outs = []
    for t in range(STEPS):
        h.actions[:] = _actions(t, n_total, tp.num_actions)[rank_slice]
        h.env_step(mnp, sp, tp, seed=7, step=t, threads=1, env_offset=offset)
        outs.append((h.obs.copy(), h.rew.copy(), h.reset.copy()))
    return outs


def _worker(rank, world, port, task, q, mode="all"):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    n_total = N_PER_RANK * world
    outs = rollout(task, N_PER_RANK, rank * N_PER_RANK, n_total, slice(rank * N_PER_RANK, (rank + 1) * N_PER_RANK))
    spec, sp, tp = _setup(task)
    g = OutputGather(N_PER_RANK, tp.num_obs, "cpu", mode=mode)
    res = []
    for obs, rew, reset in outs:
        got = g(torch.from_numpy(obs), torch.from_numpy(rew), torch.from_numpy(reset))
        if got is None:
            assert mode == "root" and rank != 0
            continue
        o, r, d = got
        res.append((o.numpy().copy(), r.numpy().copy(), d.numpy().copy()))
    if rank == 0:
        q.put(res)
    dist.barrier()
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("task,mode", [("Ant", "all"), ("Cartpole", "all"), ("Ant", "root")])
def test_sharded_rollout_equals_single_process(task, mode):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, task, q, mode)) for r in range(world)]
    for p in procs:
        p.start()
    gathered = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    n_total = N_PER_RANK * world
    single = rollout(task, n_total, 0, n_total, slice(0, n_total))
    for (o, r, d), (so, sr, sd) in zip(gathered, single):
        np.testing.assert_array_equal(o, so)
        np.testing.assert_array_equal(r, sr)
        np.testing.assert_array_equal(d, sd)
