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


MA_AGENTS = 4


def _setup(task):
    cfg = configs.task_config(task, N_PER_RANK)
    if task == "MAAnt":   # build-defined multi-agent Ant (SURVEY.md §8(a) A-MA), 4 agents per env
        cfg["env"]["numAgents"] = MA_AGENTS
        spec = M.load_builtin("ant")
        return spec, taskdefs.sim_params(cfg, 16, MA_AGENTS), taskdefs.task_params(task, cfg, spec)
    spec = M.load_builtin(taskdefs.TASK_INFO[task][1])
    return spec, taskdefs.sim_params(cfg, taskdefs.TASK_INFO[task][5]), taskdefs.task_params(task, cfg, spec)


def _agents(task):
    return MA_AGENTS if task == "MAAnt" else 1


def _actions(step, n_total, na):
    return np.random.default_rng(100 + step).uniform(-1, 1, (n_total, na)).astype(np.float32)


def rollout(task, n_envs, env_offset, n_envs_total, rank_envs):
    """n_envs envs (x agents) starting at global env env_offset, stepped STEPS times by the oracle."""
    spec, sp, tp = _setup(task)
    A = _agents(task)
    mnp = M.pack_model(spec)
    h = O.HostEnv(tp, spec, n_envs * A)
    rows = slice(rank_envs.start * A, rank_envs.stop * A)
    outs = []
    for t in range(STEPS):
        h.actions[:] = _actions(t, n_envs_total * A, tp.num_actions)[rows]
        h.env_step(mnp, sp, tp, seed=7, step=t, threads=1, env_offset=env_offset)
        outs.append((h.obs.copy(), h.rew.copy(), h.reset.copy()))
    return outs


def _worker(rank, world, port, task, q, mode="all"):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    n_total = N_PER_RANK * world
    outs = rollout(task, N_PER_RANK, rank * N_PER_RANK, n_total, slice(rank * N_PER_RANK, (rank + 1) * N_PER_RANK))
    spec, sp, tp = _setup(task)
    g = OutputGather(N_PER_RANK * _agents(task), tp.num_obs, "cpu", mode=mode)
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


def _spawn(target, world, *args):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=target, args=(r, world, port) + args + (q,)) for r in range(world)]
    for p in procs:
        p.start()
    got = q.get(timeout=180)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return got


def _worker_args(rank, world, port, task, mode, q):
    _worker(rank, world, port, task, q, mode)


@pytest.mark.parametrize("task,mode,world", [("Ant", "all", 2), ("Cartpole", "all", 2), ("Ant", "root", 2),
                                             ("MAAnt", "root", 2), ("MAAnt", "root", 4)])
def test_sharded_rollout_equals_single_process(task, mode, world):
    """MAAnt: reset noise is keyed by the global actor id env_offset * A + a, so rank 1's agents draw
    what they draw in one process (the round-1 key env_offset + a collided across ranks); world 4 checks the
    offsets of ranks past the first two."""
    gathered = _spawn(_worker_args, world, task, mode)
    n_total = N_PER_RANK * world
    single = rollout(task, n_total, 0, n_total, slice(0, n_total))
    for (o, r, d), (so, sr, sd) in zip(gathered, single):
        np.testing.assert_array_equal(o, so)
        np.testing.assert_array_equal(r, sr)
        np.testing.assert_array_equal(d, sd)


# ---------------------------------------------------------------------------------------------- ShadowHand
HAND_ENVS, HAND_STEPS = 12, 6


def _hand_setup():
    cfg = configs.task_config("ShadowHand", HAND_ENVS)
    cfg["env"]["episodeLength"] = 3   # resets (and so running-mean updates) within the rollout
    spec = taskdefs.hand_spec("block")
    tp = taskdefs.task_params("ShadowHand", cfg, spec)
    return spec, taskdefs.sim_params(cfg, 24), tp


def hand_rollout(n_envs, env_offset, rank_envs, n_total, reducer=None):
    """ShadowHand oracle rollout; with ``reducer`` the running-mean partial sums are all-reduced over
    the ranks before they are applied (defer_finalize + mg_hand_finalize, as VecTask does on RCCL)."""
    spec, sp, tp = _hand_setup()
    mnp = M.pack_model(spec)
    h = O.HandHostEnv(tp, spec, n_envs)
    h.defer_finalize = 1 if reducer else 0
    outs = []
    for t in range(HAND_STEPS):
        h.actions[:] = _actions(t, n_total, tp.num_actions)[rank_envs]
        h.env_step(mnp, sp, tp, seed=11, step=t, threads=1, env_offset=env_offset)
        if reducer:
            reducer(h.scratch)
            h.finalize(tp)
        outs.append((h.obs.copy(), h.rew.copy(), h.reset.copy(), h.cons.copy()))
    return outs


def _hand_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)

    def reducer(scratch):
        t = torch.from_numpy(scratch.view(np.int64))
        dist.all_reduce(t)

    n_total = HAND_ENVS * world
    outs = hand_rollout(HAND_ENVS, rank * HAND_ENVS, slice(rank * HAND_ENVS, (rank + 1) * HAND_ENVS), n_total,
                        reducer)
    spec, sp, tp = _hand_setup()
    g = OutputGather(HAND_ENVS, tp.num_obs, "cpu", mode="all")
    res = []
    for obs, rew, reset, cons in outs:
        o, r, d = g(torch.from_numpy(obs), torch.from_numpy(rew), torch.from_numpy(reset))
        res.append((o.numpy().copy(), r.numpy().copy(), d.numpy().copy(), cons))
    if rank == 0:
        q.put(res)
    dist.barrier()
    dist.destroy_process_group()


def test_sharded_shadowhand_equals_single_process():
    """Every rank's consecutive_successes equals the one-process value over all envs: the partial sums
    (number of resets, successes of the resetting envs) are integers, so the all-reduce is exact."""
    world = 2
    gathered = _spawn(_hand_worker, world)
    n_total = HAND_ENVS * world
    single = hand_rollout(n_total, 0, slice(0, n_total), n_total)
    assert any(s[2].any() for s in single), "rollout must contain resets"
    for (o, r, d, c), (so, sr, sd, sc) in zip(gathered, single):
        np.testing.assert_array_equal(o, so)
        np.testing.assert_array_equal(r, sr)
        np.testing.assert_array_equal(d, sd)
        np.testing.assert_array_equal(c, sc)


# ---------------------------------------------------------------------------------------------- PackedGather
def _packed_worker(rank, world, port, mode, q):
    from migym.dist import PackedGather
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    task = "Ant"
    n_total = N_PER_RANK * world
    outs = rollout(task, N_PER_RANK, rank * N_PER_RANK, n_total, slice(rank * N_PER_RANK, (rank + 1) * N_PER_RANK))
    spec, sp, tp = _setup(task)
    g = PackedGather(N_PER_RANK, tp.num_obs, "cpu", mode=mode, depth=2)
    no = tp.num_obs
    res = []
    slots = []
    for obs, rew, reset in outs:
        pk = g.next_pack()        # the kernel would write this slot (mg_task_buffers.out_pack)
        pk[:, :no] = torch.from_numpy(obs)
        pk[:, no] = torch.from_numpy(rew)
        pk[:, no + 1] = torch.from_numpy(reset.astype(np.float32))
        g.issue()
        slots.append(g.last)
        if len(slots) % 2 == 0:   # two gathers in flight, then read both slots
            g.drain()
            if g.has_full:
                for i in slots[-2:]:
                    f = g.full[i]
                    res.append((f[:, :no].numpy().copy(), f[:, no].numpy().copy(),
                                f[:, no + 1].to(torch.long).numpy().copy()))
    if rank == 0:
        q.put(res)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("mode,world", [("root", 2), ("all", 2), ("root", 4), ("all", 4)])
def test_packed_gather_double_buffers_two_steps(mode, world):
    """PackedGather (the overlapped gather of the kernel-packed rows): with two steps in flight, each
    slot holds its own step's rows from every rank, equal to the single-process rollout.  World 4: the root
    posts three receives in one batch (bench.py's default gather on a multi-GPU node is this root mode)."""
    gathered = _spawn(_packed_worker, world, mode)
    n_total = N_PER_RANK * world
    single = rollout("Ant", n_total, 0, n_total, slice(0, n_total))
    assert len(gathered) == STEPS
    for (o, r, d), (so, sr, sd) in zip(gathered, single):
        np.testing.assert_array_equal(o, so)
        np.testing.assert_array_equal(r, sr)
        np.testing.assert_array_equal(d, sd)
