"""The RCCL code path of SURVEY.md §8(e) on the one-GPU box.

A world-size-1 ``nccl`` process group (RCCL on ROCm) in this process: no second rank and no exec, so it
runs on a 1-GPU box, and every collective the multi-GPU path issues goes through RCCL for real:

  * ``PackedGather(mode="all")``: ``all_gather_into_tensor`` of the rows the fused step packed into the
    gather's message slot (``mg_task_buffers.out_pack``), double-buffered on the collective's stream;
  * ``PackedGather(mode="root")``: the root's own rows written by its kernel into its slice;
  * ShadowHand's cross-rank running mean (``globalConsecutiveSuccesses: True``): the ``post_launch``
    all-reduce of the step's integer partial sums + ``mg_hand_finalize``.

Each gathered row must equal the step's ``obs_clamped`` / ``rew`` / ``reset`` bit for bit, and the
all-reduced running mean the in-step one (reference: rlgames_utils.py:89-107, shadow_hand.py:795-798).
"""
import os
import socket

import pytest
import torch
import torch.distributed as dist

import migym
from migym import configs
from migym.dist import PackedGather

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.fixture(scope="module")
def rccl_group():
    assert torch.cuda.is_available(), "GPU tests need the MI355X"
    torch.cuda.set_device(0)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()))
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device(DEV))
    assert dist.get_backend() == "nccl"
    yield
    dist.destroy_process_group()


@pytest.mark.parametrize("mode", ["all", "root"])
@pytest.mark.parametrize("task", ["Ant", "MAAnt", "ShadowHand"])
def test_packed_gather_over_rccl_equals_step_outputs(rccl_group, task, mode):
    cfg = configs.task_config(task, 512, sim_device=DEV)
    cfg["env"]["episodeLength"] = 3   # timeouts: resets inside the rollout
    env = migym.make(seed=0, task=task, num_envs=512, sim_device=DEV, rl_device=DEV, headless=True,
                     cfg={"task": cfg})
    g = PackedGather(env.num_actors, env.num_obs, DEV, mode=mode, depth=2)
    assert not g._gloo
    env.attach_output_gather(g)
    gen = torch.Generator(device=DEV).manual_seed(0)
    any_reset = False
    for _ in range(6):
        a = torch.rand((env.num_actors, env.num_actions), device=DEV, generator=gen) * 2.4 - 1.2
        obs, rew, reset, _ = env.step(a)
        o, r, d = g.result()
        torch.cuda.synchronize()
        assert torch.equal(o, obs["obs"])
        assert torch.equal(r, rew)
        assert torch.equal(d, reset)
        any_reset = any_reset or bool(reset.any())
    assert any_reset, "the rollout must contain resets"
    g.drain()
    env.close()


def test_shadowhand_running_mean_all_reduce_over_rccl(rccl_group):
    envs = []
    for glob in (False, True):
        cfg = configs.task_config("ShadowHand", 512, sim_device=DEV)
        cfg["env"]["episodeLength"] = 4
        cfg["env"]["globalConsecutiveSuccesses"] = glob
        envs.append(migym.make(seed=0, task="ShadowHand", num_envs=512, sim_device=DEV, rl_device=DEV,
                               headless=True, cfg={"task": cfg}))
    assert not envs[0]._global_cons and envs[1]._global_cons
    gen = torch.Generator(device=DEV).manual_seed(1)
    for _ in range(10):
        a = torch.rand((512, 20), device=DEV, generator=gen) * 2 - 1
        envs[0].step(a)
        envs[1].step(a)
        torch.cuda.synchronize()
        assert torch.equal(envs[0].consecutive_successes, envs[1].consecutive_successes)
        assert int(envs[1]._reduce.abs().sum()) == 0
    assert float(envs[0].consecutive_successes) != 0.0
    for e in envs:
        e.close()
