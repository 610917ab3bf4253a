"""GPU tests of the task API around the fused step:

  * get_env_state / set_env_state: a rollout restored from a checkpointed state continues bit for bit;
  * reset_idx(env_ids): the listed envs hold their reset state right after the call (the reference
    writes it immediately, ant.py:252-279, shadow_hand.py:586-668), the other envs are untouched;
    multi-agent layouts take agent ids through the AND filter (franka_reach_MA.py:616-621, 875-889);
  * with domain randomization, the checkpointed state includes the draw counters, so a resumed rollout
    draws the same samples.
"""
import os

import numpy as np
import pytest
import torch

import migym
from migym import configs

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def make(task, n, **kw):
    assert torch.cuda.is_available(), "GPU tests need the MI355X"
    return migym.make(seed=3, task=task, num_envs=n, sim_device=DEV, rl_device=DEV, headless=True, **kw)


def actions(env, k):
    g = torch.Generator(device=DEV).manual_seed(100 + k)
    return torch.rand((env.num_actors, env.num_actions), device=DEV, generator=g) * 2 - 1


@pytest.mark.parametrize("task,n", [("Ant", 256), ("Humanoid", 64), ("MAAnt", 64), ("ShadowHand", 64)])
def test_env_state_round_trip(task, n):
    env = make(task, n)
    for k in range(4):
        env.step(actions(env, k))
    state = env.get_env_state()
    assert "root_states" in state or "root_state_tensor" in state
    assert state["control_steps"] == 4
    ref = []
    for k in range(4, 8):
        obs, rew, reset, _ = env.step(actions(env, k))
        ref.append((obs["obs"].clone(), rew.clone(), reset.clone()))
    env.set_env_state(state)
    assert env.control_steps == 4
    for k in range(4, 8):
        obs, rew, reset, _ = env.step(actions(env, k))
        o, r, d = ref[k - 4]
        torch.testing.assert_close(obs["obs"], o, rtol=0, atol=0)
        torch.testing.assert_close(rew, r, rtol=0, atol=0)
        assert torch.equal(reset, d)
    env.set_env_state(None)   # a reference checkpoint's state: no-op
    env.close()


def test_reset_idx_locomotion_writes_state_now():
    n = 128
    env = make("Ant", n)
    for k in range(3):
        env.step(actions(env, k))
    nd = env.num_dof
    before_root = env.root_states.clone()
    before_dof = env.dof_state.view(n, nd, 2).clone()
    ids = torch.tensor([1, 5, 77], device=DEV)
    u = torch.rand((n, 2 * nd), device=DEV, generator=torch.Generator(device=DEV).manual_seed(9))
    env.set_reset_noise(u)
    env.progress_buf[ids] = 17
    env.reset_buf[ids] = 1
    env.reset_idx(ids)
    torch.cuda.synchronize()
    dof = env.dof_state.view(n, nd, 2)
    # ant.py:255-265: positions U(-0.2, 0.2) about the initial pose, clamped; velocities U(-0.1, 0.1)
    pos = torch.clamp(env.initial_dof_pos[ids] + (0.4 * u[ids, :nd] - 0.2), env.dof_limits_lower,
                      env.dof_limits_upper)
    torch.testing.assert_close(dof[ids, :, 0], pos, rtol=0, atol=1e-6)
    torch.testing.assert_close(dof[ids, :, 1], 0.2 * u[ids, nd:] - 0.1, rtol=0, atol=1e-6)
    torch.testing.assert_close(env.root_states[ids], env.initial_root_states[ids], rtol=0, atol=0)
    # ant.py:268-279: potentials = prev_potentials = -|to_target (xy)| / dt
    to_t = env.targets[ids] - env.initial_root_states[ids, 0:3]
    to_t[:, 2] = 0
    pot = -torch.norm(to_t, p=2, dim=-1) / env.dt
    torch.testing.assert_close(env.potentials[ids], pot, rtol=1e-6, atol=1e-4)
    torch.testing.assert_close(env.prev_potentials[ids], pot, rtol=1e-6, atol=1e-4)
    assert (env.progress_buf[ids] == 0).all() and (env.reset_buf[ids] == 0).all()
    keep = torch.ones(n, dtype=torch.bool, device=DEV)
    keep[ids] = False
    assert torch.equal(env.root_states[keep], before_root[keep])
    assert torch.equal(dof[keep], before_dof[keep])
    env.set_reset_noise(None)
    # device RNG (no injected noise): deterministic, within the reset ranges
    env.reset_idx(ids)
    a = env.dof_state.view(n, nd, 2)[ids].clone()
    env.reset_idx(ids)
    assert torch.equal(env.dof_state.view(n, nd, 2)[ids], a)
    assert (a[..., 1].abs() <= 0.1 + 1e-6).all()
    env.step(actions(env, 9))   # the step runs on from the reset state
    assert torch.isfinite(env.obs_buf).all()
    env.close()


def test_reset_idx_cartpole():
    n = 64
    env = make("Cartpole", n)
    env.step(actions(env, 0))
    ids = torch.arange(0, n, 7, device=DEV)
    u = torch.rand((n, 4), device=DEV, generator=torch.Generator(device=DEV).manual_seed(2))
    env.set_reset_noise(u)
    env.reset_idx(ids)
    torch.cuda.synchronize()
    dof = env.dof_state.view(n, 2, 2)
    # cartpole.py:122-127: positions 0.2 (U - 0.5), velocities 0.5 (U - 0.5)
    torch.testing.assert_close(dof[ids, :, 0], 0.2 * (u[ids, :2] - 0.5), rtol=0, atol=1e-6)
    torch.testing.assert_close(dof[ids, :, 1], 0.5 * (u[ids, 2:] - 0.5), rtol=0, atol=1e-6)
    assert (env.progress_buf[ids] == 0).all() and (env.reset_buf[ids] == 0).all()
    env.close()


def test_reset_idx_shadow_hand():
    n = 32
    env = make("ShadowHand", n)
    for k in range(2):
        env.step(actions(env, k))
    ids = torch.tensor([0, 3, 30], device=DEV)
    keep = torch.ones(n, dtype=torch.bool, device=DEV)
    keep[ids] = False
    root_before = env.root_state_tensor.view(n, 3, 13).clone()
    env.successes[ids] = 3.0
    env.progress_buf[ids] = 11
    env.reset_idx(ids)
    torch.cuda.synchronize()
    nd = env.num_shadow_hand_dofs if hasattr(env, "num_shadow_hand_dofs") else env.num_dof
    dof = env.dof_state.view(n, nd, 2)
    lo, hi = env.shadow_hand_dof_lower_limits, env.shadow_hand_dof_upper_limits
    assert ((dof[ids, :, 0] >= lo - 1e-5) & (dof[ids, :, 0] <= hi + 1e-5)).all()
    # PD targets and previous targets start at the reset DOF positions (shadow_hand.py:657-661)
    torch.testing.assert_close(env.cur_targets[ids], dof[ids, :, 0], rtol=0, atol=0)
    torch.testing.assert_close(env.prev_targets[ids], dof[ids, :, 0], rtol=0, atol=0)
    root = env.root_state_tensor.view(n, 3, 13)
    assert (root[ids, 1, 7:13] == 0).all()                    # object at rest
    quat_n = root[ids, 1, 3:7].norm(dim=-1)
    torch.testing.assert_close(quat_n, torch.ones_like(quat_n), rtol=0, atol=1e-5)
    assert (env.progress_buf[ids] == 0).all() and (env.reset_buf[ids] == 0).all()
    assert (env.successes[ids] == 0).all()
    assert torch.equal(root[keep], root_before[keep])
    env.step(actions(env, 5))
    assert torch.isfinite(env.obs_buf).all()
    env.close()


def test_reset_idx_multi_agent_and_filter():
    """MA reset_idx(agent_ids): an env resets only when its ids count num_agents times (bincount, so a
    repeated id counts twice, as in the reference), and then every agent of it resets; a partially listed
    env is untouched (franka_reach_MA.py:875-885)."""
    n = 64
    env = make("MAAnt", n)
    A = env.num_agents
    assert A == 4
    for k in range(3):
        env.step(actions(env, k))
    before = env.root_states.clone()
    prog_before = env.progress_buf.clone()
    assert (prog_before > 0).all()
    # env 0 fully listed; env 1 three of four agents; env 2 two agents listed twice each; env 3 three
    # agents; plus random ids: the envs to reset are what the reference returned for this list
    G = np.load(os.path.join(os.path.dirname(__file__), "golden", "ma_conventions.npz"))
    ids = torch.tensor(G["A4_dup_ids"], device=DEV)
    full = set(G["A4_dup_env_ids"].tolist())
    assert 0 in full and 2 in full and 1 not in full and 3 not in full
    env.reset_idx(ids)
    torch.cuda.synchronize()
    for e in range(n):
        rows = slice(A * e, A * e + A)
        if e in full:
            torch.testing.assert_close(env.root_states[rows], env.initial_root_states[rows], rtol=0, atol=0)
            assert (env.progress_buf[rows] == 0).all() and (env.reset_buf[rows] == 0).all()
        else:
            assert torch.equal(env.root_states[rows], before[rows])
            assert torch.equal(env.progress_buf[rows], prog_before[rows])
    env.step(actions(env, 7))
    assert torch.isfinite(env.obs_buf).all()
    env.close()


def test_env_state_round_trip_with_randomization():
    n = 512
    cfg = configs.task_config("Ant", n, sim_device=DEV)
    cfg["task"]["randomize"] = True
    cfg["task"]["randomization_params"]["frequency"] = 1   # every reset re-randomizes
    cfg["env"]["episodeLength"] = 4                        # resets inside the resumed window
    env = make("Ant", n, cfg={"task": cfg})
    assert env.randomize
    for k in range(5):
        env.step(actions(env, k))
    state = env.get_env_state()
    assert "domain_randomization" in state
    # the state survives a checkpoint: torch.save, then torch.load with the safe (weights_only) loader
    import io
    buf = io.BytesIO()
    torch.save(state, buf)
    buf.seek(0)
    state = torch.load(buf, weights_only=True)
    ref = []
    for k in range(5, 12):
        obs, rew, reset, _ = env.step(actions(env, k))
        ref.append((obs["obs"].clone(), rew.clone(), reset.clone(), env.env_props.clone()))
    assert any(bool(r[2].any()) for r in ref), "the resumed window must contain resets (re-randomization)"
    env.set_env_state(state)
    for k in range(5, 12):
        obs, rew, reset, _ = env.step(actions(env, k))
        o, r, d, p = ref[k - 5]
        assert torch.equal(obs["obs"], o) and torch.equal(rew, r) and torch.equal(reset, d)
        assert torch.equal(env.env_props, p)
    env.close()


@pytest.mark.parametrize("task,n,how", [("Ant", 256, "sim_device"), ("ShadowHand", 64, "pipeline")])
def test_cpu_pipeline_host_views(task, n, how):
    """use_gpu_pipeline=False / sim_device='cpu' (vec_task.py:78-90): env.device is 'cpu' and every tensor the task
    exposes is a host tensor, the HIP step runs underneath (the same numbers as the GPU pipeline, bit for bit), views
    keep their base (dof_pos on dof_state), and host-side edits of the buffers take effect on the next step."""
    g = make(task, n)
    if how == "sim_device":
        c = migym.make(seed=3, task=task, num_envs=n, sim_device="cpu", rl_device=DEV, headless=True)
    else:
        cfg = configs.task_config(task, n, sim_device=DEV, pipeline="cpu")
        assert cfg["sim"]["use_gpu_pipeline"] is False
        c = migym.make(seed=3, task=task, num_envs=n, sim_device=DEV, rl_device=DEV, headless=True,
                       cfg={"task": cfg})
    assert c.device == "cpu" and c.unwrapped.device.startswith("cuda")
    for name in ("root_states", "dof_state", "obs_buf", "rew_buf", "reset_buf", "progress_buf"):
        assert getattr(c, name).device.type == "cpu", name
    pos = "shadow_hand_dof_pos" if task == "ShadowHand" else "dof_pos"
    assert getattr(c, pos).untyped_storage().data_ptr() == c.dof_state.untyped_storage().data_ptr()
    for k in range(3):
        og, rg, dg, _ = g.step(actions(g, k))
        oc, rc, dc, _ = c.step(actions(g, k).cpu())
        assert torch.equal(oc["obs"], og["obs"]) and torch.equal(rc, rg) and torch.equal(dc, dg)
        assert torch.equal(c.root_states, g.root_states.cpu()) and torch.equal(getattr(c, pos), getattr(g, pos).cpu())
        assert torch.equal(c.progress_buf, g.progress_buf.cpu())
    # a host-side edit: force resets of the first envs on both
    c.reset_buf[:5] = 1
    g.reset_buf[:5] = 1
    og, _, _, _ = g.step(actions(g, 9))
    oc, _, _, _ = c.step(actions(g, 9).cpu())
    assert torch.equal(oc["obs"], og["obs"]) and torch.equal(c.progress_buf, g.progress_buf.cpu())
    assert bool((c.progress_buf[:5] <= 1).all())
    g.close()
    c.close()


@pytest.mark.parametrize("task,filled", [("Ant", False), ("MAAnt", False), ("Cartpole", False), ("Humanoid", True),
                                         ("ShadowHand", True)])
def test_dof_force_tensor_where_the_reference_acquires_one(task, filled):
    """dof_force_tensor is filled every step where the reference task acquires a DOF-force tensor (humanoid.py:85-86,
    shadow_hand.py:157-159) and stays zero where it does not (ant.py, cartpole.py: the fused step skips it); the
    Humanoid observation's DOF-force block (obs[54:75], humanoid.py:405) is the tensor times contact_force_scale"""
    env = make(task, 64)
    for k in range(3):
        obs, _, _, _ = env.step(actions(env, k))
    torch.cuda.synchronize()
    f = env.dof_force_tensor
    if not filled:
        assert int(torch.count_nonzero(f)) == 0
        return
    assert bool(torch.isfinite(f).all()) and float(f.abs().max()) > 0.0
    if task == "Humanoid":
        ob = obs["obs"]
        torch.testing.assert_close(ob[:, 54:75], f * env.task_params.contact_force_scale, rtol=1e-6, atol=1e-6)
