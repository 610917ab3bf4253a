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
    # reset_done (the reference's base reset_done would call the two-argument reset_idx with one
    # argument and raise): the done envs reset now, each with its goal, the others untouched
    done = torch.tensor([2, 9], device=DEV)
    env.reset_buf.zero_()
    env.reset_buf[done] = 1
    env.progress_buf[done] = 5
    root_before = env.root_state_tensor.view(n, 3, 13).clone()
    obs_before = env.obs_buf.clone()
    obs, ids = env.reset_done()
    torch.cuda.synchronize()
    assert torch.equal(ids, done)
    assert (env.reset_buf == 0).all() and (env.progress_buf[done] == 0).all()
    torch.testing.assert_close(env.cur_targets[done], dof[done, :, 0], rtol=0, atol=0)
    keep = torch.ones(n, dtype=torch.bool, device=DEV)
    keep[done] = False
    assert torch.equal(root[keep], root_before[keep]) and not torch.equal(root[done], root_before[done])
    torch.testing.assert_close(obs["obs"], torch.clamp(obs_before, -env.clip_obs, env.clip_obs), rtol=0, atol=0)
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


@pytest.mark.parametrize("task", ["Ant", "Humanoid"])
def test_reset_done_replays_reference_trace(task):
    """step -> VecTask.reset_done() -> step against the reference's own reset_done (vec_task.py:442-457), traced
    on the fake gym after every step (tests/golden/make_traces.py, reset_done=True).  The steps run the device
    task layer over the trace's physics outputs (mg_post_physics on the env's own buffers); reset_done is the
    build's VecTask method, with the reference's draws injected.  Asserted: the reset rows (root exact, DOF to
    1e-7), reset_buf / progress / potentials exact, reset_done's returned obs = the terminal obs, and the next
    step's obs / rew / resets / progress (so the reset envs are not reset a second time)."""
    import ctypes as C
    from migym import _abi
    d = dict(np.load(os.path.join(os.path.dirname(__file__), "golden", f"trace_{task.lower()}_reset_done.npz")))
    Tn, N = d["actions"].shape[:2]
    env = make(task, N)
    lib, tp = env._lib, env.task_params
    tp.max_episode_length = int(d["episode_length"])
    nd = env.num_dof
    T = lambda a, dt=torch.float32: torch.as_tensor(np.ascontiguousarray(a)).to(DEV, dt)  # noqa: E731
    stream = torch.cuda.current_stream().cuda_stream
    for t in range(Tn):
        act = T(d["actions"][t]).contiguous()
        env.root_states.copy_(T(d["phys_root"][t]))
        env.dof_state.copy_(T(d["phys_dof"][t]).view(N * nd, 2))
        env.sensor_tensor.copy_(T(d["phys_sensors"][t]).view(env.sensor_tensor.shape))
        env.dof_force_tensor.copy_(T(d["phys_dof_force"][t]))
        noise = T(d["noise"][t]).contiguous()
        tb = env._tb
        tb.actions, tb.noise, tb.step_counter = act.data_ptr(), noise.data_ptr(), t
        assert torch.equal(env.reset_buf.cpu(), torch.as_tensor(d["reset_in"][t]))
        _abi.check(lib.mg_post_physics(None, C.byref(tp), C.byref(env._views), C.byref(tb), N, stream), lib)
        torch.cuda.synchronize()
        np.testing.assert_allclose(env.obs_buf.cpu().numpy(), d["obs"][t], rtol=1e-4, atol=1e-4)
        np.testing.assert_allclose(env.rew_buf.cpu().numpy(), d["rew"][t], rtol=1e-4, atol=1e-4)
        np.testing.assert_array_equal(env.reset_buf.cpu().numpy(), d["reset"][t])
        np.testing.assert_array_equal(env.progress_buf.cpu().numpy(), d["progress"][t])
        # VecTask.reset_done with the reference's reset_idx draws
        env.set_reset_noise(T(d["rd_noise"][t]))
        obs, done = env.reset_done()
        env.set_reset_noise(None)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(done.cpu().numpy(), np.nonzero(d["rd_mask"][t])[0])
        np.testing.assert_array_equal(env.root_states.cpu().numpy(), d["rd_root"][t])
        np.testing.assert_allclose(env.dof_state.view(N, nd, 2).cpu().numpy(), d["rd_dof"][t], rtol=1e-7, atol=1e-7)
        np.testing.assert_array_equal(env.reset_buf.cpu().numpy(), d["rd_reset"][t])
        np.testing.assert_array_equal(env.progress_buf.cpu().numpy(), d["rd_progress"][t])
        np.testing.assert_array_equal(env.potentials.cpu().numpy(), d["rd_potentials"][t])
        np.testing.assert_array_equal(env.prev_potentials.cpu().numpy(), d["rd_prev_potentials"][t])
        np.testing.assert_allclose(obs["obs"].cpu().numpy(), d["rd_obs"][t], rtol=1e-4, atol=1e-4)
    assert d["rd_mask"][1:].sum() > 0
    env.close()


@pytest.mark.parametrize("task,n", [("Ant", 256), ("MAAnt", 64)])
def test_reset_done_with_physics_matches_oracle(task, n):
    """reset_done between fused physics steps, device RNG: the done envs (for MAAnt: the envs whose agents are
    all done, the AND filter) hold the oracle's reset state bit for bit (orc_reset_idx on the same counter-RNG
    stream), the others keep their state; the following fused step starts the reset envs from that state, so
    their observations match the oracle's step from the same state."""
    import pyoracle as O
    from migym import model as M
    env = make(task, n)
    A = env.num_agents
    rows = n * A
    for k in range(2):
        env.step(actions(env, k))
    torch.cuda.synchronize()
    g = np.random.default_rng(4)
    mask = (g.random(rows) < 0.5).astype(np.int64)
    if A > 1:
        mask[0:A] = 1        # env 0 fully done; env 1 partly
        mask[A:2 * A] = [1] * (A - 1) + [0]
    env.reset_buf.copy_(torch.as_tensor(mask, device=DEV))
    keep_root = env.root_states.clone()
    h = O.HostEnv(env.task_params, env.model_spec, rows)
    h.root[:] = env.root_states.cpu().numpy()
    h.dof[:] = env.dof_state.view(rows, env.num_dof, 2).cpu().numpy()
    h.reset[:] = mask
    h.progress[:] = env.progress_buf.cpu().numpy()
    h.potentials[:] = env.potentials.cpu().numpy()
    h.prev_potentials[:] = env.prev_potentials.cpu().numpy()
    obs_before = env.obs_buf.clone()
    step = env.control_steps
    obs, done = env.reset_done()
    torch.cuda.synchronize()
    assert torch.equal(done.cpu(), torch.as_tensor(np.nonzero(mask)[0]))
    assert torch.equal(obs["obs"], obs_before)    # not recomputed (vec_task.py:451)
    full = (np.bincount(np.nonzero(mask)[0] // A, minlength=n) >= A) if A > 1 else mask.astype(bool)
    reset_rows = np.repeat(full, A) if A > 1 else full
    ids = np.where(reset_rows, np.arange(rows), -1)
    h.reset_idx(env.task_params, ids, seed=env.seed, step=step)
    np.testing.assert_array_equal(env.root_states.cpu().numpy(), h.root)
    np.testing.assert_array_equal(env.dof_state.view(rows, env.num_dof, 2).cpu().numpy(), h.dof)
    np.testing.assert_array_equal(env.reset_buf.cpu().numpy(), h.reset)
    np.testing.assert_array_equal(env.progress_buf.cpu().numpy(), h.progress)
    np.testing.assert_array_equal(env.potentials.cpu().numpy(), h.potentials)
    assert torch.equal(env.root_states[torch.as_tensor(~reset_rows, device=DEV)],
                       keep_root[torch.as_tensor(~reset_rows, device=DEV)])
    assert reset_rows.any() and (~reset_rows).any()
    if A > 1:
        assert reset_rows[0:A].all() and not reset_rows[A:2 * A].any()
    # the next fused step from the reset state: the reset envs' observations against the oracle's step
    a = actions(env, 5)
    env.step(a)
    torch.cuda.synchronize()
    h.actions[:] = a.cpu().numpy()
    h.env_step(M.pack_model(env.model_spec), env.sim_params, env.task_params, seed=env.seed, step=step, threads=8)
    np.testing.assert_array_equal(env.progress_buf.cpu().numpy(), h.progress)
    og = env.obs_buf.cpu().numpy()[reset_rows]
    oh = h.obs[reset_rows]
    assert (np.abs(og - oh) <= 2e-3 + 2e-3 * np.abs(oh)).mean() > 0.99
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
    # a device-side edit between calls (through env.unwrapped) is not reverted by the untouched host mirror
    c.unwrapped.reset_buf[5:8] = 1
    g.reset_buf[5:8] = 1
    og, _, dg, _ = g.step(actions(g, 10))
    oc, _, dc, _ = c.step(actions(g, 10).cpu())
    assert torch.equal(oc["obs"], og["obs"]) and torch.equal(dc, dg)
    assert torch.equal(c.progress_buf, g.progress_buf.cpu()) and bool((c.progress_buf[5:8] <= 1).all())
    # get_env_state: host tensors, with a host edit made just before it included
    c.progress_buf[0] = 123
    st = c.get_env_state()
    assert all(v.device.type == "cpu" for v in st.values() if torch.is_tensor(v))
    assert int(st["progress_buf"][0]) == 123 and int(c.unwrapped.progress_buf[0]) == 123
    # that push refreshed the snapshot: a device-side write made afterwards is not overwritten by the
    # same host bytes at the next synced call
    i = int(torch.nonzero(c.unwrapped.reset_buf == 0)[0, 0])
    c.unwrapped.progress_buf[i] = 7
    c.step(actions(g, 11).cpu())
    assert int(c.progress_buf[i]) == 8 and int(c.unwrapped.progress_buf[i]) == 8
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


@pytest.mark.parametrize("task,bodies", [("Ant", 9), ("MAAnt", 9), ("ShadowHand", 27)])
def test_net_contact_force_tensor_through_the_step(task, bodies):
    """acquire_net_contact_force_tensor / refresh_net_contact_force_tensor (franka_reach_MA.py:506, 563): the (N*A*nB, 3)
    tensor is bound into the sim and written by every fused step; before it is acquired nothing computes it.  The
    Ant's feet carry the weight (the net vertical contact force over all bodies of a resting env is about m g, gravity
    along -z), the hand's object row (body 25) is pushed up by the palm, the goal row (26) stays zero."""
    env = make(task, 64)
    t = env.acquire_net_contact_force_tensor()
    assert t.shape == (env.num_actors * bodies, 3) and t is env.acquire_net_contact_force_tensor()
    for k in range(30):
        env.step(actions(env, k) * 0.0)
        env.refresh_net_contact_force_tensor()
    torch.cuda.synchronize()
    f = t.view(env.num_actors, bodies, 3)
    assert bool(torch.isfinite(f).all()) and float(f.abs().max()) > 0.0
    if task == "ShadowHand":
        assert float(f[:, 26].abs().max()) == 0.0           # the kinematic goal never collides
        assert float(f[:, 25, 2].max()) > 0.0                # the object rests on the palm in some envs
    else:
        fz = f[..., 2].sum(dim=1)                           # every body's vertical contact force, per actor
        mg = float(env.model_spec.total_mass()) * 9.81 if hasattr(env.model_spec, "total_mass") else None
        assert float(fz.median()) > 0.0                      # the ground pushes up
        if mg is not None:
            assert abs(float(fz.median()) - mg) < 0.5 * mg
    env.close()
