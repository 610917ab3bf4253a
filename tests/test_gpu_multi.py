"""GPU side of the multi-GPU output path and of controlFrequencyInv.

  * out_pack: the fused kernels write each row [clamped obs | rew | reset] of the gather's message
    exactly equal to the buffers they write for the single-GPU caller (Ant, MA-Ant, ShadowHand);
  * defer_finalize + mg_hand_finalize: the deferred running mean equals the in-step one bit for bit;
  * controlFrequencyInv = 2: one launch runs simulate twice between one pre- and one post_physics_step,
    held to the oracle running orc_simulate twice (vec_task.py:381-384), over 3 control steps.
"""
import ctypes as C

import numpy as np
import pytest
import torch

import migym
import pyoracle as O
from migym import _abi, configs, model as M, taskdefs

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


@pytest.fixture(scope="module")
def lib():
    assert torch.cuda.is_available(), "GPU tests need the MI355X"
    return _abi.lib()


class _Pack:
    """Single-rank stand-in for PackedGather: one slot, no collective."""

    def __init__(self, rows, nobs):
        self.rows, self.nobs = rows, nobs
        self.buf = torch.full((rows, nobs + 2), float("nan"), device=DEV)

    def next_pack(self):
        return self.buf

    def issue(self):
        pass


@pytest.mark.parametrize("task", ["Ant", "MAAnt", "ShadowHand", "Cartpole"])
def test_out_pack_rows_equal_step_outputs(task):
    env = migym.make(seed=0, task=task, num_envs=256, sim_device=DEV, rl_device=DEV, headless=True)
    pk = _Pack(env.num_actors, env.num_obs)
    env.attach_output_gather(pk)
    g = torch.Generator(device=DEV).manual_seed(0)
    for _ in range(4):
        a = torch.rand((env.num_actors, env.num_actions), device=DEV, generator=g) * 2.4 - 1.2
        obs, rew, reset, _ = env.step(a)
        torch.cuda.synchronize()
        b = pk.buf
        assert torch.equal(b[:, : env.num_obs], obs["obs"])
        assert torch.equal(b[:, env.num_obs], rew)
        assert torch.equal(b[:, env.num_obs + 1], reset.float())
    env.close()


def test_deferred_running_mean_equals_in_step(lib):
    """Two identical ShadowHand envs; one defers the running mean (multi-GPU path) and finalizes after the
    step: consecutive_successes is bit-identical every step."""
    envs = []
    for defer in (0, 1):
        cfg = configs.task_config("ShadowHand", 512, sim_device=DEV)
        cfg["env"]["episodeLength"] = 4
        e = migym.make(seed=0, task="ShadowHand", num_envs=512, sim_device=DEV, rl_device=DEV, headless=True,
                       cfg={"task": cfg})
        e._tb.defer_finalize = defer
        envs.append(e)
    g = torch.Generator(device=DEV).manual_seed(1)
    for _ in range(10):
        a = torch.rand((512, 20), device=DEV, generator=g) * 2 - 1
        envs[0].step(a)
        envs[1].step(a)
        _abi.check(lib.mg_hand_finalize(C.byref(envs[1].task_params), C.byref(envs[1]._tb),
                                        torch.cuda.current_stream().cuda_stream), lib)
        torch.cuda.synchronize()
        assert torch.equal(envs[0].consecutive_successes, envs[1].consecutive_successes)
        assert int(envs[1]._reduce.abs().sum()) == 0
    assert float(envs[0].consecutive_successes) != 0.0
    for e in envs:
        e.close()


@pytest.mark.parametrize("task,n", [("Ant", 256), ("Humanoid", 128)])
def test_control_freq_inv_runs_simulate_twice(lib, task, n):
    cfg = configs.task_config(task, 16)
    cfg["env"]["controlFrequencyInv"] = 2
    spec = M.load_builtin(taskdefs.TASK_INFO[task][1])
    sp = taskdefs.sim_params(cfg, taskdefs.TASK_INFO[task][5])
    tp = taskdefs.task_params(task, cfg, spec)
    assert tp.control_freq_inv == 2
    h = O.HostEnv(tp, spec, n)
    T = lambda x, dt=torch.float32: torch.as_tensor(np.ascontiguousarray(x)).to(DEV, dt)  # noqa: E731
    dev = {k: T(getattr(h, k)) for k in ("root", "dof", "act_eff", "sensors", "dof_force", "actions",
                                          "actions_out", "obs", "obs_clamped", "rew", "potentials",
                                          "prev_potentials", "up", "heading")}
    reset, prog = T(h.reset, torch.int64), T(h.progress, torch.int64)
    timeout = torch.zeros(n, dtype=torch.bool, device=DEV)
    v = _abi.StateViews()
    v.root_states, v.dof_state, v.dof_actuation = (dev[k].data_ptr() for k in ("root", "dof", "act_eff"))
    v.sensors, v.dof_force = dev["sensors"].data_ptr(), dev["dof_force"].data_ptr()
    mnp = M.pack_model(spec)
    sim = C.c_void_p()
    _abi.check(lib.mg_sim_create(mnp.ctypes.data, C.byref(sp), n, 0, C.byref(sim)), lib)
    _abi.check(lib.mg_sim_bind(sim, C.byref(v)), lib)
    rng = np.random.default_rng(4)
    try:
        for t in range(3):
            a = rng.uniform(-1, 1, (n, tp.num_actions)).astype(np.float32)
            h.actions[:] = a
            dev["actions"].copy_(T(a))
            h.env_step(mnp, sp, tp, seed=2, step=t, threads=8)
            b = _abi.TaskBuffers()
            b.actions, b.actions_out = dev["actions"].data_ptr(), dev["actions_out"].data_ptr()
            b.obs, b.obs_clamped, b.rew = dev["obs"].data_ptr(), dev["obs_clamped"].data_ptr(), dev["rew"].data_ptr()
            b.reset, b.progress, b.timeout = reset.data_ptr(), prog.data_ptr(), timeout.data_ptr()
            b.potentials, b.prev_potentials = dev["potentials"].data_ptr(), dev["prev_potentials"].data_ptr()
            b.up_vec, b.heading_vec = dev["up"].data_ptr(), dev["heading"].data_ptr()
            b.seed, b.step_counter = 2, t
            _abi.check(lib.mg_env_step(sim, C.byref(tp), C.byref(b), torch.cuda.current_stream().cuda_stream), lib)
        torch.cuda.synchronize()
    finally:
        lib.mg_sim_destroy(sim)
    np.testing.assert_array_equal(reset.cpu().numpy(), h.reset)
    np.testing.assert_array_equal(prog.cpu().numpy(), h.progress)
    og = dev["obs"].cpu().numpy()
    bad = np.abs(og - h.obs) > (2e-2 + 2e-2 * np.abs(h.obs))
    assert bad.mean() < 1e-3, (bad.sum(), np.argwhere(bad)[:10])


@pytest.mark.parametrize("task", ["Ant", "MAAnt", "ShadowHand", "ShadowHand-asym"])
def test_non_finite_state_flags_reset(task):
    """NaN guard: a NaN injected into one env's state gives that env reset = 1 (all its
    agents under MA), reward 0 and a zero observation row (and, with asymmetric_observations, a zero
    states row); the next step's reset restores a finite state; the other envs are untouched."""
    n = 64
    asym = task.endswith("-asym")
    task = task.split("-")[0]
    cfg = configs.task_config(task, n, sim_device=DEV)
    if asym:
        cfg["env"]["asymmetric_observations"] = True
    env = migym.make(seed=0, task=task, num_envs=n, sim_device=DEV, rl_device=DEV, headless=True, cfg={"task": cfg})
    assert env.num_states == (211 if asym else 0)
    A = env.num_agents
    g = torch.Generator(device=DEV).manual_seed(0)
    act = lambda: torch.rand((env.num_actors, env.num_actions), device=DEV, generator=g) * 2 - 1  # noqa: E731
    for _ in range(3):
        env.step(act())
    e = 5
    if task == "ShadowHand":
        env.root_state_tensor[3 * e + 1, 3] = float("nan")     # the object's orientation
    else:
        env.root_states[e * A + (A - 1), 2] = float("nan")     # the last agent's torso height
    obs, rew, reset, _ = env.step(act())
    torch.cuda.synchronize()
    rows = torch.arange(e * A, (e + 1) * A, device=DEV)
    assert bool((reset[rows] == 1).all())
    assert bool((obs["obs"][rows] == 0).all()) and bool((rew[rows] == 0).all())
    others = torch.ones(env.num_actors, dtype=torch.bool, device=DEV)
    others[rows] = False
    assert bool(torch.isfinite(obs["obs"][others]).all())
    if asym:
        assert bool((obs["states"][e] == 0).all())
        keep = torch.ones(n, dtype=torch.bool, device=DEV)
        keep[e] = False
        assert bool(torch.isfinite(obs["states"][keep]).all()) and bool((obs["states"][keep] != 0).any())
    for _ in range(2):   # ShadowHand resets in pre_physics (1 step), the locomotion tasks in post_physics
        obs, rew, reset, _ = env.step(act())
    torch.cuda.synchronize()
    state = env.root_state_tensor if task == "ShadowHand" else env.root_states
    assert bool(torch.isfinite(state).all()) and bool(torch.isfinite(obs["obs"]).all())
    env.close()


def test_egg_rollout_stays_finite_after_other_kernels():
    """The egg narrowphase (GJK / MPR, convex.hpp) over a rollout that starts after other tasks' kernels
    have run on the device: every object state stays finite (the round-1 NaN came from cvx_tri's 0 / 0 on
    coincident vertices, guarded now)."""
    ant = migym.make(seed=0, task="Ant", num_envs=4096, sim_device=DEV, rl_device=DEV, headless=True)
    for _ in range(5):
        ant.step(torch.rand((4096, 8), device=DEV) * 2 - 1)
    ant.close()
    cfg = configs.task_config("ShadowHand", 4096, sim_device=DEV)
    cfg["env"]["objectType"] = "egg"
    env = migym.make(seed=0, task="ShadowHand", num_envs=4096, sim_device=DEV, rl_device=DEV, headless=True,
                     cfg={"task": cfg})
    g = torch.Generator(device=DEV).manual_seed(3)
    for _ in range(40):
        env.step(torch.rand((4096, 20), device=DEV, generator=g) * 2 - 1)
        torch.cuda.synchronize()
        assert bool(torch.isfinite(env.root_state_tensor).all()), "non-finite object state"
    env.close()
