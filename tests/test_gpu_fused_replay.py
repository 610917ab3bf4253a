"""The fused kernels the bench times (k_env_step, k_hand_step), pinned to the reference's own traces.

``mg_env_step_replay`` launches the same kernel instance as ``mg_env_step`` with gym.simulate
replaced by the trace's post-simulate state (what the traces' fake ``gym.simulate`` wrote,
tests/golden/make_traces.py).  Everything else in the launch is the bench path's code: the action
clamp and actuation / PD targets, the masked reset_idx with the reference's injected draws, the
team-parallel observation staging (``obs_head``, LDS staging, hand ``obs_map``), the team-summed
reward terms (``reward_from_sums``), ``compute_hand_reward`` and its running mean, timeouts, the obs
clamp and the write-back.

Bar (north_star: obs/reward parity within 1e-4): obs and rew rtol/atol 1e-4; reset, progress,
timeouts, reset_goal, successes exact; potentials bit-exact; pre-physics state (hand resets)
within 1e-5 relative, as the unfused replay in test_gpu_parity.py / test_gpu_hand.py.
"""
import ctypes as C
import os

import numpy as np
import pytest
import torch

import pyoracle as O
from migym import _abi, configs, model as M, taskdefs
from test_oracle_golden import HAND_TRACES, hand_noise, hand_trace_setup

pytestmark = pytest.mark.gpu
G = G_DIR = os.path.join(os.path.dirname(__file__), "golden")
DEV = "cuda:0"


@pytest.fixture(scope="module")
def lib():
    assert torch.cuda.is_available(), "GPU tests need the MI355X"
    return _abi.lib()


def T(a, dtype=torch.float32):
    return torch.as_tensor(np.ascontiguousarray(a)).to(DEV, dtype).contiguous()


def P(t):
    return None if t is None else t.data_ptr()


def np_(t):
    return t.cpu().numpy()


def stream():
    return torch.cuda.current_stream().cuda_stream


def load(name):
    return dict(np.load(os.path.join(G, name)))


def make_sim(lib, spec, sp, n, views):
    mnp = M.pack_model(spec)
    sim = C.c_void_p()
    _abi.check(lib.mg_sim_create(mnp.ctypes.data, C.byref(sp), n, 0, C.byref(sim)), lib)
    _abi.check(lib.mg_sim_bind(sim, C.byref(views)), lib)
    return sim


class LocoDev:
    """Device buffers of the locomotion task layer (layouts VecTask binds)."""

    def __init__(self, h):
        for k in ("root", "dof", "act_eff", "sensors", "dof_force", "actions", "actions_out", "obs", "obs_clamped",
                  "rew", "potentials", "prev_potentials", "up", "heading"):
            setattr(self, k, T(getattr(h, k)))
        self.reset = T(h.reset, torch.int64)
        self.progress = T(h.progress, torch.int64)
        self.timeout = torch.zeros(h.n, dtype=torch.bool, device=DEV)
        self.noise = None

    def views(self):
        v = _abi.StateViews()
        v.root_states, v.dof_state, v.dof_actuation = P(self.root), P(self.dof), P(self.act_eff)
        v.sensors, v.dof_force = P(self.sensors), P(self.dof_force)
        return v

    def buffers(self, seed=0, step=0):
        b = _abi.TaskBuffers()
        b.actions, b.actions_out, b.obs, b.obs_clamped = P(self.actions), P(self.actions_out), P(self.obs), \
            P(self.obs_clamped)
        b.rew, b.reset, b.progress, b.timeout = P(self.rew), P(self.reset), P(self.progress), P(self.timeout)
        b.potentials, b.prev_potentials = P(self.potentials), P(self.prev_potentials)
        b.up_vec, b.heading_vec = P(self.up), P(self.heading)
        b.noise = P(self.noise)
        b.seed, b.step_counter, b.env_offset = seed, step, 0
        return b


def loco_setup(task):
    cfg = configs.task_config(task, 16)
    spec = M.load_builtin(taskdefs.TASK_INFO[task][1])
    return spec, taskdefs.sim_params(cfg, taskdefs.TASK_INFO[task][5]), taskdefs.task_params(task, cfg, spec)


@pytest.mark.parametrize("task", ["Ant", "Humanoid"])
def test_fused_env_step_replays_reference_trace(lib, task):
    """k_env_step's own task layer (obs_head, LDS-staged DOF/sensor/action columns, team-summed reward
    terms, masked reset) replays trace_{ant,humanoid}.npz: ant.py:287-297, 325-408; humanoid.py:287-413."""
    d = load(f"trace_{task.lower()}.npz")
    spec, sp, tp = loco_setup(task)
    tp.max_episode_length = int(d["episode_length"])
    Tn, N = d["actions"].shape[:2]
    e = LocoDev(O.HostEnv(tp, spec, N))
    sim = make_sim(lib, spec, sp, N, e.views())
    try:
        for t in range(Tn):
            e.actions.copy_(T(d["actions"][t]))
            e.noise = T(d["noise"][t])
            ph = [T(d[k][t]) for k in ("phys_root", "phys_dof", "phys_sensors", "phys_dof_force")]
            rp = _abi.Replay()
            rp.root_states, rp.dof_state, rp.sensors, rp.dof_force = (P(x) for x in ph)
            _abi.check(lib.mg_env_step_replay(sim, C.byref(tp), C.byref(e.buffers()), C.byref(rp), stream()), lib)
            torch.cuda.synchronize()
            np.testing.assert_array_equal(np_(e.root), d["root_after"][t])
            np.testing.assert_allclose(np_(e.dof), d["dof_after"][t], rtol=1e-6, atol=1e-7)
            np.testing.assert_allclose(np_(e.obs_clamped), d["obs"][t], rtol=1e-4, atol=1e-4)
            np.testing.assert_allclose(np_(e.rew), d["rew"][t], rtol=1e-4, atol=1e-4)
            np.testing.assert_array_equal(np_(e.reset), d["reset"][t])
            np.testing.assert_array_equal(np_(e.progress), d["progress"][t])
            np.testing.assert_array_equal(np_(e.timeout).astype(np.int64), d["timeouts"][t])
            np.testing.assert_array_equal(np_(e.potentials), d["potentials"][t])
            np.testing.assert_array_equal(np_(e.prev_potentials), d["prev_potentials"][t])
            # pre_physics_step's actuation (ant.py:281-285): clamp(a) * gear * power_scale
            gear = np.array(tp.motor_effort[:spec.num_dofs], np.float32)
            a = np.clip(d["actions"][t], -tp.clip_actions, tp.clip_actions).astype(np.float32)
            np.testing.assert_allclose(np_(e.act_eff), a * gear * np.float32(tp.power_scale),
                                       rtol=1e-6, atol=1e-6)
    finally:
        lib.mg_sim_destroy(sim)


def test_fused_cartpole_replays_reference_trace(lib):
    d = load("trace_cartpole.npz")
    spec, sp, tp = loco_setup("Cartpole")
    Tn, N = d["actions"].shape[:2]
    e = LocoDev(O.HostEnv(tp, spec, N))
    sim = make_sim(lib, spec, sp, N, e.views())
    try:
        for t in range(Tn):
            e.actions.copy_(T(d["actions"][t]))
            e.noise = T(d["noise"][t])
            phd = T(d["phys_dof"][t])
            rp = _abi.Replay()
            rp.dof_state = P(phd)
            _abi.check(lib.mg_env_step_replay(sim, C.byref(tp), C.byref(e.buffers()), C.byref(rp), stream()), lib)
            torch.cuda.synchronize()
            np.testing.assert_allclose(np_(e.act_eff), d["actuation"][t], rtol=1e-6, atol=1e-6)
            np.testing.assert_allclose(np_(e.dof), d["dof_after"][t], rtol=1e-6, atol=1e-7)
            np.testing.assert_allclose(np_(e.obs_clamped), d["obs"][t], rtol=1e-4, atol=1e-4)
            np.testing.assert_allclose(np_(e.rew), d["rew"][t], rtol=1e-4, atol=1e-4)
            np.testing.assert_array_equal(np_(e.reset), d["reset"][t])
            np.testing.assert_array_equal(np_(e.progress), d["progress"][t])
            np.testing.assert_array_equal(np_(e.timeout).astype(np.int64), d["timeouts"][t])
    finally:
        lib.mg_sim_destroy(sim)


@pytest.mark.parametrize("A", [2, 4])
def test_fused_multi_agent_replay_matches_oracle_task_layer(lib, A):
    """MA-Ant through k_env_step's wave-ballot AND filter and shuffle-based others block, replayed on
    random post-simulate states, vs the oracle's MA task layer at the same 1e-4 bar; potentials
    bit-exact.  Step 3 takes the reset_buf of tests/golden/ma_conventions.npz and must reset exactly the
    agents the reference's reset_idx resets for it (franka_reach_MA.py:616-621, 875-889); step 4 places
    the agents at the fixture's positions and the others block must give the reference's cyclic shift
    (franka_reach_MA.py:604-608) once the agent's own position is added back."""
    G = np.load(os.path.join(G_DIR, "ma_conventions.npz"))
    cfg = configs.task_config("MAAnt", 16)
    cfg["env"]["numAgents"] = A
    spec = M.load_builtin("ant")
    sp, tp = taskdefs.sim_params(cfg, 16, A), taskdefs.task_params("MAAnt", cfg, spec)
    n = A * 64
    h = O.HostEnv(tp, spec, n)
    e = LocoDev(h)
    sim = make_sim(lib, spec, sp, n, e.views())
    rng = np.random.default_rng(5)
    nd = spec.num_dofs
    lo, hi = np.array(tp.dof_lower[:nd]), np.array(tp.dof_upper[:nd])
    try:
        for t in range(6):
            a = rng.uniform(-1.2, 1.2, (n, tp.num_actions)).astype(np.float32)
            root = h.root.copy()
            root[:, 0:3] += rng.normal(0, 0.05, (n, 3)).astype(np.float32)
            root[:, 2] = rng.uniform(0.2, 0.8, n)            # some torsos below the termination height
            q = rng.normal(0, 1, (n, 4))
            root[:, 3:7] = q / np.linalg.norm(q, axis=-1, keepdims=True)
            root[:, 7:13] = rng.normal(0, 1, (n, 6))
            dof = np.stack([lo + (hi - lo) * rng.uniform(-0.02, 1.02, (n, nd)), rng.normal(0, 2, (n, nd))], -1)
            sens = rng.normal(0, 5, h.sensors.shape).astype(np.float32)
            noise = rng.uniform(0, 1, (n, 2 * nd)).astype(np.float32)
            if t == 3:   # the fixture's mix of fully- and partially-done envs for the AND filter
                m = G[f"A{A}_mask"]
                assert len(m) == n
                h.reset[:] = m
                e.reset.copy_(T(m, torch.int64))
            if t == 4:   # no resets; the agents at the fixture's positions
                h.reset[:] = 0
                e.reset.zero_()
                root[:, 0:3] = G[f"A{A}_pos"].reshape(n, 3)
            # oracle: post-simulate state in place, then post_physics_step
            h.actions[:] = a
            h.root[:], h.dof[:], h.sensors[:] = root, dof, sens
            h.noise = noise
            h.post_physics(tp, seed=3, step=t)
            e.actions.copy_(T(a))
            e.noise = T(noise)
            ph = [T(root), T(dof), T(sens)]
            rp = _abi.Replay()
            rp.root_states, rp.dof_state, rp.sensors = (P(x) for x in ph)
            _abi.check(lib.mg_env_step_replay(sim, C.byref(tp), C.byref(e.buffers(seed=3, step=t)), C.byref(rp),
                                              stream()), lib)
            torch.cuda.synchronize()
            np.testing.assert_array_equal(np_(e.reset), h.reset)
            np.testing.assert_array_equal(np_(e.progress), h.progress)
            np.testing.assert_array_equal(np_(e.root), h.root)
            np.testing.assert_allclose(np_(e.dof), h.dof, rtol=1e-6, atol=1e-7)
            np.testing.assert_allclose(np_(e.obs), h.obs, rtol=1e-4, atol=1e-4)
            np.testing.assert_allclose(np_(e.rew), h.rew, rtol=1e-4, atol=1e-4)
            np.testing.assert_array_equal(np_(e.potentials), h.potentials)
            np.testing.assert_array_equal(np_(e.timeout).astype(np.uint8), h.timeout)
            assert np_(e.obs).shape[1] == 60 + 3 * (A - 1)
            if t == 3:
                reset_agents = np.zeros(n, bool)
                reset_agents[G[f"A{A}_agent_ids"]] = True
                np.testing.assert_array_equal(np_(e.progress) == 0, reset_agents)
            if t == 4:
                others = np_(e.obs)[:, 60:] + np.tile(np_(e.root)[:, 0:3], (1, A - 1))
                np.testing.assert_allclose(others, G[f"A{A}_others"], atol=2e-6)
    finally:
        lib.mg_sim_destroy(sim)


class HandDev:
    """Device mirror of pyoracle.HandHostEnv (the buffers VecTask binds for ShadowHand)."""

    def __init__(self, h):
        for k in ("root", "dof", "targets", "prev_targets", "sensors", "dof_force", "rbs", "actions", "actions_out",
                  "obs", "obs_clamped", "rew", "successes", "cons", "goal_states", "rb_forces"):
            setattr(self, k, T(getattr(h, k)))
        for k in ("reset", "reset_goal", "progress"):
            setattr(self, k, T(getattr(h, k), torch.int64))
        self.timeout = torch.zeros(h.n, dtype=torch.bool, device=DEV)
        self.scratch = torch.zeros(2, dtype=torch.int64, device=DEV)
        self.noise = None
        self.force_prob = None if h.force_prob is None else T(h.force_prob)
        self.states = None if h.states is None else T(h.states)

    def views(self):
        v = _abi.StateViews()
        v.root_states, v.dof_state = P(self.root), P(self.dof)
        v.sensors, v.dof_force, v.rigid_body_states = P(self.sensors), P(self.dof_force), P(self.rbs)
        v.dof_targets = P(self.targets)
        v.rb_forces, v.rb_force_space = P(self.rb_forces), _abi.MG_LOCAL_SPACE
        return v

    def buffers(self):
        b = _abi.TaskBuffers()
        b.actions, b.actions_out, b.obs, b.obs_clamped = P(self.actions), P(self.actions_out), P(self.obs), \
            P(self.obs_clamped)
        b.rew, b.reset, b.progress, b.timeout = P(self.rew), P(self.reset), P(self.progress), P(self.timeout)
        b.noise = P(self.noise)
        b.prev_targets, b.goal_states, b.reset_goal = P(self.prev_targets), P(self.goal_states), P(self.reset_goal)
        b.successes, b.consecutive_successes, b.reduce_scratch = P(self.successes), P(self.cons), P(self.scratch)
        b.states, b.random_force_prob = P(self.states), P(self.force_prob)
        return b


@pytest.mark.parametrize("trace", HAND_TRACES)
def test_fused_hand_step_replays_reference_trace(lib, trace):
    """k_hand_step's own pre_physics_step (goal / env resets with the reference's draws, PD targets,
    random forces), observation staging through obs_map (every observationType, asymmetric states),
    compute_hand_reward and the running mean: shadow_hand.py:437-471, 528-668, 670-800."""
    d = load(trace)
    spec, tp = hand_trace_setup(d)
    cfg = configs.task_config("ShadowHand", 16)
    sp = taskdefs.sim_params(cfg, 24)
    Tn, N = d["actions"].shape[:2]
    h = O.HandHostEnv(tp, spec, N)
    h.root[:] = d["init_root"]
    h.goal_states[:] = d["init_goal_states"]
    forces = "force_scale" in d
    if forces:
        h.force_prob = O.f32(d["init_force_prob"]).copy()
        h.states = np.zeros((N, tp.num_states), np.float32)
    e = HandDev(h)
    sim = make_sim(lib, spec, sp, N, e.views())
    pre_root = torch.zeros_like(e.root)
    pre_dof = torch.zeros_like(e.dof)
    nb = len(spec.bodies)
    try:
        for t in range(Tn):
            e.actions.copy_(T(d["actions"][t]))
            e.noise = T(hand_noise(d, t))
            ph = {k: T(d[k][t]) for k in ("phys_root", "phys_dof", "phys_rbs", "phys_sensors", "phys_dof_force")}
            rp = _abi.Replay()
            rp.root_states, rp.dof_state, rp.rigid_body_states = P(ph["phys_root"]), P(ph["phys_dof"]), \
                P(ph["phys_rbs"])
            rp.sensors, rp.dof_force = P(ph["phys_sensors"]), P(ph["phys_dof_force"])
            rp.pre_root_states, rp.pre_dof_state = P(pre_root), P(pre_dof)
            _abi.check(lib.mg_env_step_replay(sim, C.byref(tp), C.byref(e.buffers()), C.byref(rp), stream()), lib)
            torch.cuda.synchronize()
            # pre_physics_step: what simulate would have started from
            np.testing.assert_allclose(np_(pre_root), d["root_pre"][t], rtol=1e-5, atol=1e-6)
            np.testing.assert_allclose(np_(pre_dof), d["dof_pre"][t], rtol=1e-5, atol=1e-6)
            np.testing.assert_allclose(np_(e.targets), d["targets"][t], rtol=1e-5, atol=1e-6)
            np.testing.assert_allclose(np_(e.goal_states), d["goal_states"][t], rtol=1e-5, atol=1e-6)
            if forces:
                np.testing.assert_allclose(np_(e.rb_forces), d["rb_forces"][t], rtol=1e-5, atol=1e-6)
                np.testing.assert_allclose(np_(e.force_prob), d["force_prob"][t], rtol=1e-5)
            # post_physics_step on the injected state
            np.testing.assert_allclose(np_(e.root), d["phys_root"][t], rtol=1e-5, atol=1e-6)
            np.testing.assert_array_equal(np_(e.rbs)[:, :nb], d["phys_rbs"][t][:, :nb])
            np.testing.assert_allclose(np_(e.obs_clamped), d["obs"][t], rtol=1e-4, atol=1e-4)
            np.testing.assert_allclose(np_(e.rew), d["rew"][t], rtol=1e-4, atol=1e-4)
            np.testing.assert_array_equal(np_(e.reset), d["reset"][t])
            np.testing.assert_array_equal(np_(e.reset_goal), d["reset_goal"][t])
            np.testing.assert_array_equal(np_(e.progress), d["progress"][t])
            np.testing.assert_array_equal(np_(e.successes), d["successes"][t])
            np.testing.assert_allclose(np_(e.cons), d["cons"][t], rtol=1e-6)
            np.testing.assert_array_equal(np_(e.timeout).astype(np.int64), d["timeouts"][t])
            assert int(e.scratch.abs().sum()) == 0
            if forces:
                np.testing.assert_allclose(np.clip(np_(e.states), -tp.clip_obs, tp.clip_obs), d["states"][t],
                                           rtol=1e-4, atol=1e-4)
    finally:
        lib.mg_sim_destroy(sim)
