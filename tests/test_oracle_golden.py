"""The oracle's task layer vs the reference's own outputs (golden fixtures).

Pins oracle/oracle_task.c to tasks/ant.py:325-408, tasks/humanoid.py:323-413,
tasks/cartpole.py:131-196 and the VecTask.step ordering
(tasks/base/vec_task.py:362-410) via tests/golden/*.npz, which
tests/golden/make_golden.py / make_traces.py produced by running the reference
code.  Tolerance: the oracle computes in fp32 like the reference, so 2e-5
relative + 2e-5 absolute (transcendental ulp differences), exact for ints.
"""
import os

import numpy as np
import pytest

import pyoracle as O
from migym import _abi, model as M, taskdefs, configs

G = os.path.join(os.path.dirname(__file__), "golden")
RTOL, ATOL = 2e-5, 2e-5


def load(name):
    return dict(np.load(os.path.join(G, name)))


def tparams(task):
    cfg = configs.task_config(task, 16)
    spec = M.load_builtin(taskdefs.TASK_INFO[task][1])
    return taskdefs.task_params(task, cfg, spec), spec


def _obs_case(task, d, nsens):
    tp, spec = tparams(task)
    n = d["root"].shape[0]
    nd = tp.num_actions
    # golden limits are the reference's dof limits; they must equal the model's
    np.testing.assert_allclose(np.array(tp.dof_lower[:nd]), d["lo"], rtol=0, atol=1e-6)
    np.testing.assert_allclose(np.array(tp.dof_upper[:nd]), d["hi"], rtol=0, atol=1e-6)
    root = O.f32(d["root"])
    dof = O.f32(np.stack([d["dof_pos"], d["dof_vel"]], -1))
    dforce = O.f32(d.get("dof_force", np.zeros((n, nd))))
    sens = O.f32(d["sensors"])
    act = O.f32(d["actions"])
    pot = O.f32(d["potentials_in"]).copy()
    prev = np.zeros(n, np.float32)
    up = np.zeros((n, 3), np.float32)
    hd = np.zeros((n, 3), np.float32)
    obs = np.zeros((n, tp.num_obs), np.float32)
    O.compute_observations(tp, root, dof, dforce, sens, act, pot, prev, up, hd, obs)
    return tp, obs, pot, prev, up, hd


@pytest.mark.parametrize("task", ["Ant", "Humanoid"])
def test_locomotion_observations_match_reference(task):
    d = load(f"jit_{task.lower()}.npz")
    tp, obs, pot, prev, up, hd = _obs_case(task, d, 4 if task == "Ant" else 2)
    np.testing.assert_allclose(obs, d["obs"], rtol=RTOL, atol=ATOL)
    np.testing.assert_array_equal(pot, d["potentials"])            # fp32 order reproduced exactly
    np.testing.assert_array_equal(prev, d["prev_potentials"])
    np.testing.assert_allclose(up, d["up_vec"], rtol=RTOL, atol=ATOL)
    np.testing.assert_allclose(hd, d["heading_vec"], rtol=RTOL, atol=ATOL)


@pytest.mark.parametrize("task", ["Ant", "Humanoid"])
def test_locomotion_reward_match_reference(task):
    d = load(f"jit_{task.lower()}.npz")
    tp, _ = tparams(task)
    obs = O.f32(d["obs"])
    n = obs.shape[0]
    reset = O.i64(d["reset_buf"]).copy()
    rew = np.zeros(n, np.float32)
    O.compute_reward(tp, obs, O.f32(d["actions"]), O.f32(d["potentials"]), O.f32(d["prev_potentials"]),
                     O.i64(d["progress"]), reset, rew)
    np.testing.assert_allclose(rew, d["rew"], rtol=RTOL, atol=ATOL)
    np.testing.assert_array_equal(reset, d["reset"])


def test_cartpole_reward_match_reference():
    d = load("jit_cartpole.npz")
    tp, _ = tparams("Cartpole")
    obs = O.f32(d["obs"])
    n = obs.shape[0]
    reset = O.i64(d["reset_buf"]).copy()
    rew = np.zeros(n, np.float32)
    O.compute_reward(tp, obs, np.zeros((n, 1), np.float32), np.zeros(n, np.float32), np.zeros(n, np.float32),
                     O.i64(d["progress"]), reset, rew)
    np.testing.assert_allclose(rew, d["rew"], rtol=RTOL, atol=ATOL)
    np.testing.assert_array_equal(reset, d["reset"])


@pytest.mark.parametrize("task", ["Ant", "Humanoid"])
def test_full_step_trace_matches_reference(task):
    """Replays the reference's physics-free VecTask.step trace through the oracle's
    post-physics path with the reference's own reset-noise draws injected."""
    d = load(f"trace_{task.lower()}.npz")
    tp, spec = tparams(task)
    tp.max_episode_length = int(d["episode_length"])
    T, N = d["actions"].shape[:2]
    h = O.HostEnv(tp, spec, N)
    for t in range(T):
        h.actions[:] = d["actions"][t]
        h.root[:] = d["phys_root"][t]
        h.dof[:] = d["phys_dof"][t]
        h.sensors[:] = d["phys_sensors"][t]
        h.dof_force[:] = d["phys_dof_force"][t]
        h.noise = O.f32(d["noise"][t])
        np.testing.assert_array_equal(h.reset, d["reset_in"][t])
        np.testing.assert_array_equal(h.progress, d["progress_in"][t])
        h.post_physics(tp)
        np.testing.assert_allclose(h.root, d["root_after"][t], rtol=0, atol=0)
        np.testing.assert_allclose(h.dof, d["dof_after"][t], rtol=1e-7, atol=1e-7)
        np.testing.assert_allclose(h.obs_clamped, d["obs"][t], rtol=RTOL, atol=ATOL)
        np.testing.assert_allclose(h.rew, d["rew"][t], rtol=RTOL, atol=ATOL)
        np.testing.assert_array_equal(h.reset, d["reset"][t])
        np.testing.assert_array_equal(h.progress, d["progress"][t])
        np.testing.assert_array_equal(h.timeout, d["timeouts"][t])
        np.testing.assert_array_equal(h.potentials, d["potentials"][t])
        np.testing.assert_array_equal(h.prev_potentials, d["prev_potentials"][t])


@pytest.mark.parametrize("task", ["Ant", "Humanoid"])
def test_reset_done_trace_matches_reference(task):
    """step -> reset_done -> step: the reference's own VecTask.reset_done (vec_task.py:442-457) after every
    physics-free step (make_traces.py run_locomotion(reset_done=True)), replayed through the oracle's post-physics
    and reset_idx with the reference's draws injected: the reset state written, reset_buf / progress cleared, the
    returned observations the terminal ones, and the next step simulating from the reset state without a second
    reset."""
    d = load(f"trace_{task.lower()}_reset_done.npz")
    tp, spec = tparams(task)
    tp.max_episode_length = int(d["episode_length"])
    T, N = d["actions"].shape[:2]
    h = O.HostEnv(tp, spec, N)
    assert d["rd_mask"][1:].sum() > 0 and d["timeouts"].sum() > 0   # the trace exercises both kinds of done
    for t in range(T):
        h.actions[:] = d["actions"][t]
        h.root[:] = d["phys_root"][t]
        h.dof[:] = d["phys_dof"][t]
        h.sensors[:] = d["phys_sensors"][t]
        h.dof_force[:] = d["phys_dof_force"][t]
        h.noise = O.f32(d["noise"][t])
        np.testing.assert_array_equal(h.reset, d["reset_in"][t])
        h.post_physics(tp)
        np.testing.assert_allclose(h.obs_clamped, d["obs"][t], rtol=RTOL, atol=ATOL)
        np.testing.assert_allclose(h.rew, d["rew"][t], rtol=RTOL, atol=ATOL)
        np.testing.assert_array_equal(h.reset, d["reset"][t])
        # reset_done: reset_idx(reset_buf.nonzero())
        ids = np.nonzero(h.reset)[0]
        np.testing.assert_array_equal(ids, np.nonzero(d["rd_mask"][t])[0])
        h.noise = O.f32(d["rd_noise"][t])
        h.reset_idx(tp, ids)
        np.testing.assert_array_equal(h.root, d["rd_root"][t])
        np.testing.assert_allclose(h.dof, d["rd_dof"][t], rtol=1e-7, atol=1e-7)
        np.testing.assert_array_equal(h.reset, d["rd_reset"][t])
        np.testing.assert_array_equal(h.progress, d["rd_progress"][t])
        np.testing.assert_array_equal(h.potentials, d["rd_potentials"][t])
        np.testing.assert_array_equal(h.prev_potentials, d["rd_prev_potentials"][t])
        np.testing.assert_allclose(h.obs_clamped, d["rd_obs"][t], rtol=RTOL, atol=ATOL)   # terminal obs, unchanged


def test_cartpole_trace_matches_reference():
    d = load("trace_cartpole.npz")
    tp, spec = tparams("Cartpole")
    T, N = d["actions"].shape[:2]
    h = O.HostEnv(tp, spec, N)
    for t in range(T):
        h.actions[:] = d["actions"][t]
        h.dof[:] = d["phys_dof"][t]
        h.noise = O.f32(d["noise"][t])
        h.post_physics(tp)
        np.testing.assert_allclose(h.dof, d["dof_after"][t], rtol=1e-7, atol=1e-7)
        np.testing.assert_allclose(h.obs_clamped, d["obs"][t], rtol=RTOL, atol=ATOL)
        np.testing.assert_allclose(h.rew, d["rew"][t], rtol=RTOL, atol=ATOL)
        np.testing.assert_array_equal(h.reset, d["reset"][t])
        np.testing.assert_array_equal(h.progress, d["progress"][t])
        np.testing.assert_array_equal(h.timeout, d["timeouts"][t])
        # actuation written by pre_physics_step: 400 * clamp(a) on DOF 0 only (cartpole.py:159-163)
        a = np.clip(d["actions"][t][:, 0], -1, 1) * 400.0
        np.testing.assert_allclose(d["actuation"][t][:, 0], a, rtol=1e-6)
        assert np.all(d["actuation"][t][:, 1] == 0)


def test_shadowhand_reward_and_rotation_match_reference():
    """compute_hand_reward incl. the global running mean, randomize_rotation (shadow_hand.py:746-806)."""
    d = load("jit_shadowhand.npz")
    tp, _ = tparams("ShadowHand")
    np.testing.assert_allclose(O.randomize_rotation(d["r0"], d["r1"]), d["rand_rot"], rtol=RTOL, atol=ATOL)
    reset, rg = O.i64(d["reset_buf"]).copy(), O.i64(d["reset_goal_buf"]).copy()
    prog, succ = O.i64(d["progress"]).copy(), O.f32(d["successes"]).copy()
    rew, cons = O.hand_reward(tp, 600.0, d["object_pos"], d["object_rot"], d["target_pos"], d["target_rot"],
                              d["actions"], reset, rg, prog, succ, float(d["cons_in"]))
    np.testing.assert_allclose(rew, d["rew"], rtol=RTOL, atol=ATOL)
    np.testing.assert_array_equal(reset, d["reset"])
    np.testing.assert_array_equal(rg, d["goal_reset"])
    np.testing.assert_array_equal(prog, d["progress_out"])
    np.testing.assert_array_equal(succ, d["successes_out"])
    np.testing.assert_allclose(cons, d["cons_out"], rtol=1e-6)


def hand_noise(d, t):
    """Injected noise row of step t, padded to the 66 columns of the current layout (the traces made
    before the random-force columns existed hold the first 61)."""
    x = O.f32(d["noise"][t])
    return np.ascontiguousarray(np.pad(x, ((0, 0), (0, _abi.HAND_NOISE_COLS - x.shape[1]))))


def hand_trace_setup(d, n=16):
    """Task params of a ShadowHand trace: observation type, episode length, and for the forces trace
    forceScale / forceProbRange / asymmetric states with the fake gym's object mass."""
    cfg = configs.task_config("ShadowHand", n)
    cfg["env"]["observationType"] = str(d["obs_type"])
    if "force_scale" in d and float(d["force_scale"]) > 0:
        cfg["env"]["forceScale"] = float(d["force_scale"])
        cfg["env"]["forceProbRange"] = [0.2, 0.8]
        cfg["env"]["asymmetric_observations"] = d["states"].shape[-1] > 0
    if "object_type" in d:   # objectType pen: pen start pose, randomize_rotation_pen, ignore_z_rot
        cfg["env"]["objectType"] = str(d["object_type"])
    spec = taskdefs.hand_spec(cfg["env"].get("objectType", "block"))
    tp = taskdefs.task_params("ShadowHand", cfg, spec)
    tp.max_episode_length = int(d["episode_length"])
    if "object_mass" in d:
        tp.object_rb_mass = float(d["object_mass"])
    return spec, tp


HAND_TRACES = ["trace_shadowhand.npz", "trace_shadowhand_full.npz", "trace_shadowhand_full_no_vel.npz",
               "trace_shadowhand_openai.npz", "trace_shadowhand_forces.npz", "trace_shadowhand_pen.npz"]


@pytest.mark.parametrize("trace", HAND_TRACES)
def test_shadowhand_trace_matches_reference(trace):
    """Whole physics-free ShadowHand VecTask.step (pre_physics resets + PD targets, observations of
    every observationType, reward, running mean, timeouts) replayed with the reference's own reset
    draws injected.  The forces trace adds random object forces (forceScale 2, rb_forces after the
    decay / redraw, the per-env probability redrawn on reset) and the asymmetric states buffer."""
    d = load(trace)
    spec, tp = hand_trace_setup(d)
    mnp = M.pack_model(spec)
    T, N = d["actions"].shape[:2]
    h = O.HandHostEnv(tp, spec, N)
    h.root[:] = d["init_root"]
    h.goal_states[:] = d["init_goal_states"]
    forces = "force_scale" in d
    if forces:
        h.force_prob = O.f32(d["init_force_prob"]).copy()
        h.states = np.zeros((N, tp.num_states), np.float32)
    for t in range(T):
        h.actions[:] = d["actions"][t]
        h.noise = hand_noise(d, t)
        np.testing.assert_array_equal(h.reset, d["reset_in"][t])
        np.testing.assert_array_equal(h.reset_goal, d["reset_goal_in"][t])
        np.testing.assert_array_equal(h.progress, d["progress_in"][t])
        h.pre_physics(mnp, tp)
        np.testing.assert_allclose(h.root, d["root_pre"][t], rtol=1e-6, atol=1e-7)
        np.testing.assert_allclose(h.dof, d["dof_pre"][t], rtol=1e-6, atol=1e-7)
        np.testing.assert_allclose(h.targets, d["targets"][t], rtol=1e-6, atol=1e-7)
        np.testing.assert_allclose(h.prev_targets, d["prev_targets"][t], rtol=1e-6, atol=1e-7)
        np.testing.assert_allclose(h.goal_states, d["goal_states"][t], rtol=1e-6, atol=1e-7)
        if forces:
            np.testing.assert_allclose(h.rb_forces, d["rb_forces"][t], rtol=1e-6, atol=1e-7)
            np.testing.assert_allclose(h.force_prob, d["force_prob"][t], rtol=1e-6)
        # "physics": the trace's injected post-simulate state
        h.root[:] = d["phys_root"][t]
        h.dof[:] = d["phys_dof"][t]
        h.rbs[:] = d["phys_rbs"][t]
        h.sensors[:] = d["phys_sensors"][t]
        h.dof_force[:] = d["phys_dof_force"][t]
        h.post_physics(mnp, tp)
        np.testing.assert_allclose(h.obs_clamped, d["obs"][t], rtol=RTOL, atol=ATOL)
        np.testing.assert_allclose(h.rew, d["rew"][t], rtol=RTOL, atol=ATOL)
        np.testing.assert_array_equal(h.reset, d["reset"][t])
        np.testing.assert_array_equal(h.reset_goal, d["reset_goal"][t])
        np.testing.assert_array_equal(h.progress, d["progress"][t])
        np.testing.assert_array_equal(h.successes, d["successes"][t])
        np.testing.assert_allclose(h.cons, d["cons"][t], rtol=1e-6)
        np.testing.assert_array_equal(h.timeout, d["timeouts"][t])
        if forces:  # get_state() = clamp(states_buf, +-clipObservations)
            np.testing.assert_allclose(np.clip(h.states, -tp.clip_obs, tp.clip_obs), d["states"][t], rtol=RTOL,
                                       atol=ATOL)
