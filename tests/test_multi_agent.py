"""Multi-agent layout (SURVEY.md §8(a) row A-MA) on the CPU oracle.

The conventions restated from the fork's MA tasks:
  * buffers are (num_envs * num_agents, ...) env-major   franka_reach_MA.py:22-38
  * an env resets only when ALL its agents are done      franka_reach_MA.py:616-626, 875-885
    (``_agent_ids_to_env_ids(use_AND_filter=True)``: bincount(agent_ids // A) >= A)
  * the reset clears progress/reset of every agent of those envs   :677-679, 887-889
  * "others" obs block: cyclic shift starting after self            :604-608
"""
import numpy as np
import pytest

import pyoracle as O
from migym import configs, model as M, taskdefs


def ma_setup(A=4, n_env=8):
    cfg = configs.task_config("MAAnt", n_env)
    cfg["env"]["numAgents"] = A
    spec = M.load_builtin("ant")
    tp = taskdefs.task_params("MAAnt", cfg, spec)
    sp = taskdefs.sim_params(cfg, 16, A)
    return cfg, spec, tp, sp


def reference_and_filter(reset_buf, A):
    """Restatement of franka_reach_MA.py:875-885 on a reset mask (agent ids -> env ids)."""
    agent_ids = np.nonzero(reset_buf)[0]
    env_ids = agent_ids // A
    counts = np.bincount(env_ids, minlength=len(reset_buf) // A)
    return np.nonzero(counts >= A)[0]


def test_obs_width_and_offsets():
    _, spec, tp, _ = ma_setup()
    assert tp.num_agents == 4 and tp.num_obs == 69
    offs = np.array([list(tp.agent_offset[k]) for k in range(4)])
    assert np.allclose(offs[:, :2], [[-1, -1], [1, -1], [-1, 1], [1, 1]])


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_and_filter_matches_reference_semantics(seed):
    A, n_env = 4, 16
    _, spec, tp, _ = ma_setup(A, n_env)
    n = A * n_env
    h = O.HostEnv(tp, spec, n)
    h.post_physics(tp, seed=3, step=0)                     # first step: everything resets
    rng = np.random.default_rng(seed)
    mask = (rng.random(n) < 0.7).astype(np.int64)
    mask[0:4] = 1                                          # env 0 fully done
    mask[4:8] = [1, 1, 1, 0]                               # env 1 not
    h.reset[:] = mask
    prog_before = h.progress.copy()
    h.post_physics(tp, seed=3, step=1)
    envs = set(reference_and_filter(mask, A).tolist())
    assert 0 in envs and 1 not in envs
    for e in range(n_env):
        agents = range(A * e, A * e + A)
        if e in envs:
            assert all(h.progress[a] == 0 for a in agents)
        else:
            assert all(h.progress[a] == prog_before[a] + 1 for a in agents)
            # done agents of a not-yet-reset env stay done (reward keeps reset_buf)
            assert all(h.reset[a] >= mask[a] for a in agents)


def test_others_block_is_cyclic_relative_positions():
    A, n_env = 4, 3
    _, spec, tp, _ = ma_setup(A, n_env)
    n = A * n_env
    h = O.HostEnv(tp, spec, n)
    h.post_physics(tp, seed=0, step=0)
    rng = np.random.default_rng(0)
    h.root[:, 0:3] += rng.normal(size=(n, 3)).astype(np.float32)
    h.reset[:] = 0
    h.post_physics(tp, seed=0, step=1)
    for e in range(n_env):
        for k in range(A):
            a = A * e + k
            block = h.obs[a, 60:69].reshape(3, 3)
            for j in range(1, A):
                b = A * e + (k + j) % A
                np.testing.assert_allclose(block[j - 1], h.root[b, 0:3] - h.root[a, 0:3], atol=1e-6)


def test_single_agent_obs_prefix_equals_ant():
    """Each agent's first 60 obs are the Ant obs of that agent (translated by its offset)."""
    A, n_env = 4, 4
    _, spec, tp, sp = ma_setup(A, n_env)
    n = A * n_env
    h = O.HostEnv(tp, spec, n)
    mnp = M.pack_model(spec)
    rng = np.random.default_rng(1)
    for t in range(3):
        h.actions[:] = rng.uniform(-1, 1, h.actions.shape)
        h.env_step(mnp, sp, tp, seed=1, step=t)
    # same physics per agent as a single Ant whose origin is shifted by the agent offset
    cfg1 = configs.task_config("Ant", n)
    tp1 = taskdefs.task_params("Ant", cfg1, spec)
    h1 = O.HostEnv(tp1, spec, n)
    h1.root[:] = h.root
    h1.dof[:] = h.dof
    offs = np.tile(np.array([list(tp.agent_offset[k]) for k in range(A)], np.float32), (n_env, 1))
    h1.root[:, 0:3] -= offs
    h1.sensors[:] = h.sensors
    h1.potentials[:] = h.prev_potentials
    h1.actions[:] = h.actions
    h1.reset[:] = 0
    h1.progress[:] = h.progress - 1
    h1.post_physics(tp1, seed=1, step=99)
    np.testing.assert_allclose(h1.obs[:, 1:60], h.obs[:, 1:60], atol=2e-4)
