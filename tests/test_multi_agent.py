"""Multi-agent layout (SURVEY.md §8(a) row A-MA) on the CPU oracle, pinned to the reference's own code.

The conventions of the fork's MA tasks:
  * buffers are (num_envs * num_agents, ...) env-major   franka_reach_MA.py:22-38
  * an env resets only when ALL its agents are done      franka_reach_MA.py:616-626, 875-885
    (``_agent_ids_to_env_ids(use_AND_filter=True)``: bincount(agent_ids // A) >= A)
  * the reset clears progress/reset of every agent of those envs   :677-679, 887-889
  * "others" obs block: cyclic shift starting after self            :604-608

``tests/golden/ma_conventions.npz`` holds what the reference's ``_agent_ids_to_env_ids`` /
``_env_ids_to_agent_ids`` / ``compute_observations`` return on seeded masks, id lists and positions
(tests/golden/make_ma_golden.py calls the reference methods unmodified); the oracle is checked against it.
MAAnt's "others" block holds the other agents' root positions relative to the agent (a translation of
the reference's absolute end-effector positions, same cyclic order).
"""
import os

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


G = np.load(os.path.join(os.path.dirname(__file__), "golden", "ma_conventions.npz"))


def test_fixture_conventions_are_self_consistent():
    """The fixture's env / agent ids (what the reference returned) obey the stated rule."""
    for A in (2, 4):
        mask = G[f"A{A}_mask"]
        counts = np.bincount(np.nonzero(mask)[0] // A, minlength=len(mask) // A)
        np.testing.assert_array_equal(G[f"A{A}_env_ids_and"], np.nonzero(counts >= A)[0])
        np.testing.assert_array_equal(G[f"A{A}_env_ids_or"], np.unique(np.nonzero(mask)[0] // A))
        np.testing.assert_array_equal(G[f"A{A}_agent_ids"],
                                      (G[f"A{A}_env_ids_and"][:, None] * A + np.arange(A)).ravel())
        assert 0 in G[f"A{A}_env_ids_and"] and 1 not in G[f"A{A}_env_ids_and"]


def test_obs_width_and_offsets():
    _, spec, tp, _ = ma_setup()
    assert tp.num_agents == 4 and tp.num_obs == 69
    offs = np.array([list(tp.agent_offset[k]) for k in range(4)])
    assert np.allclose(offs[:, :2], [[-1, -1], [1, -1], [-1, 1], [1, 1]])


@pytest.mark.parametrize("A", [2, 4])
def test_and_filter_matches_reference(A):
    """The oracle's post_physics resets exactly the agents the reference's reset_idx resets for the same
    reset_buf (the fixture's ``_env_ids_to_agent_ids(_agent_ids_to_env_ids(nonzero(mask)))``)."""
    mask = G[f"A{A}_mask"]
    n = len(mask)
    _, spec, tp, _ = ma_setup(A, n // A)
    h = O.HostEnv(tp, spec, n)
    h.post_physics(tp, seed=3, step=0)                     # first step: everything resets
    h.reset[:] = mask
    prog_before = h.progress.copy()
    h.post_physics(tp, seed=3, step=1)
    reset_agents = np.zeros(n, bool)
    reset_agents[G[f"A{A}_agent_ids"]] = True
    np.testing.assert_array_equal(h.progress == 0, reset_agents)
    np.testing.assert_array_equal(h.progress[~reset_agents], prog_before[~reset_agents] + 1)
    # done agents of a not-yet-reset env stay done (reward keeps reset_buf)
    assert (h.reset[~reset_agents] >= mask[~reset_agents]).all()


@pytest.mark.parametrize("A", [2, 4])
def test_others_block_matches_reference_shift(A):
    """Others block + own position = the reference's cyclic shift of the agents' positions
    (compute_observations on the same positions, from the fixture)."""
    pos = G[f"A{A}_pos"]
    n_env = pos.shape[0]
    n = A * n_env
    _, spec, tp, _ = ma_setup(A, n_env)
    h = O.HostEnv(tp, spec, n)
    h.post_physics(tp, seed=0, step=0)
    h.root[:, 0:3] = pos.reshape(n, 3)
    h.reset[:] = 0
    h.post_physics(tp, seed=0, step=1)
    w = 60 + 3 * (A - 1)
    assert h.obs.shape[1] == w
    others = h.obs[:, 60:w] + np.tile(h.root[:, 0:3], (1, A - 1))
    np.testing.assert_allclose(others, G[f"A{A}_others"], atol=2e-6)


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
