#!/usr/bin/env python3
"""Multi-agent conventions from the reference's own code (SURVEY.md §8(a) A-MA, §8(c)).

Run in the build container only (needs /root/reference):

    python tests/golden/make_ma_golden.py

The fork's multi-agent layer lives in ``FrankaReachMA`` (isaacgymenvs/tasks/franka_reach_MA.py).  Its
conventions are plain torch methods, so they are called here unmodified, bound to a minimal stand-in
``self`` (only the attributes the methods read):

  * ``_agent_ids_to_env_ids(agent_ids, use_AND_filter=True/False)``   franka_reach_MA.py:875-885
  * ``_env_ids_to_agent_ids(env_ids)``                                 franka_reach_MA.py:887-889
  * ``compute_observations`` (for its "others" block, the cyclic shift of the agents' positions,
    franka_reach_MA.py:582-611) on random end-effector positions.

Inputs are seeded masks (some envs fully done, some partially), id lists with repeated ids (bincount
counts a repeat twice) and random positions; outputs are what the reference returns.  The fixture holds
data only: tests/golden/ma_conventions.npz.
"""
import os
import sys
import types

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import _refshim  # noqa: E402

_refshim.install()
from isaacgymenvs.tasks.franka_reach_MA import FrankaReachMA  # noqa: E402

N_ENV = {2: 64, 4: 64}


def fake(num_envs, num_agents, states=None):
    s = types.SimpleNamespace(num_envs=num_envs, num_agents=num_agents, states=states or {}, device="cpu")
    s._refresh = lambda: None
    return s


def main():
    out = {}
    rng = np.random.default_rng(20261017)
    for A, N in N_ENV.items():
        n = N * A
        f = fake(N, A)
        # a reset_buf: ~70 % of agents done, env 0 fully done, env 1 all but one, env 2 none
        mask = (rng.random(n) < 0.7).astype(np.int64)
        mask[0:A] = 1
        mask[A:2 * A] = 1
        mask[2 * A - 1] = 0
        mask[2 * A:3 * A] = 0
        agent_ids = torch.from_numpy(np.nonzero(mask)[0])      # post_physics_step's reset_buf.nonzero()
        env_and = FrankaReachMA._agent_ids_to_env_ids(f, agent_ids, use_AND_filter=True)
        env_or = FrankaReachMA._agent_ids_to_env_ids(f, agent_ids, use_AND_filter=False)
        out[f"A{A}_mask"] = mask
        out[f"A{A}_env_ids_and"] = env_and.numpy().astype(np.int64)
        out[f"A{A}_env_ids_or"] = env_or.numpy().astype(np.int64)
        out[f"A{A}_agent_ids"] = FrankaReachMA._env_ids_to_agent_ids(f, env_and).numpy().astype(np.int64)
        # an explicit id list with repeats (a caller's reset_idx(ids)): env 2 listed as pairs of one agent
        dup = np.concatenate([np.arange(A), np.repeat(np.arange(2 * A, 2 * A + A // 2), 2),
                              np.arange(3 * A, 4 * A - 1), rng.integers(0, n, 40)])
        env_dup = FrankaReachMA._agent_ids_to_env_ids(f, torch.from_numpy(dup), use_AND_filter=True)
        out[f"A{A}_dup_ids"] = dup.astype(np.int64)
        out[f"A{A}_dup_env_ids"] = env_dup.numpy().astype(np.int64)
        out[f"A{A}_dup_agent_ids"] = FrankaReachMA._env_ids_to_agent_ids(f, env_dup).numpy().astype(np.int64)
        # the "others" block: compute_observations on random positions; the block is the last 3 (A-1) columns
        pos = rng.normal(0, 2, (N, A, 3)).astype(np.float32)
        states = {"cubeA_pos": torch.zeros(N, 1, 3), "eef_quat": torch.zeros(N, A, 4),
                  "eef_pos": torch.from_numpy(pos), "cubeA_pos_min_relative": torch.zeros(N, A, 3)}
        obs = FrankaReachMA.compute_observations(fake(N, A, states))
        out[f"A{A}_pos"] = pos
        out[f"A{A}_others"] = obs[:, obs.shape[1] - 3 * (A - 1):].numpy().astype(np.float32)
    path = os.path.join(HERE, "ma_conventions.npz")
    np.savez_compressed(path, **out)
    print("wrote", path, {k: v.shape for k, v in out.items()})


if __name__ == "__main__":
    main()
