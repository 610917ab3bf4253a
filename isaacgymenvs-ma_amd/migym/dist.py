"""Multi-GPU sharding of the env batch (one process per GPU, torchrun).

Envs are independent, so rank r of P simulates its own contiguous block of envs
(global ids [r*N, (r+1)*N), the layout of rlgames_utils.py:89-107 where every
rank owns ``numEnvs`` envs on ``cuda:LOCAL_RANK``).  Reset noise is keyed by the
global env id, so a rollout is invariant to P.  The data path has no
collective; :class:`OutputGather` is the optional single all-gather that
concatenates obs / rew / reset of all ranks onto every rank's rl_device (the
north_star's "RCCL all-gather over xGMI"), packed into ONE buffer so each step
issues exactly one collective.
"""
from __future__ import annotations

import os

import torch
import torch.distributed as dist


def rank_info():
    return (int(os.getenv("RANK", "0")), int(os.getenv("WORLD_SIZE", "1")), int(os.getenv("LOCAL_RANK", "0")))


def env_offset(num_envs_per_rank: int, rank: int) -> int:
    return rank * num_envs_per_rank


class OutputGather:
    """Packs [obs | rew | reset] of the local shard and all-gathers it (RCCL on GPU, gloo on CPU)."""

    def __init__(self, num_rows: int, num_obs: int, device, group=None):
        self.group = group
        self.world = dist.get_world_size(group)
        self.rows, self.nobs = num_rows, num_obs
        self.width = num_obs + 2
        self.local = torch.empty((num_rows, self.width), device=device, dtype=torch.float32)
        self.full = torch.empty((self.world * num_rows, self.width), device=device, dtype=torch.float32)
        self._gloo = dist.get_backend(group) == "gloo"

    def __call__(self, obs: torch.Tensor, rew: torch.Tensor, reset: torch.Tensor):
        self.local[:, : self.nobs].copy_(obs)
        self.local[:, self.nobs].copy_(rew)
        self.local[:, self.nobs + 1].copy_(reset)
        if self._gloo:
            parts = list(self.full.chunk(self.world, 0))
            dist.all_gather(parts, self.local, group=self.group)
        else:
            dist.all_gather_into_tensor(self.full, self.local, group=self.group)
        obs_all = self.full[:, : self.nobs]
        rew_all = self.full[:, self.nobs]
        reset_all = self.full[:, self.nobs + 1].to(torch.long)
        return obs_all, rew_all, reset_all
