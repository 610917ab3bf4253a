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
    """Packs [obs | rew | reset] of the local shard into one buffer and concatenates the shards.

    mode="all": one all-gather (RCCL on GPU, gloo on CPU): every rank gets every shard.
    mode="root": the shards go only to rank ``root``: the other ranks each send one
    message and the root posts one receive per peer in a single batch, so on an 8-GPU node the root
    takes the 7 shards over its 7 xGMI links at once instead of a ring's 7 sequential hops.  Ranks other
    than the root get ``None`` back.
    """

    def __init__(self, num_rows: int, num_obs: int, device, group=None, mode: str = "all", root: int = 0):
        if mode not in ("all", "root"):
            raise ValueError(f"mode must be 'all' or 'root', got {mode!r}")
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.mode, self.root = mode, root
        self.rows, self.nobs = num_rows, num_obs
        self.width = num_obs + 2
        self.local = torch.empty((num_rows, self.width), device=device, dtype=torch.float32)
        need_full = mode == "all" or self.rank == root
        self.full = torch.empty((self.world * num_rows, self.width), device=device, dtype=torch.float32) \
            if need_full else None
        self._gloo = dist.get_backend(group) == "gloo"

    def __call__(self, obs: torch.Tensor, rew: torch.Tensor, reset: torch.Tensor):
        self.local[:, : self.nobs].copy_(obs)
        self.local[:, self.nobs].copy_(rew)
        self.local[:, self.nobs + 1].copy_(reset)
        if self.mode == "root":
            if self.rank != self.root:
                dist.send(self.local, dst=self.root, group=self.group)
                return None
            parts = list(self.full.chunk(self.world, 0))
            parts[self.root].copy_(self.local)
            ops = [dist.P2POp(dist.irecv, parts[r], r, self.group) for r in range(self.world) if r != self.root]
            for w in dist.batch_isend_irecv(ops):
                w.wait()
        elif self._gloo:
            parts = list(self.full.chunk(self.world, 0))
            dist.all_gather(parts, self.local, group=self.group)
        else:
            dist.all_gather_into_tensor(self.full, self.local, group=self.group)
        obs_all = self.full[:, : self.nobs]
        rew_all = self.full[:, self.nobs]
        reset_all = self.full[:, self.nobs + 1].to(torch.long)
        return obs_all, rew_all, reset_all


class PackedGather:
    """The obs/rew/reset gather of SURVEY.md §8(e), overlapped with the next step.

    The fused step writes each actor's row ``[clamped obs | rew | reset]`` straight into a message
    buffer (``mg_task_buffers.out_pack``), so packing costs no extra kernel or copy.  Message buffers
    rotate over ``depth`` slots: the gather of step k (issued right after step k's launch, on the
    collective's own stream) runs while step k+1 computes into the next slot; a slot is reused only
    after its gather has completed (a stream wait, not a host block).

    mode="root": every rank sends its rows to ``root`` (one message; the root posts one receive per
    peer in a single batch, so on one node the 7 shards arrive over 7 xGMI links at once); the root's
    own rows are written by its kernel directly into its slice of the gathered buffer.  mode="all":
    one all-gather, every rank gets every shard.

    Use: ``VecTask.attach_output_gather(g)``; after a step, ``g.result()`` waits for the latest gather and
    returns ``(obs, rew, reset)`` of all ranks (``None`` on non-root ranks in root mode).
    """

    def __init__(self, num_rows: int, num_obs: int, device, group=None, mode: str = "root", root: int = 0,
                 depth: int = 2):
        if mode not in ("all", "root"):
            raise ValueError(f"mode must be 'all' or 'root', got {mode!r}")
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.mode, self.root, self.depth = mode, root, depth
        self.rows, self.nobs, self.width = num_rows, num_obs, num_obs + 2
        self._gloo = dist.get_backend(group) == "gloo"
        self.has_full = mode == "all" or self.rank == root
        self.full, self.pack = [], []
        for _ in range(depth):
            if self.has_full:
                f = torch.empty((self.world * num_rows, self.width), device=device, dtype=torch.float32)
                self.full.append(f)
                self.pack.append(f[self.rank * num_rows:(self.rank + 1) * num_rows])  # contiguous row block
            else:
                self.pack.append(torch.empty((num_rows, self.width), device=device, dtype=torch.float32))
        self.works = [None] * depth
        self.k = 0
        self.last = None
        # one full-group collective before the first point-to-point message, so every rank has created
        # the group's communicator before the root's batched receives (torch's batch_isend_irecv rule)
        dist.barrier(group=group)

    def next_pack(self) -> torch.Tensor:
        """The slot the next step writes; waits (stream-ordered) for the gather that last used it."""
        i = self.k % self.depth
        self._wait(i)
        return self.pack[i]

    def issue(self):
        """Start the gather of the slot the step just launched wrote (async on the collective stream)."""
        i = self.k % self.depth
        buf = self.pack[i]
        if self.mode == "root":
            if self.rank != self.root:
                works = dist.batch_isend_irecv([dist.P2POp(dist.isend, buf, self.root, self.group)])
            else:
                parts = self.full[i].chunk(self.world, 0)
                ops = [dist.P2POp(dist.irecv, parts[r], r, self.group) for r in range(self.world) if r != self.root]
                works = dist.batch_isend_irecv(ops) if ops else []
        elif self._gloo:
            works = [dist.all_gather(list(self.full[i].chunk(self.world, 0)), buf, group=self.group, async_op=True)]
        else:
            works = [dist.all_gather_into_tensor(self.full[i], buf, group=self.group, async_op=True)]
        self.works[i] = works
        self.last = i
        self.k += 1

    def _wait(self, i):
        if self.works[i]:
            for w in self.works[i]:
                w.wait()
        self.works[i] = None

    def result(self):
        """(obs, rew, reset) of all ranks for the latest issued step (root / all ranks), else None."""
        if self.last is None:
            return None
        self._wait(self.last)
        if not self.has_full:
            return None
        f = self.full[self.last]
        return f[:, : self.nobs], f[:, self.nobs], f[:, self.nobs + 1].to(torch.long)

    def drain(self):
        for i in range(self.depth):
            self._wait(i)
