"""``use_gpu_pipeline=False`` / ``sim_device='cpu'`` as a drop-in (reference: tasks/base/vec_task.py:78-90).

The reference's CPU pipeline runs PhysX on the host and keeps every gym tensor and task buffer in host memory
(``env.device == 'cpu'``); ``step()`` still returns its outputs on ``rl_device``.  This build has no CPU physics
engine (the CPU oracle is test infrastructure, never the product path), so the CPU pipeline keeps the HIP step
on the MI355X and exposes host-side views of the task:

  * the task is built on the GPU pipeline (``cuda:<device id>``, device 0 for ``sim_device='cpu'``);
  * every device tensor attribute of the task (gym state, task buffers, views of them) is mirrored in pinned
    host memory, storage by storage, so a view keeps its relation to its base tensor (``dof_pos`` is a view of
    ``dof_state`` on the host as on the device);
  * the mirrors are pulled after each call that changes the state (step, reset, reset_idx, reset_done,
    set_env_state, apply_randomizations) and pushed back before it and before get_env_state, so host-side edits
    (``env.reset_buf[ids] = 1``, ``env.root_states[...] = ...`` before ``reset_idx``) take effect on the next
    step, as the reference's set_*_tensor calls make them take effect.  Only storages whose host bytes changed
    since the last pull are pushed (each mirror keeps a snapshot of what it pulled), so a device-side write made
    between calls through ``env.unwrapped`` is not reverted by a stale host copy;
  * ``get_env_state()`` returns host tensors, like every other tensor of a CPU-pipeline task;
  * ``env.device`` is ``'cpu'``; ``step()`` returns on ``rl_device`` exactly as the GPU pipeline does.

Transfers cost PCIe time per step (the whole mirrored set each way); the CPU pipeline is a compatibility mode,
not the measured path.
"""
from __future__ import annotations

import torch

_SYNCED = ("step", "reset", "reset_idx", "reset_done", "set_env_state", "apply_randomizations", "get_env_state")


def _to_host(x):
    if torch.is_tensor(x):
        return x.cpu()
    if isinstance(x, dict):
        return {k: _to_host(v) for k, v in x.items()}
    if isinstance(x, (list, tuple)):
        return type(x)(_to_host(v) for v in x)
    return x


class HostPipeline:
    def __init__(self, task):
        object.__setattr__(self, "_task", task)
        # device storage ptr -> (device bytes, host bytes, snapshot of the host bytes as last pulled)
        object.__setattr__(self, "_host", {})
        object.__setattr__(self, "_mirror", {})    # attribute -> host tensor
        object.__setattr__(self, "device", "cpu")
        object.__setattr__(self, "sim_device_internal", task.device)
        self._pull()

    # ------------------------------------------------------------------ mirrors
    def _device_tensors(self):
        t = self._task
        return {k: v for k, v in vars(t).items() if torch.is_tensor(v) and v.device.type == "cuda"}

    def _pull(self):
        """(re)map every device tensor attribute onto a host storage mirror and copy the device contents in"""
        tens = self._device_tensors()
        host, mirror = {}, {}
        for k, v in tens.items():
            st = v.untyped_storage()
            key = st.data_ptr()
            if key not in host:
                old = self._host.get(key)
                if old is not None and old[1].numel() == st.nbytes():
                    hb = old[1]
                else:
                    hb = torch.empty(st.nbytes(), dtype=torch.uint8, pin_memory=True)
                dev_bytes = torch.empty(0, dtype=torch.uint8, device=v.device).set_(st)
                host[key] = (dev_bytes, hb, old[2] if old is not None and old[1] is hb else torch.empty_like(hb))
            hb = host[key][1]
            mirror[k] = torch.empty(0, dtype=v.dtype).set_(hb.untyped_storage(), v.storage_offset(), v.size(),
                                                           v.stride())
        torch.cuda.synchronize(self._task.device)
        for dev_bytes, hb, _ in host.values():
            hb.copy_(dev_bytes, non_blocking=True)
        torch.cuda.synchronize(self._task.device)
        for _, hb, snap in host.values():
            snap.copy_(hb)
        object.__setattr__(self, "_host", host)
        object.__setattr__(self, "_mirror", mirror)

    def _push(self):
        """host mirrors the caller edited since the last pull -> device (the others are left alone, so a device-side
        change made in between through env.unwrapped survives)"""
        for dev_bytes, hb, snap in self._host.values():
            if not torch.equal(hb, snap):
                dev_bytes.copy_(hb, non_blocking=True)
                snap.copy_(hb)   # the device now holds these bytes: the next push leaves them alone

    # ------------------------------------------------------------------ attribute surface
    def __getattr__(self, name):
        m = self._mirror.get(name)
        if m is not None:
            return m
        v = getattr(self._task, name)
        if name in _SYNCED and callable(v):
            def synced(*a, **kw):
                self._push()
                out = v(*a, **kw)
                if name == "get_env_state":   # a read: host copies of the state, nothing to pull
                    torch.cuda.synchronize(self._task.device)
                    return _to_host(out)
                self._pull()
                return out
            return synced
        return v

    def __setattr__(self, name, value):
        m = self._mirror.get(name)
        if m is not None and torch.is_tensor(value):
            m.copy_(value)
            return
        setattr(self._task, name, value)

    @property
    def unwrapped(self):
        """the GPU-pipeline task underneath (its tensors are the device buffers)"""
        return self._task
