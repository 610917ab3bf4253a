"""rl_games-facing wrappers (reference: isaacgymenvs/utils/rlgames_utils.py:53-127, 242-424).

rl_games itself is not a dependency; ``RLGPUEnv`` keeps the same methods and the
fork's multi-agent ``get_env_info()['agents']`` contract (rlgames_utils.py:258-263).
``ComplexObsRLGPUEnv`` restates rlgames_utils.py:300-424.  The wrappers take the env either directly
(``env=``) or through ``config_name``, looked up in :data:`env_configurations` (the counterpart of
rl_games' ``env_configurations.configurations`` registry, filled with :func:`register_env_creator`).
"""
from __future__ import annotations

from typing import Any, Dict, Tuple

import numpy as np

# name -> {"env_creator": callable(**kwargs) -> env, "vecenv_type": str}
env_configurations: Dict[str, Dict[str, Any]] = {}


def register_env_creator(name, creator, vecenv_type="RLGPU"):
    """``env_configurations.register(name, {'env_creator': ..., 'vecenv_type': ...})`` (train.py:160-180)."""
    env_configurations[name] = {"env_creator": creator, "vecenv_type": vecenv_type}


def _create_env(env, config_name, kwargs):
    if env is None and config_name is not None and not isinstance(config_name, str):
        env = config_name   # RLGPUEnv(env): an env object in the config-name position
    if env is not None:
        return env
    if config_name is None or config_name not in env_configurations:
        raise KeyError(f"no env creator registered as {config_name!r} (register_env_creator)")
    return env_configurations[config_name]["env_creator"](**kwargs)


def get_rlgames_env_creator(seed, task_config, task_name, sim_device, rl_device, graphics_device_id, headless,
                            multi_gpu=False, post_create_hook=None, virtual_screen_capture=False,
                            force_render=False):
    def create_rlgpu_env():
        from ..tasks import isaacgym_task_map
        nonlocal sim_device, rl_device
        cfg = dict(task_config)
        if multi_gpu:
            import os
            local_rank = int(os.getenv("LOCAL_RANK", "0"))
            global_rank = int(os.getenv("RANK", "0"))
            world = int(os.getenv("WORLD_SIZE", "1"))
            import torch
            ndev = max(torch.cuda.device_count(), 1)
            sim_device = f"cuda:{local_rank % ndev}"
            rl_device = f"cuda:{local_rank % ndev}"
            cfg["rank"] = global_rank
            cfg["world_size"] = world
            cfg["env_offset"] = global_rank * int(cfg["env"]["numEnvs"])
        cfg["seed"] = seed
        # the CPU pipeline (vec_task.py:78-90: use_gpu_pipeline False, or a non-GPU sim_device): the HIP step on the
        # GPU with host-side views of every tensor (migym/host_pipeline.py)
        dev_type, _, dev_id = str(sim_device).partition(":")
        host = not cfg.get("sim", {}).get("use_gpu_pipeline", True) or dev_type.lower() not in ("cuda", "gpu")
        if host:
            if dev_type.lower() not in ("cuda", "gpu"):
                print("GPU Pipeline can only be used with GPU simulation. Forcing CPU Pipeline.")
            cfg["sim"] = dict(cfg["sim"], use_gpu_pipeline=True)
            sim_device = f"cuda:{int(dev_id) if dev_id and dev_type.lower() in ('cuda', 'gpu') else 0}"
        env = isaacgym_task_map[task_name](cfg=cfg, rl_device=rl_device, sim_device=sim_device,
                                           graphics_device_id=graphics_device_id, headless=headless,
                                           virtual_screen_capture=virtual_screen_capture, force_render=force_render)
        if host:
            from ..host_pipeline import HostPipeline
            env = HostPipeline(env)
        if post_create_hook is not None:
            post_create_hook()
        return env

    return create_rlgpu_env


class RLGPUEnv:
    def __init__(self, config_name=None, num_actors=None, env=None, **kwargs):
        self.env = _create_env(env, config_name, kwargs)

    def step(self, actions):
        return self.env.step(actions)

    def reset(self):
        return self.env.reset()

    def reset_done(self):
        return self.env.reset_done()

    def get_number_of_agents(self):
        return self.env.num_agents

    def get_env_info(self):
        info = {"action_space": self.env.action_space, "observation_space": self.env.observation_space,
                "agents": self.env.num_agents}
        if self.env.num_states > 0:
            info["state_space"] = self.env.state_space
        return info

    def set_train_info(self, env_frames, *args_, **kwargs_):
        if hasattr(self.env, "set_train_info"):
            self.env.set_train_info(env_frames, *args_, **kwargs_)

    def get_env_state(self):
        return self.env.get_env_state() if hasattr(self.env, "get_env_state") else None

    def set_env_state(self, env_state):
        if hasattr(self.env, "set_env_state"):
            self.env.set_env_state(env_state)


class ComplexObsRLGPUEnv:
    """RLGPU wrapper with named observation groups (rlgames_utils.py:300-424).

    obs_spec: ``{rl_games key: {'names': [env observation names], 'concat': bool, 'space_name': str}}``, e.g.
    ``{'obs': {'names': ['obs'], 'concat': True, 'space_name': 'observation_space'},
    'states': {'names': ['states'], 'concat': True, 'space_name': 'state_space'}}``.  With ``concat`` the named
    (num_envs, k) tensors are concatenated along dim 1, otherwise passed on as a dict.  The env's
    observation names are the keys of its ``obs_dict``; their spaces come from ``observation_space[name]`` when
    the env exposes a Dict space, else ``obs`` -> ``observation_space`` and ``states`` -> ``state_space``."""

    def __init__(self, config_name=None, num_actors=None, obs_spec: Dict[str, Dict] = None, env=None, **kwargs):
        self.env = _create_env(env, config_name, kwargs)
        if not obs_spec:
            raise ValueError("ComplexObsRLGPUEnv needs an obs_spec")
        self.obs_spec = obs_spec

    def _generate_obs(self, env_obs: Dict[str, Any]) -> Dict[str, Any]:
        return {k: self.gen_obs_dict(env_obs, v["names"], v["concat"]) for k, v in self.obs_spec.items()}

    def step(self, action) -> Tuple[Dict[str, Any], Any, Any, Dict[str, Any]]:
        env_obs, rewards, dones, infos = self.env.step(action)
        return self._generate_obs(env_obs), rewards, dones, infos

    def reset(self) -> Dict[str, Any]:
        return self._generate_obs(self.env.reset())

    def get_number_of_agents(self) -> int:
        if hasattr(self.env, "get_number_of_agents"):
            return self.env.get_number_of_agents()
        return getattr(self.env, "num_agents", 1)

    def get_env_info(self) -> Dict[str, Any]:
        info = {"action_space": self.env.action_space}
        for v in self.obs_spec.values():
            info[v["space_name"]] = self.gen_obs_space(v["names"], v["concat"])
        return info

    def gen_obs_dict(self, obs_dict, obs_names, concat):
        import torch
        if concat:
            return torch.cat([obs_dict[name] for name in obs_names], dim=1)
        return {k: obs_dict[k] for k in obs_names}

    def _space(self, name):
        space = self.env.observation_space
        if hasattr(space, "keys") and name in space:
            return space[name]
        if name == "obs":
            return space
        if name == "states" and getattr(self.env, "num_states", 0) > 0:
            return self.env.state_space
        raise KeyError(f"the env has no observation named {name!r}")

    def gen_obs_space(self, obs_names, concat):
        from ..spaces import Box, Dict as DictSpace
        if concat:
            return Box(low=-np.inf, high=np.inf, shape=(sum(self._space(s).shape[0] for s in obs_names),),
                       dtype=np.float32)
        return DictSpace({k: self._space(k) for k in obs_names})

    def set_train_info(self, env_frames, *args_, **kwargs_):
        if hasattr(self.env, "set_train_info"):
            self.env.set_train_info(env_frames, *args_, **kwargs_)

    def get_env_state(self):
        return self.env.get_env_state() if hasattr(self.env, "get_env_state") else None

    def set_env_state(self, env_state):
        if hasattr(self.env, "set_env_state"):
            self.env.set_env_state(env_state)
