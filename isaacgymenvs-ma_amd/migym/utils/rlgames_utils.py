"""rl_games-facing wrappers (reference: isaacgymenvs/utils/rlgames_utils.py:53-127, 242-297).

rl_games itself is not a dependency; ``RLGPUEnv`` keeps the same methods and the
fork's multi-agent ``get_env_info()['agents']`` contract (rlgames_utils.py:258-263).
"""
from __future__ import annotations


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
        env = isaacgym_task_map[task_name](cfg=cfg, rl_device=rl_device, sim_device=sim_device,
                                           graphics_device_id=graphics_device_id, headless=headless,
                                           virtual_screen_capture=virtual_screen_capture, force_render=force_render)
        if post_create_hook is not None:
            post_create_hook()
        return env

    return create_rlgpu_env


class RLGPUEnv:
    def __init__(self, env=None, config_name=None, num_actors=None, **kwargs):
        self.env = env

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
