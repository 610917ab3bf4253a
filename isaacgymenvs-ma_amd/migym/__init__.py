"""migym — MI355X-native physics-step + observation/reward pipeline behind the
isaacgymenvs ``make()`` / ``VecTask.step()`` / ``reset()`` API.

    import migym
    env = migym.make(seed=0, task="Ant", num_envs=16384, sim_device="cuda:0", rl_device="cuda:0")
    obs, rew, done, extras = env.step(actions)

``make`` mirrors isaacgymenvs/__init__.py:14-55 (same signature); hydra is
replaced by the eager resolver in :mod:`migym.configs`.
"""
from __future__ import annotations

__version__ = "0.1.0"


def make(seed: int, task: str, num_envs: int, sim_device: str, rl_device: str, graphics_device_id: int = -1,
         headless: bool = False, multi_gpu: bool = False, virtual_screen_capture: bool = False,
         force_render: bool = True, cfg=None):
    from .configs import task_config
    from .utils.rlgames_utils import get_rlgames_env_creator
    if cfg is None:
        cfg_dict = task_config(task, num_envs, sim_device=sim_device)
    else:
        c = cfg["task"] if isinstance(cfg, dict) and "task" in cfg else getattr(cfg, "task", cfg)
        cfg_dict = dict(c)
        task = cfg_dict.get("name", task)
    creator = get_rlgames_env_creator(seed=seed, task_config=cfg_dict, task_name=cfg_dict["name"],
                                      sim_device=sim_device, rl_device=rl_device,
                                      graphics_device_id=graphics_device_id, headless=headless,
                                      multi_gpu=multi_gpu, virtual_screen_capture=virtual_screen_capture,
                                      force_render=force_render)
    return creator()
