"""Cartpole on the MI355X path (reference: tasks/cartpole.py).

4-d obs [x, xdot, theta, thetadot], 1 action -> 400 N on the slider DOF,
episode length 500 (hard-coded at cartpole.py:44), obs clamp +-5."""
from __future__ import annotations

from .base.vec_task import VecTask


class Cartpole(VecTask):
    task_name = "Cartpole"

    def __init__(self, cfg, rl_device, sim_device, graphics_device_id, headless, virtual_screen_capture=False,
                 force_render=False):
        self.reset_dist = cfg["env"]["resetDist"]
        self.max_push_effort = cfg["env"]["maxEffort"]
        self.max_episode_length = 500
        cfg["env"]["numObservations"] = 4
        cfg["env"]["numActions"] = 1
        super().__init__(cfg, rl_device, sim_device, graphics_device_id, headless, virtual_screen_capture,
                         force_render)
