"""Ant / Humanoid / multi-agent Ant on the MI355X path.

Reference counterparts: tasks/ant.py (Ant: 60-d obs, 8 actions, 4 foot force
sensors), tasks/humanoid.py (108-d obs, 21 actions, 2 foot sensors + DOF
forces).  Their jit observation/reward functions, reset_idx and
post_physics_step run inside the fused ``mg_env_step`` kernel (csrc/task.hpp).
"""
from __future__ import annotations

from .base.vec_task import VecTask


class _Locomotion(VecTask):
    task_name = None
    num_obs_default = 0
    num_act_default = 0

    def __init__(self, cfg, rl_device, sim_device, graphics_device_id, headless, virtual_screen_capture=False,
                 force_render=False):
        env = cfg["env"]
        self.max_episode_length = env["episodeLength"]
        self.dof_vel_scale = env["dofVelocityScale"]
        self.contact_force_scale = env["contactForceScale"]
        self.power_scale = env["powerScale"]
        self.heading_weight = env["headingWeight"]
        self.up_weight = env["upWeight"]
        self.actions_cost_scale = env["actionsCost"]
        self.energy_cost_scale = env["energyCost"]
        self.joints_at_limit_cost_scale = env["jointsAtLimitCost"]
        self.death_cost = env["deathCost"]
        self.termination_height = env["terminationHeight"]
        env["numObservations"] = self.num_obs_default
        env["numActions"] = self.num_act_default
        self.up_axis_idx = 2
        super().__init__(cfg, rl_device, sim_device, graphics_device_id, headless, virtual_screen_capture,
                         force_render)
        self.joint_gears = self.dof_actuation.new_tensor([a["gear"] for a in self.model_spec.actuators])
        self.motor_efforts = self.joint_gears
        self.max_motor_effort = float(self.task_params.max_motor_effort)
        self.torso_index = 0

    def post_step_extras(self):
        pass


class Ant(_Locomotion):
    task_name = "Ant"
    num_obs_default = 60
    num_act_default = 8
    dr_actor_names = {"ant": "articulation"}

    def post_step_extras(self):
        # compute_true_objective (ant.py:245-250): forward velocity of the torso
        self.extras["true_objective"] = self.root_states[:, 7]


class Humanoid(_Locomotion):
    task_name = "Humanoid"
    num_obs_default = 108
    num_act_default = 21
    dr_actor_names = {"humanoid": "articulation"}
    acquires_dof_force = True   # humanoid.py:85-86


class MAAnt(_Locomotion):
    """Multi-agent Ant (build-defined, SURVEY.md §8(a) row A-MA).

    ``numAgents`` (default 4) ant actors per env on a square grid ``agentSpacing`` apart.
    Buffers are ``(num_envs * num_agents, ...)`` env-major like the fork's MA tasks
    (franka_reach_MA.py:22-38); obs per agent = the 60-d Ant obs + the other agents' torso
    positions relative to self in cyclic-shift order (franka_reach_MA.py:604-608) = 69-d for
    A = 4; reward per agent = compute_ant_reward; an env resets only when all of its agents
    are done (AND filter, franka_reach_MA.py:875-885).  Agents do not collide with each other
    (each is an independent articulation).
    """
    task_name = "MAAnt"
    num_obs_default = 60
    num_act_default = 8
    dr_actor_names = {"ant": "articulation"}

    def __init__(self, cfg, rl_device, sim_device, graphics_device_id, headless, virtual_screen_capture=False,
                 force_render=False):
        A = int(cfg["env"].get("numAgents", 4))
        cfg["env"]["numAgents"] = A
        self.num_obs_default = 60 + 3 * (A - 1)
        super().__init__(cfg, rl_device, sim_device, graphics_device_id, headless, virtual_screen_capture,
                         force_render)
