"""ShadowHand in-hand cube reorientation on the MI355X path.

Reference counterpart: tasks/shadow_hand.py (ShadowHand, every observationType,
20 actions, 24 DOFs, objectType block / egg / pen).  pre_physics_step (masked goal /
env resets and PD targets, :670-698), the physics (PD drives, tendons, hand-cube
contacts), compute_full_state (:528-584) and compute_hand_reward (:746-800) run in
the fused ``mg_env_step`` kernel (csrc/hand_task.hpp, team_physics.hpp); the global
running mean of consecutive successes is one 1-thread finishing kernel.

Tensors mirror the reference's names and layouts: ``root_state_tensor`` (N*3, 13)
with actors [hand, object, goal] per env and global actor indices ``hand_indices``
/ ``object_indices`` / ``goal_object_indices``; ``rigid_body_states`` (N, 27, 13);
``prev_targets`` / ``cur_targets`` (N, 24); ``goal_states`` (N, 13);
``reset_goal_buf``; ``successes``; ``consecutive_successes`` (1,).
"""
from __future__ import annotations

import torch

from .. import _abi
from .. import model as M
from .. import taskdefs
from .base.vec_task import VecTask


class ShadowHand(VecTask):
    task_name = "ShadowHand"
    dr_actor_names = {"hand": "articulation", "object": "object", "goal_object": "none"}
    dr_reset_in_pre_physics = True
    acquires_dof_force = True   # shadow_hand.py:157-159 (bound in create_sim below)

    def __init__(self, cfg, rl_device, sim_device, graphics_device_id, headless, virtual_screen_capture=False,
                 force_render=False):
        env = cfg["env"]
        self.obs_type = env.get("observationType", "full_state")
        self.object_type = env.get("objectType", "block")
        self.max_episode_length = env["episodeLength"]
        self.num_fingertips = 5
        env["numObservations"] = taskdefs.HAND_OBS.get(self.obs_type, (0, 211))[1]
        self.asymmetric_obs = bool(env.get("asymmetric_observations", False))
        env["numStates"] = 211 if self.asymmetric_obs else 0   # shadow_hand.py:125-131
        self.force_scale = float(env.get("forceScale", 0.0))
        self.force_prob_range = env.get("forceProbRange", [0.001, 0.1])
        self.force_decay = env.get("forceDecay", 0.99)
        self.force_decay_interval = env.get("forceDecayInterval", 0.08)
        env["numActions"] = 20
        self.up_axis_idx = 2
        super().__init__(cfg, rl_device, sim_device, graphics_device_id, headless, virtual_screen_capture,
                         force_render)

    # ---------------------------------------------------------------------------------- setup
    def create_sim(self):
        _, table, _, _, _, max_contacts = taskdefs.TASK_INFO["ShadowHand"]
        spec = taskdefs.hand_spec(self.object_type)   # block / egg / pen object (shadow_hand.py:86-100)
        self.model_spec = spec
        self.num_dof = self.num_shadow_hand_dofs = spec.num_dofs
        self.num_shadow_hand_bodies = len(spec.bodies)
        self.num_bodies = self.num_shadow_hand_bodies + 2
        self.num_actors = self.num_envs
        self.sim_params = taskdefs.sim_params(self.cfg, max_contacts, 1)
        self.task_params = tp = taskdefs.task_params("ShadowHand", self.cfg, spec)
        self._model_np = _abi.model_bytes(spec)
        torch.cuda.set_device(self.device_id)
        h = _abi.C.c_void_p()
        _abi.check(self._lib.mg_sim_create(self._model_np.ctypes.data, _abi.C.byref(self.sim_params),
                                           self.num_envs, self.device_id, _abi.C.byref(h)), self._lib)
        self.sim = h
        dev, f, N, nd = self.device, torch.float32, self.num_envs, self.num_dof
        # actor root states [hand, object, goal] per env (shadow_hand.py:356-384, 400-405)
        self.root_state_tensor = torch.zeros((N * 3, 13), device=dev, dtype=f)
        rs = self.root_state_tensor.view(N, 3, 13)
        rs[:, 0, 0:3] = torch.tensor(list(tp.start_pos), device=dev)
        rs[:, 0, 3:7] = torch.tensor(list(tp.start_rot), device=dev)
        obj = torch.tensor(list(tp.object_start), device=dev)
        rs[:, 1, 0:3] = obj
        rs[:, 1, 6] = 1.0
        self.object_init_state = rs[:, 1].clone()
        self.goal_states = self.object_init_state.clone()
        self.goal_states[:, self.up_axis_idx] += tp.goal_dz
        self.goal_init_state = self.goal_states.clone()
        self.goal_displacement_tensor = torch.tensor(list(tp.goal_displacement), device=dev)
        rs[:, 2, 0:3] = self.goal_states[:, 0:3] + self.goal_displacement_tensor
        rs[:, 2, 6] = 1.0
        self.hand_start_states = rs[:, 0].clone()
        self.root_states = self.root_state_tensor
        ar = torch.arange(N, device=dev, dtype=torch.long)
        self.hand_indices, self.object_indices, self.goal_object_indices = 3 * ar, 3 * ar + 1, 3 * ar + 2
        self.dof_state = torch.zeros((N * nd, 2), device=dev, dtype=f)
        self.shadow_hand_dof_state = self.dof_state.view(N, nd, 2)
        self.shadow_hand_dof_pos = self.shadow_hand_dof_state[..., 0]
        self.shadow_hand_dof_vel = self.shadow_hand_dof_state[..., 1]
        self.rigid_body_states = torch.zeros((N, self.num_bodies, 13), device=dev, dtype=f)
        self.sensor_tensor = torch.zeros((N * self.num_fingertips, 6), device=dev, dtype=f)
        self.vec_sensor_tensor = self.sensor_tensor.view(N, self.num_fingertips * 6)
        self.dof_force_tensor = torch.zeros((N, nd), device=dev, dtype=f)
        self.prev_targets = torch.zeros((N, nd), device=dev, dtype=f)
        self.cur_targets = torch.zeros((N, nd), device=dev, dtype=f)
        self.shadow_hand_dof_lower_limits = torch.tensor([n.lower for n in spec.nodes[1:]], device=dev, dtype=f)
        self.shadow_hand_dof_upper_limits = torch.tensor([n.upper for n in spec.nodes[1:]], device=dev, dtype=f)
        self.actuated_dof_indices = torch.tensor([spec.dof_index(a["joint"]) for a in spec.actuators], device=dev,
                                                 dtype=torch.long)
        self.fingertip_handles = torch.tensor(list(spec.sensors), device=dev, dtype=torch.long)
        v = _abi.StateViews()
        v.root_states, v.dof_state = _abi.ptr(self.root_state_tensor), _abi.ptr(self.dof_state)
        v.dof_actuation, v.sensors = None, _abi.ptr(self.sensor_tensor)
        v.dof_force, v.rigid_body_states = _abi.ptr(self.dof_force_tensor), _abi.ptr(self.rigid_body_states)
        v.dof_targets = _abi.ptr(self.cur_targets)
        # apply_rigid_body_force_tensors(sim, rb_forces, None, LOCAL_SPACE) (shadow_hand.py:708): the fused
        # step updates and applies the object row every step (zero while forceScale is 0)
        self.rb_forces = torch.zeros((N, self.num_bodies, 3), device=dev, dtype=f)
        self.object_rb_handles = torch.tensor([self.num_shadow_hand_bodies], device=dev, dtype=torch.long)
        self.object_rb_masses = torch.tensor([tp.object_rb_mass], device=dev, dtype=f)
        v.rb_forces, v.rb_force_space = _abi.ptr(self.rb_forces), _abi.MG_LOCAL_SPACE
        self._views = v
        _abi.check(self._lib.mg_sim_bind(self.sim, _abi.C.byref(v)), self._lib)

    env_state_tensors = VecTask.env_state_tensors + (
        "root_state_tensor", "rigid_body_states", "prev_targets", "cur_targets", "goal_states", "reset_goal_buf",
        "successes", "consecutive_successes", "rb_forces", "random_force_prob")

    def allocate_buffers(self):
        super().allocate_buffers()
        dev, N = self.device, self.num_envs
        self.reset_goal_buf = self.reset_buf.clone()
        self.successes = torch.zeros(N, device=dev, dtype=torch.float)
        self.consecutive_successes = torch.zeros(1, device=dev, dtype=torch.float)
        self._reduce = torch.zeros(2, device=dev, dtype=torch.int64)
        tb = self._tb
        tb.potentials = tb.prev_potentials = tb.up_vec = tb.heading_vec = None
        tb.prev_targets, tb.goal_states = _abi.ptr(self.prev_targets), _abi.ptr(self.goal_states)
        tb.reset_goal, tb.successes = _abi.ptr(self.reset_goal_buf), _abi.ptr(self.successes)
        tb.consecutive_successes, tb.reduce_scratch = _abi.ptr(self.consecutive_successes), _abi.ptr(self._reduce)
        # random force probability per env (shadow_hand.py:196-199), redrawn on reset inside the step
        lo, hi = (torch.tensor(float(x), device=dev) for x in self.force_prob_range)
        self.random_force_prob = torch.exp((torch.log(lo) - torch.log(hi)) * torch.rand(N, device=dev) + torch.log(hi))
        tb.random_force_prob = _abi.ptr(self.random_force_prob)
        tb.states = _abi.ptr(self.states_buf) if self.num_states > 0 else None
        # multi-GPU: the running mean over the envs of all ranks; the step leaves its
        # partial sums, post_launch all-reduces them (16 bytes) and applies shadow_hand.py:795-798.
        # Off by default: the reference's statistic is per rank (shadow_hand.py:795-798); set
        # env.globalConsecutiveSuccesses: True to opt in to the node-wide mean (one 16-byte all-reduce per step).
        self._global_cons = bool(self.cfg["env"].get("globalConsecutiveSuccesses", False)) and \
            torch.distributed.is_available() and torch.distributed.is_initialized()
        tb.defer_finalize = 1 if self._global_cons else 0

    def post_launch(self):
        if self._global_cons:
            torch.distributed.all_reduce(self._reduce)
            _abi.check(self._lib.mg_hand_finalize(_abi.C.byref(self.task_params), _abi.C.byref(self._tb),
                                                  self._stream()), self._lib)

    def post_step_extras(self):
        self.extras["consecutive_successes"] = self.consecutive_successes.mean()

    def set_reset_noise(self, noise):
        """Inject per-env rows (N, 66) = [goal-only 4 | reset_idx 53 | reset_target_pose 4 | force probability
        redraw 1 | force selection 1 (all U(0,1)) | force direction 3 (N(0,1))]."""
        super().set_reset_noise(noise)
