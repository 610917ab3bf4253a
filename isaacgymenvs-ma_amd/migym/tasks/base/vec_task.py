"""VecTask on the MI355X path — same contract as the reference's
``isaacgymenvs/tasks/base/vec_task.py`` (Env 67-206, VecTask 208-457).

The reference drives PhysX through ``gym.simulate`` plus a dozen ATen kernels
per step and synchronises with the host every step (``reset_buf.nonzero()``,
ant.py:291-293).  Here one ``mg_env_step`` launch runs the whole
``VecTask.step`` for every env (clamp -> pre_physics_step -> simulate ->
post_physics_step -> timeout -> obs clamp), with no host synchronisation.

Kept reference semantics:
  * ``reset_buf`` starts at ones, so the first ``step`` resets every env;
    ``reset()`` returns the current (unclamped-then-clamped) obs without computing
    observations (vec_task.py:428-440).
  * resets requested by a step's reward are applied at the start of the next
    step's post-physics phase, before observations (ant.py:287-297).
  * ``extras['time_outs']`` is a bool tensor (vec_task.py:396, 402).
  * observations are clamped to ``clipObservations`` and moved to ``rl_device``.
Differences (documented in DESIGN.md / INTEGRATION.md): reset noise comes from a
counter-based device RNG keyed by (seed, global env id, control step) instead
of the global torch generator; returned obs/rew/reset tensors are persistent
buffers overwritten by the next step (rl_games copies them immediately).
"""
from __future__ import annotations

import abc
import math
from typing import Any, Dict, Tuple

import numpy as np
import torch

from ... import _abi
from ... import model as M
from ...dr import DomainRandomizationMixin
from ... import spaces
from ... import taskdefs


class Env(abc.ABC):
    def __init__(self, config: Dict[str, Any], rl_device: str, sim_device: str, graphics_device_id: int,
                 headless: bool):
        split = sim_device.split(":")
        self.device_type = split[0]
        self.device_id = int(split[1]) if len(split) > 1 else 0
        self.device = "cpu"
        if config["sim"]["use_gpu_pipeline"]:
            if self.device_type.lower() in ("cuda", "gpu"):
                self.device = "cuda:" + str(self.device_id)
            else:
                config["sim"]["use_gpu_pipeline"] = False
        self.rl_device = rl_device
        self.headless = headless
        self.graphics_device_id = graphics_device_id
        env = config["env"]
        self.num_environments = env["numEnvs"]
        self.num_agents = env.get("numAgents", 1)
        self.num_observations = env.get("numObservations", 0)
        self.num_states = env.get("numStates", 0)
        self.obs_space = spaces.Box(np.ones(self.num_obs) * -np.inf, np.ones(self.num_obs) * np.inf)
        self.state_space = spaces.Box(np.ones(self.num_states) * -np.inf, np.ones(self.num_states) * np.inf)
        self.num_actions = env["numActions"]
        self.control_freq_inv = env.get("controlFrequencyInv", 1)
        self.act_space = spaces.Box(np.ones(self.num_actions) * -1.0, np.ones(self.num_actions) * 1.0)
        self.clip_obs = env.get("clipObservations", math.inf)
        self.clip_actions = env.get("clipActions", math.inf)
        self.total_train_env_frames = 0
        self.control_steps = 0

    @property
    def observation_space(self):
        return self.obs_space

    @property
    def action_space(self):
        return self.act_space

    @property
    def num_envs(self) -> int:
        return self.num_environments

    @property
    def num_acts(self) -> int:
        return self.num_actions

    @property
    def num_obs(self) -> int:
        return self.num_observations

    def set_train_info(self, env_frames, *args, **kwargs):
        self.total_train_env_frames = env_frames

    def get_env_state(self):
        return None

    def set_env_state(self, env_state):
        pass


class VecTask(DomainRandomizationMixin, Env):
    """Base class of the MI355X tasks.  Subclasses set ``task_name`` and fill
    ``cfg['env']['numObservations'/'numActions']`` before calling ``__init__``."""

    metadata = {"render.modes": ["human", "rgb_array"], "video.frames_per_second": 24}
    task_name = None
    # domain randomization (migym/dr.py): actor names of task.randomization_params.actor_params, and
    # whether the task resets (and so randomizes) in pre_physics_step (ShadowHand) or post_physics_step
    dr_actor_names = {}
    dr_reset_in_pre_physics = False
    # whether the reference task calls gym.acquire_dof_force_tensor (humanoid.py:85-86, shadow_hand.py:157-159): the
    # DOF-force view is bound, and the fused step computes the forces, only then
    acquires_dof_force = False

    def __init__(self, config, rl_device, sim_device, graphics_device_id, headless, virtual_screen_capture=False,
                 force_render=False):
        self.cfg = config
        super().__init__(config, rl_device, sim_device, graphics_device_id, headless)
        if self.device == "cpu":
            raise RuntimeError("migym simulates on the MI355X: for the CPU pipeline (use_gpu_pipeline=False or "
                               "sim_device='cpu') create the task through migym.make / isaacgymenvs.make, which runs "
                               "the HIP step and exposes host-side views (migym/host_pipeline.py)")
        if not torch.cuda.is_available():
            raise RuntimeError("migym needs a HIP device (torch.cuda.is_available() is False)")
        self.virtual_screen_capture = virtual_screen_capture
        self.force_render = force_render
        self.dt = float(config["sim"]["dt"])
        self.control_freq_inv = int(config["env"].get("controlFrequencyInv", 1))
        self.viewer = None
        self.seed = int(config.get("seed", 0) or 0)
        self.env_offset = int(config.get("env_offset", 0))
        self._lib = _abi.lib()
        self._gather = None
        self.launch_events = None
        self.create_sim()
        self.allocate_buffers()
        self.obs_dict = {}
        self.extras = {}
        self._dr_init()
        self.sim_initialized = True

    # ---------------------------------------------------------------------------------- setup
    def create_sim(self):
        base = "Ant" if self.task_name == "MAAnt" else self.task_name
        _, table, _, _, _, max_contacts = taskdefs.TASK_INFO[base]
        self.model_spec = M.load_builtin(table)
        self.num_dof = self.model_spec.num_dofs
        self.num_bodies = len(self.model_spec.bodies)
        self.num_actors = self.num_envs * self.num_agents
        self.sim_params = taskdefs.sim_params(self.cfg, max_contacts, self.num_agents)
        self.task_params = taskdefs.task_params(self.task_name, self.cfg, self.model_spec)
        self._model_np = _abi.model_bytes(self.model_spec)
        torch.cuda.set_device(self.device_id)
        h = _abi.C.c_void_p()
        _abi.check(self._lib.mg_sim_create(self._model_np.ctypes.data, _abi.C.byref(self.sim_params),
                                           self.num_actors, self.device_id, _abi.C.byref(h)), self._lib)
        self.sim = h
        dev, f = self.device, torch.float32
        A, nd, ns = self.num_actors, self.num_dof, len(self.model_spec.sensors)
        # gym-visible state tensors (acquire_*_tensor + wrap_tensor): zero-copy, owned by torch
        self.root_states = torch.zeros((A, 13), device=dev, dtype=f)
        self.root_states[:, 0:3] = torch.tensor(list(self.task_params.start_pos), device=dev)
        if self.num_agents > 1:
            offs = torch.tensor([list(self.task_params.agent_offset[k]) for k in range(self.num_agents)],
                                device=dev, dtype=f)
            self.root_states[:, 0:3] += offs.repeat(self.num_envs, 1)
        self.root_states[:, 3:7] = torch.tensor(list(self.task_params.start_rot), device=dev)
        self.initial_root_states = self.root_states.clone()
        self.initial_root_states[:, 7:13] = 0
        self.dof_state = torch.zeros((A * nd, 2), device=dev, dtype=f)
        self.dof_pos = self.dof_state.view(A, nd, 2)[..., 0]
        self.dof_vel = self.dof_state.view(A, nd, 2)[..., 1]
        self.dof_actuation = torch.zeros((A * nd,), device=dev, dtype=f)
        self.sensor_tensor = torch.zeros((A * max(ns, 1), 6), device=dev, dtype=f)
        self.vec_sensor_tensor = self.sensor_tensor.view(A, max(ns, 1) * 6)
        self.dof_force_tensor = torch.zeros((A, nd), device=dev, dtype=f)
        lo, hi = taskdefs.dof_limits(self.model_spec)
        self.dof_limits_lower = torch.tensor(lo, device=dev, dtype=f)
        self.dof_limits_upper = torch.tensor(hi, device=dev, dtype=f)
        self.initial_dof_pos = torch.tensor(list(self.task_params.initial_dof_pos)[:nd], device=dev,
                                            dtype=f).repeat(A, 1)
        v = _abi.StateViews()
        v.root_states, v.dof_state = _abi.ptr(self.root_states), _abi.ptr(self.dof_state)
        v.dof_actuation, v.sensors = _abi.ptr(self.dof_actuation), _abi.ptr(self.sensor_tensor)
        # the DOF-force view only where the reference acquires one (humanoid.py:85-86: acquires_dof_force); Ant and
        # Cartpole never do (ant.py, cartpole.py), so the fused step skips their DOF forces and dof_force_tensor
        # stays zero
        v.dof_force = _abi.ptr(self.dof_force_tensor) if self.acquires_dof_force else None
        v.rigid_body_states = None
        self._views = v
        _abi.check(self._lib.mg_sim_bind(self.sim, _abi.C.byref(v)), self._lib)

    def allocate_buffers(self):
        dev, A = self.device, self.num_actors
        self.obs_buf = torch.zeros((A, self.num_obs), device=dev, dtype=torch.float)
        self.states_buf = torch.zeros((self.num_envs, self.num_states), device=dev, dtype=torch.float)
        self.rew_buf = torch.zeros(A, device=dev, dtype=torch.float)
        self.reset_buf = torch.ones(A, device=dev, dtype=torch.long)
        self.timeout_buf = torch.zeros(A, device=dev, dtype=torch.bool)
        self.progress_buf = torch.zeros(A, device=dev, dtype=torch.long)
        self.randomize_buf = torch.zeros(self.num_envs, device=dev, dtype=torch.long)
        self.actions = torch.zeros((A, self.num_actions), device=dev, dtype=torch.float)
        self._clamp_obs = math.isfinite(float(self.clip_obs))
        self.obs_clamped = torch.zeros_like(self.obs_buf) if self._clamp_obs else self.obs_buf
        pot = -1000.0 / self.dt
        self.potentials = torch.full((A,), pot, device=dev, dtype=torch.float)
        self.prev_potentials = self.potentials.clone()
        self.up_vec = torch.zeros((A, 3), device=dev, dtype=torch.float)
        self.up_vec[:, 2] = 1.0
        self.heading_vec = torch.zeros((A, 3), device=dev, dtype=torch.float)
        self.heading_vec[:, 0] = 1.0
        self.targets = torch.tensor([[1000.0, 0.0, 0.0]], device=dev).repeat(A, 1)
        if self.num_agents > 1:
            self.targets += self.root_states[:, 0:3] - self.root_states[:, 0:3].new_tensor(
                list(self.task_params.start_pos))
            self.targets[:, 2] = 0.0
        self._noise = None
        tb = _abi.TaskBuffers()
        tb.actions_out, tb.obs = _abi.ptr(self.actions), _abi.ptr(self.obs_buf)
        tb.obs_clamped = _abi.ptr(self.obs_clamped) if self._clamp_obs else None
        tb.rew, tb.reset, tb.progress = _abi.ptr(self.rew_buf), _abi.ptr(self.reset_buf), _abi.ptr(self.progress_buf)
        tb.timeout = _abi.ptr(self.timeout_buf)
        tb.potentials, tb.prev_potentials = _abi.ptr(self.potentials), _abi.ptr(self.prev_potentials)
        tb.up_vec, tb.heading_vec = _abi.ptr(self.up_vec), _abi.ptr(self.heading_vec)
        tb.seed, tb.env_offset = self.seed, self.env_offset
        self._tb = tb

    # ---------------------------------------------------------------------------------- hot path
    def _stream(self):
        return torch.cuda.current_stream(self.device).cuda_stream

    def step(self, actions: torch.Tensor) -> Tuple[Dict[str, torch.Tensor], torch.Tensor, torch.Tensor,
                                                   Dict[str, Any]]:
        """VecTask.step (vec_task.py:362-410) as one fused device launch per control step."""
        a = actions
        if a.device != torch.device(self.device) or a.dtype != torch.float32 or not a.is_contiguous():
            a = a.to(device=self.device, dtype=torch.float32).contiguous()
        if a.shape != (self.num_actors, self.num_actions):
            raise ValueError(f"actions must be {(self.num_actors, self.num_actions)}, got {tuple(a.shape)}")
        dr = self.randomize and self._dr is not None
        if dr:
            a = self._dr_actions(a)   # vec_task.py:372-374
            if self.dr_reset_in_pre_physics:   # reset_idx in pre_physics_step (shadow_hand.py:599-607)
                self._dr_step(self.reset_buf, pending_increment=self.control_steps > 0)
            else:
                self._dr["mask"].copy_(self.reset_buf)   # the resets post_physics_step will apply
        self._actions_in = a   # keep alive until the launch has consumed it
        tb = self._tb
        tb.actions = a.data_ptr()
        tb.noise = _abi.ptr(self._noise)
        g = self._gather
        tb.out_pack = _abi.ptr(g.next_pack()) if g is not None else None
        stream = self._stream()
        # one launch: pre_physics_step, gym.simulate x controlFrequencyInv (task_params.control_freq_inv),
        # post_physics_step (vec_task.py:376-396)
        tb.step_counter = self.control_steps
        ev = self.launch_events   # optional (start, end) torch.cuda.Event pair around the launch (bench.py)
        if ev is not None:
            ev[0].record(torch.cuda.current_stream(self.device))
        _abi.check(self._lib.mg_env_step(self.sim, _abi.C.byref(self.task_params), _abi.C.byref(tb), stream),
                   self._lib)
        if ev is not None:
            ev[1].record(torch.cuda.current_stream(self.device))
        self.post_launch()
        if g is not None:
            g.issue()   # gather of this step's rows, overlapped with the next step (migym/dist.py)
        self.control_steps += 1
        self.frame_count += self.control_freq_inv
        if dr:
            if not self.dr_reset_in_pre_physics:   # reset_idx in post_physics_step (ant.py:287-293)
                self._dr_step(self._dr["mask"], pending_increment=True)
            self._dr_observations()   # vec_task.py:398-400
        self.extras["time_outs"] = self.timeout_buf.to(self.rl_device)
        self.post_step_extras()
        self.obs_dict["obs"] = self.obs_clamped.to(self.rl_device)
        if self.num_states > 0:
            self.obs_dict["states"] = self.get_state()
        return self.obs_dict, self.rew_buf.to(self.rl_device), self.reset_buf.to(self.rl_device), self.extras

    def _dr_step(self, mask, pending_increment):
        """apply_randomizations as reset_idx calls it (only when some env resets: with dr_exact_trigger this
        is checked with one host synchronisation, otherwise assumed), plus post_physics_step's
        randomize_buf += 1 that precedes it."""
        if (not self.dr_exact_trigger) or bool(mask.any()):
            self.apply_randomizations(self.randomization_params, reset_mask=mask, increment=pending_increment)
        elif pending_increment:
            self.randomize_buf_actors += 1

    # ---------------------------------------------------------------------------------- gym tensor API
    def acquire_net_contact_force_tensor(self) -> torch.Tensor:
        """gym.acquire_net_contact_force_tensor + gymtorch.wrap_tensor (franka_reach_MA.py:506): the (N*A*nB, 3)
        world-frame net contact force on each rigid body (hand tasks: the hand's bodies, the object, the goal) over
        the last substep, in the rigid-body layout.  Binding it (mg_state_views.net_contact_forces) makes the fused
        step and mg_sim_simulate write it every step; unbound, nothing computes it (the reference's Ant, Humanoid,
        ShadowHand and Cartpole never acquire it).  Zero-copy, like every gym tensor here."""
        t = getattr(self, "net_contact_force_tensor", None)
        if t is None:
            t = torch.zeros((self.num_actors * self.num_bodies, 3), device=self.device, dtype=torch.float32)
            self.net_contact_force_tensor = t
            self._views.net_contact_forces = _abi.ptr(t)
            _abi.check(self._lib.mg_sim_bind(self.sim, _abi.C.byref(self._views)), self._lib)
        return t

    def refresh_net_contact_force_tensor(self):
        """gym.refresh_net_contact_force_tensor (franka_reach_MA.py:563): a no-op -- the bound tensor is written by
        the step itself"""

    def kernel_span_begin(self, n: int):
        """record the device-side duration (first wave start -> last wave end, GPU wall clock) of the next n fused
        step launches (mg_kernel_span_begin; 0 stops recording).  A measurement aid: bench.py's kernel_ms"""
        _abi.check(self._lib.mg_kernel_span_begin(self.sim, int(n)), self._lib)

    def kernel_span_read(self, n: int):
        """the recorded spans in ms, in launch order (synchronises the device)"""
        buf = np.zeros(max(int(n), 1), np.float64)
        got = _abi.C.c_int32(0)
        _abi.check(self._lib.mg_kernel_span_read(self.sim, buf.ctypes.data, int(n), _abi.C.byref(got)), self._lib)
        return buf[:got.value]

    def post_launch(self):
        """Device work that follows the fused launch in stream order (ShadowHand: the cross-rank
        running-mean reduction)."""

    def attach_output_gather(self, gather):
        """Route every step's [clamped obs | rew | reset] rows into ``gather`` (migym.dist.PackedGather):
        the kernel writes them into the gather's message slot and the gather overlaps the next step."""
        if gather is not None and (gather.rows != self.num_actors or gather.nobs != self.num_obs):
            raise ValueError("gather shape does not match (num_actors, num_obs)")
        self._gather = gather

    def post_step_extras(self):
        """Task-specific extras (e.g. Ant's true_objective); cheap device views only."""

    # ---------------------------------------------------------------------------------- env state
    # device tensors that carry a rollout from one step to the next (the gym-visible state and the task
    # buffers the fused kernel reads back); subclasses extend the list
    env_state_tensors = ("root_states", "dof_state", "dof_actuation", "sensor_tensor", "dof_force_tensor",
                         "obs_buf", "obs_clamped", "states_buf", "rew_buf", "reset_buf", "timeout_buf",
                         "progress_buf", "randomize_buf", "actions", "potentials", "prev_potentials", "up_vec",
                         "heading_vec", "env_props", "randomize_buf_actors")
    env_state_scalars = ("control_steps", "frame_count", "last_step", "last_rand_step")

    def get_env_state(self):
        """Serializable env state for a checkpoint (the reference's hook, vec_task.py:197-205, returns None;
        SURVEY.md §5 asks for the SoA state tensors): a dict of clones of every per-env device tensor that
        carries the rollout, plus the step counters.  ``set_env_state`` of it resumes the rollout exactly
        (the reset RNG is keyed by (seed, env, control step), so the counters are part of the state); with
        domain randomization the draw counters, noise state and randomized sim params are part of it too."""
        out, seen = {}, set()
        for k in self.env_state_tensors:
            t = getattr(self, k, None)
            if isinstance(t, torch.Tensor) and t.data_ptr() not in seen:
                seen.add(t.data_ptr())
                out[k] = t.detach().clone()
        for k in self.env_state_scalars:
            if hasattr(self, k):
                out[k] = getattr(self, k)
        dr = self._dr_get_state()
        if dr is not None:
            out["domain_randomization"] = dr
        return out

    def set_env_state(self, env_state):
        """Restore ``get_env_state``'s dict in place (the sim keeps pointers to these tensors). ``None`` (what
        a reference checkpoint holds) is a no-op."""
        if env_state is None:
            return
        for k, v in env_state.items():
            cur = getattr(self, k, None)
            if isinstance(cur, torch.Tensor):
                if tuple(cur.shape) != tuple(v.shape):
                    raise ValueError(f"set_env_state: {k} has shape {tuple(v.shape)}, expected {tuple(cur.shape)}")
                cur.copy_(v.to(cur.device, cur.dtype))
            elif k in self.env_state_scalars:
                setattr(self, k, v)
            elif k == "domain_randomization":
                self._dr_set_state(v)

    # ---------------------------------------------------------------------------------- API
    def get_state(self):
        return torch.clamp(self.states_buf, -self.clip_obs, self.clip_obs).to(self.rl_device)

    def zero_actions(self) -> torch.Tensor:
        return torch.zeros([self.num_actors, self.num_actions], dtype=torch.float32, device=self.rl_device)

    def reset(self):
        """Returns the current observations without computing them (vec_task.py:428-440)."""
        self.obs_dict["obs"] = torch.clamp(self.obs_buf, -self.clip_obs, self.clip_obs).to(self.rl_device)
        if self.num_states > 0:
            self.obs_dict["states"] = self.get_state()
        return self.obs_dict

    def reset_idx(self, env_ids, goal_env_ids=None):
        """reset_idx (ant.py:252-279, humanoid.py:251-278, cartpole.py:122-136, shadow_hand.py:586-668):
        the listed envs (MA layouts: agent ids, kept only where every agent of the env is listed -- the AND
        filter below; a partial agent list resets nothing) get their reset state written now, by one device launch
        (``mg_reset_idx``): DOF noise, root rows and potentials, or ShadowHand's goal, object, hand DOFs and
        PD targets; progress / reset (/ successes) cleared.  A caller reading ``root_states`` right after
        sees the reset state, as with the reference.  Inside ``step`` the fused kernel applies
        ``reset_buf``'s resets itself.  ``goal_env_ids`` (ShadowHand) are reset with the env (their goal is
        redrawn as part of the env reset).

        Multi-agent layouts (num_agents > 1) take agent ids, as the fork's MA tasks do
        (franka_reach_MA.py:616-621, 875-889): ``_agent_ids_to_env_ids(use_AND_filter=True)`` keeps the envs
        whose ids count at least num_agents times (``bincount(agent_ids // A) >= A``), and every agent of
        those envs is reset (``_env_ids_to_agent_ids``).  The filter runs on the device: the launch gets all
        N*A actor rows, -1 for the rows it skips, so there is no host synchronisation.

        With domain randomization on, ``apply_randomizations`` runs first, as the reference's reset_idx does
        (ant.py:254-256); like the reference's, it selects the envs to randomize from ``reset_buf``."""
        ids = torch.as_tensor(env_ids, device=self.device).flatten().to(torch.int64)
        if ids.numel() == 0:
            return
        if self.num_agents > 1:
            A, N = self.num_agents, self.num_envs
            full = torch.bincount(ids // A, minlength=N)[:N] >= A
            rows = torch.arange(N * A, device=self.device, dtype=torch.int64)
            ids = torch.where(full.repeat_interleave(A), rows, torch.full_like(rows, -1))
        ids = ids.to(torch.int32).contiguous()
        n = int(ids.numel())
        if self.randomize and self._dr is not None:
            self.apply_randomizations(self.randomization_params, reset_mask=self.reset_buf, increment=False)
        self._reset_ids = ids   # alive until the launch has consumed it
        tb = self._tb
        tb.step_counter = self.control_steps
        tb.noise = _abi.ptr(self._noise)
        _abi.check(self._lib.mg_reset_idx(self.sim, _abi.C.byref(self.task_params), _abi.C.byref(tb), ids.data_ptr(),
                                          n, self._stream()), self._lib)

    def reset_done(self):
        """reset_done (vec_task.py:442-457): ``reset_idx`` of every env whose ``reset_buf`` is set, applied now (one
        ``mg_reset_idx`` launch: noise, root/DOF rows, potentials; progress and reset_buf cleared), then the current
        observations clamped -- not recomputed, so they stay the terminal ones, as in the reference -- and the done
        ids.  The next ``step`` then simulates those envs from their reset state and does not reset them again.
        Multi-agent layouts: the ids are agent ids and ``reset_idx``'s AND filter applies (franka_reach_MA.py:
        616-621), so an env resets only when all its agents are done.  The ``nonzero`` is a host synchronisation,
        as in the reference; ``step`` itself never needs one."""
        done_env_ids = self.reset_buf.nonzero(as_tuple=False).flatten()
        if len(done_env_ids) > 0:
            self.reset_idx(done_env_ids)
        self.obs_dict["obs"] = torch.clamp(self.obs_buf, -self.clip_obs, self.clip_obs).to(self.rl_device)
        if self.num_states > 0:
            self.obs_dict["states"] = self.get_state()
        return self.obs_dict, done_env_ids

    def set_reset_noise(self, noise: torch.Tensor | None):
        """Inject per-env U(0,1) reset noise rows (N*A, 2*nD) instead of the device RNG
        (parity tests replay the reference's torch draws through this)."""
        self._noise = None if noise is None else noise.to(self.device, torch.float32).contiguous()

    def render(self, mode="rgb_array"):
        return None

    def close(self):
        if getattr(self, "sim", None) is not None:
            self._lib.mg_sim_destroy(self.sim)
            self.sim = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
