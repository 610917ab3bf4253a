"""Per-task constants -> ``mg_task_params`` / ``mg_sim_params``.

What the reference task constructors compute once at setup
(tasks/ant.py:43-114 + 135-212, tasks/humanoid.py:43-117 + 138-217,
tasks/cartpole.py:36-113, tasks/shadow_hand.py:40-400) and then pass to their jit
functions every step.
"""
from __future__ import annotations

import math

from . import _abi
from . import model as M

TASK_INFO = {
    # name: (task_id, model table, num_obs, num_actions, start z, max_contacts)
    "Cartpole": (_abi.MG_TASK_CARTPOLE, "cartpole", 4, 1, 2.0, 4),
    "Ant": (_abi.MG_TASK_ANT, "ant", 60, 8, 0.44, 16),
    "Humanoid": (_abi.MG_TASK_HUMANOID, "humanoid", 108, 21, 1.34, 32),
    "ShadowHand": (_abi.MG_TASK_SHADOW_HAND, "shadow_hand", 211, 20, 0.5, 24),
}
# observationType -> (layout id, obs size) (shadow_hand.py:108-113; layouts in csrc/hand_task.hpp)
HAND_OBS = {"full_state": (0, 211), "full": (1, 157), "full_no_vel": (2, 77), "openai": (3, 42)}
TASK_INFO["MAAnt"] = TASK_INFO["Ant"]   # per-agent physics/obs of the multi-agent Ant are the Ant's

# build-defined solver constants
BAUMGARTE = 0.2
LIMIT_MARGIN = 0.1


def sim_params(cfg: dict, max_contacts: int, agents: int = 1) -> _abi.SimParams:
    s = cfg["sim"]
    px = s.get("physx", {})
    p = _abi.SimParams()
    p.dt = float(s["dt"])
    p.substeps = int(s.get("substeps", 2))
    for i, g in enumerate(s.get("gravity", [0.0, 0.0, -9.81])):
        p.gravity[i] = float(g)
    p.pos_iters = int(px.get("num_position_iterations", 4))
    p.contact_offset = float(px.get("contact_offset", 0.02))
    p.rest_offset = float(px.get("rest_offset", 0.0))
    p.max_depen_vel = float(px.get("max_depenetration_velocity", 10.0))
    plane = cfg["env"].get("plane", {})
    p.friction = float(plane.get("staticFriction", 1.0))
    p.baumgarte = BAUMGARTE
    p.limit_margin = LIMIT_MARGIN
    p.max_contacts = int(max_contacts)
    p.agents = int(agents)
    # the solver: north_star fixes PGS for this build, so the reference's `physx.solver_type` (config.yaml:31, 1 = TGS
    # by default) does not select it; `physx.solver: tgs` opts in to the build's TGS
    solver = str(px.get("solver", "pgs")).lower()
    if solver not in ("pgs", "tgs"):
        raise ValueError(f"sim.physx.solver must be 'pgs' or 'tgs', got {solver!r}")
    p.solver_type = _abi.MG_SOLVER_TGS if solver == "tgs" else _abi.MG_SOLVER_PGS
    p.vel_iters = int(px.get("num_velocity_iterations", 0))
    return p


def dof_limits(spec: M.ModelSpec):
    """lower/upper as the reference reads them (swapped when lower > upper: ant.py:199-206)."""
    lo, hi = [], []
    for n in spec.nodes[1:]:
        a, b = n.lower, n.upper
        if a > b:
            a, b = b, a
        lo.append(a)
        hi.append(b)
    return lo, hi


def agent_offsets(A: int, spacing: float):
    """Agent k of an env starts at (col, row) of a ceil(sqrt(A))-wide grid, centred on the env origin."""
    cols = int(math.ceil(math.sqrt(A)))
    rows = int(math.ceil(A / cols))
    out = []
    for k in range(A):
        c, r = k % cols, k // cols
        out.append(((c - (cols - 1) / 2.0) * spacing, (r - (rows - 1) / 2.0) * spacing, 0.0))
    return out


def hand_spec(object_type: str = "block") -> M.ModelSpec:
    """The ShadowHand model table with the free object of ``objectType`` (shadow_hand.py:86-100, 229-232)."""
    spec = M.load_builtin("shadow_hand")
    spec.obj = M.hand_object(object_type)
    return spec


def hand_task_params(cfg: dict, spec: M.ModelSpec) -> _abi.TaskParams:
    """ShadowHand constants (shadow_hand.py:46-118, 220-330)."""
    env = cfg["env"]
    obs_type = env.get("observationType", "full_state")
    if obs_type not in HAND_OBS:
        raise ValueError(f"Unknown type of observations! observationType should be one of: {sorted(HAND_OBS)}")
    object_type = env.get("objectType", "block")
    if object_type not in ("block", "egg", "pen"):   # shadow_hand.py:86-87
        raise ValueError(f"objectType must be one of block, egg, pen, got {object_type!r}")
    if spec.obj is None or spec.obj["type"] != M.hand_object(object_type)["type"]:
        raise ValueError(f"model's object does not match objectType {object_type!r} (use taskdefs.hand_spec)")
    tp = _abi.TaskParams()
    tp.task_id = _abi.MG_TASK_SHADOW_HAND
    tp.num_agents = 1
    tp.control_freq_inv = max(1, int(env.get("controlFrequencyInv", 1)))   # vec_task.py:381-384
    tp.obs_type, tp.num_obs = HAND_OBS[obs_type]
    tp.num_actions = len(spec.actuators)
    tp.dt = float(cfg["sim"]["dt"])
    tp.clip_actions = float(env.get("clipActions", math.inf))
    tp.clip_obs = float(env.get("clipObservations", math.inf))
    tp.max_episode_length = int(env["episodeLength"])
    if env.get("resetTime", -1.0) > 0.0:   # shadow_hand.py:127-131
        tp.max_episode_length = int(round(env["resetTime"] / (env.get("controlFrequencyInv", 1) * tp.dt)))
    nd = spec.num_dofs
    for j, n in enumerate(spec.nodes[1:]):
        tp.dof_lower[j], tp.dof_upper[j], tp.initial_dof_pos[j] = n.lower, n.upper, 0.0
    for i, a in enumerate(spec.actuators):
        tp.actuated_dof[i] = spec.dof_index(a["joint"])
    tp.rb_per_env = len(spec.bodies) + 2
    tp.num_dofs = spec.num_dofs
    tp.num_fingertips = len(spec.sensors)
    for i, b in enumerate(spec.sensors):
        tp.fingertip_body[i] = b
    tp.max_consecutive_successes = int(env.get("maxConsecutiveSuccesses", 0))
    tp.use_relative_control = int(bool(env.get("useRelativeControl", False)))
    tp.ignore_z_rot = int(object_type == "pen")   # shadow_hand.py:89, 421; also selects randomize_rotation_pen
    tp.dof_speed_scale = float(env["dofSpeedScale"])
    tp.act_moving_average = float(env["actionsMovingAverage"])
    tp.dist_reward_scale = float(env["distRewardScale"])
    tp.rot_reward_scale = float(env["rotRewardScale"])
    tp.rot_eps = float(env["rotEps"])
    tp.action_penalty_scale = float(env["actionPenaltyScale"])
    tp.success_tolerance = float(env["successTolerance"])
    tp.reach_goal_bonus = float(env["reachGoalBonus"])
    tp.fall_dist = float(env["fallDistance"])
    tp.fall_penalty = float(env["fallPenalty"])
    tp.av_factor = float(env.get("averFactor", 0.1))
    tp.vel_obs_scale = 0.2
    tp.force_torque_obs_scale = 10.0
    tp.reset_position_noise = float(env["resetPositionNoise"])
    tp.reset_dof_pos_noise = float(env["resetDofPosRandomInterval"])
    tp.reset_dof_vel_noise = float(env["resetDofVelRandomInterval"])
    # hand at (0, 0, 0.5); object at hand + (0, -0.39, 0.10); goal = object - 0.04 z, drawn displaced
    tp.start_pos[:] = (0.0, 0.0, 0.5)
    tp.start_rot[:] = (0.0, 0.0, 0.0, 1.0)
    tp.object_start[:] = (0.0, 0.0 + -0.39, 0.5 + (0.02 if object_type == "pen" else 0.10))  # :315-318
    tp.goal_displacement[:] = (-0.2, -0.06, 0.12)
    tp.goal_dz = -0.04
    # asymmetric actor-critic: states_buf (N, 211) = compute_full_state(asymm_obs=True) (shadow_hand.py:125-131)
    tp.num_states = 211 if env.get("asymmetric_observations", False) else 0
    # random object forces (shadow_hand.py:69-72, 196-199, 700-706); the per-step decay factor is
    # torch.pow(float32 forceDecay, dt / forceDecayInterval) exactly as the reference evaluates it
    import torch
    tp.object_rb = len(spec.bodies)
    tp.object_rb_mass = float(spec.obj["mass"]) if spec.obj else 0.0
    tp.force_scale = float(env.get("forceScale", 0.0))
    lo, hi = env.get("forceProbRange", [0.001, 0.1])
    tp.force_prob_lo, tp.force_prob_hi = float(lo), float(hi)
    decay = torch.tensor(float(env.get("forceDecay", 0.99)), dtype=torch.float32)
    dt32 = float(torch.tensor(float(cfg["sim"]["dt"]), dtype=torch.float32))  # gymapi.SimParams.dt is a C float
    tp.force_decay_step = float(torch.pow(decay, dt32 / float(env.get("forceDecayInterval", 0.08))))
    del nd
    return tp


def task_params(task: str, cfg: dict, spec: M.ModelSpec) -> _abi.TaskParams:
    if task == "ShadowHand":
        return hand_task_params(cfg, spec)
    base = "Ant" if task == "MAAnt" else task
    task_id, _, nobs, nact, z0, _ = TASK_INFO[base]
    env = cfg["env"]
    tp = _abi.TaskParams()
    tp.task_id = task_id
    tp.num_agents = 1
    tp.control_freq_inv = max(1, int(env.get("controlFrequencyInv", 1)))   # vec_task.py:381-384
    if task == "MAAnt":
        # build-defined multi-agent Ant (SURVEY.md §8(a) A-MA): A ants on a square grid,
        # obs = Ant obs + the other agents' torso positions relative to self (3 (A-1))
        A = int(env.get("numAgents", 4))
        if A < 1 or A > 8 or 64 % A:
            raise ValueError("numAgents must be 1, 2, 4 or 8")
        tp.num_agents = A
        nobs = nobs + 3 * (A - 1)
        for k, off in enumerate(agent_offsets(A, float(env.get("agentSpacing", 2.0)))):
            tp.agent_offset[k][:] = off
    tp.num_obs = nobs
    tp.num_actions = nact
    tp.dt = float(cfg["sim"]["dt"])
    tp.clip_actions = float(env.get("clipActions", math.inf))
    tp.clip_obs = float(env.get("clipObservations", math.inf))
    tp.target[:] = (1000.0, 0.0, 0.0)
    tp.start_pos[:] = (0.0, 0.0, z0)
    tp.start_rot[:] = (0.0, 0.0, 0.0, 1.0)
    if base == "Cartpole":
        tp.max_episode_length = 500                       # cartpole.py:44 (hard-coded)
        tp.power_scale = float(env["maxEffort"])
        tp.reset_dist = float(env["resetDist"])
        return tp
    tp.max_episode_length = int(env["episodeLength"])
    tp.power_scale = float(env["powerScale"])
    tp.dof_vel_scale = float(env["dofVelocityScale"])
    tp.angular_velocity_scale = float(env.get("angularVelocityScale", 0.1))
    tp.contact_force_scale = float(env["contactForceScale"])
    tp.heading_weight = float(env["headingWeight"])
    tp.up_weight = float(env["upWeight"])
    tp.actions_cost_scale = float(env["actionsCost"])
    tp.energy_cost_scale = float(env["energyCost"])
    tp.joints_at_limit_cost_scale = float(env["jointsAtLimitCost"])
    tp.death_cost = float(env["deathCost"])
    tp.termination_height = float(env["terminationHeight"])
    # actuator gears in MJCF actuator order, applied by DOF position (ant.py:159-161, humanoid.py:160-161)
    gears = [a["gear"] for a in spec.actuators]
    for i, g in enumerate(gears):
        tp.motor_effort[i] = float(g)
    tp.max_motor_effort = float(max(gears)) if gears else 1.0
    lo, hi = dof_limits(spec)
    for i, (a, b) in enumerate(zip(lo, hi)):
        tp.dof_lower[i] = a
        tp.dof_upper[i] = b
        # initial_dof_pos: 0 clamped into the limits (ant.py:96-99)
        tp.initial_dof_pos[i] = a if a > 0 else (b if b < 0 else 0.0)
    return tp
