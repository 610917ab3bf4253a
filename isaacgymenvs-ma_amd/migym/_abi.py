"""ctypes mirror of ``include/migym.h`` and the loader for ``libmigym.so``.

The product path calls ONLY the HIP library built from ``csrc/`` (see
``build.py``).  If the library is missing, :func:`lib` raises: there is no CPU
fallback on the product path.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

from . import model as _model

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(PKG_DIR, "_lib", "libmigym.so")

MG_TASK_CARTPOLE, MG_TASK_ANT, MG_TASK_HUMANOID, MG_TASK_SHADOW_HAND = 0, 1, 2, 3
MG_SET_ROOT_STATE, MG_SET_DOF_STATE, MG_SET_DOF_TARGET = 0, 1, 2
MG_MAX_HAND_DOFS = 32
# [goal-only 4 | reset_idx 53 | reset_target_pose 4 | force-prob redraw 1 | force select 1 | force dir 3]
# (shadow_hand.py:587, 610, 642-643, 704-706)
HAND_NOISE_COLS = 66
MG_ENV_SPACE, MG_LOCAL_SPACE, MG_GLOBAL_SPACE = 0, 1, 2


class SimParams(C.Structure):
    _fields_ = [("dt", C.c_float), ("substeps", C.c_int32), ("gravity", C.c_float * 3),
                ("pos_iters", C.c_int32), ("contact_offset", C.c_float), ("rest_offset", C.c_float),
                ("max_depen_vel", C.c_float), ("friction", C.c_float), ("baumgarte", C.c_float),
                ("limit_margin", C.c_float), ("max_contacts", C.c_int32), ("agents", C.c_int32),
                ("solver_type", C.c_int16), ("vel_iters", C.c_int16)]


MG_SOLVER_PGS, MG_SOLVER_TGS = 0, 1


class StateViews(C.Structure):
    _fields_ = [("root_states", C.c_void_p), ("dof_state", C.c_void_p), ("dof_actuation", C.c_void_p),
                ("sensors", C.c_void_p), ("dof_force", C.c_void_p), ("rigid_body_states", C.c_void_p),
                ("dof_targets", C.c_void_p), ("rb_forces", C.c_void_p), ("rb_force_space", C.c_int32),
                ("env_props_stride", C.c_int32), ("env_props", C.c_void_p), ("net_contact_forces", C.c_void_p)]


# ---- domain randomization (include/migym.h; vec_task.py:612-842, dr_utils.py)
MG_EP_NODE, MG_EP_GEOM, MG_EP_TENDON, MG_EP_OBJECT = 0, 1, 2, 3
MG_EP_NODE_WIDTH = 9   # [mass, armature, damping, stiffness, lower, upper, drive kp, effort, frictionloss]
MG_DR_UNIFORM, MG_DR_GAUSSIAN, MG_DR_LOGUNIFORM = 0, 1, 2
MG_DR_ADDITIVE, MG_DR_SCALING = 0, 1
MG_DR_SCHED_NONE, MG_DR_SCHED_LINEAR, MG_DR_SCHED_CONSTANT = 0, 1, 2


class DrDesc(C.Structure):
    _fields_ = [("distribution", C.c_int32), ("operation", C.c_int32), ("schedule", C.c_int32),
                ("schedule_steps", C.c_int32), ("num_buckets", C.c_int32), ("after_setup", C.c_int32),
                ("range", C.c_float * 2)]


class DrAttr(C.Structure):
    _fields_ = [("slot", C.c_int32), ("desc", C.c_int32), ("og", C.c_float), ("pad", C.c_int32)]


class DrApplyArgs(C.Structure):
    _fields_ = [("descs", C.c_void_p), ("attrs", C.c_void_p), ("nattr", C.c_int32), ("stride", C.c_int32),
                ("n", C.c_int32), ("frequency", C.c_int32), ("first", C.c_int32), ("increment", C.c_int32),
                ("last_step", C.c_int64), ("env_props", C.c_void_p), ("reset_mask", C.c_void_p),
                ("randomize_buf", C.c_void_p), ("samples", C.c_void_p), ("seed", C.c_uint64),
                ("counter", C.c_uint64), ("env_offset", C.c_int64)]


class DrNoiseArgs(C.Structure):
    _fields_ = [("x", C.c_void_p), ("x_clamped", C.c_void_p), ("clip", C.c_float), ("distribution", C.c_int32),
                ("operation", C.c_int32), ("refresh_corr", C.c_int32), ("corr", C.c_void_p), ("n", C.c_int64),
                ("scale", C.c_float), ("shift", C.c_float), ("c_scale", C.c_float), ("c_shift", C.c_float),
                ("injected", C.c_void_p), ("injected_corr", C.c_void_p), ("seed", C.c_uint64),
                ("counter", C.c_uint64), ("elem_offset", C.c_int64), ("key", C.c_uint32), ("pad", C.c_int32)]


class TaskParams(C.Structure):
    _fields_ = [("task_id", C.c_int32), ("num_obs", C.c_int32), ("num_actions", C.c_int32),
                ("max_episode_length", C.c_int32), ("dt", C.c_float), ("clip_actions", C.c_float),
                ("clip_obs", C.c_float), ("power_scale", C.c_float), ("dof_vel_scale", C.c_float),
                ("angular_velocity_scale", C.c_float), ("contact_force_scale", C.c_float),
                ("heading_weight", C.c_float), ("up_weight", C.c_float), ("actions_cost_scale", C.c_float),
                ("energy_cost_scale", C.c_float), ("joints_at_limit_cost_scale", C.c_float),
                ("death_cost", C.c_float), ("termination_height", C.c_float), ("max_motor_effort", C.c_float),
                ("reset_dist", C.c_float), ("target", C.c_float * 3), ("start_pos", C.c_float * 3),
                ("start_rot", C.c_float * 4), ("motor_effort", C.c_float * 64), ("dof_lower", C.c_float * 64),
                ("dof_upper", C.c_float * 64), ("initial_dof_pos", C.c_float * 64),
                ("num_agents", C.c_int32), ("control_freq_inv", C.c_int32), ("agent_offset", (C.c_float * 3) * 8),
                # in-hand manipulation (MG_TASK_SHADOW_HAND)
                ("num_fingertips", C.c_int32), ("fingertip_body", C.c_int32 * 8),
                ("actuated_dof", C.c_int32 * MG_MAX_HAND_DOFS), ("max_consecutive_successes", C.c_int32),
                ("use_relative_control", C.c_int32), ("ignore_z_rot", C.c_int32), ("obs_type", C.c_int32),
                ("rb_per_env", C.c_int32), ("num_dofs", C.c_int32),
                ("dof_speed_scale", C.c_float), ("act_moving_average", C.c_float),
                ("dist_reward_scale", C.c_float), ("rot_reward_scale", C.c_float), ("rot_eps", C.c_float),
                ("action_penalty_scale", C.c_float), ("success_tolerance", C.c_float),
                ("reach_goal_bonus", C.c_float), ("fall_dist", C.c_float), ("fall_penalty", C.c_float),
                ("av_factor", C.c_float), ("vel_obs_scale", C.c_float), ("force_torque_obs_scale", C.c_float),
                ("reset_position_noise", C.c_float), ("reset_dof_pos_noise", C.c_float),
                ("reset_dof_vel_noise", C.c_float), ("object_start", C.c_float * 3),
                ("goal_displacement", C.c_float * 3), ("goal_dz", C.c_float),
                ("num_states", C.c_int32), ("object_rb", C.c_int32), ("force_scale", C.c_float),
                ("force_decay_step", C.c_float), ("force_prob_lo", C.c_float), ("force_prob_hi", C.c_float),
                ("object_rb_mass", C.c_float), ("obs_map", C.c_uint16 * 256), ("state_map", C.c_uint16 * 256)]


class TaskBuffers(C.Structure):
    _fields_ = [("actions", C.c_void_p), ("actions_out", C.c_void_p), ("obs", C.c_void_p),
                ("obs_clamped", C.c_void_p), ("rew", C.c_void_p), ("reset", C.c_void_p),
                ("progress", C.c_void_p), ("timeout", C.c_void_p), ("potentials", C.c_void_p),
                ("prev_potentials", C.c_void_p), ("up_vec", C.c_void_p), ("heading_vec", C.c_void_p),
                ("noise", C.c_void_p), ("seed", C.c_uint64), ("step_counter", C.c_uint64),
                ("env_offset", C.c_int64),
                ("prev_targets", C.c_void_p), ("goal_states", C.c_void_p), ("reset_goal", C.c_void_p),
                ("successes", C.c_void_p), ("consecutive_successes", C.c_void_p), ("reduce_scratch", C.c_void_p),
                ("states", C.c_void_p), ("random_force_prob", C.c_void_p), ("out_pack", C.c_void_p),
                ("defer_finalize", C.c_int32), ("pad_tb", C.c_int32)]


class Replay(C.Structure):
    """mg_replay: the post-simulate state mg_env_step_replay injects in place of gym.simulate (tests)."""
    _fields_ = [("root_states", C.c_void_p), ("dof_state", C.c_void_p), ("sensors", C.c_void_p),
                ("dof_force", C.c_void_p), ("rigid_body_states", C.c_void_p), ("pre_root_states", C.c_void_p),
                ("pre_dof_state", C.c_void_p)]


def model_bytes(spec) -> np.ndarray:
    """mg_model POD for a ModelSpec (numpy structured scalar; pass .ctypes.data)."""
    return np.ascontiguousarray(_model.pack_model(spec))


def ptr(t):
    """data_ptr of a torch tensor / numpy array, or None."""
    if t is None:
        return None
    if hasattr(t, "data_ptr"):
        return t.data_ptr()
    return t.ctypes.data


# ---------------------------------------------------------------------------------------------
EXPORTS = {
    "mg_last_error": (C.c_char_p, []),
    "mg_version": (C.c_int, []),
    "mg_model_sizeof": (C.c_size_t, []),
    "mg_task_params_sizeof": (C.c_size_t, []),
    "mg_task_buffers_sizeof": (C.c_size_t, []),
    "mg_sim_params_sizeof": (C.c_size_t, []),
    "mg_state_views_sizeof": (C.c_size_t, []),
    "mg_debug_phase_cycles": (C.c_int, [C.c_void_p, C.c_int32]),
    "mg_debug_phase_waves": (C.c_int, [C.c_void_p, C.c_int32]),
    "mg_sim_create": (C.c_int, [C.c_void_p, C.POINTER(SimParams), C.c_int32, C.c_int32, C.POINTER(C.c_void_p)]),
    "mg_sim_bind": (C.c_int, [C.c_void_p, C.POINTER(StateViews)]),
    "mg_sim_simulate": (C.c_int, [C.c_void_p, C.c_void_p]),
    "mg_sim_destroy": (C.c_int, [C.c_void_p]),
    "mg_set_indexed": (C.c_int, [C.c_void_p, C.c_int32, C.c_void_p, C.c_void_p, C.c_int32, C.c_void_p]),
    "mg_compute_observations": (C.c_int, [C.POINTER(TaskParams), C.c_int32] + [C.c_void_p] * 10 + [C.c_void_p]),
    "mg_compute_reward": (C.c_int, [C.POINTER(TaskParams), C.c_int32] + [C.c_void_p] * 7 + [C.c_void_p]),
    "mg_post_physics": (C.c_int, [C.c_void_p, C.POINTER(TaskParams), C.POINTER(StateViews),
                                  C.POINTER(TaskBuffers), C.c_int32, C.c_void_p]),
    "mg_pre_physics": (C.c_int, [C.c_void_p, C.POINTER(TaskParams), C.POINTER(StateViews),
                                 C.POINTER(TaskBuffers), C.c_int32, C.c_void_p]),
    "mg_env_step": (C.c_int, [C.c_void_p, C.POINTER(TaskParams), C.POINTER(TaskBuffers), C.c_void_p]),
    "mg_hand_finalize": (C.c_int, [C.POINTER(TaskParams), C.POINTER(TaskBuffers), C.c_void_p]),
    "mg_kernel_span_begin": (C.c_int, [C.c_void_p, C.c_int32]),
    "mg_kernel_span_read": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int32, C.POINTER(C.c_int32)]),
    "mg_kernel_span_waves": (C.c_int, [C.c_void_p, C.c_int32, C.c_void_p, C.c_int32, C.POINTER(C.c_int32)]),
    "mg_work_order": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int32, C.POINTER(C.c_int32),
                                C.POINTER(C.c_int32)]),
    "mg_sim_kernel_layout": (C.c_int, [C.c_void_p, C.POINTER(C.c_int32), C.POINTER(C.c_int32)]),
    "mg_reset_idx": (C.c_int, [C.c_void_p, C.POINTER(TaskParams), C.POINTER(TaskBuffers), C.c_void_p, C.c_int32,
                               C.c_void_p]),
    "mg_env_step_replay": (C.c_int, [C.c_void_p, C.POINTER(TaskParams), C.POINTER(TaskBuffers), C.POINTER(Replay),
                                     C.c_void_p]),
    "mg_dr_desc_sizeof": (C.c_size_t, []),
    "mg_dr_apply_args_sizeof": (C.c_size_t, []),
    "mg_dr_noise_args_sizeof": (C.c_size_t, []),
    "mg_env_props_layout": (C.c_int, [C.c_void_p, C.c_void_p]),
    "mg_env_props_defaults": (C.c_int, [C.c_void_p, C.c_void_p]),
    "mg_dr_apply": (C.c_int, [C.POINTER(DrApplyArgs), C.c_void_p]),
    "mg_dr_noise": (C.c_int, [C.POINTER(DrNoiseArgs), C.c_void_p]),
    "mg_sim_set_params": (C.c_int, [C.c_void_p, C.POINTER(SimParams)]),
}

_LIB = None


class MigymError(RuntimeError):
    pass


def _bind(lib):
    for name, (res, args) in EXPORTS.items():
        f = getattr(lib, name)
        f.restype = res
        f.argtypes = args
    return lib


def check_layout(lib):
    sizes = {"mg_model_sizeof": _model.MODEL_DTYPE.itemsize, "mg_task_params_sizeof": C.sizeof(TaskParams),
             "mg_task_buffers_sizeof": C.sizeof(TaskBuffers), "mg_sim_params_sizeof": C.sizeof(SimParams),
             "mg_state_views_sizeof": C.sizeof(StateViews), "mg_dr_desc_sizeof": C.sizeof(DrDesc),
             "mg_dr_apply_args_sizeof": C.sizeof(DrApplyArgs), "mg_dr_noise_args_sizeof": C.sizeof(DrNoiseArgs)}
    for fn, py in sizes.items():
        c = getattr(lib, fn)()
        if c != py:
            raise MigymError(f"ABI layout mismatch: {fn}() = {c}, Python mirror = {py}")


def lib(path: str | None = None):
    """Load the HIP library (raises if it was not built)."""
    global _LIB
    if _LIB is not None and path is None:
        return _LIB
    p = path or os.environ.get("MIGYM_LIB", LIB_PATH)
    if not os.path.exists(p):
        raise MigymError(f"libmigym.so not found at {p}: run `python __graft_entry__.py build` "
                         "(the product path has no CPU fallback)")
    handle = _bind(C.CDLL(p))
    check_layout(handle)
    if path is None:
        _LIB = handle
    return handle


def check(rc, l=None):
    if rc != 0:
        l = l or lib()
        msg = l.mg_last_error()
        raise MigymError(f"migym call failed ({rc}): {msg.decode() if msg else ''}")
