"""ctypes binding of the CPU oracle (TEST INFRASTRUCTURE ONLY).

Imported by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg —
never by the product package.  Parity status: see oracle.h.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
# MG_ORACLE_LIB: an alternative build of the checker (the sanitizer build, `make sanitize`;
# tests/test_oracle_sanitize.py runs the oracle tests against it)
LIB = os.environ.get("MG_ORACLE_LIB") or os.path.join(HERE, "build", "liboracle.so")
sys.path.insert(0, os.path.join(HERE, "..", "isaacgymenvs-ma_amd"))
from migym import _abi  # noqa: E402  (struct mirrors only)

LIB_F32 = os.path.join(HERE, "build", "liboracle_f32.so")
_lib = None
_lib32 = None


def build():
    subprocess.check_call(["make", "-s", "-C", HERE])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        l = C.CDLL(LIB)
        P = C.c_void_p
        l.orc_uniform.restype = C.c_float
        l.orc_uniform.argtypes = [C.c_uint64, C.c_uint64, C.c_uint64, C.c_uint32]
        l.orc_simulate.argtypes = [P, C.POINTER(_abi.SimParams), C.c_int32, P, P, P, P, P, C.c_int32]
        l.orc_mass_matrix.argtypes = [P, C.POINTER(_abi.SimParams), P, P, P]
        l.orc_free_acceleration.argtypes = [P, C.POINTER(_abi.SimParams), P, P, P, P]
        l.orc_contacts.argtypes = [P, C.POINTER(_abi.SimParams), P, P, P, C.c_int32]
        l.orc_rigid_body_states.argtypes = [P, P, P, P]
        l.orc_compute_observations.argtypes = [C.POINTER(_abi.TaskParams), C.c_int32] + [P] * 10
        l.orc_compute_reward.argtypes = [C.POINTER(_abi.TaskParams), C.c_int32] + [P] * 7
        l.orc_post_physics.argtypes = [C.POINTER(_abi.TaskParams), C.POINTER(_abi.StateViews),
                                       C.POINTER(_abi.TaskBuffers), C.c_int32]
        l.orc_env_step.argtypes = [P, C.POINTER(_abi.SimParams), C.POINTER(_abi.TaskParams),
                                   C.POINTER(_abi.StateViews), C.POINTER(_abi.TaskBuffers), C.c_int32, C.c_int32]
        l.orc_reset_idx.argtypes = [C.POINTER(_abi.TaskParams), C.POINTER(_abi.StateViews),
                                    C.POINTER(_abi.TaskBuffers), P, C.c_int32, C.c_int32]
        l.orc_simulate_views.argtypes = [P, C.POINTER(_abi.SimParams), C.c_int32, C.POINTER(_abi.StateViews),
                                         C.c_int32]
        l.orc_randomize_rotation.restype = None
        l.orc_randomize_rotation.argtypes = [C.c_float, C.c_float, P]
        l.orc_hand_reward.argtypes = [C.POINTER(_abi.TaskParams), C.c_int32, C.c_float] + [P] * 11
        for f in ("orc_hand_pre_physics", "orc_hand_post_physics"):
            getattr(l, f).argtypes = [P, C.POINTER(_abi.TaskParams), C.POINTER(_abi.StateViews),
                                      C.POINTER(_abi.TaskBuffers), C.c_int32]
        l.orc_hand_env_step.argtypes = [P, C.POINTER(_abi.SimParams), C.POINTER(_abi.TaskParams),
                                        C.POINTER(_abi.StateViews), C.POINTER(_abi.TaskBuffers), C.c_int32,
                                        C.c_int32]
        l.orc_hand_finalize.argtypes = [C.POINTER(_abi.TaskParams), C.POINTER(_abi.TaskBuffers)]
        l.orc_ellipsoid_contact.argtypes = [C.c_int32, P, C.c_double, P, P]
        l.orc_box_box_edge.argtypes = [P, P, C.c_double, P]
        l.orc_hull_distance.argtypes = [P, P, C.c_int32, P]
        l.orc_hull_core_contact.argtypes = [P, P, C.c_double, C.c_double, P]
        l.orc_step_flips.argtypes = [P, C.POINTER(_abi.SimParams), C.POINTER(_abi.StateViews), C.c_int32, C.c_double,
                                     C.c_double]
        l.orc_dr_apply.argtypes = [C.POINTER(_abi.DrApplyArgs)]
        l.orc_dr_noise.argtypes = [C.POINTER(_abi.DrNoiseArgs)]
        _lib = l
    return _lib


def lib_f32():
    """The fp32 physics build (bench.py's timed CPU baseline; the tests' checker is lib())."""
    global _lib32
    if _lib32 is None:
        if not os.path.exists(LIB_F32):
            build()
        l = C.CDLL(LIB_F32)
        P = C.c_void_p
        l.orc_env_step.argtypes = [P, C.POINTER(_abi.SimParams), C.POINTER(_abi.TaskParams),
                                   C.POINTER(_abi.StateViews), C.POINTER(_abi.TaskBuffers), C.c_int32, C.c_int32]
        l.orc_hand_env_step.argtypes = l.orc_env_step.argtypes
        l.orc_simulate.argtypes = [P, C.POINTER(_abi.SimParams), C.c_int32, P, P, P, P, P, C.c_int32]
        l.orc_simulate_views.argtypes = [P, C.POINTER(_abi.SimParams), C.c_int32, C.POINTER(_abi.StateViews),
                                         C.c_int32]
        _lib32 = l
    return _lib32


def f32(a):
    return np.ascontiguousarray(a, dtype=np.float32)


def i64(a):
    return np.ascontiguousarray(a, dtype=np.int64)


def p(a):
    return None if a is None else a.ctypes.data


def simulate(model_np, sp, root, dof, act=None, sensors=None, dof_force=None, threads=0, fp32=False):
    n = root.shape[0]
    (lib_f32() if fp32 else lib()).orc_simulate(model_np.ctypes.data, C.byref(sp), n, p(root), p(dof), p(act), p(sensors), p(dof_force),
                       threads)


def mass_matrix(model_np, sp, root13, dof2):
    out = np.zeros(46 * 46)
    nv = lib().orc_mass_matrix(model_np.ctypes.data, C.byref(sp), p(f32(root13)), p(f32(dof2)), p(out))
    return out[: nv * nv].reshape(nv, nv)


def free_acceleration(model_np, sp, root13, dof2, tau=None):
    out = np.zeros(46)
    nv = lib().orc_free_acceleration(model_np.ctypes.data, C.byref(sp), p(f32(root13)), p(f32(dof2)),
                                     p(None if tau is None else f32(tau)), p(out))
    return out[:nv]


def contacts(model_np, sp, root13, dof2, cap=64):
    out = np.zeros(9 * cap)
    n = lib().orc_contacts(model_np.ctypes.data, C.byref(sp), p(f32(root13)), p(f32(dof2)), p(out), cap)
    return out[: 9 * n].reshape(n, 9)


def box_box_edge(c, R, h, hb, off):
    """edge-edge contact of hand box (c, R, h) against the object box hb (object frame): None or
    (point, normal from the object to the hand box, separation)"""
    sh = np.concatenate([np.asarray(c, np.float64), np.asarray(R, np.float64).ravel(), np.asarray(h, np.float64)])
    out = np.zeros(7)
    ok = lib().orc_box_box_edge(p(sh), p(np.ascontiguousarray(hb, dtype=np.float64)), float(off), p(out))
    return (out[0:3], out[3:6], out[6]) if ok else None


def hull_distance(model_np, pts):
    """plane distance of geom-frame points to the model's convex-mesh hull: (distances, faces)"""
    pl = np.ascontiguousarray(pts, dtype=np.float64).reshape(-1, 3)
    out = np.zeros((len(pl), 2))
    lib().orc_hull_distance(model_np.ctypes.data, p(pl), len(pl), p(out))
    return out[:, 0], out[:, 1].astype(int)


def hull_core_contact(model_np, kind, shape, radius, off):
    """the exact hull candidates (oracle hull_core_contacts) against a core in the hull's geom frame: kind 0 =
    segment (shape = p0, p1), 1 = box (shape = c, R row-major, h); a list of (point, normal from the core to the
    hull, gap), at most 2"""
    sh = np.concatenate([[float(kind)], np.asarray(shape, np.float64).ravel()])
    out = np.zeros(14)
    n = lib().orc_hull_core_contact(model_np.ctypes.data, p(sh), float(radius), float(off), p(out))
    return [(out[7 * i:7 * i + 3], out[7 * i + 3:7 * i + 6], out[7 * i + 6]) for i in range(n)]


def ellipsoid_contact(kind, shape, radius, e):
    """egg narrowphase (oracle cvx_contact): returns (point, normal, signed distance)"""
    sh = np.ascontiguousarray(shape, dtype=np.float64).ravel()
    ev = np.ascontiguousarray(e, dtype=np.float64)
    out = np.zeros(7)
    lib().orc_ellipsoid_contact(int(kind), p(sh), float(radius), p(ev), p(out))
    return out[0:3], out[3:6], out[6]


def step_flips(model_np, sp, host, delta=1e-4, df=1e-2):
    """per env of a HostEnv / HandHostEnv holding a step's physics input (after pre-physics): the bit mask of
    orc_step_flips (1 contact threshold in use, 2 limit threshold in use, 4 drive near saturation, 8 seg_box_sat
    tie) over the substeps of one gym.simulate"""
    v = host.views()
    return np.array([lib().orc_step_flips(model_np.ctypes.data, C.byref(sp), C.byref(v), e, delta, df)
                     for e in range(host.n)], np.int32)


def rigid_body_states(model_np, root13, dof2, nbodies):
    out = np.zeros((nbodies, 13), dtype=np.float32)
    lib().orc_rigid_body_states(model_np.ctypes.data, p(f32(root13)), p(f32(dof2)), p(out))
    return out


def compute_observations(tp, root, dof, dof_force, sensors, actions, potentials, prev_potentials, up, heading,
                         obs):
    lib().orc_compute_observations(C.byref(tp), root.shape[0], p(root), p(dof), p(dof_force), p(sensors),
                                   p(actions), p(potentials), p(prev_potentials), p(up), p(heading), p(obs))


def compute_reward(tp, obs, actions, potentials, prev_potentials, progress, reset, rew):
    lib().orc_compute_reward(C.byref(tp), obs.shape[0], p(obs), p(actions), p(potentials), p(prev_potentials),
                             p(progress), p(reset), p(rew))


def randomize_rotation(r0, r1):
    out = np.zeros((len(r0), 4), np.float32)
    for i, (a, b) in enumerate(zip(r0, r1)):
        lib().orc_randomize_rotation(float(a), float(b), out[i].ctypes.data)
    return out


def hand_reward(tp, max_episode_length, object_pos, object_rot, target_pos, target_rot, actions, reset, reset_goal,
                progress, successes, cons):
    """compute_hand_reward (shadow_hand.py:746-800); buffers updated in place, returns (rew, cons)."""
    n = object_pos.shape[0]
    rew = np.zeros(n, np.float32)
    c = np.array([cons], np.float32)
    lib().orc_hand_reward(C.byref(tp), n, max_episode_length, p(f32(object_pos)), p(f32(object_rot)),
                          p(f32(target_pos)), p(f32(target_rot)), p(f32(actions)), p(reset), p(reset_goal),
                          p(progress), p(successes), p(c), p(rew))
    return rew, float(c[0])


def uniform(seed, env, counter, k):
    return lib().orc_uniform(seed, env, counter, k)


class HostEnv:
    """Host buffers for the oracle's full step (same layout the GPU path binds)."""

    def __init__(self, tp, spec, n, agents=1):
        nd = spec.num_dofs
        na, no = tp.num_actions, tp.num_obs
        ns = len(spec.sensors)
        self.n = n
        self.root = np.zeros((n, 13), np.float32)
        self.root[:, 0:3] = np.array(tp.start_pos[:3], np.float32)
        self.root[:, 3:7] = np.array(tp.start_rot[:4], np.float32)
        A = max(int(tp.num_agents), 1)
        if A > 1:
            offs = np.array([list(tp.agent_offset[k]) for k in range(A)], np.float32)
            self.root[:, 0:3] += np.tile(offs, (n // A, 1))
        self.dof = np.zeros((n, nd, 2), np.float32)
        self.act_eff = np.zeros((n, nd), np.float32)
        self.sensors = np.zeros((n, max(ns, 1) * 6), np.float32)
        self.dof_force = np.zeros((n, nd), np.float32)
        self.actions = np.zeros((n, na), np.float32)
        self.actions_out = np.zeros((n, na), np.float32)
        self.obs = np.zeros((n, no), np.float32)
        self.obs_clamped = np.zeros((n, no), np.float32)
        self.rew = np.zeros(n, np.float32)
        self.reset = np.ones(n, np.int64)
        self.progress = np.zeros(n, np.int64)
        self.timeout = np.zeros(n, np.uint8)
        pot = -1000.0 / tp.dt
        self.potentials = np.full(n, pot, np.float32)
        self.prev_potentials = np.full(n, pot, np.float32)
        self.up = np.zeros((n, 3), np.float32)
        self.heading = np.zeros((n, 3), np.float32)
        self.noise = None
        self.env_props = None   # (n, stride) domain-randomized properties, or None
        self.ncf = None         # (n, num_bodies, 3) net contact forces when bound (acquire_net_contact_force_tensor)

    def views(self):
        v = _abi.StateViews()
        v.root_states, v.dof_state, v.dof_actuation = p(self.root), p(self.dof), p(self.act_eff)
        v.sensors, v.dof_force, v.rigid_body_states = p(self.sensors), p(self.dof_force), None
        v.net_contact_forces = p(self.ncf)
        if self.env_props is not None:
            v.env_props, v.env_props_stride = p(self.env_props), self.env_props.shape[1]
        return v

    def buffers(self, seed=0, step=0, env_offset=0):
        b = _abi.TaskBuffers()
        b.actions, b.actions_out, b.obs, b.obs_clamped = p(self.actions), p(self.actions_out), p(self.obs), \
            p(self.obs_clamped)
        b.rew, b.reset, b.progress, b.timeout = p(self.rew), p(self.reset), p(self.progress), p(self.timeout)
        b.potentials, b.prev_potentials = p(self.potentials), p(self.prev_potentials)
        b.up_vec, b.heading_vec = p(self.up), p(self.heading)
        b.noise = p(self.noise)
        b.seed, b.step_counter, b.env_offset = seed, step, env_offset
        return b

    def post_physics(self, tp, seed=0, step=0, env_offset=0):
        v, b = self.views(), self.buffers(seed, step, env_offset)
        lib().orc_post_physics(C.byref(tp), C.byref(v), C.byref(b), self.n)

    def simulate(self, model_np, sp, threads=0, fp32=False):
        """gym.simulate alone on these buffers (orc_simulate_views: net contact forces too when self.ncf is set)"""
        v = self.views()
        (lib_f32() if fp32 else lib()).orc_simulate_views(model_np.ctypes.data, C.byref(sp), self.n, C.byref(v),
                                                           threads)

    def env_step(self, model_np, sp, tp, seed=0, step=0, threads=0, env_offset=0, fp32=False):
        v, b = self.views(), self.buffers(seed, step, env_offset)
        (lib_f32() if fp32 else lib()).orc_env_step(model_np.ctypes.data, C.byref(sp), C.byref(tp), C.byref(v),
                                                     C.byref(b), self.n, threads)

    def reset_idx(self, tp, ids, seed=0, step=0, env_offset=0):
        """reset_idx(ids) now (orc_reset_idx; ids < 0 skipped, noise rows by actor)"""
        ids = np.ascontiguousarray(ids, np.int32)
        v, b = self.views(), self.buffers(seed, step, env_offset)
        rc = lib().orc_reset_idx(C.byref(tp), C.byref(v), C.byref(b), p(ids), len(ids), self.n)
        assert rc == 0


class HandHostEnv:
    """Host buffers of one ShadowHand shard (layouts the GPU path binds: root rows
    [hand, object, goal] per env, rigid bodies [hand bodies, object, goal])."""

    def __init__(self, tp, spec, n):
        nd, na, no = spec.num_dofs, tp.num_actions, tp.num_obs
        nb = len(spec.bodies) + 2
        self.n, self.nd = n, nd
        self.root = np.zeros((n, 3, 13), np.float32)
        self.root[:, 0, 0:3] = np.array(tp.start_pos[:3], np.float32)
        self.root[:, 0, 3:7] = np.array(tp.start_rot[:4], np.float32)
        obj = np.array(tp.object_start[:3], np.float32)
        self.root[:, 1, 0:3] = obj
        self.root[:, 1, 6] = 1.0
        self.goal_states = np.zeros((n, 13), np.float32)
        self.goal_states[:, 0:3] = obj
        self.goal_states[:, 2] += np.float32(tp.goal_dz)
        self.goal_states[:, 6] = 1.0
        self.root[:, 2, 0:3] = self.goal_states[:, 0:3] + np.array(tp.goal_displacement[:3], np.float32)
        self.root[:, 2, 6] = 1.0
        self.dof = np.zeros((n, nd, 2), np.float32)
        self.targets = np.zeros((n, nd), np.float32)
        self.prev_targets = np.zeros((n, nd), np.float32)
        self.sensors = np.zeros((n, len(spec.sensors) * 6), np.float32)
        self.dof_force = np.zeros((n, nd), np.float32)
        self.rbs = np.zeros((n, nb, 13), np.float32)
        self.ncf = None   # (n, nb, 3) net contact forces when bound (acquire_net_contact_force_tensor)
        self.actions = np.zeros((n, na), np.float32)
        self.actions_out = np.zeros((n, na), np.float32)
        self.obs = np.zeros((n, no), np.float32)
        self.obs_clamped = np.zeros((n, no), np.float32)
        self.rew = np.zeros(n, np.float32)
        self.reset = np.ones(n, np.int64)
        self.reset_goal = np.ones(n, np.int64)
        self.progress = np.zeros(n, np.int64)
        self.timeout = np.zeros(n, np.uint8)
        self.successes = np.zeros(n, np.float32)
        self.cons = np.zeros(1, np.float32)
        self.noise = None
        # random object forces (apply_rigid_body_force_tensors, LOCAL_SPACE) and asymmetric states
        self.rb_forces = np.zeros((n, nb, 3), np.float32)
        self.force_prob = None
        self.states = None
        # running-mean partial sums left for a cross-rank all-reduce (defer_finalize)
        self.scratch = np.zeros(2, np.uint64)
        self.defer_finalize = 0
        self.env_props = None   # (n, stride) domain-randomized properties, or None

    def views(self):
        v = _abi.StateViews()
        v.root_states, v.dof_state, v.dof_actuation = p(self.root), p(self.dof), None
        v.sensors, v.dof_force, v.rigid_body_states = p(self.sensors), p(self.dof_force), p(self.rbs)
        v.dof_targets = p(self.targets)
        v.rb_forces, v.rb_force_space = p(self.rb_forces), _abi.MG_LOCAL_SPACE
        v.net_contact_forces = p(self.ncf)
        if self.env_props is not None:
            v.env_props, v.env_props_stride = p(self.env_props), self.env_props.shape[1]
        return v

    def buffers(self, seed=0, step=0, env_offset=0):
        b = _abi.TaskBuffers()
        b.actions, b.actions_out, b.obs, b.obs_clamped = p(self.actions), p(self.actions_out), p(self.obs), \
            p(self.obs_clamped)
        b.states, b.random_force_prob = p(self.states), p(self.force_prob)
        b.rew, b.reset, b.progress, b.timeout = p(self.rew), p(self.reset), p(self.progress), p(self.timeout)
        b.noise = p(self.noise)
        b.seed, b.step_counter, b.env_offset = seed, step, env_offset
        b.prev_targets, b.goal_states, b.reset_goal = p(self.prev_targets), p(self.goal_states), p(self.reset_goal)
        b.successes, b.consecutive_successes = p(self.successes), p(self.cons)
        b.reduce_scratch, b.defer_finalize = p(self.scratch), self.defer_finalize
        return b

    def finalize(self, tp):
        """mg_hand_finalize: the running mean from the (all-reduced) partial sums in ``scratch``."""
        b = self.buffers()
        lib().orc_hand_finalize(C.byref(tp), C.byref(b))

    def pre_physics(self, model_np, tp, seed=0, step=0, env_offset=0):
        v, b = self.views(), self.buffers(seed, step, env_offset)
        lib().orc_hand_pre_physics(model_np.ctypes.data, C.byref(tp), C.byref(v), C.byref(b), self.n)

    def post_physics(self, model_np, tp, seed=0, step=0, env_offset=0):
        v, b = self.views(), self.buffers(seed, step, env_offset)
        lib().orc_hand_post_physics(model_np.ctypes.data, C.byref(tp), C.byref(v), C.byref(b), self.n)

    def simulate(self, model_np, sp, threads=0, fp32=False):
        v = self.views()
        (lib_f32() if fp32 else lib()).orc_simulate_views(model_np.ctypes.data, C.byref(sp), self.n, C.byref(v), threads)

    def env_step(self, model_np, sp, tp, seed=0, step=0, threads=0, env_offset=0, fp32=False):
        v, b = self.views(), self.buffers(seed, step, env_offset)
        (lib_f32() if fp32 else lib()).orc_hand_env_step(model_np.ctypes.data, C.byref(sp), C.byref(tp),
                                                          C.byref(v), C.byref(b), self.n, threads)
