"""GPU parity of the ShadowHand path through the C ABI.

  * task layer vs the reference's own physics-free trace (tests/golden/trace_shadowhand.npz):
    mg_pre_physics (masked goal/env resets, PD targets) and mg_post_physics (full_state obs,
    compute_hand_reward, the running mean) with the reference's reset draws injected;
    rtol/atol 1e-4 on floats, exact on ints.
  * physics step and the fused mg_env_step vs the fp64 oracle from identical states.  Contacts
    are decided by fp32 vs fp64 distance tests, so an env whose candidate sits within rounding of
    the contact offset may differ: every env must agree within the tolerances of tests/test_gpu_parity.py
    (positions 2e-4, velocities 2e-3 + 2e-3 |v|) unless orc_step_flips puts its step at a discontinuity, and
    those exemptions may reach at most 5 % of the env-steps (tests/parity_stats.py).
"""
import copy
import ctypes as C
import os

import numpy as np
import pytest
import torch

import parity_stats as PS
import pyoracle as O
from migym import _abi, configs, model as M, taskdefs
from test_oracle_golden import HAND_TRACES, hand_noise, hand_trace_setup

pytestmark = pytest.mark.gpu
G = os.path.join(os.path.dirname(__file__), "golden")
DEV = "cuda:0"


@pytest.fixture(scope="module")
def lib():
    assert torch.cuda.is_available(), "GPU tests need the MI355X"
    return _abi.lib()


def T(a, dtype=torch.float32):
    return torch.as_tensor(np.ascontiguousarray(a)).to(DEV, dtype).contiguous()


def P(t):
    return None if t is None else t.data_ptr()


def stream():
    return torch.cuda.current_stream().cuda_stream


def setup(n=16, kind="block"):
    cfg = configs.task_config("ShadowHand", n)
    cfg["env"]["objectType"] = kind
    spec = taskdefs.hand_spec(kind)
    return spec, taskdefs.sim_params(cfg, 24), taskdefs.task_params("ShadowHand", cfg, spec)


# object drop below its reset pose that puts it on / just above the palm
PALM_DZ = {"block": 0.07, "egg": 0.065, "pen": 0.012}


class DevHandEnv:
    """Device mirror of pyoracle.HandHostEnv."""

    def __init__(self, h):
        self.h = h
        for k in ("root", "dof", "targets", "prev_targets", "sensors", "dof_force", "rbs", "actions", "actions_out",
                  "obs", "obs_clamped", "rew", "successes", "cons", "goal_states"):
            setattr(self, k, T(getattr(h, k)))
        for k in ("reset", "reset_goal", "progress"):
            setattr(self, k, T(getattr(h, k), torch.int64))
        self.timeout = torch.zeros(h.n, dtype=torch.bool, device=DEV)
        self.scratch = torch.zeros(2, dtype=torch.int64, device=DEV)
        self.noise = None
        self.rb_forces = T(h.rb_forces)
        self.force_prob = None if h.force_prob is None else T(h.force_prob)
        self.states = None if h.states is None else T(h.states)
        self.ncf = None if h.ncf is None else T(h.ncf)

    def views(self):
        v = _abi.StateViews()
        v.root_states, v.dof_state, v.dof_actuation = P(self.root), P(self.dof), None
        v.sensors, v.dof_force, v.rigid_body_states = P(self.sensors), P(self.dof_force), P(self.rbs)
        v.dof_targets = P(self.targets)
        v.rb_forces, v.rb_force_space = P(self.rb_forces), _abi.MG_LOCAL_SPACE
        v.net_contact_forces = P(self.ncf)
        return v

    def buffers(self, seed=0, step=0):
        b = _abi.TaskBuffers()
        b.actions, b.actions_out, b.obs, b.obs_clamped = P(self.actions), P(self.actions_out), P(self.obs), \
            P(self.obs_clamped)
        b.rew, b.reset, b.progress, b.timeout = P(self.rew), P(self.reset), P(self.progress), P(self.timeout)
        b.noise = P(self.noise)
        b.seed, b.step_counter, b.env_offset = seed, step, 0
        b.prev_targets, b.goal_states, b.reset_goal = P(self.prev_targets), P(self.goal_states), P(self.reset_goal)
        b.successes, b.consecutive_successes, b.reduce_scratch = P(self.successes), P(self.cons), P(self.scratch)
        b.states, b.random_force_prob = P(self.states), P(self.force_prob)
        return b


def np_(t):
    return t.cpu().numpy()


@pytest.mark.parametrize("trace", HAND_TRACES)
def test_hand_task_layer_replays_reference_trace(lib, trace):
    d = dict(np.load(os.path.join(G, trace)))
    spec, tp = hand_trace_setup(d)
    Tn, N = d["actions"].shape[:2]
    h = O.HandHostEnv(tp, spec, N)
    h.root[:] = d["init_root"]
    h.goal_states[:] = d["init_goal_states"]
    forces = "force_scale" in d
    if forces:
        h.force_prob = O.f32(d["init_force_prob"]).copy()
        h.states = np.zeros((N, tp.num_states), np.float32)
    e = DevHandEnv(h)
    for t in range(Tn):
        e.actions.copy_(T(d["actions"][t]))
        e.noise = T(hand_noise(d, t))
        _abi.check(lib.mg_pre_physics(None, C.byref(tp), C.byref(e.views()), C.byref(e.buffers()), N, stream()), lib)
        torch.cuda.synchronize()
        np.testing.assert_allclose(np_(e.root), d["root_pre"][t], rtol=1e-5, atol=1e-6)
        np.testing.assert_allclose(np_(e.dof), d["dof_pre"][t], rtol=1e-5, atol=1e-6)
        np.testing.assert_allclose(np_(e.targets), d["targets"][t], rtol=1e-5, atol=1e-6)
        np.testing.assert_allclose(np_(e.goal_states), d["goal_states"][t], rtol=1e-5, atol=1e-6)
        if forces:
            np.testing.assert_allclose(np_(e.rb_forces), d["rb_forces"][t], rtol=1e-5, atol=1e-6)
            np.testing.assert_allclose(np_(e.force_prob), d["force_prob"][t], rtol=1e-5)
        e.root.copy_(T(d["phys_root"][t]))
        e.dof.copy_(T(d["phys_dof"][t]))
        e.rbs.copy_(T(d["phys_rbs"][t]))
        e.sensors.copy_(T(d["phys_sensors"][t]))
        e.dof_force.copy_(T(d["phys_dof_force"][t]))
        _abi.check(lib.mg_post_physics(None, C.byref(tp), C.byref(e.views()), C.byref(e.buffers()), N, stream()),
                   lib)
        torch.cuda.synchronize()
        np.testing.assert_allclose(np_(e.obs_clamped), d["obs"][t], rtol=1e-4, atol=1e-4)
        np.testing.assert_allclose(np_(e.rew), d["rew"][t], rtol=1e-4, atol=1e-4)
        np.testing.assert_array_equal(np_(e.reset), d["reset"][t])
        np.testing.assert_array_equal(np_(e.reset_goal), d["reset_goal"][t])
        np.testing.assert_array_equal(np_(e.progress), d["progress"][t])
        np.testing.assert_array_equal(np_(e.successes), d["successes"][t])
        np.testing.assert_allclose(np_(e.cons), d["cons"][t], rtol=1e-6)
        np.testing.assert_array_equal(np_(e.timeout).astype(np.int64), d["timeouts"][t])
        assert int(e.scratch.abs().sum()) == 0  # the finishing kernel clears the partial sums
        if forces:
            np.testing.assert_allclose(np.clip(np_(e.states), -tp.clip_obs, tp.clip_obs), d["states"][t],
                                       rtol=1e-4, atol=1e-4)


def hand_states(spec, tp, n, rng, dz=0.07, pen=False):
    """Object on / just above the palm with random orientation and twist, random hand pose and targets."""
    h = O.HandHostEnv(tp, spec, n)
    lo = np.array([x.lower for x in spec.nodes[1:]])
    hi = np.array([x.upper for x in spec.nodes[1:]])
    h.dof[:, :, 0] = lo + (hi - lo) * rng.uniform(0.0, 0.6, (n, spec.num_dofs))
    h.dof[:, :, 1] = rng.normal(0, 0.5, (n, spec.num_dofs))
    h.targets[:] = lo + (hi - lo) * rng.uniform(0, 1, (n, spec.num_dofs))
    ob = h.root[:, 1]
    ob[:, 0:3] = np.array(tp.object_start[:3]) + rng.normal(0, 0.01, (n, 3)) - np.array([0, 0, dz])
    q = rng.normal(0, 1, (n, 4))
    ob[:, 3:7] = q / np.linalg.norm(q, axis=-1, keepdims=True)
    if pen:   # lying across the palm as reset_idx places it (randomize_rotation_pen), 0-8 mm above rest,
              # fingers near the zero pose (curled fingers would cut through a 0.2 m pen)
        h.dof[:, :, 0] = np.clip(rng.normal(0, 0.05, (n, spec.num_dofs)), lo, hi)
        r0 = rng.uniform(-1, 1, n)
        ha, hz = 0.5 * (0.5 * np.pi + 0.02 * r0), 0.5 * np.pi * r0   # tilt within 0.02 rad
        ob[:, 3:7] = np.stack([np.sin(ha) * np.cos(hz), -np.sin(ha) * np.sin(hz), np.cos(ha) * np.sin(hz),
                               np.cos(ha) * np.cos(hz)], -1)
        ob[:, 2] = tp.object_start[2] - dz + rng.uniform(0.0, 0.008, n)
    ob[:, 7:13] = rng.normal(0, 0.2, (n, 6))
    return h


def _physics_vs_oracle(lib, spec, sp, h, rng, n, reach_cap=PS.REACH_CAP):
    """one simulate of the states h on the GPU and in the oracle; asserts determinism and per-env agreement"""
    # applied object forces (LOCAL_SPACE) on half of the envs
    h.rb_forces[: n // 2, len(spec.bodies)] = rng.normal(0, 0.3, (n // 2, 3))
    # the net contact force tensor bound on both sides (acquire_net_contact_force_tensor, franka_reach_MA.py:506)
    h.ncf = np.zeros((n, len(spec.bodies) + 2, 3), np.float32)
    e = DevHandEnv(h)
    h0 = copy.deepcopy(h)
    mnp = M.pack_model(spec)
    h.simulate(mnp, sp, threads=8)
    sim = C.c_void_p()
    _abi.check(lib.mg_sim_create(mnp.ctypes.data, C.byref(sp), n, 0, C.byref(sim)), lib)
    _abi.check(lib.mg_sim_bind(sim, C.byref(e.views())), lib)
    _abi.check(lib.mg_sim_simulate(sim, stream()), lib)
    torch.cuda.synchronize()
    rg, dg = np_(e.root), np_(e.dof)
    # the same step again from the same states must be bit-identical (the egg kernels once changed with
    # unrelated edits to the calling kernel: convex.hpp, cvx_contact_v)
    e2 = DevHandEnv(h0)
    _abi.check(lib.mg_sim_bind(sim, C.byref(e2.views())), lib)
    _abi.check(lib.mg_sim_simulate(sim, stream()), lib)
    torch.cuda.synchronize()
    lib.mg_sim_destroy(sim)
    np.testing.assert_array_equal(np_(e2.root), rg)
    np.testing.assert_array_equal(np_(e2.dof), dg)
    assert np.isfinite(rg).all() and np.isfinite(dg).all()
    np.testing.assert_array_equal(rg[:, 0], h.root[:, 0])       # fixed hand root untouched
    np.testing.assert_array_equal(rg[:, 2], h.root[:, 2])       # goal actor untouched
    # every env must agree, unless its step passes a discontinuity of the physics (orc_step_flips: a contact or
    # limit threshold in use, a drive at saturation, a seg_box_sat tie); the error statistics and the exemptions'
    # reach go to MIGYM_PARITY_REPORT
    test = os.environ.get("PYTEST_CURRENT_TEST", "hand").split(" ")[0]
    scale = max(1.0, np.abs(h.sensors).max())
    ncf_scale = max(1.0, np.abs(h.ncf).max())
    assert np.array_equal(np_(e2.ncf), np_(e.ncf)) and float(np.abs(h.ncf).max()) > 0.0
    checks = [("net contact forces", np_(e.ncf), h.ncf, 1e-2 * ncf_scale, 0),("object pose", rg[:, 1, 0:7], h.root[:, 1, 0:7], 2e-4, 0), ("object twist", rg[:, 1, 7:13], h.root[:, 1, 7:13], 2e-3, 2e-3),
              ("dof pos", dg[..., 0], h.dof[..., 0], 2e-4, 0), ("dof vel", dg[..., 1], h.dof[..., 1], 2e-3, 2e-3),
              ("dof force", np_(e.dof_force), h.dof_force, 1e-2, 1e-2), ("rigid bodies", np_(e.rbs), h.rbs, 2e-3, 2e-3),
              ("sensors", np_(e.sensors), h.sensors, 1e-2 * scale, 0)]
    bad = np.zeros(n, bool)
    for name, a, b, atol, rtol in checks:
        eb = PS.env_bad(a, b, atol, rtol)
        PS.record(test, name, a, b, envs_outside=int(eb.sum()), atol=atol, rtol=rtol)
        bad |= eb
    flags = PS.step_flags(mnp, sp, h0)   # h0: the targets and object forces this simulate used
    PS.assert_steps_explained(test, bad[None], flags[None], reach_cap=reach_cap)
    return mnp, h0


@pytest.mark.parametrize("kind", ["block", "egg", "pen"])
def test_hand_physics_step_matches_oracle(lib, kind):
    """One simulate from random states; egg = GJK / MPR narrowphase, pen = capsule contacts."""
    spec, sp, tp = setup(kind=kind)
    n = 256
    rng = np.random.default_rng(5)
    h = hand_states(spec, tp, n, rng, PALM_DZ[kind], pen=kind == "pen")
    mnp, h0 = _physics_vs_oracle(lib, spec, sp, h, rng, n)
    # the states exercise the object contacts
    ncon = [len(O.contacts(mnp, sp, h0.root[i].ravel(), h0.dof[i], 64)) for i in range(32)]
    assert max(ncon) >= 3


def test_hand_finger_pairs_match_oracle(lib):
    """Curled fingers and thumb (60-95 % of their flexion range, object parked away): the MJCF's explicit
    finger / thumb / palm pairs (frictionless, from zero distance) are in contact in most envs; one simulate on
    the GPU against the oracle, every env, as _physics_vs_oracle."""
    spec, sp, tp = setup(kind="block")
    n = 256
    rng = np.random.default_rng(17)
    h = hand_states(spec, tp, n, rng)
    lo = np.array([x.lower for x in spec.nodes[1:]])
    hi = np.array([x.upper for x in spec.nodes[1:]])
    h.dof[:, :, 0] = lo + (hi - lo) * rng.uniform(0.6, 0.95, (n, spec.num_dofs))
    h.root[:, 1, 0:3] = (5.0, 5.0, 3.0)
    mnp, h0 = _physics_vs_oracle(lib, spec, sp, h, rng, n)
    spec0 = copy.deepcopy(spec)
    spec0.pairs = []
    m0 = M.pack_model(spec0)
    npair = [len(O.contacts(mnp, sp, h0.root[i].ravel(), h0.dof[i], 64)) - len(O.contacts(m0, sp, h0.root[i].ravel(), h0.dof[i], 64))
             for i in range(64)]
    assert sum(1 for k in npair if k > 0) >= 32, npair


def forearm_top(spec, h):
    """world position of the forearm hull's highest vertex (geom frame of node 0 = the hand's root row)"""
    g = spec.geoms[spec.hull["geom"]]

    def rot(q):
        a, b, c, w = q
        return np.array([[1 - 2 * (b * b + c * c), 2 * (a * b - c * w), 2 * (a * c + b * w)],
                         [2 * (a * b + c * w), 1 - 2 * (a * a + c * c), 2 * (b * c - a * w)],
                         [2 * (a * c - b * w), 2 * (b * c + a * w), 1 - 2 * (a * a + b * b)]])
    Rn = rot(h.root[0, 0, 3:7].astype(np.float64))
    c = h.root[0, 0, 0:3] + Rn @ np.asarray(g.pos)
    vw = c + np.array(spec.hull["verts"]) @ (Rn @ rot(g.quat)).T
    return vw[np.argmax(vw[:, 2])]


@pytest.mark.parametrize("kind", ["block", "egg", "pen"])
def test_hand_physics_near_forearm_matches_oracle(lib, kind):
    """The forearm's convex-hull geom (robot.xml:8): objects dropped on / into the hull top
    (block: vertex-face both ways; egg: GJK / MPR on the hull's support function; pen: hull vertices vs its
    segment, its ends vs the hull's faces), GPU vs oracle like the palm states."""
    spec, sp, tp = setup(kind=kind)
    n = 256
    rng = np.random.default_rng(11)
    h = hand_states(spec, tp, n, rng, PALM_DZ[kind], pen=kind == "pen")
    top = forearm_top(spec, h)
    ob = h.root[:, 1]
    reach = {"block": 0.025, "egg": 0.03, "pen": 0.008}[kind]
    ob[:, 0:3] = top + np.c_[rng.normal(0, 0.02, (n, 2)), reach * rng.uniform(0.6, 1.4, n)]
    ob[:, 7:13] = rng.normal(0, 0.1, (n, 6))
    h.dof[:, :, 0] = 0.0   # fingers straight and away from the forearm
    mnp, h0 = _physics_vs_oracle(lib, spec, sp, h, rng, n)
    hull_geom = spec.hull["geom"]
    touching = 0
    for i in range(64):
        cs = O.contacts(mnp, sp, h0.root[i].ravel(), h0.dof[i], 64)
        touching += any(int(c[0]) == spec.geoms[hull_geom].node and int(c[8]) == -2 for c in cs)
    assert touching >= 16, touching


def _forearm_world(spec, h):
    """world centre and axes of the forearm hull's geom frame (node 0 = the hand's fixed root row)"""
    g = spec.geoms[spec.hull["geom"]]
    from scipy.spatial.transform import Rotation
    Rn = Rotation.from_quat(h.root[0, 0, 3:7].astype(np.float64)).as_matrix()
    return h.root[0, 0, 0:3] + Rn @ np.asarray(g.pos), Rn @ Rotation.from_quat(np.asarray(g.quat, np.float64)).as_matrix()


def hull_exact_states(kind, n, rng):
    """the exact-hull placements (hull.hpp / oracle hull_core_contact): the cube with an edge across one of the
    hull's upper edges, or the pen lying across one of its upper faces with its ends overhanging, at gaps of
    -0.5 .. 1.5 mm (tests/test_step_flags.py uses them on the CPU too)"""
    from scipy.spatial.transform import Rotation
    from test_oracle_hand_physics import _cube_across_edge, _hull_edges
    spec, sp, tp = setup(kind=kind)
    h = hand_states(spec, tp, n, rng, PALM_DZ[kind], pen=kind == "pen")
    h.dof[:, :, 0] = 0.0   # fingers straight and away from the forearm
    c, R = _forearm_world(spec, h)
    edges, V, P, on = _hull_edges(spec)
    ob = h.root[:, 1]
    if kind == "block":
        up = [e for e in edges if e[1] > 10 and e[0] > 0.03 and (R @ (P[e[4], :3] + P[e[5], :3]))[2] > 0]
        assert len(up) >= 4
        for i in range(n):
            (_, _, a, b, f1, f2) = up[i % len(up)]
            cl, Rl, _, _ = _cube_across_edge(V, P, a, b, f1, f2, rng.uniform(-5e-4, 1.5e-3))
            ob[i, 0:3] = c + R @ cl
            ob[i, 3:7] = Rotation.from_matrix(R @ Rl).as_quat()
    else:
        faces = [f for f in range(len(P)) if (R @ P[f, :3])[2] > 0.3]
        assert len(faces) >= 8
        for i in range(n):
            f = faces[i % len(faces)]
            nf = P[f, :3]
            t = np.cross(nf, rng.normal(size=3))
            t /= np.linalg.norm(t)
            ctr = V[on[:, f]].mean(0) + nf * (0.008 + rng.uniform(-5e-4, 1.5e-3))
            Rl = np.stack([nf, np.cross(t, nf), t], 1)      # the pen's axis (object z) along t
            ob[i, 0:3] = c + R @ ctr
            ob[i, 3:7] = Rotation.from_matrix(R @ Rl).as_quat()
    ob[:, 7:13] = rng.normal(0, 0.05, (n, 6))
    # these placements sit on the hull's features by construction (an edge across an edge, a segment across a
    # face next to its ridges), so the feature-decision band (bit 16) reaches more of them than of random states
    return spec, sp, tp, h


@pytest.mark.parametrize("kind", ["block", "pen"])
def test_hand_physics_hull_exact_matches_oracle(lib, kind):
    """A6, the exact hull candidate (hull.hpp / oracle hull_core_contact): the cube with an edge across one of the
    hull's upper edges, or the pen lying across one of its upper faces with its ends overhanging, at gaps of
    -0.5 .. 1.5 mm, where the vertex-face candidates see nothing (test_oracle_hand_physics.py KATs).  GPU vs
    oracle like the palm states; most envs must be in contact with the hull."""
    n = 256
    rng = np.random.default_rng(13)
    spec, sp, tp, h = hull_exact_states(kind, n, rng)
    mnp, h0 = _physics_vs_oracle(lib, spec, sp, h, rng, n, reach_cap=0.10)
    node = spec.geoms[spec.hull["geom"]].node
    touching = 0
    for i in range(n):
        cs = O.contacts(mnp, sp, h0.root[i].ravel(), h0.dof[i], 64)
        touching += any(int(x[0]) == node and int(x[8]) == -2 for x in cs)
    assert touching >= n // 2, touching


def _hand_teacher_forced(lib, test, spec, sp, tp, h, steps, actions, seed, extra=None, obs_tol=2e-3,
                         reach_cap=PS.REACH_CAP, north_star=False, threads=8):
    """mg_env_step vs orc_hand_env_step step by step, both sides started each step from the oracle's state (all
    buffers reloaded: DOF / root / rigid-body state, targets, goal, resets, successes, running mean, forces), so a
    step's fp32-vs-fp64 difference cannot grow chaotically over the next ones.  Per step: progress, targets and goals
    exact (within 1e-5); every env's obs within obs_tol (1 + |x|), reward within 5e-3 (1 + |r|) and the same resets,
    unless orc_step_flips puts that env's step at a discontinuity (or the oracle itself is sensitive there); the
    exemptions' reach is capped (parity_stats.assert_steps_explained).  extra(e, h) -> per-env bad flags of more
    outputs."""
    n = h.n
    mnp = M.pack_model(spec)
    sim = C.c_void_p()
    _abi.check(lib.mg_sim_create(mnp.ctypes.data, C.byref(sp), n, 0, C.byref(sim)), lib)
    bad = np.zeros((steps, n), bool)
    flags = np.zeros((steps, n), np.int32)
    pres, outs, rews = [], [], []
    ncon = 0
    try:
        for t in range(steps):
            h.actions[:] = actions[t]
            e = DevHandEnv(h)
            _abi.check(lib.mg_sim_bind(sim, C.byref(e.views())), lib)
            flags[t] = PS.step_flags(mnp, sp, PS.hand_physics_input(h, mnp, tp, seed, t))
            pres.append(copy.deepcopy(h))
            h.env_step(mnp, sp, tp, seed=seed, step=t, threads=threads)
            _abi.check(lib.mg_env_step(sim, C.byref(tp), C.byref(e.buffers(seed=seed, step=t)), stream()), lib)
            torch.cuda.synchronize()
            np.testing.assert_array_equal(np_(e.progress), h.progress)
            np.testing.assert_allclose(np_(e.targets), h.targets, rtol=1e-5, atol=1e-6)
            np.testing.assert_allclose(np_(e.prev_targets), h.prev_targets, rtol=1e-5, atol=1e-6)
            np.testing.assert_allclose(np_(e.goal_states), h.goal_states, rtol=1e-5, atol=1e-6)
            og = np_(e.obs)
            b = (PS.env_bad(og, h.obs, obs_tol, obs_tol) | PS.env_bad(np_(e.rew)[:, None], h.rew[:, None], 5e-3, 5e-3)
                 | (np_(e.reset) != h.reset) | (np_(e.reset_goal) != h.reset_goal))
            if extra is not None:
                b |= extra(e, h)
            bad[t] = b
            outs.append((og, h.obs.copy()))
            rews.append((np_(e.rew), h.rew.copy()))
            PS.record(test, f"obs step {t}", og, h.obs, envs_outside=int(b.sum()))
            ncon = sum(len(O.contacts(mnp, sp, h.root[i].ravel(), h.dof[i], 64)) > 0 for i in range(n))
            np.testing.assert_allclose(np_(e.cons), h.cons, atol=2e-2)
    finally:
        lib.mg_sim_destroy(sim)
    sens = lambda t, i: PS.oracle_sensitive_step(mnp, sp, tp, pres[t], actions[t], i, outs[t][0][i], outs[t][1][i],
                                                 seed=seed, step=t, hand=True)
    PS.assert_steps_explained(test, bad, flags, sens, reach_cap=reach_cap)
    if not north_star:
        return ncon
    # per column group against north_star's 1e-4 relative over the unflagged env-steps that agree within the step's
    # tolerances (a disagreeing one is explained above: a discontinuity, or the oracle's own sensitivity), with the
    # oracle's fp32 twin from the same states (test_gpu_parity._teacher_forced)
    keep = ((flags == 0) & ~bad).ravel()
    groups = PS.OBS_GROUPS[tp.num_obs]
    og, oh = np.concatenate([o[0] for o in outs]), np.concatenate([o[1] for o in outs])
    rg, rh = np.concatenate([r[0] for r in rews])[:, None], np.concatenate([r[1] for r in rews])[:, None]
    cols = PS.column_stats(test, "columns vs 1e-4 rel (agreeing unflagged env-steps)", og, oh, keep, groups)
    cols.update(PS.column_stats(test, "reward vs 1e-4 rel (agreeing unflagged env-steps)", rg, rh, keep, {"reward": [0]}))
    o32, r32 = [], []
    for t in range(steps):
        g = copy.deepcopy(pres[t])
        g.env_step(mnp, sp, tp, seed=seed, step=t, threads=threads, fp32=True)
        o32.append(g.obs.copy())
        r32.append(g.rew.copy())
    twin = PS.column_stats(test, "fp32 twin: columns vs 1e-4 rel", np.concatenate(o32), oh, keep, groups)
    twin.update(PS.column_stats(test, "fp32 twin: reward vs 1e-4 rel", np.concatenate(r32)[:, None], rh, keep,
                                {"reward": [0]}))
    return ncon, (cols, twin, 0.0)


@pytest.mark.parametrize("kind", ["block", "egg", "pen"])
def test_hand_fused_env_step_matches_oracle(lib, kind):
    """mg_env_step (the bench path) vs orc_hand_env_step over 12 teacher-forced control steps (the block and the
    egg start 0.1 m above the palm and land on it after ~9), device RNG resets (pen: randomize_rotation_pen,
    ignore_z_rot success tolerance, reset poses through the palm box)."""
    spec, sp, tp = setup(kind=kind)
    n = 192
    h = O.HandHostEnv(tp, spec, n)
    rng = np.random.default_rng(3)
    acts = [rng.uniform(-1.2, 1.2, (n, tp.num_actions)).astype(np.float32) for _ in range(12)]
    ncon = _hand_teacher_forced(lib, f"test_hand_fused_env_step_matches_oracle[{kind}]", spec, sp, tp, h, 12, acts, 5)
    assert ncon >= n // 2   # the objects are on the hand by now


def test_hand_fused_parity_at_baseline_shard(lib):
    """BASELINE.json configs[4] (ShadowHand, 32,768 envs over 8 GPUs) at its per-GPU shard, 4,096 envs: the oracle
    rolls every env 12 steps on from the all-reset start (random actions: objects dropped, caught, some reset), then 3
    fused steps are teacher-forced as in test_hand_fused_env_step_matches_oracle, and every obs column group and the
    reward are held to north_star's 1e-4 relative (test_gpu_parity.assert_north_star_rtol: 1e-4 of the group's scale,
    or 4x what the oracle's own fp32 build needs from the same states)"""
    from test_gpu_parity import assert_north_star_rtol
    spec, sp, tp = setup(n=4096, kind="block")
    n = 4096
    h = O.HandHostEnv(tp, spec, n)
    mnp = M.pack_model(spec)
    rng = np.random.default_rng(37)
    for t in range(12):
        h.actions[:] = rng.uniform(-1, 1, (n, tp.num_actions)).astype(np.float32)
        h.env_step(mnp, sp, tp, seed=11, step=200 + t, threads=16)
    acts = [rng.uniform(-1.2, 1.2, (n, tp.num_actions)).astype(np.float32) for _ in range(3)]
    ncon, res = _hand_teacher_forced(lib, "test_hand_fused_parity_at_baseline_shard[block-4096]", spec, sp, tp, h, 3,
                                     acts, 11, north_star=True, threads=16)
    assert ncon >= n // 4
    assert_north_star_rtol(res)


def test_hand_fused_forces_and_states_match_oracle(lib):
    """mg_env_step with random object forces (forceScale 2, forceProbRange [0.2, 0.8]) and asymmetric
    states vs the oracle over 3 teacher-forced control steps with the device RNG: force draws, probability
    redraws and the applied force in the object's dynamics."""
    cfg = configs.task_config("ShadowHand", 16)
    cfg["env"]["forceScale"] = 2.0
    cfg["env"]["forceProbRange"] = [0.2, 0.8]
    cfg["env"]["asymmetric_observations"] = True
    spec = taskdefs.hand_spec("block")
    sp, tp = taskdefs.sim_params(cfg, 24), taskdefs.task_params("ShadowHand", cfg, spec)
    assert tp.num_states == 211 and tp.force_scale == 2.0
    n = 128
    h = O.HandHostEnv(tp, spec, n)
    h.force_prob = np.full(n, 0.5, np.float32)
    h.states = np.zeros((n, 211), np.float32)
    rng = np.random.default_rng(11)
    acts = [rng.uniform(-1, 1, (n, tp.num_actions)).astype(np.float32) for _ in range(3)]
    nb = len(spec.bodies)
    drawn = []

    def extra(e, hh):
        np.testing.assert_allclose(np_(e.rb_forces), hh.rb_forces, rtol=1e-4, atol=1e-6)
        np.testing.assert_allclose(np_(e.force_prob), hh.force_prob, rtol=1e-5)
        np.testing.assert_allclose(np_(e.states)[:, 211 - 20:], np_(e.obs)[:, 211 - 20:])  # actions block
        drawn.append(np.abs(hh.rb_forces[:, nb]).sum(-1).astype(bool).mean())
        return (PS.env_bad(np_(e.root)[:, 1], hh.root[:, 1], 2e-3, 2e-3)
                | PS.env_bad(np_(e.states), hh.states, 2e-3, 2e-3))
    _hand_teacher_forced(lib, "test_hand_fused_forces_and_states_match_oracle", spec, sp, tp, h, 3, acts, 9, extra)
    assert max(drawn) > 0.3   # forces were drawn


def test_hand_set_indexed_maps_actor_ids(lib):
    spec, sp, tp = setup()
    n = 50
    h = O.HandHostEnv(tp, spec, n)
    e = DevHandEnv(h)
    mnp = M.pack_model(spec)
    sim = C.c_void_p()
    _abi.check(lib.mg_sim_create(mnp.ctypes.data, C.byref(sp), n, 0, C.byref(sim)), lib)
    _abi.check(lib.mg_sim_bind(sim, C.byref(e.views())), lib)
    src = torch.randn((n, 24, 2), device=DEV)
    tsrc = torch.randn((n, 24), device=DEV)
    rsrc = torch.randn((n * 3, 13), device=DEV)
    envs = torch.tensor([1, 7, 30], device=DEV)
    hand_ids = (3 * envs).to(torch.int32)
    obj_ids = (3 * envs + 1).to(torch.int32)
    _abi.check(lib.mg_set_indexed(sim, _abi.MG_SET_DOF_STATE, P(src), P(hand_ids), 3, stream()), lib)
    _abi.check(lib.mg_set_indexed(sim, _abi.MG_SET_DOF_TARGET, P(tsrc), P(hand_ids), 3, stream()), lib)
    _abi.check(lib.mg_set_indexed(sim, _abi.MG_SET_ROOT_STATE, P(rsrc), P(obj_ids), 3, stream()), lib)
    torch.cuda.synchronize()
    lib.mg_sim_destroy(sim)
    assert torch.equal(e.dof[envs], src[envs]) and torch.equal(e.targets[envs], tsrc[envs])
    assert torch.equal(e.root.view(n * 3, 13)[obj_ids.long()], rsrc[obj_ids.long()])
    mask = torch.ones(n, dtype=torch.bool, device=DEV)
    mask[envs] = False
    assert float(e.dof[mask].abs().sum()) == 0.0


@pytest.mark.parametrize("obs_type", ["full", "openai"])
def test_hand_fused_obs_types_match_oracle(lib, obs_type):
    """the full (157) and openai (42) observation layouts through the fused step, teacher-forced over 2 steps"""
    cfg = configs.task_config("ShadowHand", 16)
    cfg["env"]["observationType"] = obs_type
    spec = taskdefs.hand_spec("block")
    sp, tp = taskdefs.sim_params(cfg, 24), taskdefs.task_params("ShadowHand", cfg, spec)
    n = 64
    h = O.HandHostEnv(tp, spec, n)
    rng = np.random.default_rng(8)
    acts = [rng.uniform(-1, 1, (n, tp.num_actions)).astype(np.float32) for _ in range(2)]
    assert tp.num_obs == taskdefs.HAND_OBS[obs_type][1]
    _hand_teacher_forced(lib, f"test_hand_fused_obs_types_match_oracle[{obs_type}]", spec, sp, tp, h, 2, acts, 2)


def test_hand_make_full_size():
    import migym
    n = 4096
    env = migym.make(seed=0, task="ShadowHand", num_envs=n, sim_device=DEV, rl_device=DEV, headless=True)
    assert env.num_obs == 211 and env.num_actions == 20
    g = torch.Generator(device=DEV).manual_seed(0)
    for _ in range(40):
        a = torch.rand((n, 20), device=DEV, generator=g) * 2 - 1
        obs, rew, reset, extras = env.step(a)
    torch.cuda.synchronize()
    o = obs["obs"]
    assert o.shape == (n, 211) and torch.isfinite(o).all() and torch.isfinite(rew).all()
    assert float(o.abs().max()) <= 5.0
    assert "consecutive_successes" in extras and torch.isfinite(extras["consecutive_successes"])
    obj = env.root_state_tensor.view(n, 3, 13)[:, 1]
    assert torch.isfinite(obj).all() and float(obj[:, 7:13].abs().max()) < 100.0
    # the cube stays with the hand for most envs (falls reset them; fall distance 0.24)
    assert float((obj[:, 2] > 0.2).float().mean()) > 0.9
    env.close()


def test_hand_make_asymmetric_with_forces():
    """make() with asymmetric_observations and forceScale > 0: obs_dict['states'] (N, 211) clamped to
    clipObservations, rb_forces (N, 27, 3) populated on the object row only."""
    import migym
    n = 512
    cfg = configs.task_config("ShadowHand", n, sim_device=DEV)
    cfg["env"]["asymmetric_observations"] = True
    cfg["env"]["forceScale"] = 1.0
    cfg["env"]["forceProbRange"] = [0.1, 0.5]
    env = migym.make(seed=0, task="ShadowHand", num_envs=n, sim_device=DEV, rl_device=DEV, headless=True,
                     cfg={"task": cfg})
    assert env.num_states == 211 and env.states_buf.shape == (n, 211)
    g = torch.Generator(device=DEV).manual_seed(0)
    for _ in range(10):
        obs, rew, reset, extras = env.step(torch.rand((n, 20), device=DEV, generator=g) * 2 - 1)
    torch.cuda.synchronize()
    st = obs["states"]
    assert st.shape == (n, 211) and torch.isfinite(st).all() and float(st.abs().max()) <= 5.0
    # states = full_state layout: actions block equals the obs actions block (obs is full_state too)
    assert torch.equal(st[:, 191:], obs["obs"][:, 191:])
    obj = len(env.model_spec.bodies)
    f = env.rb_forces
    assert float(f[:, obj].abs().sum()) > 0 and float(f[:, :obj].abs().sum()) == 0.0
    p = env.random_force_prob
    assert float(p.min()) >= 0.1 - 1e-6 and float(p.max()) <= 0.5 + 1e-6
    env.close()


@pytest.mark.parametrize("kind", ["egg", "pen"])
def test_hand_make_object_types(kind):
    """make(..., objectType egg / pen) through the fused step: finite state, the object held near the hand,
    pen resets with randomize_rotation_pen (axis near horizontal: |R e_z . e_z| = |cos(pi/2 + 0.3 r)| <= sin 0.3
    at the reset, before contacts act)."""
    import migym
    n = 1024
    cfg = configs.task_config("ShadowHand", n, sim_device=DEV)
    cfg["env"]["objectType"] = kind
    env = migym.make(seed=0, task="ShadowHand", num_envs=n, sim_device=DEV, rl_device=DEV, headless=True,
                     cfg={"task": cfg})
    assert env.model_spec.obj["type"] == (M.GT_ELLIPSOID if kind == "egg" else M.GT_CAPSULE)
    g = torch.Generator(device=DEV).manual_seed(0)
    obs, rew, reset, extras = env.step(torch.zeros((n, 20), device=DEV))
    obj = env.root_state_tensor.view(n, 3, 13)[:, 1]
    if kind == "pen":   # every env reset on the first step
        q = obj[:, 3:7]
        zz = 1 - 2 * (q[:, 0] ** 2 + q[:, 1] ** 2)
        assert float(zz.abs().mean()) <= float(np.sin(0.3))   # after one step of contact physics
    for _ in range(20):
        obs, rew, reset, extras = env.step(torch.rand((n, 20), device=DEV, generator=g) * 2 - 1)
    torch.cuda.synchronize()
    o = obs["obs"]
    assert torch.isfinite(o).all() and torch.isfinite(rew).all()
    obj = env.root_state_tensor.view(n, 3, 13)[:, 1]
    assert torch.isfinite(obj).all()
    # a light object squeezed by random finger motions can be flung (max_depenetration_velocity 1000):
    # bound the bulk, not the rarest env
    assert float((obj[:, 7:13].abs().amax(1) < 100.0).float().mean()) >= 0.99
    assert float((obj[:, 2] > 0.2).float().mean()) > 0.8
    env.close()
