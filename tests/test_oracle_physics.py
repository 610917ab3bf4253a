"""Known-answer tests pinning the fp64 physics oracle (oracle/oracle_physics.c).

The reference physics (closed PhysX) cannot run anywhere in this pipeline, so
these analytic checks are what establish the oracle; the HIP kernels are then
held to the oracle (tests/test_gpu_parity.py).  Checks:
  * Ant total mass == MJCF geom-density mass (0.911 kg)
  * joint-space inertia is symmetric positive definite and its kinetic energy
    equals the sum of the rigid bodies' kinetic energies
  * free fall follows the discrete semi-implicit Euler law exactly
  * with gravity and contact off, linear and angular momentum are conserved
    under internal actuation
  * a frictionless pendulum (cartpole) conserves energy to O(h)
  * joint limits hold under saturating torque; a dropped Ant comes to rest
"""
import math

import numpy as np
import pytest

import pyoracle as O
from migym import model as M, taskdefs, configs


def setup(task, **sp_over):
    cfg = configs.task_config(task, 4)
    spec = M.load_builtin(taskdefs.TASK_INFO[task][1])
    sp = taskdefs.sim_params(cfg, 32)
    for k, v in sp_over.items():
        if k == "gravity":
            for i in range(3):
                sp.gravity[i] = v[i]
        else:
            setattr(sp, k, v)
    tp = taskdefs.task_params(task, cfg, spec)
    return spec, M.pack_model(spec), sp, tp


def body_momenta(spec, mnp, root, dof):
    rb = O.rigid_body_states(mnp, root, dof, len(spec.bodies)).astype(np.float64)
    P = np.zeros(3)
    L = np.zeros(3)
    KE = 0.0
    for b, body in enumerate(spec.bodies):
        if body.mass <= 0:
            continue
        q = rb[b, 3:7]
        R = M.qmat(q)
        c = rb[b, 0:3] + R @ np.array(body.com)
        v, w = rb[b, 7:10], rb[b, 10:13]
        Ib = body_inertia(spec, b)
        Iw = R @ Ib @ R.T
        P += body.mass * v
        L += np.cross(c, body.mass * v) + Iw @ w
        KE += 0.5 * body.mass * v @ v + 0.5 * w @ Iw @ w
    return P, L, KE


def body_inertia(spec, b):
    """inertia about the body COM in body frame, rebuilt from the geoms (model-independent path)."""
    acc = M._MassAccum()
    density = 5.0 if spec.name == "ant" else 1000.0
    for g in spec.geoms:
        if g.body != b:
            continue
        m, Ig = M.geom_mass_inertia(g.gtype, g.size, density)
        body = spec.bodies[b]
        # geom pose in body frame = inverse(body in node) * geom in node
        Rb = M.qmat(body.quat)
        pos = Rb.T @ (np.array(g.pos) - np.array(body.pos))
        Rg = Rb.T @ M.qmat(g.quat)
        acc.add(m, pos, Rg @ Ig @ Rg.T)
    m, c, Ic = acc.result()
    return Ic


def rand_state(spec, tp, rng, z=2.0):
    nd = spec.num_dofs
    root = np.zeros(13, np.float32)
    root[2] = z
    q = rng.normal(size=4)
    root[3:7] = q / np.linalg.norm(q)
    root[7:13] = rng.normal(size=6)
    lo, hi = np.array(tp.dof_lower[:nd]), np.array(tp.dof_upper[:nd])
    dof = np.zeros((nd, 2), np.float32)
    dof[:, 0] = lo + (hi - lo) * rng.uniform(0.2, 0.8, nd)
    dof[:, 1] = rng.normal(size=nd)
    return root, dof


def test_ant_mass_matches_mjcf_geoms():
    spec = M.load_builtin("ant")
    assert abs(spec.total_mass() - 0.9109) < 5e-4


@pytest.mark.parametrize("task", ["Ant", "Humanoid"])
def test_mass_matrix_spd_and_kinetic_energy(task):
    spec, mnp, sp, tp = setup(task)
    mnp["armature"][:] = 0
    mnp["damping"][:] = 0
    mnp["stiffness"][:] = 0
    rng = np.random.default_rng(0)
    for _ in range(5):
        root, dof = rand_state(spec, tp, rng)
        Mm = O.mass_matrix(mnp, sp, root, dof)
        np.testing.assert_allclose(Mm, Mm.T, atol=1e-12)
        assert np.linalg.eigvalsh(Mm).min() > 0
        np.testing.assert_allclose(Mm[3:6, 3:6], np.eye(3) * spec.total_mass(), rtol=1e-6)
        # generalized velocity nu = [w, v_o, qd], v_o = v_com - w x (R com_b0)
        R = M.qmat(root[3:7].astype(np.float64) / np.linalg.norm(root[3:7]))
        w = root[10:13].astype(np.float64)
        vo = root[7:10] - np.cross(w, R @ np.array(spec.bodies[0].com))
        nu = np.concatenate([w, vo, dof[:, 1]])
        ke_m = 0.5 * nu @ Mm @ nu
        _, _, ke_b = body_momenta(spec, mnp, root, dof)
        assert abs(ke_m - ke_b) < 1e-4 * max(1.0, ke_b)


def test_free_fall_is_discrete_semi_implicit_euler():
    spec, mnp, sp, tp = setup("Ant")
    root = np.zeros((1, 13), np.float32)
    root[0, 2] = 3.0
    root[0, 6] = 1.0
    dof = np.zeros((1, 8, 2), np.float32)
    dof[0, :, 0] = 0.5 * (np.array(tp.dof_lower[:8]) + np.array(tp.dof_upper[:8]))  # mid-range
    steps = 10
    for _ in range(steps):
        O.simulate(mnp, sp, root, dof)
    h = sp.dt / sp.substeps
    n = steps * sp.substeps
    z = 3.0 - 9.81 * h * h * n * (n + 1) / 2
    assert abs(root[0, 2] - z) < 2e-5
    assert abs(root[0, 9] - (-9.81 * h * n)) < 1e-4
    assert np.abs(dof[0, :, 1]).max() < 1e-5


def test_momentum_conserved_without_gravity_or_contact():
    """Internal actuation conserves momentum; the discrete drift is O(h) (converges 10x per 10x dt)."""
    drifts = []
    for dt in (0.0166, 0.00166):
        spec, mnp, sp, tp = setup("Ant", gravity=(0.0, 0.0, 0.0), max_contacts=0)
        mnp["damping"][:] = 0
        sp.dt = dt
        sp.limit_margin = -1.0   # limits off: a pure internal-force test
        rng = np.random.default_rng(1)
        root, dof = rand_state(spec, tp, rng, z=5.0)
        root[7:13] *= 0.3
        dof[:, 1] *= 0.3
        root, dof = root[None].copy(), dof[None].copy()
        P0, L0, _ = body_momenta(spec, mnp, root[0], dof[0])
        act = (rng.uniform(-1, 1, (1, 8)) * 0.5).astype(np.float32)
        for _ in range(int(round(0.0664 / dt))):
            O.simulate(mnp, sp, root, dof, act)
        P1, L1, _ = body_momenta(spec, mnp, root[0], dof[0])
        drifts.append(np.abs(np.concatenate([P1 - P0, L1 - L0])).max())
    assert drifts[1] < 0.15 * drifts[0], drifts
    assert drifts[1] < 2e-3, drifts


def test_cartpole_pendulum_energy():
    """Unactuated, undamped cart + inverted pendulum released at 1 rad: energy error is O(h)."""
    drift = []
    for dt in (0.0166, 0.00166):
        spec, mnp, sp, tp = setup("Cartpole")
        mnp["damping"][:] = 0
        mnp["armature"][:] = 0
        sp.dt = dt
        root = np.zeros((1, 13), np.float32)
        root[0, 2] = 2.0
        root[0, 6] = 1.0
        dof = np.zeros((1, 2, 2), np.float32)
        dof[0, 1, 0] = 1.0
        mp = spec.nodes[2].mass

        def energy():
            rb = O.rigid_body_states(mnp, root[0], dof[0], len(spec.bodies))
            Mm = O.mass_matrix(mnp, sp, root[0], dof[0])
            nu = dof[0, :, 1].astype(np.float64)
            R = M.qmat(rb[2, 3:7].astype(np.float64))
            cz = rb[2, 2] + (R @ np.array(spec.bodies[2].com))[2]
            return 0.5 * nu @ Mm @ nu + mp * 9.81 * cz

        e0 = energy()
        es = []
        for _ in range(int(round(3.32 / dt))):
            O.simulate(mnp, sp, root, dof)
            es.append(energy())
        drift.append(max(abs(e - e0) for e in es) / e0)
    assert drift[0] < 0.03 and drift[1] < 0.2 * drift[0], drift


def test_joint_limit_holds_under_saturating_torque():
    spec, mnp, sp, tp = setup("Ant", gravity=(0.0, 0.0, 0.0))
    root = np.zeros((1, 13), np.float32)
    root[0, 2] = 3.0
    root[0, 6] = 1.0
    dof = np.zeros((1, 8, 2), np.float32)
    dof[0, :, 0] = np.array(tp.initial_dof_pos[:8]) + 0.3
    act = np.full((1, 8), 15.0, np.float32)  # push every joint towards its upper limit
    for _ in range(60):
        O.simulate(mnp, sp, root, dof, act)
    hi = np.array(tp.dof_upper[:8])
    assert np.all(dof[0, :, 0] <= hi + 0.02), (dof[0, :, 0], hi)


def test_dropped_ant_comes_to_rest_on_the_plane():
    spec, mnp, sp, tp = setup("Ant")
    root = np.zeros((1, 13), np.float32)
    root[0, 2] = 0.44
    root[0, 6] = 1.0
    dof = np.zeros((1, 8, 2), np.float32)
    dof[0, :, 0] = np.array(tp.initial_dof_pos[:8])
    sens = np.zeros((1, 24), np.float32)
    for _ in range(300):
        O.simulate(mnp, sp, root, dof, None, sens)
    assert 0.15 < root[0, 2] < 0.44
    assert np.abs(root[0, 7:13]).max() < 0.05
    # feet carry the weight: summed vertical contact force ~ m g
    fz = 0.0
    rb = O.rigid_body_states(mnp, root[0], dof[0], len(spec.bodies))
    for s, b in enumerate(spec.sensors):
        R = M.qmat(rb[b, 3:7].astype(np.float64))
        fz += (R @ sens[0, 6 * s:6 * s + 3])[2]
    assert abs(fz - spec.total_mass() * 9.81) < 0.15 * spec.total_mass() * 9.81


def test_fp32_restatement_tracks_fp64_checker():
    """liboracle_f32.so (bench.py's timed CPU baseline) computes the same step as the fp64 checker:
    5 Ant control steps from the reset state agree to fp32 rounding (obs within 2e-3)."""
    from migym import configs
    cfg = configs.task_config("Ant", 256)
    spec = M.load_builtin("ant")
    sp, tp = taskdefs.sim_params(cfg, 16), taskdefs.task_params("Ant", cfg, spec)
    mnp = M.pack_model(spec)
    obs = []
    for fp32 in (False, True):
        h = O.HostEnv(tp, spec, 256)
        rng = np.random.default_rng(0)
        for t in range(5):
            h.actions[:] = rng.uniform(-1, 1, h.actions.shape)
            h.env_step(mnp, sp, tp, 0, t, 4, fp32=fp32)
        obs.append(h.obs.copy())
    np.testing.assert_allclose(obs[1], obs[0], atol=2e-3, rtol=2e-3)
