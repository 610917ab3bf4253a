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
        mnp["link_ang_damping"] = 0   # gym's default link damping 0.5 would drain the pendulum
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


# ------------------------------------------------------------------ link damping and the angular velocity cap
def free_link_spec(c, W, inertia=(0.02, 0.02, 0.02)):
    """one free rigid body (spherical inertia: no gyroscopic torque), no geoms"""
    node = M.Node(name="link", parent=-1, jtype=M.JT_FREE, t=[0, 0, 0], r0=[0, 0, 0, 1], axis=[0, 0, 1], body=0,
                  mass=1.0, inertia=list(inertia) + [0.0, 0.0, 0.0])
    body = M.Body(name="link", node=0, pos=[0, 0, 0], quat=[0, 0, 0, 1], parent_body=-1, mass=1.0)
    return M.ModelSpec(name="link", fixed_base=0, nodes=[node], bodies=[body], geoms=[], pairs=[], actuators=[],
                       dof_names=[], angular_damping=c, max_angular_velocity=W)


def test_asset_options_follow_the_tasks():
    """gym AssetOptions per task (ant.py:152, humanoid.py:153-154, shadow_hand.py:240; Cartpole and the hand
    objects keep gym's defaults 0.5 / 64)"""
    want = {"ant": (0.0, 64.0), "humanoid": (0.01, 100.0), "shadow_hand": (0.01, 64.0), "cartpole": (0.5, 64.0)}
    for name, (c, W) in want.items():
        m = M.pack_model(M.load_builtin(name))
        assert m["link_ang_damping"] == np.float32(c) and m["link_max_ang_vel"] == np.float32(W), name
    m = M.pack_model(taskdefs.hand_spec("block"))
    assert m["obj_ang_damping"] == np.float32(0.5) and m["obj_max_ang_vel"] == np.float32(64.0)


def test_free_link_angular_damping_decays_per_substep():
    """a spinning free link (no gravity, spherical inertia): w -> w / (1 + h c) per substep, v untouched"""
    c = 0.5
    spec = free_link_spec(c, 0.0)
    mnp = M.pack_model(spec)
    sp = taskdefs.sim_params(configs.task_config("Ant", 1), 0)
    for i in range(3):
        sp.gravity[i] = 0.0
    root = np.zeros((1, 13), np.float32)
    root[0, 2] = 1.0
    root[0, 6] = 1.0
    root[0, 7:10] = (0.3, -0.2, 0.1)
    root[0, 10:13] = (3.0, -2.0, 1.0)
    w0, v0 = root[0, 10:13].astype(np.float64), root[0, 7:10].copy()
    h = sp.dt / sp.substeps
    steps = 5
    for _ in range(steps):
        O.simulate(mnp, sp, root, np.zeros((1, 0, 2), np.float32))
    want = w0 / (1.0 + h * c) ** (steps * sp.substeps)
    np.testing.assert_allclose(root[0, 10:13], want, rtol=1e-6)
    np.testing.assert_allclose(root[0, 7:10], v0, atol=1e-7)
    # c = 0: no decay
    mnp["link_ang_damping"] = 0.0
    root[0, 10:13] = (3.0, -2.0, 1.0)
    O.simulate(mnp, sp, root, np.zeros((1, 0, 2), np.float32))
    np.testing.assert_allclose(root[0, 10:13], (3.0, -2.0, 1.0), rtol=1e-7)


def test_free_link_angular_velocity_is_capped_keeping_com_velocity():
    spec = free_link_spec(0.0, 10.0)
    spec.nodes[0].com = [0.1, 0.0, 0.0]          # COM off the origin: the cap keeps v_com, not v_o
    spec.bodies[0].com = [0.1, 0.0, 0.0]
    mnp = M.pack_model(spec)
    sp = taskdefs.sim_params(configs.task_config("Ant", 1), 0)
    for i in range(3):
        sp.gravity[i] = 0.0
    sp.substeps = 1
    root = np.zeros((1, 13), np.float32)
    root[0, 2] = 1.0
    root[0, 6] = 1.0
    root[0, 7:10] = (0.5, 0.0, 0.0)
    root[0, 10:13] = (0.0, 0.0, 25.0)   # about z through the origin: no gyroscopic term for I = diag(.02) + m c c
    O.simulate(mnp, sp, root, np.zeros((1, 0, 2), np.float32))
    assert abs(np.linalg.norm(root[0, 10:13]) - 10.0) < 1e-5, root[0, 10:13]
    np.testing.assert_allclose(root[0, 10:13], (0.0, 0.0, 10.0), atol=1e-5)


@pytest.mark.parametrize("task,DOF,rate", [("Cartpole", 1, 200.0), ("Humanoid", 14, 400.0), ("Ant", 1, 300.0)])
def test_link_angular_velocity_cap(task, DOF, rate):
    """one hinge spun far past the cap (gravity and contacts off): every link's |w| ends at <= W (Cartpole's
    pole exactly at gym's default 64; a free base's links within the axes' motion over the step)"""
    spec, mnp, sp, tp = setup(task, gravity=(0.0, 0.0, 0.0), max_contacts=0)
    sp.limit_margin = -1.0
    sp.substeps = 1   # the clamp is the last velocity update of a substep
    W = float(mnp["link_max_ang_vel"])
    nd = spec.num_dofs
    root = np.zeros((1, 13), np.float32)
    root[0, 2] = 5.0
    root[0, 6] = 1.0
    dof = np.zeros((1, nd, 2), np.float32)
    dof[0, :, 0] = np.array(tp.initial_dof_pos[:nd])
    dof[0, DOF, 1] = rate
    root0, dof0 = root.copy(), dof.copy()
    O.simulate(mnp, sp, root, dof)
    # the links' w in the frame the clamp acts in: the step's start pose with the new velocities
    mix_r, mix_d = root0[0].copy(), dof0[0].copy()
    mix_r[7:13] = root[0, 7:13]
    mix_d[:, 1] = dof[0, :, 1]
    rb = O.rigid_body_states(mnp, mix_r, mix_d, len(spec.bodies))
    wn = np.linalg.norm(rb[:, 10:13].astype(np.float64), axis=1)
    if task == "Cartpole":
        assert abs(abs(dof[0, 1, 1]) - W) < 1e-4 * W, dof[0, :, 1]
    assert wn.max() <= W * (1 + 1e-6), (wn, W)
    assert wn.max() >= W * (1 - 1e-6), (wn, W)       # the cap is what stopped it
    # below the cap the clamp changes nothing: an uncapped model gives the same step bit for bit
    root2 = np.zeros((1, 13), np.float32)
    root2[0, 2] = 5.0
    root2[0, 6] = 1.0
    dof2 = np.zeros((1, nd, 2), np.float32)
    dof2[0, :, 0] = np.array(tp.initial_dof_pos[:nd])
    dof2[0, DOF, 1] = 0.2 * W
    outs = []
    for cap in (W, 0.0):
        mm = mnp.copy()
        mm["link_max_ang_vel"] = cap
        r, d = root2.copy(), dof2.copy()
        O.simulate(mm, sp, r, d)
        outs.append((r, d))
    np.testing.assert_array_equal(outs[0][0], outs[1][0])
    np.testing.assert_array_equal(outs[0][1], outs[1][1])


# ------------------------------------------------------------------ the build-defined TGS solver
def test_tgs_selected_by_config():
    """sim.physx.solver picks the solver ('pgs', north_star's, by default; 'tgs' opts in); num_velocity_iterations
    goes to vel_iters; anything else is refused"""
    cfg = configs.task_config("Ant", 4)
    assert taskdefs.sim_params(cfg, 16).solver_type == 0
    cfg["sim"]["physx"]["solver"] = "TGS"
    cfg["sim"]["physx"]["num_velocity_iterations"] = 6
    sp = taskdefs.sim_params(cfg, 16)
    assert (sp.solver_type, sp.vel_iters) == (1, 6)
    cfg["sim"]["physx"]["solver"] = "sor"
    with pytest.raises(ValueError):
        taskdefs.sim_params(cfg, 16)


def test_tgs_without_rows_is_pgs():
    """no contact or limit rows (in the air, limits off): the sub-steps move the positions by sum (h / N) nu = h nu,
    so TGS is the PGS step up to the rounding of that sum"""
    out = []
    for st in (0, 1):
        spec, mnp, sp, tp = setup("Ant", gravity=(0.0, 0.0, -9.81), max_contacts=0)
        sp.limit_margin = -1.0
        sp.solver_type = st
        rng = np.random.default_rng(4)
        root, dof = rand_state(spec, tp, rng, z=5.0)
        dof[:, 0] = 0.5 * (np.array(tp.dof_lower[:8]) + np.array(tp.dof_upper[:8]))   # mid-range
        dof[:, 1] *= 0.2
        root, dof = root[None].copy(), dof[None].copy()
        act = (rng.uniform(-1, 1, (1, 8)) * 2).astype(np.float32)
        for _ in range(5):
            O.simulate(mnp, sp, root, dof, act)
            # the joints stay inside their limits (a limit row would make the solvers differ)
            assert np.all((dof[0, :, 0] > tp.dof_lower[:8]) & (dof[0, :, 0] < tp.dof_upper[:8]))
        out.append((root, dof))
    np.testing.assert_allclose(out[1][0], out[0][0], atol=2e-6, rtol=1e-6)
    np.testing.assert_allclose(out[1][1], out[0][1], atol=2e-6, rtol=1e-6)


def _settled_ant(solver, steps=300):
    spec, mnp, sp, tp = setup("Ant")
    sp.solver_type = solver
    root = np.zeros((1, 13), np.float32)
    root[0, 2] = 0.44
    root[0, 6] = 1.0
    dof = np.zeros((1, 8, 2), np.float32)
    dof[0, :, 0] = np.array(tp.initial_dof_pos[:8])
    for _ in range(steps):
        O.simulate(mnp, sp, root, dof)
    return mnp, sp, root, dof


def test_tgs_corrects_penetration_without_momentum():
    """A settled Ant pushed 2 cm into the plane: TGS moves the torso out through the sub-steps' displacement and its
    velocity sweeps take the depenetration velocity back out -- it is nearly out after one step and never rises above
    its rest height -- while PGS (Baumgarte, 0.2 per substep) needs ~10 steps"""
    tr = {}
    for st in (0, 1):
        mnp, sp, root, dof = _settled_ant(st)
        z0 = float(root[0, 2])
        assert np.abs(root[0, 7:13]).max() < 0.05
        root[0, 2] -= 0.02
        root[0, 7:13] = 0
        dof[0, :, 1] = 0
        tr[st] = []
        for _ in range(20):
            O.simulate(mnp, sp, root, dof)
            tr[st].append(float(root[0, 2]) - z0)
    pgs, tgs = np.array(tr[0]), np.array(tr[1])
    assert tgs[0] > -0.01 and abs(tgs[2]) < 1e-3, tgs       # measured: -6.6 mm after 1 step, -0.3 mm after 3
    assert abs(pgs[2]) > 4e-3                                # PGS: -5.2 mm after 3
    assert tgs.max() < 1e-3, tgs                             # no pop above the rest height (no injected momentum)
    assert abs(tgs[-1]) < 1e-4 and abs(pgs[-1]) < 1e-4


def test_tgs_dropped_ant_rests_and_holds_limits():
    """TGS keeps the contact / limit behaviour: a dropped Ant rests on its feet, and saturating torque does not
    push a joint through its limit"""
    mnp, sp, root, dof = _settled_ant(1)
    assert 0.3 < root[0, 2] < 0.44 and np.abs(root[0, 7:13]).max() < 0.05
    spec, mnp, sp, tp = setup("Ant", gravity=(0.0, 0.0, 0.0))
    sp.solver_type = 1
    root = np.zeros((1, 13), np.float32)
    root[0, 2] = 3.0
    root[0, 6] = 1.0
    dof = np.zeros((1, 8, 2), np.float32)
    dof[0, :, 0] = np.array(tp.initial_dof_pos[:8]) + 0.3
    act = np.full((1, 8), 15.0, np.float32)
    for _ in range(60):
        O.simulate(mnp, sp, root, dof, act)
    assert np.all(dof[0, :, 0] <= np.array(tp.dof_upper[:8]) + 0.02)


# ------------------------------------------------------------------ dry joint friction (MJCF frictionloss)
def hinge_link_spec(f, I=0.02):
    """a fixed base and one hinge link (COM on the axis, inertia I about it), MJCF frictionloss f"""
    root = M.Node(name="base", parent=-1, jtype=M.JT_FIXED, t=[0, 0, 0], r0=[0, 0, 0, 1], axis=[0, 0, 1], body=0)
    link = M.Node(name="hinge", parent=0, jtype=M.JT_HINGE, t=[0, 0, 0], r0=[0, 0, 0, 1], axis=[0, 0, 1], body=1,
                  mass=1.0, inertia=[I, I, I, 0.0, 0.0, 0.0], limited=0, frictionloss=f)
    bodies = [M.Body(name="base", node=0, pos=[0, 0, 0], quat=[0, 0, 0, 1], parent_body=-1, mass=0.0),
              M.Body(name="link", node=1, pos=[0, 0, 0], quat=[0, 0, 0, 1], parent_body=0, mass=1.0)]
    return M.ModelSpec(name="hinge", fixed_base=1, nodes=[root, link], bodies=bodies, geoms=[], pairs=[],
                       actuators=[], dof_names=["hinge"], angular_damping=0.0, max_angular_velocity=0.0)


def test_frictionloss_is_read_from_the_mjcf():
    """shared.xml:13's default joint class gives every hand joint frictionloss 0.001; the locomotion MJCFs none"""
    hand = M.pack_model(taskdefs.hand_spec("block"))
    assert np.all(hand["frictionloss"][1:25] == np.float32(0.001)) and hand["frictionloss"][0] == 0
    for name in ("ant", "humanoid", "cartpole"):
        assert not M.pack_model(M.load_builtin(name))["frictionloss"].any(), name


def test_frictionloss_decelerates_then_creeps():
    """-f tanh(qd / v_s) (v_s = MG_FRICTIONLOSS_VS 0.01): a hinge spun at 2 rad/s with no other force slows at
    f / I (Coulomb) and comes to rest; a constant torque 0.5 f then drives the creep rate v_s atanh(0.5)"""
    f, I = 0.01, 0.02
    mnp = M.pack_model(hinge_link_spec(f, I))
    sp = taskdefs.sim_params(configs.task_config("Ant", 1), 0)
    for i in range(3):
        sp.gravity[i] = 0.0
    sp.limit_margin = -1.0
    root = np.zeros((1, 13), np.float32)
    root[0, 6] = 1.0
    dof = np.zeros((1, 1, 2), np.float32)
    dof[0, 0, 1] = 2.0
    steps = 60                                  # 0.996 s: 2 - 0.5 t stays well above v_s
    for _ in range(steps):
        O.simulate(mnp, sp, root, dof)
    t = steps * sp.dt
    assert abs(dof[0, 0, 1] - (2.0 - f / I * t)) < 1e-3, dof[0, 0, 1]
    for _ in range(300):                         # ~4 s more: stopped (the law is smooth: |qd| << v_s at rest)
        O.simulate(mnp, sp, root, dof)
    assert abs(dof[0, 0, 1]) < 1e-4
    act = np.full((1, 1), 0.5 * f, np.float32)
    for _ in range(200):
        O.simulate(mnp, sp, root, dof, act)
    np.testing.assert_allclose(dof[0, 0, 1], 0.01 * np.arctanh(0.5), rtol=1e-3)
