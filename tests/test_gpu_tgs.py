"""GPU parity of the build-defined TGS solver (sim.physx.solver: tgs) against the oracle's TGS
(oracle/oracle_physics.c substep: N position sub-steps of h / N with per-sweep targets from the moved gaps, then
max(N, num_velocity_iterations) bias-free velocity sweeps, positions from the accumulated displacement).

The same gates as the PGS path: one simulate from random states (tests/test_gpu_parity.py tolerances, every env
unless orc_step_flips puts its step at a discontinuity), the fused step teacher-forced against orc_env_step with
north_star's per-column-group 1e-4 relative, the ShadowHand fused step (block / egg / pen), and a full-size make()
rollout.  The reference's TGS is PhysX's (closed): this solver's parity is to its own oracle, "parity unpinned"
against the reference's physics as the PGS path's is.
"""

import numpy as np
import pytest
import torch

import parity_stats as PS
import pyoracle as O
import test_gpu_hand as GH
import test_gpu_parity as GP
from migym import _abi, configs, model as M

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


@pytest.fixture(scope="module")
def lib():
    assert torch.cuda.is_available(), "GPU tests need the MI355X"
    return _abi.lib()


def tgs(sp):
    sp.solver_type = _abi.MG_SOLVER_TGS
    return sp


@pytest.mark.parametrize("task,n,z", [("Ant", 512, (0.25, 0.7)), ("Humanoid", 256, (0.6, 1.4)),
                                      ("Cartpole", 256, (2.0, 2.0))])
def test_tgs_physics_step_matches_oracle(lib, task, n, z):
    """one gym.simulate (TGS) from random states (deep contacts, joints up to 5 % past their limits) against the
    oracle's TGS: positions 2e-4, velocities 2e-3 + 2e-3 |v|, every env unless its step is flagged"""
    spec, sp, tp = GP.setup(task)
    tgs(sp)
    rng = np.random.default_rng(19)
    root, dof = GP.random_states(spec, tp, n, rng, z)
    if task == "Cartpole":
        root[:, :] = 0
        root[:, 2] = 2.0
        root[:, 6] = 1.0
    act = (rng.uniform(-1, 1, (n, spec.num_dofs)) * (15.0 if task == "Ant" else 50.0)).astype(np.float32)
    ns = max(len(spec.sensors), 1)
    sens_h = np.zeros((n, ns * 6), np.float32)
    dfor_h = np.zeros((n, spec.num_dofs), np.float32)
    mnp = M.pack_model(spec)
    r_h, d_h = root.copy(), dof.copy()
    O.simulate(mnp, sp, r_h, d_h, act, sens_h, dfor_h, threads=8)
    rg, dg, sg, fg = GP._gpu_simulate(lib, mnp, sp, root, dof, act, ns)
    if task != "Cartpole":   # the solver really is another one: the same states under PGS end elsewhere (the
        sp_pgs = GP.setup(task)[1]   # cart and pole here meet no limit: no rows, the two solvers coincide)
        r_p, d_p = root.copy(), dof.copy()
        O.simulate(mnp, sp_pgs, r_p, d_p, act, threads=8)
        assert np.abs(d_p[..., 1] - d_h[..., 1]).max() > 1e-2
    test = f"test_tgs_physics_step_matches_oracle[{task}]"
    checks = [("root pose", rg[:, 0:7], r_h[:, 0:7], 2e-4, 0), ("dof pos", dg[..., 0], d_h[..., 0], 2e-4, 0),
              ("root twist", rg[:, 7:13], r_h[:, 7:13], 2e-3, 2e-3), ("dof vel", dg[..., 1], d_h[..., 1], 2e-3, 2e-3)]
    if len(spec.sensors):
        checks.append(("sensors", sg, sens_h, 1e-2 * max(1.0, np.abs(sens_h).max()), 0))
    checks.append(("dof force", fg, dfor_h, 1e-2 * max(1.0, np.abs(dfor_h).max()), 0))
    bad = np.zeros(n, bool)
    for name, a, b, atol, rtol in checks:
        eb = PS.env_bad(a, b, atol, rtol)
        PS.record(test, name, a, b, envs_outside=int(eb.sum()), atol=atol, rtol=rtol)
        bad |= eb
    pre = O.HostEnv(tp, spec, n)
    pre.root[:], pre.dof[:], pre.act_eff[:] = root, dof, act
    PS.assert_steps_explained(test, bad[None], PS.step_flags(mnp, sp, pre)[None], sens=None)


@pytest.mark.parametrize("layout", ["auto", "compact"])
@pytest.mark.parametrize("task,n", [("Ant", 256), ("Humanoid", 128)])
def test_tgs_fused_env_step_matches_oracle(lib, task, n, layout, monkeypatch):
    """mg_env_step with the TGS instances vs orc_env_step (TGS) over 4 teacher-forced control steps, device-RNG
    resets; north_star's 1e-4 relative per column group (test_gpu_parity.assert_north_star_rtol).  `compact` pins
    the 12-wave team layout the big batches run (the default picks the classic one at these sizes)"""
    monkeypatch.setenv("MIGYM_LAYOUT", layout)
    spec, sp, tp = GP.setup(task)
    tgs(sp)
    h = O.HostEnv(tp, spec, n)
    rng = np.random.default_rng(23)
    acts = [rng.uniform(-1.2, 1.2, (n, tp.num_actions)).astype(np.float32) for _ in range(4)]
    res = GP._teacher_forced(lib, f"test_tgs_fused_env_step_matches_oracle[{task}-{layout}]", spec, sp, tp, h, 4, acts,
                             seed=5)
    GP.assert_north_star_rtol(res)


def test_tgs_multi_agent_env_step_matches_oracle(lib):
    """MAAnt (4 agents) with TGS: the fused step vs the oracle, teacher-forced"""
    spec, sp, tp = GP.ma_setup(4)
    tgs(sp)
    n = 4 * 64
    h = O.HostEnv(tp, spec, n)
    rng = np.random.default_rng(29)
    acts = [rng.uniform(-1, 1, (n, tp.num_actions)).astype(np.float32) for _ in range(3)]
    GP._teacher_forced(lib, "test_tgs_multi_agent_env_step_matches_oracle", spec, sp, tp, h, 3, acts, seed=9)


@pytest.mark.parametrize("kind", ["block", "egg", "pen"])
def test_tgs_hand_fused_env_step_matches_oracle(lib, kind):
    """ShadowHand (8 position sub-steps, the free object's columns in the displacement) with TGS: mg_env_step vs
    orc_hand_env_step over 12 teacher-forced control steps, as test_gpu_hand.test_hand_fused_env_step_matches_oracle"""
    spec, sp, tp = GH.setup(kind=kind)
    tgs(sp)
    n = 192
    h = O.HandHostEnv(tp, spec, n)
    rng = np.random.default_rng(3)
    acts = [rng.uniform(-1.2, 1.2, (n, tp.num_actions)).astype(np.float32) for _ in range(12)]
    # the exemption predicates' reach: bit 1 (a contact candidate within rounding of the contact offset) flags 4.0 /
    # 3.6 / 5.1 % of the block / egg / pen env-steps (PGS 2.0 / 1.9 / 1.7 %: the sub-steps' displacement leaves the
    # pen lying nearer the offset), 4.5 / 4.6 / 5.5 % in all; of those only 4 pen env-steps disagree (round 5)
    ncon = GH._hand_teacher_forced(lib, f"test_tgs_hand_fused_env_step_matches_oracle[{kind}]", spec, sp, tp, h, 12,
                                   acts, 5, reach_cap=0.08)
    assert ncon >= n // 2


def test_tgs_hand_physics_step_matches_oracle(lib):
    """one simulate of the block on the palm (object contacts in most envs) with TGS, every env against the oracle"""
    spec, sp, tp = GH.setup(kind="block")
    tgs(sp)
    n = 256
    rng = np.random.default_rng(5)
    h = GH.hand_states(spec, tp, n, rng, GH.PALM_DZ["block"])
    GH._physics_vs_oracle(lib, spec, sp, h, rng, n)


@pytest.mark.parametrize("task,n", [("Ant", 16384), ("ShadowHand", 4096)])
def test_tgs_make_rollout(task, n):
    """migym.make with sim.physx.solver: tgs at a bench size: 20 steps stay finite, the torsos above the ground /
    the objects in the scene, and the run differs from the PGS one of the same seed (the TGS kernels ran)"""
    import migym
    finals = []
    for solver in ("pgs", "tgs"):
        cfg = configs.task_config(task, n, sim_device=DEV)
        cfg["sim"]["physx"]["solver"] = solver
        env = migym.make(seed=0, task=task, num_envs=n, sim_device=DEV, rl_device=DEV, headless=True,
                         cfg={"task": cfg})
        assert env.sim_params.solver_type == (_abi.MG_SOLVER_TGS if solver == "tgs" else _abi.MG_SOLVER_PGS)
        g = torch.Generator(device=DEV).manual_seed(0)
        for _ in range(20):
            a = torch.rand((n, env.num_actions), device=DEV, generator=g) * 2 - 1
            obs_dict, rew, reset, extras = env.step(a)
        torch.cuda.synchronize()
        obs = obs_dict["obs"]
        assert torch.isfinite(obs).all() and torch.isfinite(rew).all() and torch.isfinite(env.root_states).all()
        if task == "Ant":
            assert float(env.root_states[:, 2].min()) > 0.0
        finals.append(obs.clone())
        env.close()
    assert not torch.equal(finals[0], finals[1])
