"""The step flags (oracle orc_step_flips, tests/parity_stats.py) on the CPU, against a second fp32 implementation.

The GPU parity tests accept an env-step where the kernel (fp32) and the checker (fp64) part ways only when
orc_step_flips puts that step at a discontinuity of the physics.  The oracle's fp32 build (liboracle_f32.so, the
same C restated in float; bench.py's CPU baseline) rounds differently from both, so it is an independent witness
for the flags: on the stress states of the GPU tests, every env where it leaves the GPU tests' tolerances of the
fp64 result must be flagged, within the same reach caps; and calm free-flight states must raise no flag at all.
"""
import copy

import numpy as np
import pytest

import parity_stats as PS
import pyoracle as O
from migym import model as M
from test_gpu_hand import hull_exact_states
from test_gpu_parity import random_states, setup as loco_setup


def _spin_states(task, n, seed, rate=40.0, spin=80.0):
    """test_gpu_parity.py fast = 1: in the air, joint rates ~N(0, rate), root spins ~N(0, spin/2)"""
    spec, sp, tp = loco_setup(task)
    rng = np.random.default_rng(seed)
    root, dof = random_states(spec, tp, n, rng, (4.0, 5.0))
    dof[:, :, 1] *= rate
    root[:, 10:13] *= spin
    act = (rng.uniform(-1, 1, (n, spec.num_dofs)) * (15.0 if task == "Ant" else 50.0)).astype(np.float32)
    return spec, sp, tp, root, dof, act


def _simulate(mnp, spec, sp, root, dof, act, fp32):
    r, d = root.copy(), dof.copy()
    n = len(r)
    sens = np.zeros((n, max(len(spec.sensors), 1) * 6), np.float32)
    dfor = np.zeros((n, spec.num_dofs), np.float32)
    O.simulate(mnp, sp, r, d, act, sens, dfor, threads=8, fp32=fp32)
    return r, d


@pytest.mark.parametrize("task,n", [("Ant", 2048), ("Humanoid", 4096)])
def test_fp32_build_disagreements_are_flagged_at_spin(task, n):
    """fast-spin states: the angular-velocity cap acts in every env; every fp32-vs-fp64 disagreement beyond the
    spin-scaled tolerance (PS.spin_bad) is flagged, and the flags reach at most 12 % (the GPU test's cap)"""
    spec, sp, tp, root, dof, act = _spin_states(task, n, seed=8)
    mnp = M.pack_model(spec)
    r64, d64 = _simulate(mnp, spec, sp, root, dof, act, False)
    r32, d32 = _simulate(mnp, spec, sp, root, dof, act, True)
    assert np.abs(d32 - d64).max() > 0  # two implementations, not one
    bad = PS.spin_bad(r32, d32, r64, d64, root, dof, sp.dt)
    pre = O.HostEnv(tp, spec, n)
    pre.root[:], pre.dof[:], pre.act_eff[:] = root, dof, act
    flags = PS.step_flags(mnp, sp, pre)
    assert (flags & 64).any()   # the cap-interval bit is what these states exercise
    # the rest only where the fp64 dynamics themselves carry the first substep's fp32 position drift (~3e-6 here) to
    # a quarter of the gap (a limb deep past its limit under ~100 rad/s spins: velocity per position ~4e3 / s, the
    # top 3 % of these states), within the 1 % sensitivity cap
    out32 = np.concatenate([r32, d32.reshape(n, -1)], 1)
    out64 = np.concatenate([r64, d64.reshape(n, -1)], 1)
    drift = PS.first_substep_drift(mnp, sp, root, dof, act)
    sens = lambda t, i: PS.simulate_sensitive(mnp, sp, root, dof, act, i, out32, out64, eps=drift[i])
    PS.assert_steps_explained(f"test_step_flags[{task}-spin]", bad[None], flags[None], sens=sens, reach_cap=0.12)


@pytest.mark.parametrize("kind", ["block", "pen"])
def test_fp32_build_disagreements_are_flagged_on_hull_features(kind):
    """the exact-hull placements of test_gpu_hand.py (an edge across a hull edge, a pen across a face next to its
    ridges, gaps -0.5 .. 1.5 mm): every fp32-vs-fp64 disagreement is flagged, reach at most 10 %"""
    n = 1024
    rng = np.random.default_rng(13)
    spec, sp, tp, h = hull_exact_states(kind, n, rng)
    h.rb_forces[: n // 2, len(spec.bodies)] = rng.normal(0, 0.3, (n // 2, 3))
    mnp = M.pack_model(spec)
    h0, h32 = copy.deepcopy(h), copy.deepcopy(h)
    h.simulate(mnp, sp, threads=8)
    h32.simulate(mnp, sp, threads=8, fp32=True)
    assert np.abs(h32.root - h.root).max() > 0
    bad = np.zeros(n, bool)
    for a, b, atol, rtol in ((h32.root[:, 1, 0:7], h.root[:, 1, 0:7], 2e-4, 0),
                             (h32.root[:, 1, 7:13], h.root[:, 1, 7:13], 2e-3, 2e-3),
                             (h32.dof[..., 0], h.dof[..., 0], 2e-4, 0), (h32.dof[..., 1], h.dof[..., 1], 2e-3, 2e-3)):
        bad |= PS.env_bad(a, b, atol, rtol)
    PS.assert_steps_explained(f"test_step_flags[hull-{kind}]", bad[None], PS.step_flags(mnp, sp, h0)[None],
                              reach_cap=0.10)


@pytest.mark.parametrize("task", ["Ant", "Humanoid"])
def test_flags_quiet_in_calm_free_flight(task):
    """in the air (no contact candidate within reach), joints mid-range, rates well below the cap, actuation well
    below the effort limits: no predicate may fire, and the two builds agree to the plain tolerances"""
    spec, sp, tp = loco_setup(task)
    n = 512
    rng = np.random.default_rng(3)
    root, dof = random_states(spec, tp, n, rng, (4.0, 5.0))
    lo, hi = np.array(tp.dof_lower[:spec.num_dofs]), np.array(tp.dof_upper[:spec.num_dofs])
    dof[:, :, 0] = lo + (hi - lo) * rng.uniform(0.3, 0.7, (n, spec.num_dofs))
    dof[:, :, 1] *= 0.2
    root[:, 7:13] *= 0.2
    act = (rng.uniform(-1, 1, (n, spec.num_dofs)) * 2.0).astype(np.float32)
    mnp = M.pack_model(spec)
    pre = O.HostEnv(tp, spec, n)
    pre.root[:], pre.dof[:], pre.act_eff[:] = root, dof, act
    flags = PS.step_flags(mnp, sp, pre)
    assert (flags == 0).all(), np.unique(flags[flags != 0])
    r64, d64 = _simulate(mnp, spec, sp, root, dof, act, False)
    r32, d32 = _simulate(mnp, spec, sp, root, dof, act, True)
    np.testing.assert_allclose(r32[:, 0:7], r64[:, 0:7], atol=2e-4)
    np.testing.assert_allclose(d32[..., 0], d64[..., 0], atol=2e-4)
    np.testing.assert_allclose(r32[:, 7:13], r64[:, 7:13], atol=2e-3, rtol=2e-3)
    np.testing.assert_allclose(d32[..., 1], d64[..., 1], atol=2e-3, rtol=2e-3)
