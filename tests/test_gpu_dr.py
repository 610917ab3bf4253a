"""Domain randomization on the GPU, through the C ABI.

* mg_dr_apply / mg_dr_noise replay the reference's recorded draws (tests/golden/trace_ant_dr.npz, the
  same replay as tests/test_dr.py's oracle check): property values within 1e-6 relative, noise lambdas
  through the reference's actuation and observations (fp32 op order), randomize_buf exact.
* the physics kernels with an env_props table (the domain-randomized instances) vs the oracle applying
  the same rows to its fp64 model, for Ant and ShadowHand, from identical random states — the bars of
  tests/test_gpu_parity.py / test_gpu_hand.py.
* make() with task.randomize for Ant / Humanoid / ShadowHand: the shipped randomization_params run
  through the fused step, properties land in their ranges, and the per-env rows differ.
"""
import ctypes as C

import numpy as np
import pytest
import torch

import copy

import parity_stats as PS
import pyoracle as O
from migym import _abi, configs, model as M, taskdefs
from dr_trace import defaults, layout
from test_dr import replay_dr_trace

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


@pytest.fixture(scope="module")
def lib():
    assert torch.cuda.is_available(), "GPU tests need the MI355X"
    return _abi.lib()


class DeviceBackend:
    """mg_dr_apply / mg_dr_noise: the argument struct's host arrays are mirrored on the device"""

    OUT = {"x", "corr", "env_props", "randomize_buf"}

    def __init__(self, lib):
        self.lib = lib

    def _run(self, fn, args_bufs):
        a, bufs = args_bufs
        dev = {}
        for k, v in bufs.items():
            if v is None:
                continue
            t = torch.from_numpy(np.ascontiguousarray(v)).to(DEV)
            dev[k] = t
            setattr(a, k, t.data_ptr())
        _abi.check(fn(C.byref(a), torch.cuda.current_stream().cuda_stream), self.lib)
        torch.cuda.synchronize()
        for k in self.OUT & dev.keys():
            bufs[k][...] = dev[k].cpu().numpy().reshape(bufs[k].shape)

    def apply(self, args_bufs):
        self._run(self.lib.mg_dr_apply, args_bufs)

    def noise(self, args_bufs):
        self._run(self.lib.mg_dr_noise, args_bufs)


def test_dr_trace_matches_reference_gpu(lib):
    replay_dr_trace(DeviceBackend(lib))


def random_props(spec, n, rng):
    """env_props rows with every supported property perturbed"""
    stride, offs = layout(spec)
    props = np.tile(defaults(spec), (n, 1))
    nn = len(spec.nodes)
    for i in range(nn):
        r = props[:, _abi.MG_EP_NODE_WIDTH * i:_abi.MG_EP_NODE_WIDTH * (i + 1)]
        r[:, 0] *= rng.uniform(0.5, 1.5, n)          # mass
        r[:, 1] *= rng.uniform(0.5, 1.5, n)          # armature
        r[:, 2] *= rng.uniform(0.3, 3.0, n)          # damping
        r[:, 3] *= rng.uniform(0.5, 1.5, n)          # stiffness
        r[:, 4] += rng.normal(0, 0.02, n)            # lower
        r[:, 5] += rng.normal(0, 0.02, n)            # upper
        r[:, 6] *= rng.uniform(0.75, 1.5, n)         # drive kp
        r[:, 8] *= rng.uniform(0.3, 3.0, n)          # frictionloss (the hand's 0.001; 0 elsewhere)
    props[:, offs[1]:offs[1] + len(spec.geoms)] *= rng.uniform(0.3, 1.3, (n, len(spec.geoms)))
    nt = len(spec.tendons)
    props[:, offs[2]:offs[2] + 2 * nt] *= rng.uniform(0.3, 3.0, (n, 2 * nt))
    if spec.obj:
        props[:, offs[3] + 0] *= rng.uniform(0.5, 1.5, n)
        props[:, offs[3] + 1] *= rng.uniform(0.3, 1.3, n)
        props[:, offs[3] + 2] = rng.uniform(0.9, 1.1, n)
    return props


def agreement(a, b, atol, rtol):
    a = a.reshape(a.shape[0], -1)
    b = b.reshape(b.shape[0], -1)
    return ((np.abs(a - b) <= atol + rtol * np.abs(b)).all(axis=1)).mean()


def _physics_sensitive(mnp, sp, pre, i, checks, hand, eps=1e-6, ratio=0.25):
    """the oracle's own sensitivity at env i: its physics step alone from `pre`, once as given and once with the
    positions moved by eps; True if some element outside its tolerance moves by >= ratio x the largest such gap
    (e.g. several capsules a centimetre or two inside the egg, whose depenetration a 1e-6 m change moves by 1e-3)"""
    outs = []
    for pert in (0.0, eps):
        g = PS.env_slice(pre, i)
        if hand:
            g.root[:, 1, 0:3] += pert
        else:
            g.root[:, 0:3] += pert
        g.dof[..., 0] += pert
        O.lib().orc_simulate_views(mnp.ctypes.data, C.byref(sp), 1, C.byref(g.views()), 1)
        outs.append(g)
    for name, a, b, atol, rtol, pick in checks:
        ai, bi = np.ravel(a[i]).astype(np.float64), np.ravel(b[i]).astype(np.float64)
        diff = np.abs(ai - bi)
        out = diff > atol + rtol * np.abs(bi)   # the elements outside their tolerance
        if not out.any():
            continue
        moved = np.abs(np.ravel(pick(outs[1])).astype(np.float64) - np.ravel(pick(outs[0])))[out].max()
        if moved >= ratio * diff[out].max():
            return True
    return False


def _dr_explained(test, mnp, sp, pre, checks, hand):
    """every env within each check's tolerance unless orc_step_flips (with the env's own env_props row) puts its
    step at a discontinuity or the oracle is itself sensitive there (_physics_sensitive, capped at 1%); the
    exemptions' reach is capped (tests/parity_stats.py).  checks: (name, gpu, oracle, atol, rtol, pick) with
    pick(host) selecting the quantity from a one-env oracle copy"""
    bad = np.zeros(pre.n, bool)
    for name, a, b, atol, rtol, _ in checks:
        eb = PS.env_bad(a, b, atol, rtol)
        PS.record(test, name, a, b, envs_outside=int(eb.sum()), atol=atol, rtol=rtol)
        bad |= eb
    flags = PS.step_flags(mnp, sp, pre)
    PS.assert_steps_explained(test, bad[None], flags[None],
                              sens=lambda t, i: _physics_sensitive(mnp, sp, pre, i, checks, hand))


@pytest.mark.parametrize("layout", ["auto", "compact"])
@pytest.mark.parametrize("solver", ["pgs", "tgs"])
def test_dr_physics_matches_oracle_ant(lib, solver, layout, monkeypatch):
    """env_props rows on the GPU vs the oracle (solver tgs: the DR instance of the TGS kernels); at this
    batch the default picks the classic team layout, `compact` pins the 12-wave one (big batches)"""
    monkeypatch.setenv("MIGYM_LAYOUT", layout)
    cfg = configs.task_config("Ant", 16)
    cfg["sim"]["physx"]["solver"] = solver
    spec = M.load_builtin("ant")
    sp = taskdefs.sim_params(cfg, 16)
    n = 384
    rng = np.random.default_rng(21)
    props = random_props(spec, n, rng)
    root = np.zeros((n, 13), np.float32)
    root[:, 2] = rng.uniform(0.3, 0.6, n)
    q = rng.normal(0, 1, (n, 4)) * np.array([0.15, 0.15, 1.0, 1.0])
    root[:, 3:7] = q / np.linalg.norm(q, axis=1, keepdims=True)
    root[:, 7:13] = rng.normal(0, 0.5, (n, 6))
    lo = np.array([x.lower for x in spec.nodes[1:]])
    hi = np.array([x.upper for x in spec.nodes[1:]])
    dof = np.stack([lo + (hi - lo) * rng.uniform(0, 1, (n, 8)), rng.normal(0, 1, (n, 8))], -1).astype(np.float32)
    act = rng.uniform(-15, 15, (n, 8)).astype(np.float32)
    sens = np.zeros((n, 24), np.float32)
    mnp = M.pack_model(spec)
    # oracle
    h = O.HostEnv(taskdefs.task_params("Ant", cfg, spec), spec, n)
    h.root[:], h.dof[:], h.act_eff[:] = root, dof, act
    h.env_props = np.ascontiguousarray(props, np.float32)
    pre = copy.deepcopy(h)
    O.lib().orc_simulate_views(mnp.ctypes.data, C.byref(sp), n, C.byref(h.views()), 8)
    # GPU
    tr, td, ta = (torch.from_numpy(x).to(DEV) for x in (root, dof, act))
    ts, tf = torch.zeros((n, 24), device=DEV), torch.zeros((n, 8), device=DEV)
    tp = torch.from_numpy(np.ascontiguousarray(props, np.float32)).to(DEV)
    v = _abi.StateViews()
    v.root_states, v.dof_state, v.dof_actuation, v.sensors, v.dof_force = (x.data_ptr() for x in (tr, td, ta, ts, tf))
    v.env_props, v.env_props_stride = tp.data_ptr(), props.shape[1]
    sim = C.c_void_p()
    _abi.check(lib.mg_sim_create(mnp.ctypes.data, C.byref(sp), n, 0, C.byref(sim)), lib)
    _abi.check(lib.mg_sim_bind(sim, C.byref(v)), lib)
    _abi.check(lib.mg_sim_simulate(sim, torch.cuda.current_stream().cuda_stream), lib)
    torch.cuda.synchronize()
    lib.mg_sim_destroy(sim)
    rg, dg = tr.cpu().numpy(), td.cpu().numpy()
    assert np.isfinite(rg).all() and np.isfinite(dg).all()
    _dr_explained(f"test_dr_physics_matches_oracle_ant[{solver}-{layout}]", mnp, sp, pre,
                  [("root pose", rg[:, 0:7], h.root[:, 0:7], 2e-4, 0, lambda g: g.root[0, 0:7]),
                   ("root twist", rg[:, 7:13], h.root[:, 7:13], 2e-3, 2e-3, lambda g: g.root[0, 7:13]),
                   ("dof pos", dg[..., 0], h.dof[..., 0], 2e-4, 0, lambda g: g.dof[0, :, 0]),
                   ("dof vel", dg[..., 1], h.dof[..., 1], 2e-3, 2e-3, lambda g: g.dof[0, :, 1])], hand=False)
    # the properties matter: the same states without them end elsewhere
    h2 = O.HostEnv(taskdefs.task_params("Ant", cfg, spec), spec, n)
    h2.root[:], h2.dof[:], h2.act_eff[:] = root, dof, act
    O.lib().orc_simulate_views(mnp.ctypes.data, C.byref(sp), n, C.byref(h2.views()), 8)
    assert agreement(h2.dof[..., 1], h.dof[..., 1], 2e-3, 2e-3) < 0.5


@pytest.mark.parametrize("kind,solver", [("block", "pgs"), ("egg", "pgs"), ("pen", "pgs"), ("block", "tgs")])
def test_dr_physics_matches_oracle_hand(lib, kind, solver):
    """env_props rows (masses, drives, friction, object mass / friction / scale) on the GPU vs the oracle;
    the object's scale reaches every shape's size (box half extents, egg semi-axes, pen radius + length)."""
    from test_gpu_hand import DevHandEnv, PALM_DZ, hand_states, setup
    spec, sp, tp = setup(kind=kind)
    sp.solver_type = _abi.MG_SOLVER_TGS if solver == "tgs" else _abi.MG_SOLVER_PGS
    n = 192
    rng = np.random.default_rng(23)
    h = hand_states(spec, tp, n, rng, PALM_DZ[kind], pen=kind == "pen")
    props = np.ascontiguousarray(random_props(spec, n, rng), np.float32)
    e = DevHandEnv(h)
    mnp = M.pack_model(spec)
    h.env_props = props
    pre = copy.deepcopy(h)
    O.lib().orc_simulate_views(mnp.ctypes.data, C.byref(sp), n, C.byref(h.views()), 8)
    tp_ = torch.from_numpy(props).to(DEV)
    vg = e.views()
    vg.env_props, vg.env_props_stride = tp_.data_ptr(), props.shape[1]
    sim = C.c_void_p()
    _abi.check(lib.mg_sim_create(mnp.ctypes.data, C.byref(sp), n, 0, C.byref(sim)), lib)
    _abi.check(lib.mg_sim_bind(sim, C.byref(vg)), lib)
    _abi.check(lib.mg_sim_simulate(sim, torch.cuda.current_stream().cuda_stream), lib)
    torch.cuda.synchronize()
    lib.mg_sim_destroy(sim)
    rg, dg = e.root.cpu().numpy(), e.dof.cpu().numpy()
    assert np.isfinite(rg).all() and np.isfinite(dg).all()
    _dr_explained(f"test_dr_physics_matches_oracle_hand[{kind}{'-tgs' if solver == 'tgs' else ''}]", mnp, sp, pre,
                  [("object pose", rg[:, 1, 0:7], h.root[:, 1, 0:7], 2e-4, 0, lambda g: g.root[0, 1, 0:7]),
                   ("object twist", rg[:, 1, 7:13], h.root[:, 1, 7:13], 2e-3, 2e-3, lambda g: g.root[0, 1, 7:13]),
                   ("dof pos", dg[..., 0], h.dof[..., 0], 2e-4, 0, lambda g: g.dof[0, :, 0]),
                   ("dof vel", dg[..., 1], h.dof[..., 1], 2e-3, 2e-3, lambda g: g.dof[0, :, 1])], hand=True)


@pytest.mark.parametrize("task,n", [("Ant", 4096), ("Humanoid", 2048), ("ShadowHand", 1024)])
def test_make_with_randomize(task, n):
    """the shipped randomization_params of each task YAML through make() and the fused step"""
    import migym
    cfg = configs.task_config(task, n, sim_device=DEV)
    cfg["task"]["randomize"] = True
    env = migym.make(seed=3, task=task, num_envs=n, sim_device=DEV, rl_device=DEV, headless=True, cfg={"task": cfg})
    assert env.randomize and env.env_props.shape[0] == env.num_actors
    spec = env.model_spec
    props = env.env_props.cpu().numpy()
    base = defaults(spec)
    W = _abi.MG_EP_NODE_WIDTH
    mass = np.stack([props[:, W * b.node] for b in spec.bodies], 1)
    m0 = np.array([base[W * b.node] for b in spec.bodies])
    r = mass / np.where(m0 > 0, m0, 1)
    assert r[:, m0 > 0].min() >= 0.5 - 1e-6 and r[:, m0 > 0].max() <= 1.5 + 1e-6
    if task == "Humanoid":   # mass is setup_only with a linear schedule: scale 0 at setup, never randomized
        assert np.all(r[:, m0 > 0] == 1.0)
    else:
        assert np.std(r[:, m0 > 0]) > 0.1        # per-env draws differ
    g = torch.Generator(device=DEV).manual_seed(0)
    for _ in range(20):
        obs, rew, reset, extras = env.step(torch.rand((env.num_actors, env.num_actions), device=DEV, generator=g) * 2 - 1)
    torch.cuda.synchronize()
    assert torch.isfinite(obs["obs"]).all() and torch.isfinite(rew).all()
    assert "actions" in env.dr_randomizations and "observations" in env.dr_randomizations
    if task == "ShadowHand":   # gravity noise without a schedule (Humanoid's starts at scale 0)
        assert tuple(env.sim_params.gravity) != (0.0, 0.0, -9.81)
    env.close()


class _Gen:
    """actor_params_generator stand-in: a known vector per call (vec_task.py:736-760)"""

    def __init__(self, n):
        self.n, self.calls = n, 0

    def sample(self):
        self.calls += 1
        return 1.0 + 0.01 * np.arange(self.n) + 0.1 * self.calls


def test_actor_params_generator_ant():
    """get_actor_params_info + actor_params_generator: the randomized envs take og * sample (scaling) /
    og + sample (additive) from the generator's vector, setup_only entries (mass) are ignored, the other
    envs keep their rows, and a vector of the wrong length raises."""
    import migym
    n = 64
    cfg = configs.task_config("Ant", n, sim_device=DEV)
    cfg["task"]["randomize"] = True
    env = migym.make(seed=3, task="Ant", num_envs=n, sim_device=DEV, rl_device=DEV, headless=True, cfg={"task": cfg})
    dr = env.randomization_params
    params, names, lows, highs = env.get_actor_params_info(dr, 5)
    assert len(params) == len(names) == len(lows) == len(highs)
    nd = env.num_dof
    assert "dof_properties_0_damping_0" in names and f"dof_properties_0_damping_{nd - 1}" in names
    assert "rigid_body_properties_0_mass" in names
    i_lo = names.index("dof_properties_0_lower_0")
    assert lows[i_lo] == -np.inf and highs[i_lo] == np.inf          # gaussian: unbounded
    i_d = names.index("dof_properties_0_damping_3")
    assert (lows[i_d], highs[i_d]) == (0.5, 1.5)
    spec = env.model_spec
    base = defaults(spec)
    stride, offs = layout(spec)
    assert params[i_d] == pytest.approx(float(env.env_props[5, offs[0] + _abi.MG_EP_NODE_WIDTH * 4 + 2]), rel=0, abs=0)
    before = env.env_props.clone()
    gen = _Gen(len(names))
    env.actor_params_generator = gen
    ids = torch.tensor([2, 9, 40], device=DEV)
    mask = torch.zeros(n, dtype=torch.long, device=DEV)
    mask[ids] = 1
    env.randomize_buf_actors[:] = 10 ** 6
    env.apply_randomizations(dr, reset_mask=mask, increment=False)
    torch.cuda.synchronize()
    assert gen.calls == 3 and sorted(env.extern_actor_params) == [2, 9, 40]
    props = env.env_props.cpu().numpy()
    keep = np.ones(n, bool)
    keep[ids.cpu().numpy()] = False
    assert np.array_equal(props[keep], before.cpu().numpy()[keep])
    for e in (2, 9, 40):
        ext = env.extern_actor_params[e]
        for d in range(nd):
            col = offs[0] + _abi.MG_EP_NODE_WIDTH * (d + 1)
            j = names.index(f"dof_properties_0_damping_{d}")
            assert props[e, col + 2] == pytest.approx(base[col + 2] * ext[j], rel=1e-6, abs=1e-7)
            j = names.index(f"dof_properties_0_lower_{d}")
            assert props[e, col + 4] == pytest.approx(base[col + 4] + ext[j], rel=1e-6, abs=1e-6)
        # mass is setup_only: unchanged by the generator
        W = _abi.MG_EP_NODE_WIDTH
        assert np.array_equal(props[e, offs[0]::W][:len(spec.nodes)], before.cpu().numpy()[e, offs[0]::W][:len(spec.nodes)])
    env.actor_params_generator = _Gen(len(names) + 1)
    env.randomize_buf_actors[:] = 10 ** 6      # the call above restarted the randomized envs' counters
    with pytest.raises(Exception, match="extern_sample size"):
        env.apply_randomizations(dr, reset_mask=mask, increment=False)
    env.close()
