"""Domain randomization against the reference.

tests/golden/trace_ant_dr.npz is the reference's Ant with ``task.randomize`` run on the fake gym
(make_traces.py ``run_ant_dr``): every numpy draw of apply_randomizations, every torch draw of the
observation / action noise lambdas, and the property values the reference hands to the gym setters
are recorded.  The build replays them injected:

* mg_dr_apply / orc_dr_apply: actor properties of the randomized envs (first call: every env with the
  setup_only mass; later: randomize_buf >= frequency on a resetting step), operations, schedules,
  buckets, and the randomize_buf bookkeeping — property values within 1e-6 relative (the reference's
  numpy arithmetic is float64 before the gym's float32 store);
* mg_dr_noise / orc_dr_noise: the noise lambdas with the persistent correlated noise, checked through the
  actuation the reference sets (actions) and the observations it returns — fp32 op order, rtol 1e-6.

The physical effect of the properties (PhysX) is unpinned like the rest of the physics; the GPU
physics with an env_props table is held to the oracle's (which applies the same rows to its fp64 model)
in tests/test_gpu_dr.py.
"""
import ctypes as C

import numpy as np
import pytest

import pyoracle as O
from migym import _abi, configs, dr as DR, model as M, taskdefs
from dr_trace import (dr_tensor_props, defaults, layout, load_dr_trace, pack, samples_for_step, tables,
                      trace_params)

RTOL = 1e-6


class _Host(DR.DomainRandomizationMixin):
    """the mixin's host-side parameter bookkeeping without a sim (noise-lambda parameters)"""

    def __init__(self):
        self.dr_randomizations = {}
        self.last_step = 0


def noise_args(entry, x, corr, refresh, z, c):
    a = _abi.DrNoiseArgs()
    a.x, a.x_clamped, a.clip = x.ctypes.data, None, float("inf")
    a.operation = _abi.MG_DR_ADDITIVE if entry["op"].__name__ == "add" else _abi.MG_DR_SCALING
    if "mu" in entry:
        a.distribution = _abi.MG_DR_GAUSSIAN
        a.scale, a.shift, a.c_scale, a.c_shift = entry["var"], entry["mu"], entry["var_corr"], entry["mu_corr"]
    else:
        a.distribution = _abi.MG_DR_UNIFORM
        a.scale, a.shift = entry["hi"] - entry["lo"], entry["lo"]
        a.c_scale, a.c_shift = entry["hi_corr"] - entry["lo_corr"], entry["lo_corr"]
    a.refresh_corr, a.corr, a.n = int(refresh), corr.ctypes.data, x.size
    a.injected = z.ctypes.data
    a.injected_corr = c.ctypes.data if refresh else None
    return a, {"x": x, "corr": corr, "injected": z, "injected_corr": c if refresh else None}


def apply_args(db, ab, nlive, stride, n, freq, first, inc, last_step, props, mask, rb, samples):
    a = _abi.DrApplyArgs()
    a.descs, a.attrs, a.nattr, a.stride = db.ctypes.data, ab.ctypes.data, nlive, stride
    a.n, a.frequency, a.first, a.increment, a.last_step = n, freq, int(first), int(inc), last_step
    a.env_props = props.ctypes.data
    a.reset_mask = None if mask is None else mask.ctypes.data
    a.randomize_buf, a.samples = rb.ctypes.data, samples.ctypes.data
    return a, {"descs": db, "attrs": ab, "env_props": props, "reset_mask": mask, "randomize_buf": rb,
               "samples": samples}


def test_env_props_layout_matches_c_abi():
    """the Python statement of the layout / defaults used by the tests equals the C ABI's (host code only)"""
    lib = _abi.lib()
    for name in ("ant", "humanoid", "shadow_hand"):
        spec = M.load_builtin(name)
        mnp = _abi.model_bytes(spec)
        offs = (C.c_int32 * 4)()
        stride = lib.mg_env_props_layout(mnp.ctypes.data, offs)
        assert (stride, tuple(offs)) == layout(spec)
        row = np.zeros(stride, np.float32)
        assert lib.mg_env_props_defaults(mnp.ctypes.data, row.ctypes.data) == 0
        np.testing.assert_array_equal(row, defaults(spec))


def test_actor_attr_tables_follow_reference_order():
    spec = M.load_builtin("ant")
    params = trace_params()
    descs, live, names, live_of, setup_only = tables(params, spec, {"ant": "articulation"})
    # rigid_body (9 bodies x mass) | rigid_shape (13 geoms x [friction, restitution]) | dof 4 attrs x 8
    assert len(names) == 9 + 2 * len(spec.geoms) + 4 * 8
    assert names[0] == ("ant", "rigid_body_properties", 0, "mass") and setup_only[0]
    assert names[9] == ("ant", "rigid_shape_properties", 0, "friction")
    assert names[10] == ("ant", "rigid_shape_properties", 0, "restitution") and live_of[10] == -1
    assert names[-1] == ("ant", "dof_properties", 7, "upper")
    assert len(live) == 9 + len(spec.geoms) + 32


def test_unsupported_attributes_raise():
    spec = M.load_builtin("ant")
    with pytest.raises(NotImplementedError):
        DR.build_actor_attrs({"ant": {"dof_properties": {"velocity": {"range": [0, 1], "operation": "additive",
                                                                      "distribution": "uniform"}}}},
                             {"ant": "articulation"}, spec, layout(spec)[1])
    with pytest.raises(NotImplementedError):
        DR.build_actor_attrs({"ant": {"scale": {"range": [0.9, 1.1], "operation": "scaling",
                                                "distribution": "uniform"}}}, {"ant": "articulation"}, spec,
                             layout(spec)[1])


def test_dof_friction_randomizes_the_frictionloss_column():
    """dof_properties.friction (vec_task.py:780-800) targets the node rows' frictionloss column (MG_EP_NODE_WIDTH 9,
    column 8) with the model's frictionloss as the original value (the hand's 0.001, shared.xml:13)"""
    from migym import taskdefs
    spec = taskdefs.hand_spec("block")
    _, attrs, names = DR.build_actor_attrs({"hand": {"dof_properties": {"friction": {
        "range": [0.5, 2.0], "operation": "scaling", "distribution": "uniform"}}}}, {"hand": "articulation"}, spec,
        layout(spec)[1])
    slots = [a[0] for a in attrs]
    assert [a[2] for a in attrs] == [np.float32(0.001)] * spec.num_dofs   # the original values
    W = _abi.MG_EP_NODE_WIDTH
    assert sorted(slots) == [W * (d + 1) + 8 for d in range(spec.num_dofs)]
    row = defaults(spec)
    assert all(row[s] == np.float32(0.001) for s in slots)


class OracleBackend:
    """orc_dr_apply / orc_dr_noise on host buffers"""

    def __init__(self):
        self.lib = O.lib()

    def apply(self, args_bufs):
        self.lib.orc_dr_apply(C.byref(args_bufs[0]))

    def noise(self, args_bufs):
        self.lib.orc_dr_noise(C.byref(args_bufs[0]))


def replay_dr_trace(backend):
    """Replays trace_ant_dr.npz through ``backend.apply`` / ``backend.noise`` (host-pointer argument
    structs; a device backend copies in and out) and the oracle's post-physics task layer."""
    d = load_dr_trace()
    params = trace_params()
    spec = M.load_builtin("ant")
    descs, live, names, live_of, setup_only = tables(params, spec, {"ant": "articulation"})
    db, ab = pack(descs, live)
    T, N = d["actions"].shape[:2]
    stride, _ = layout(spec)
    props = np.tile(defaults(spec), (N, 1))
    rb = np.zeros(N, np.int64)
    # ---- the first call (create_sim): gravity draws (3, schedule 0), then every env incl. setup_only mass
    init = d["init_np"].ravel()
    smp = samples_for_step(init[3:], range(N), N, names, live_of, setup_only, len(live), first=True)
    backend.apply(apply_args(db, ab, len(live), stride, N, 3, True, False, 0, props, None, rb, smp))
    mass, fric, dof = dr_tensor_props(props, spec, d)
    np.testing.assert_allclose(mass, d["init_mass"][0], rtol=RTOL)
    np.testing.assert_allclose(fric, d["init_fric"][0], rtol=RTOL)
    np.testing.assert_allclose(dof, d["init_dof"][0], rtol=RTOL, atol=1e-7)
    np.testing.assert_allclose(d["init_sim"][0], [0.0, 0.0, -9.81] + init[:3], rtol=1e-12)
    og_g = d["init_sim"][0]   # the first draw stays in the aliased "original" gravity
    # ---- the steps
    cfg = configs.task_config("Ant", N)
    tp = taskdefs.task_params("Ant", cfg, spec)
    tp.max_episode_length = int(d["episode_length"])
    h = O.HostEnv(tp, spec, N)
    host = _Host()
    corr_a = np.zeros(N * 8, np.float32)
    corr_o = np.zeros(N * 60, np.float32)
    npd, npl = d["np_draws"].ravel(), d["np_draws_len"]
    sset, frame, last_rand = d["sim_set"], 0, 0
    for name in ("observations", "actions"):   # the first call's noise parameters
        host._dr_nonphysical(name, params[name])
    k0 = 0
    for t in range(T):
        # vec_task.py:372-374: actions = noise_lambda(actions) before the clamp
        entry = host.dr_randomizations["actions"]
        x = np.ascontiguousarray(d["actions"][t], np.float32).copy()
        c, z = d["act_draws"][t]
        refresh = not np.isnan(c).all()
        backend.noise(noise_args(entry, x, corr_a, refresh, np.ascontiguousarray(z, np.float32),
                                 np.ascontiguousarray(c, np.float32)))
        np.testing.assert_allclose(np.clip(x, -1, 1) * 15.0, d["actuation"][t], rtol=RTOL, atol=1e-7)
        # post_physics_step on the injected physics output
        h.actions[:] = x
        h.root[:], h.dof[:], h.sensors[:] = d["phys_root"][t], d["phys_dof"][t], d["phys_sensors"][t]
        h.noise = O.f32(d["noise"][t])
        np.testing.assert_array_equal(h.reset, d["reset_in"][t])
        mask = h.reset.copy()
        h.post_physics(tp)
        frame += 1
        # reset_idx -> apply_randomizations (the reference calls it when some env resets)
        draws = npd[k0:k0 + npl[t]]
        k0 += npl[t]
        if mask.any():
            if frame - last_rand >= 3:   # do_nonenv_randomize
                last_rand = frame
                g = draws[:3]
                draws = draws[3:]
                host.last_step = frame
                for name in ("observations", "actions"):
                    host._dr_nonphysical(name, params[name])
                assert abs(DR.sched_scaling(params["sim_params"]["gravity"], frame) - min(frame, 6) / 6) < 1e-12
                np.testing.assert_allclose(sset[t], og_g + g, rtol=1e-12)
            rand = (rb + 1 >= 3) & (mask != 0)
            smp = samples_for_step(draws, np.nonzero(rand)[0], N, names, live_of, setup_only, len(live), first=False)
            backend.apply(apply_args(db, ab, len(live), stride, N, 3, False, True, frame, props, mask, rb, smp))
        else:
            rb += 1
            assert len(draws) == 0
        np.testing.assert_array_equal(rb, d["randomize_buf"][t])
        mass, fric, dof = dr_tensor_props(props, spec, d)
        np.testing.assert_allclose(mass, d["mass_set"][t], rtol=RTOL)
        np.testing.assert_allclose(fric, d["fric_set"][t], rtol=RTOL)
        np.testing.assert_allclose(dof, d["dof_set"][t], rtol=RTOL, atol=1e-7)
        # vec_task.py:398-400: obs_buf = noise_lambda(obs_buf)
        entry = host.dr_randomizations["observations"]
        o = h.obs.copy()
        c, z = d["obs_draws"][t]
        refresh = not np.isnan(c).all()
        backend.noise(noise_args(entry, o, corr_o, refresh, np.ascontiguousarray(z, np.float32),
                                 np.ascontiguousarray(c, np.float32)))
        np.testing.assert_allclose(o, d["obs"][t], rtol=RTOL, atol=1e-6)
        np.testing.assert_allclose(h.rew, d["rew"][t], rtol=1e-5, atol=1e-5)
        np.testing.assert_array_equal(h.reset, d["reset"][t])
    # the trace exercises re-randomization after setup and the bucketing
    assert (d["randomize_buf"] == 0).any()
    f = d["fric_set"][-1]
    assert len(np.unique(np.round(f, 6))) < f.size   # bucketed values repeat


def test_dr_trace_matches_reference_oracle():
    replay_dr_trace(OracleBackend())
