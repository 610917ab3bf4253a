"""Helpers of the domain-randomization parity tests (tests/test_dr*.py).

The reference run on the fake gym (tests/golden/make_traces.py ``run_ant_dr``) records every numpy draw
of apply_randomizations in call order, per step.  ``samples_for_step`` turns one step's draws into the
build's injected-sample matrix (actors x live attributes, the column order of ``migym.dr``) by walking
the same loops the reference walks (vec_task.py:733-833): the randomized envs in ascending order, then
the actor's properties, list properties element-major and array properties attribute-major; setup_only
attributes draw nothing after the first call.
"""
import os

import numpy as np

from migym import _abi, dr as DR

G = os.path.join(os.path.dirname(__file__), "golden")


def load_dr_trace():
    return dict(np.load(os.path.join(G, "trace_ant_dr.npz")))


def trace_params():
    import sys
    sys.path.insert(0, G)
    # the generator's parameter dict is plain data; importing make_traces would need the reference
    return {
        "frequency": 3,
        "observations": {"range": [0, .002], "range_correlated": [0, .001], "operation": "additive",
                         "distribution": "gaussian"},
        "actions": {"range": [0., .05], "range_correlated": [0, .015], "operation": "additive",
                    "distribution": "uniform"},
        "sim_params": {"gravity": {"range": [0, 0.4], "operation": "additive", "distribution": "gaussian",
                                   "schedule": "linear", "schedule_steps": 6}},
        "actor_params": {"ant": {
            "color": True,
            "rigid_body_properties": {"mass": {"range": [0.5, 1.5], "operation": "scaling",
                                               "distribution": "uniform", "setup_only": True}},
            "rigid_shape_properties": {"friction": {"num_buckets": 40, "range": [0.7, 1.3], "operation": "scaling",
                                                    "distribution": "uniform", "schedule": "linear",
                                                    "schedule_steps": 6},
                                       "restitution": {"range": [0., 0.7], "operation": "scaling",
                                                       "distribution": "uniform"}},
            "dof_properties": {"damping": {"range": [0.5, 1.5], "operation": "scaling", "distribution": "uniform",
                                           "schedule": "linear", "schedule_steps": 6},
                               "stiffness": {"range": [0.5, 1.5], "operation": "scaling",
                                             "distribution": "loguniform"},
                               "lower": {"range": [0, 0.01], "operation": "additive", "distribution": "gaussian"},
                               "upper": {"range": [0, 0.01], "operation": "additive", "distribution": "gaussian"}}}},
    }


def layout(spec):
    """Python statement of mg_env_props_layout (include/migym.h)."""
    nn, ng, nt = len(spec.nodes), len(spec.geoms), len(spec.tendons)
    W = _abi.MG_EP_NODE_WIDTH
    offs = (0, W * nn, W * nn + ng, W * nn + ng + 2 * nt)
    return (offs[3] + 4 + 3) & ~3, offs


def defaults(spec):
    """Python statement of mg_env_props_defaults."""
    stride, offs = layout(spec)
    row = np.zeros(stride, np.float32)
    for i, n in enumerate(spec.nodes):
        W = _abi.MG_EP_NODE_WIDTH
        row[W * i:W * i + W] = [n.mass, n.armature, n.damping, n.stiffness, n.lower, n.upper, n.drive_kp,
                                n.effort_limit, n.frictionloss]
    row[offs[1]:offs[1] + len(spec.geoms)] = 1.0
    for q, t in enumerate(spec.tendons):
        row[offs[2] + 2 * q:offs[2] + 2 * q + 2] = [t["limit_stiffness"], t["damping"]]
    row[offs[3]:offs[3] + 4] = [spec.obj["mass"] if spec.obj else 0.0, 1.0, 1.0, 0.0]
    return row


def tables(params, spec, actors):
    """(descs, live attrs (slot, desc, og), names, live index per name or -1, setup_only flag per name)."""
    stride, offs = layout(spec)
    descs, attrs, names = DR.build_actor_attrs(params["actor_params"], actors, spec, offs)
    live, live_of = [], []
    for (slot, d, og) in attrs:
        live_of.append(len(live) if slot is not None else -1)
        if slot is not None:
            live.append((slot, d, og))
    setup_only = [bool(params["actor_params"][a][p][at].get("setup_only", False)) if p != "scale" else
                  bool(params["actor_params"][a][p].get("setup_only", False)) for (a, p, e, at) in names]
    return descs, live, names, live_of, setup_only


def samples_for_step(draws, env_ids, n, names, live_of, setup_only, nlive, first):
    """Injected sample matrix (n, nlive) from one apply_randomizations call's numpy draws (after any
    sim_params draws have been taken off the front)."""
    out = np.zeros((n, max(nlive, 1)), np.float32)
    k = 0
    for e in env_ids:
        for i, _ in enumerate(names):
            if setup_only[i] and not first:
                continue
            if live_of[i] >= 0:
                out[e, live_of[i]] = draws[k]
            k += 1
    assert k == len(draws), (k, len(draws))
    return out


def pack(descs, live):
    """device/host byte tables of mg_dr_desc / mg_dr_attr"""
    db = np.frombuffer(b"".join(bytes(d) for d in descs), np.uint8).copy()
    ab = np.zeros((max(len(live), 1), 4), np.int32)
    for i, (s, d, og) in enumerate(live):
        ab[i, 0], ab[i, 1] = s, d
        ab[i, 2] = np.array([og], np.float32).view(np.int32)[0]
    return db, ab


def dr_tensor_props(env_props, spec, d_t):
    """(masses per body, frictions per geom, dof [damping, stiffness, lower, upper]) from env_props rows,
    in the layout of the reference's recorded setter values."""
    stride, offs = layout(spec)
    W = _abi.MG_EP_NODE_WIDTH
    mass = np.stack([env_props[:, W * b.node] for b in spec.bodies], 1)
    fric = env_props[:, offs[1]:offs[1] + len(spec.geoms)]
    nd = spec.num_dofs
    cols = {"damping": 2, "stiffness": 3, "lower": 4, "upper": 5}
    dof = np.stack([np.stack([env_props[:, W * (j + 1) + cols[k]] for j in range(nd)], 1)
                    for k in ("damping", "stiffness", "lower", "upper")])
    return mass, fric, dof
