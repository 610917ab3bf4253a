"""Helpers of the GPU-vs-oracle physics tests (test infrastructure): error statistics, and the
discontinuities of the build's physics that let an fp32 (GPU) and an fp64 (oracle) step of the same state
part ways:

  * contact threshold: a candidate whose gap lies within `delta` of contact_offset is a contact on one side
    and not on the other (detected by regenerating the oracle's contacts with the offset moved by +-delta; the hand's explicit
    MJCF pairs switch on at distance 0, and their threshold is moved by +-delta the same way);
  * joint-limit rows: a DOF within `dq` of the limit margin (limit_margin 0.1 rad from a limit);
  * PD drive saturation (hand tasks): an explicit drive force within `df` of its effort limit;
  * deep penetration (a contact deeper than 5 mm, reachable only where a reset places the object into hand
    geometry): the normal of a point inside a box is its nearest face's, a discontinuous function of position.

  * any other state where the oracle itself is sensitive: replayed alone from step 1 with positions
    perturbed by 1e-6, the oracle moves by at least a quarter of the GPU-vs-oracle difference
    (oracle_sensitive; e.g. a separating-axis tie between a face and an edge axis, a friction-cone clamp).

An env whose GPU and oracle results disagree is accepted only when one of these holds for it.  Set
MIGYM_PARITY_REPORT=<path> to collect the max / 99.9th-percentile errors of every check into a JSON file.
"""
import copy
import json
import os

import numpy as np

import pyoracle as O

_REPORT = {}


def err_stats(a, b):
    d = np.abs(np.asarray(a, np.float64) - np.asarray(b, np.float64)).ravel()
    if d.size == 0:
        return {"max": 0.0, "p999": 0.0, "p99": 0.0}
    return {"max": float(d.max()), "p999": float(np.quantile(d, 0.999)), "p99": float(np.quantile(d, 0.99))}


def record(test, name, a, b, **extra):
    st = err_stats(a, b)
    st.update({k: (float(v) if isinstance(v, (float, np.floating)) else v) for k, v in extra.items()})
    _REPORT.setdefault(test, {})[name] = st
    return st


def write_report():
    path = os.environ.get("MIGYM_PARITY_REPORT")
    if path and _REPORT:
        os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
        old = {}
        if os.path.exists(path):
            with open(path) as f:
                old = json.load(f)
        old.update(_REPORT)
        with open(path, "w") as f:
            json.dump(old, f, indent=1, sort_keys=True)


def env_bad(a, b, atol, rtol):
    """per-env: some element outside atol + rtol |b|"""
    a = np.asarray(a).reshape(len(a), -1)
    b = np.asarray(b).reshape(len(b), -1)
    return ~((np.abs(a - b) <= atol + rtol * np.abs(b)).all(axis=1))


def contact_flips(mnp, sp, roots, dofs, delta=1e-4, cap=64):
    """per env: the oracle's contact set changes when contact_offset moves by +-delta"""
    lo, hi = copy.copy(sp), copy.copy(sp)
    lo.contact_offset = sp.contact_offset - delta
    hi.contact_offset = sp.contact_offset + delta
    out = np.zeros(len(roots), bool)
    for i in range(len(roots)):
        r = np.ascontiguousarray(roots[i], np.float32).ravel()
        d = np.ascontiguousarray(dofs[i], np.float32)
        out[i] = len(O.contacts(mnp, lo, r, d, cap)) != len(O.contacts(mnp, hi, r, d, cap))
    if int(mnp["pair_mjcf"]) and int(mnp["num_pairs"]) > 0:
        # explicit MJCF pairs switch on at distance 0, not at the offset: count the pair contacts alone (the
        # model with pairs minus the model without) with the pairs' threshold moved to +-delta
        mp, m0 = mnp.copy(), mnp.copy()
        mp["pair_mjcf"] = 0
        m0["num_pairs"] = 0
        lo0, hi0 = copy.copy(sp), copy.copy(sp)
        lo0.contact_offset, hi0.contact_offset = -delta, delta
        for i in range(len(roots)):
            r = np.ascontiguousarray(roots[i], np.float32).ravel()
            d = np.ascontiguousarray(dofs[i], np.float32)
            npl = len(O.contacts(mp, lo0, r, d, cap)) - len(O.contacts(m0, lo0, r, d, cap))
            nph = len(O.contacts(mp, hi0, r, d, cap)) - len(O.contacts(m0, hi0, r, d, cap))
            out[i] |= npl != nph
    return out


def deep_contacts(mnp, sp, roots, dofs, depth=5e-3, cap=64):
    """per env: an oracle contact deeper than `depth`"""
    out = np.zeros(len(roots), bool)
    for i in range(len(roots)):
        cs = O.contacts(mnp, sp, np.ascontiguousarray(roots[i], np.float32).ravel(),
                        np.ascontiguousarray(dofs[i], np.float32), cap)
        out[i] = any(c[7] < -depth for c in cs)
    return out


def limit_flips(q, lower, upper, margin, dq=1e-4):
    """per env: a DOF position within dq of the joint-limit row threshold (limit_margin from a limit)"""
    q = np.asarray(q, np.float64)
    lo = np.abs((q - np.asarray(lower)) - margin) < dq
    hi = np.abs((np.asarray(upper) - q) - margin) < dq
    return (lo | hi).reshape(len(q), -1).any(axis=1)


def drive_flips(q, qd, targets, kp, damping, effort, df=1e-2):
    """per env: an explicit PD force kp (q* - q) - b qd within df (relative) of its effort limit"""
    fe = np.asarray(kp) * (np.asarray(targets) - q) - np.asarray(damping) * qd
    lim = np.asarray(effort)
    near = (np.asarray(kp) > 0) & (np.abs(np.abs(fe) - lim) < df * np.maximum(lim, 1e-6))
    return near.reshape(len(q), -1).any(axis=1)


def assert_explained(bad, explained, what):
    """every disagreeing env must sit at one of the discontinuities"""
    unexplained = np.flatnonzero(bad & ~explained)
    assert unexplained.size == 0, (f"{what}: {unexplained.size} of {int(bad.sum())} disagreeing envs are not at a "
                                   f"contact / limit / drive threshold or a deep penetration: {unexplained[:10].tolist()}")


def env_slice(h, i):
    """a one-env copy of a pyoracle HostEnv / HandHostEnv (every per-env array sliced)"""
    g = copy.copy(h)
    for k, v in vars(h).items():
        if isinstance(v, np.ndarray):
            setattr(g, k, v[i:i + 1].copy() if v.shape[:1] == (h.n,) else v.copy())
    g.n = 1
    return g


def oracle_sensitive(mnp, sp, tp, pre, actions, i, gpu_out, oracle_out, seed, hand, t0=1, eps=1e-6, ratio=0.25):
    """the oracle's own sensitivity at env i: replay steps t0.. of env i alone (RNG keyed by its index), once as
    recorded and once with its positions perturbed by eps; True if the perturbed replay's final observation
    moves by >= ratio x the GPU-vs-oracle difference"""
    runs = []
    for pert in (0.0, eps):
        g = env_slice(pre[t0], i)
        if hand:
            g.root[:, 1, 0:3] += pert
        else:
            g.root[:, 0:3] += pert
        g.dof[..., 0] += pert
        for t in range(t0, len(actions)):
            g.actions[:] = actions[t][i:i + 1]
            g.env_step(mnp, sp, tp, seed=seed, step=t, threads=1, env_offset=i)
        runs.append(g.obs[0].astype(np.float64).copy())
    moved = np.abs(runs[1] - runs[0]).max()
    gap = np.abs(np.asarray(gpu_out, np.float64) - np.asarray(oracle_out, np.float64)).max()
    return moved >= ratio * gap
