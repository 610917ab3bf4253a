"""Domain randomization on the MI355X path.

Reference: ``VecTask.apply_randomizations`` (tasks/base/vec_task.py:612-842) with
``utils/dr_utils.py`` (generate_random_samples, get_bucketed_val, apply_random_samples).  The
reference re-sets gym actor properties in a per-env Python loop inside ``reset_idx``, which needs
the host to know which envs reset (``reset_buf.nonzero()``).  Here:

* the per-actor physical properties live in one device table ``env_props`` (N*A rows, layout of
  ``mg_env_props_layout``) bound to the sim; ``mg_dr_apply`` rewrites the rows of the actors being
  randomized (first call: every actor; later: ``randomize_buf >= frequency`` on a resetting step)
  on the device, one thread per actor, and the physics kernels read the table;
* the observation / action noise lambdas are one elementwise HIP kernel each (``mg_dr_noise``),
  with the reference's fp32 operation order and its persistent correlated-noise tensor;
* ``sim_params`` attributes (gravity, rest_offset) are drawn on the host with ``np.random`` like the
  reference and pushed with ``mg_sim_set_params``.

Supported actor properties (everything the shipped task configs randomize):
  dof_properties       damping, stiffness (the PD drive's kp on position-driven DOFs), lower, upper,
                       armature, effort, friction (the joint's dry friction bound, mg_model.frictionloss:
                       randomizing it scales the MuJoCo-style frictionloss torque bound f, DESIGN.md §4, not a
                       PhysX-style joint friction coefficient -- parity unpinned)
  rigid_body_properties  mass (inertia rescaled with it, recomputeInertia=True)
  rigid_shape_properties friction (a contact's friction is the mean of its two shapes'), restitution
                       (accepted; the build's contacts are inelastic, so it has no effect)
  tendon_properties    damping, limit_stiffness (stiffness accepted: the fixed-tendon model has none)
  scale                the free object only (half extents x s, mass x s^3, inertia x s^5)
  color                ignored (no renderer)
Anything else raises ``NotImplementedError`` at setup.

External samples (vec_task.py:566-604, 736-760, 832-840): ``get_actor_params_info`` lists the randomized
actor parameters (values of an env's row, names ``<prop>_<element>_<attr>[_<dof>]``, uniform ranges or
+-inf) in the reference's draw order, and an ``actor_params_generator`` (any object with ``sample()``
returning one flat vector of that length per env) replaces the per-attribute draws of every env being
randomized: the value is scheduled like dr_utils.generate_random_samples' ``extern_sample`` branch and
applied with the attribute's operation and buckets.  The reference resolves the vector's slices with a
helper it never defines (``get_attr_val_from_sample`` is not in its tree), so the slicing here is this
build's: the vector has get_actor_params_info's length and order (a generator sized from it fits), the
entries of setup_only attributes are ignored after setup, and a vector of any other length raises.  The
generator path needs the host to know which envs are randomized, so it costs one synchronisation per
resetting step (like ``dr_exact_trigger``).

The reference evaluates apply_randomizations only on steps where some env resets; without a host
synchronisation this build evaluates it every step (identical once any env resets each step, which is
the case at the benchmark sizes).  ``VecTask.dr_exact_trigger = True`` restores the reference's rule
at the cost of one ``reset_buf.any()`` synchronisation per step (the parity tests use it).
"""
from __future__ import annotations

import operator
from typing import Any, Dict, List, Tuple

import numpy as np
import torch

from . import _abi

_DIST = {"uniform": _abi.MG_DR_UNIFORM, "gaussian": _abi.MG_DR_GAUSSIAN, "loguniform": _abi.MG_DR_LOGUNIFORM}
_OPS = {"additive": _abi.MG_DR_ADDITIVE, "scaling": _abi.MG_DR_SCALING}
_SCHED = {None: _abi.MG_DR_SCHED_NONE, "linear": _abi.MG_DR_SCHED_LINEAR, "constant": _abi.MG_DR_SCHED_CONSTANT}
# dof_properties attribute -> column of a node row [mass, armature, damping, stiffness, lower, upper, kp, effort]
_DOF_COL = {"armature": 1, "damping": 2, "stiffness": 3, "lower": 4, "upper": 5, "effort": 7, "friction": 8}
_W = _abi.MG_EP_NODE_WIDTH
_NOOP_ATTRS = {("rigid_shape_properties", "restitution"), ("tendon_properties", "stiffness")}
_LIST_PROPS = ("rigid_body_properties", "rigid_shape_properties", "tendon_properties")


def sched_scaling(params: Dict[str, Any], step: int) -> float:
    """dr_utils.py:76-81 / vec_task.py:662-669."""
    kind = params.get("schedule", None) if "schedule" in params else None
    steps = params.get("schedule_steps", None) if "schedule" in params else None
    if kind == "linear":
        return 1.0 / steps * min(step, steps)
    if kind == "constant":
        return 0 if step < steps else 1
    return 1


def generate_random_samples(params: Dict[str, Any], shape, step: int) -> np.ndarray:
    """dr_utils.generate_random_samples on the host (np.random, as the reference): sim_params only."""
    lo, hi = params["range"]
    dist, op = params["distribution"], params["operation"]
    s = sched_scaling(params, step)
    if dist == "gaussian":
        if op == "additive":
            lo, hi = lo * s, hi * s
        elif op == "scaling":
            hi = hi * s
            lo = lo * s + 1 * (1 - s)
        return np.random.normal(lo, hi, shape)
    if op == "additive":
        lo, hi = lo * s, hi * s
    elif op == "scaling":
        lo, hi = lo * s + 1 * (1 - s), hi * s + 1 * (1 - s)
    if dist == "loguniform":
        return np.exp(np.random.uniform(np.log(lo), np.log(hi), shape))
    return np.random.uniform(lo, hi, shape)


def _desc(params: Dict[str, Any], after_setup: bool) -> _abi.DrDesc:
    d = _abi.DrDesc()
    if params["distribution"] not in _DIST or params["operation"] not in _OPS:
        raise ValueError(f"unsupported randomization {params}")
    d.distribution, d.operation = _DIST[params["distribution"]], _OPS[params["operation"]]
    d.schedule = _SCHED[params.get("schedule", None)]
    d.schedule_steps = int(params.get("schedule_steps", 0) or 0)
    d.num_buckets = int(params.get("num_buckets", 0) or 0)
    d.after_setup = int(after_setup)
    d.range[0], d.range[1] = float(params["range"][0]), float(params["range"][1])
    return d


def build_actor_attrs(actor_params: Dict[str, Any], actors: Dict[str, str], spec, offsets) -> Tuple[list, list, list]:
    """Descriptors and per-element attributes of ``actor_params``, in the reference's draw order
    (vec_task.py:746-833: actor, prop, then list props element-major / array props attr-major).

    actors: actor name -> "articulation" | "object" | "none".  Returns (descs, attrs, names) with
    names[i] = (actor, prop, element, attr) for the test harness's sample mapping."""
    o_node, o_geom, o_ten, o_obj = offsets
    descs: List[_abi.DrDesc] = []
    attrs: List[Tuple[int, int, float]] = []
    names: List[tuple] = []
    nd = spec.num_dofs
    for actor, props in actor_params.items():
        kind = actors.get(actor)
        if kind is None:
            raise NotImplementedError(f"domain randomization: unknown actor {actor!r} (have {sorted(actors)})")
        for prop, pattrs in props.items():
            if prop == "color" or kind == "none":
                continue
            if prop == "scale":
                if kind != "object":
                    raise NotImplementedError("actor scale randomization is supported for the free object only")
                descs.append(_desc(pattrs, not pattrs.get("setup_only", False)))
                attrs.append((o_obj + 2, len(descs) - 1, 1.0))
                names.append((actor, prop, 0, "scale"))
                continue
            # a property holding a setup_only attribute is not re-set after the first call (vec_task.py:800-830)
            after = not any(a.get("setup_only", False) for a in pattrs.values())
            base = len(descs)
            keys = list(pattrs.keys())
            for a in keys:
                descs.append(_desc(pattrs[a], after))
            if kind == "object":
                table = {("rigid_body_properties", "mass"): (o_obj + 0, float(spec.obj["mass"])),
                         ("rigid_shape_properties", "friction"): (o_obj + 1, 1.0)}
                for j, a in enumerate(keys):
                    if (prop, a) in _NOOP_ATTRS:
                        slot = None
                    elif (prop, a) in table:
                        slot, og = table[(prop, a)]
                    else:
                        raise NotImplementedError(f"domain randomization of object {prop}.{a}")
                    attrs.append((slot, base + j, og if slot is not None else 0.0))
                    names.append((actor, prop, 0, a))
                continue
            if prop == "dof_properties":   # ndarray property: one draw of shape (nD,) per attribute
                for j, a in enumerate(keys):
                    if a not in _DOF_COL:
                        raise NotImplementedError(f"domain randomization of dof_properties.{a}")
                    for d in range(nd):
                        n = spec.nodes[d + 1]
                        col = _DOF_COL[a]
                        og = {1: n.armature, 2: n.damping, 3: n.stiffness, 4: n.lower, 5: n.upper,
                              7: n.effort_limit, 8: n.frictionloss}[col]
                        if a == "stiffness" and n.drive_kp > 0:   # DOF_MODE_POS: stiffness is the drive's kp
                            col, og = 6, n.drive_kp
                        attrs.append((o_node + _W * (d + 1) + col, base + j, float(og)))
                        names.append((actor, prop, d, a))
                continue
            if prop not in _LIST_PROPS:
                raise NotImplementedError(f"domain randomization of {prop}")
            if prop == "rigid_body_properties":
                elems = [(o_node + _W * b.node, {"mass": float(spec.nodes[b.node].mass)}) for b in spec.bodies]
            elif prop == "rigid_shape_properties":
                elems = [(o_geom + g, {"friction": 1.0}) for g in range(len(spec.geoms))]
            else:
                elems = [(o_ten + 2 * q, {"limit_stiffness": float(t["limit_stiffness"]), "damping": float(t["damping"])})
                         for q, t in enumerate(spec.tendons)]
            cols = {"mass": 0, "friction": 0, "limit_stiffness": 0, "damping": 1}
            for e, (slot0, ogs) in enumerate(elems):
                for j, a in enumerate(keys):
                    if (prop, a) in _NOOP_ATTRS:
                        attrs.append((None, base + j, 0.0))
                    elif a in ogs:
                        attrs.append((slot0 + cols[a], base + j, ogs[a]))
                    else:
                        raise NotImplementedError(f"domain randomization of {prop}.{a}")
                    names.append((actor, prop, e, a))
    return descs, attrs, names


class NoiseLambda:
    """dr_randomizations[name]['noise_lambda'] (vec_task.py:684-720) as a HIP kernel: applies the noise to
    ``x`` in place (and writes ``clamp(x)`` into ``out`` if given) and returns ``x``."""

    def __init__(self, owner, name: str, key: int):
        self.owner, self.name, self.key = owner, name, key
        self.corr = None
        self.refresh = True
        self.inject = None        # tests: (z, corr) tensors replacing the device draws
        self.calls = 0

    def __call__(self, x: torch.Tensor, out: torch.Tensor = None, clip: float = float("inf")) -> torch.Tensor:
        p = self.owner.dr_randomizations[self.name]
        if self.corr is None or self.corr.numel() != x.numel():
            self.corr = torch.zeros(x.numel(), device=x.device, dtype=torch.float32)
            self.refresh = True
        a = _abi.DrNoiseArgs()
        a.x, a.x_clamped, a.clip = x.data_ptr(), None if out is None else out.data_ptr(), float(clip)
        a.operation = _abi.MG_DR_ADDITIVE if p["op"] is operator.add else _abi.MG_DR_SCALING
        if "mu" in p:
            a.distribution = _abi.MG_DR_GAUSSIAN
            a.scale, a.shift, a.c_scale, a.c_shift = p["var"], p["mu"], p["var_corr"], p["mu_corr"]
        else:
            a.distribution = _abi.MG_DR_UNIFORM
            a.scale, a.shift = p["hi"] - p["lo"], p["lo"]
            a.c_scale, a.c_shift = p["hi_corr"] - p["lo_corr"], p["lo_corr"]
        a.refresh_corr = int(self.refresh)
        a.corr, a.n = self.corr.data_ptr(), x.numel()
        inj = self.inject
        a.injected = None if inj is None else inj[0].data_ptr()
        a.injected_corr = None if inj is None or inj[1] is None else inj[1].data_ptr()
        a.seed, a.counter = self.owner.seed, self.calls
        a.elem_offset, a.key = self.owner.env_offset * (x.numel() // max(self.owner.num_envs, 1)), self.key
        _abi.check(self.owner._lib.mg_dr_noise(_abi.C.byref(a), self.owner._stream()), self.owner._lib)
        self.refresh = False
        self.calls += 1
        return x


class DomainRandomizationMixin:
    """The VecTask side of domain randomization; call ``_dr_init`` after the sim and buffers exist."""

    # actor name of the articulation in cfg['task']['randomization_params']['actor_params']
    dr_actor_names: Dict[str, str] = {}

    def _dr_init(self):
        task = self.cfg.get("task", {}) if isinstance(self.cfg, dict) else {}
        self.randomize = bool(task.get("randomize", False))
        self.randomization_params = task.get("randomization_params", {}) if self.randomize else {}
        self.dr_randomizations = {}
        self.first_randomization = True
        self.original_props = {}
        self.actor_params_generator = None
        self.extern_actor_params = {}
        self.last_step = -1
        self.last_rand_step = -1
        self.frame_count = 0
        self.dr_exact_trigger = False
        self.sim_initialized = False
        self._dr = None
        if not self.randomize or not self.dr_actor_names:   # Cartpole's reset_idx never randomizes (cartpole.py)
            self.randomize = False
            return
        dr = self.randomization_params
        spec = self.model_spec
        offs = (_abi.C.c_int32 * 4)()
        stride = self._lib.mg_env_props_layout(self._model_np.ctypes.data, offs)
        offsets = tuple(int(x) for x in offs)
        actors = dict(self.dr_actor_names)
        descs, attrs, names = build_actor_attrs(dr.get("actor_params", {}), actors, spec, offsets)
        self._dr_offsets = offsets
        self._dr_attrs = attrs
        row = np.zeros(stride, np.float32)
        _abi.check(self._lib.mg_env_props_defaults(self._model_np.ctypes.data, row.ctypes.data), self._lib)
        dev = self.device
        self.env_props = torch.tensor(row, device=dev).repeat(self.num_actors, 1).contiguous()
        live = [(s, d, og) for (s, d, og) in attrs if s is not None]
        self._dr_names = names
        self._dr_live = [i for i, (s, _, _) in enumerate(attrs) if s is not None]   # columns of injected samples
        dbytes = np.frombuffer(b"".join(bytes(d) for d in descs), np.uint8) if descs else np.zeros(1, np.uint8)
        abytes = np.zeros((max(len(live), 1), 4), np.int32)
        for i, (s, d, og) in enumerate(live):
            abytes[i, 0], abytes[i, 1] = s, d
            abytes[i, 2] = np.array([og], np.float32).view(np.int32)[0]
        self._dr = {"stride": stride, "descs": torch.tensor(dbytes, device=dev),
                    "attrs": torch.tensor(abytes.view(np.uint8).ravel(), device=dev), "nattr": len(live),
                    "mask": torch.zeros(self.num_actors, device=dev, dtype=torch.long),
                    "samples": None, "gravity_inject": [], "calls": 0}
        # VecTask.randomize_buf is per env (vec_task.py:323); with several agents per env every actor keeps
        # its own counter (the agents of an env reset together, so they stay equal)
        self.randomize_buf_actors = (self.randomize_buf if self.num_actors == self.num_envs
                                     else torch.zeros(self.num_actors, device=dev, dtype=torch.long))
        v = self._views
        v.env_props, v.env_props_stride = self.env_props.data_ptr(), stride
        _abi.check(self._lib.mg_sim_bind(self.sim, _abi.C.byref(v)), self._lib)
        self._og_sim_params = {"gravity": tuple(self.sim_params.gravity), "rest_offset": self.sim_params.rest_offset}
        # If randomizing, apply once immediately on startup before the first sim step (ant.py:125-126)
        self.apply_randomizations(dr)

    # -------------------------------------------------------------------------------------------
    def apply_randomizations(self, dr_params, reset_mask: torch.Tensor = None, increment: bool = False):
        """vec_task.py:612-842.  ``reset_mask``: the reset_buf of the resetting step (None on the first
        call); ``increment``: post_physics_step's ``randomize_buf += 1`` is still pending."""
        rand_freq = dr_params.get("frequency", 1)
        self.last_step = self.frame_count
        if self.first_randomization:
            do_nonenv_randomize = True
        else:
            do_nonenv_randomize = (self.last_step - self.last_rand_step) >= rand_freq
        if do_nonenv_randomize:
            self.last_rand_step = self.last_step
        for name in ("observations", "actions"):
            if name in dr_params and do_nonenv_randomize:
                self._dr_nonphysical(name, dr_params[name])
        if "sim_params" in dr_params and do_nonenv_randomize:
            self._dr_sim_params(dr_params["sim_params"])
        d = self._dr
        if d["nattr"] > 0:
            a = _abi.DrApplyArgs()
            a.descs, a.attrs, a.nattr, a.stride = d["descs"].data_ptr(), d["attrs"].data_ptr(), d["nattr"], d["stride"]
            a.n, a.frequency = self.num_actors, int(rand_freq)
            a.first, a.increment, a.last_step = int(self.first_randomization), int(increment), int(self.last_step)
            a.env_props = self.env_props.data_ptr()
            a.reset_mask = None if reset_mask is None else reset_mask.data_ptr()
            a.randomize_buf = self.randomize_buf_actors.data_ptr()
            smp = d["samples"]
            if smp is None and self.actor_params_generator is not None and not self.first_randomization:
                smp = self._extern_samples(dr_params, reset_mask, increment, int(rand_freq))
            a.samples = None if smp is None else smp.data_ptr()
            a.seed, a.counter, a.env_offset = self.seed, d["calls"], self.env_offset * self.num_agents
            _abi.check(self._lib.mg_dr_apply(_abi.C.byref(a), self._stream()), self._lib)
            d["calls"] += 1
        self.first_randomization = False

    def get_actor_params_info(self, dr_params: Dict[str, Any], env: int = 0):
        """vec_task.py:566-604: (params, names, lows, highs) of the randomized actor attributes, one entry per
        element in the reference's order; ``params`` are env ``env``'s current values (its first actor's
        env_props row).  lows / highs: the range for uniform / loguniform draws, +-inf otherwise."""
        if "actor_params" not in dr_params:
            return None
        _, attrs, names = build_actor_attrs(dr_params["actor_params"], dict(self.dr_actor_names), self.model_spec,
                                            self._dr_offsets)
        row = self.env_props[env * self.num_agents].cpu().numpy() if self._dr is not None else None
        params, out_names, lows, highs = [], [], [], []
        for (slot, _, og), (actor, prop, elem, attr) in zip(attrs, names):
            if prop == "scale":
                continue
            rp = dr_params["actor_params"][actor][prop][attr]
            if prop == "dof_properties":
                out_names.append(f"{prop}_0_{attr}_{elem}")
            else:
                out_names.append(f"{prop}_{elem}_{attr}")
            params.append(float(row[slot]) if (row is not None and slot is not None) else float(og))
            lo, hi = rp["range"] if "uniform" in rp["distribution"] else (-float("inf"), float("inf"))
            lows.append(lo)
            highs.append(hi)
        return params, out_names, lows, highs

    def _extern_layout(self, dr_params):
        """per live attribute column: (index into the extern vector or -1 for a setup_only attribute, schedule
        scale, op is scaling), and the vector length (get_actor_params_info's)"""
        names = self._dr_names
        pos, n = {}, 0
        for j, (actor, prop, elem, attr) in enumerate(names):
            if prop == "scale":
                continue
            if not dr_params["actor_params"][actor][prop][attr].get("setup_only", False):
                pos[j] = n
            n += 1
        cols = []
        for j in self._dr_live:
            actor, prop, elem, attr = names[j]
            rp = dr_params["actor_params"][actor][prop][attr] if prop != "scale" else dr_params["actor_params"][actor][prop]
            cols.append((pos.get(j, -1), sched_scaling(rp, self.last_step), rp["operation"] == "scaling"))
        return cols, n

    def _extern_samples(self, dr_params, reset_mask, increment, freq) -> torch.Tensor:
        """vec_task.py:736-760: actor_params_generator.sample() for every env the kernel will randomize on
        this call (randomize_buf >= frequency on a resetting env), scheduled as dr_utils' extern_sample
        branch, as the (num_actors, live attributes) sample table mg_dr_apply reads."""
        cols, n = self._extern_layout(dr_params)
        rb = self.randomize_buf_actors + (1 if increment else 0)
        doit = (rb >= freq) & (reset_mask != 0)
        ids = torch.nonzero(doit).flatten().cpu().numpy()
        smp = np.zeros((self.num_actors, max(len(cols), 1)), np.float32)
        env_ids = np.unique(ids // self.num_agents)
        ext = np.zeros((len(env_ids), n), np.float64)
        for k, env_id in enumerate(env_ids):
            v = np.asarray(self.actor_params_generator.sample(), np.float64).ravel()
            if v.shape[0] != n:
                raise Exception(f"Invalid extern_sample size: env {env_id} needs {n} values, got {v.shape[0]}")
            self.extern_actor_params[int(env_id)] = v
            ext[k] = v
        row = np.searchsorted(env_ids, ids // self.num_agents)
        for i, (p, s, scaling) in enumerate(cols):
            if p >= 0:
                x = ext[row, p]
                smp[ids, i] = x * s + (1.0 - s) if scaling else x * s
        t = torch.from_numpy(smp).to(self.device)
        self._dr_extern_keep = t          # alive until the kernel has read it (stream order)
        return t

    def _dr_nonphysical(self, name, p):
        """vec_task.py:646-720: the noise parameters after the schedule; the correlated noise is redrawn."""
        dist, op_type = p["distribution"], p["operation"]
        s = sched_scaling(p, self.last_step)
        op = operator.add if op_type == "additive" else operator.mul
        lam = self.dr_randomizations.get(name, {}).get("noise_lambda") or NoiseLambda(self, name, 1 if name == "actions" else 2)
        lam.refresh = True
        if dist == "gaussian":
            mu, var = p["range"]
            mu_corr, var_corr = p.get("range_correlated", [0., 0.])
            if op_type == "additive":
                mu, var, mu_corr, var_corr = mu * s, var * s, mu_corr * s, var_corr * s
            elif op_type == "scaling":
                var = var * s
                mu = mu * s + 1.0 * (1.0 - s)
                var_corr = var_corr * s
                mu_corr = mu_corr * s + 1.0 * (1.0 - s)
            self.dr_randomizations[name] = {"mu": mu, "var": var, "mu_corr": mu_corr, "var_corr": var_corr,
                                            "op": op, "noise_lambda": lam}
        elif dist == "uniform":
            lo, hi = p["range"]
            lo_corr, hi_corr = p.get("range_correlated", [0., 0.])
            if op_type == "additive":
                lo, hi, lo_corr, hi_corr = lo * s, hi * s, lo_corr * s, hi_corr * s
            elif op_type == "scaling":
                lo, hi = lo * s + 1.0 * (1.0 - s), hi * s + 1.0 * (1.0 - s)
                lo_corr, hi_corr = lo_corr * s + 1.0 * (1.0 - s), hi_corr * s + 1.0 * (1.0 - s)
            self.dr_randomizations[name] = {"lo": lo, "hi": hi, "lo_corr": lo_corr, "hi_corr": hi_corr,
                                            "op": op, "noise_lambda": lam}

    def _dr_sim_params(self, prop_attrs):
        """dr_utils.apply_random_samples on gym.SimParams (gravity, rest_offset) + gym.set_sim_params."""
        sp = self.sim_params
        for attr, params in prop_attrs.items():
            if attr == "gravity":
                inj = self._dr["gravity_inject"]
                sample = inj.pop(0) if inj else generate_random_samples(params, 3, self.last_step)
                og = self._og_sim_params["gravity"]
                for k in range(3):
                    v = og[k] * sample[k] if params["operation"] == "scaling" else og[k] + sample[k]
                    sp.gravity[k] = float(v)
                if self.first_randomization:
                    # the reference's original_props['sim_params']['gravity'] aliases the Vec3 of the
                    # SimParams object it randomizes on the first call (vec_task.py:726-731), so the
                    # first draw stays in the "original" gravity of every later call
                    self._og_sim_params["gravity"] = tuple(float(x) for x in sp.gravity)
            elif attr == "rest_offset":
                sp.rest_offset = float(generate_random_samples(params, 1, self.last_step))
            else:
                raise NotImplementedError(f"domain randomization of sim_params.{attr}")
        _abi.check(self._lib.mg_sim_set_params(self.sim, _abi.C.byref(sp)), self._lib)

    # -------------------------------------------------------------------------------------------
    def _dr_get_state(self):
        """The randomization state a resumed rollout needs to draw the same samples as an uninterrupted one:
        the counters that key the device draws (``mg_dr_apply``'s call counter, each noise lambda's call
        counter and its correlated-noise tensor), the schedule / first-call flags, the current noise
        parameters, the randomized sim params and the extern samples.  None without randomization."""
        if self._dr is None:
            return None
        # only tensors, numbers, strings and containers of them: rl_games saves env_state with torch.save, and
        # torch.load(weights_only=True) (the default) refuses functions and numpy arrays
        noise = {}
        for name, p in self.dr_randomizations.items():
            lam = p.get("noise_lambda")
            noise[name] = {k: v for k, v in p.items() if k not in ("noise_lambda", "op")}
            if "op" in p:
                noise[name]["op_type"] = "additive" if p["op"] is operator.add else "scaling"
            if lam is not None:
                noise[name]["_lambda"] = (lam.calls, lam.refresh, None if lam.corr is None else lam.corr.clone())
        return {"calls": self._dr["calls"], "first_randomization": self.first_randomization, "noise": noise,
                "gravity": tuple(float(x) for x in self.sim_params.gravity),
                "rest_offset": float(self.sim_params.rest_offset),
                "og_gravity": tuple(float(x) for x in self._og_sim_params["gravity"]),
                "extern_actor_params": {int(k): torch.from_numpy(np.array(v, copy=True))
                                        for k, v in self.extern_actor_params.items()}}

    def _dr_set_state(self, st):
        if st is None or self._dr is None:
            return
        self._dr["calls"] = st["calls"]
        self.first_randomization = st["first_randomization"]
        for name, p in st["noise"].items():
            p = dict(p)
            calls, refresh, corr = p.pop("_lambda", (0, True, None))
            if "op_type" in p:
                p["op"] = operator.add if p.pop("op_type") == "additive" else operator.mul
            lam = self.dr_randomizations.get(name, {}).get("noise_lambda") or \
                NoiseLambda(self, name, 1 if name == "actions" else 2)
            lam.calls, lam.refresh = calls, refresh
            lam.corr = None if corr is None else corr.to(self.device).clone()
            p["noise_lambda"] = lam
            self.dr_randomizations[name] = p
        sp = self.sim_params
        for k in range(3):
            sp.gravity[k] = st["gravity"][k]
        sp.rest_offset = st["rest_offset"]
        self._og_sim_params["gravity"] = st["og_gravity"]
        _abi.check(self._lib.mg_sim_set_params(self.sim, _abi.C.byref(sp)), self._lib)
        self.extern_actor_params = {int(k): (v.numpy() if torch.is_tensor(v) else np.asarray(v)).copy()
                                    for k, v in st["extern_actor_params"].items()}

    def _dr_any_reset(self) -> bool:
        return (not self.dr_exact_trigger) or bool(self.reset_buf.any())

    def _dr_actions(self, actions: torch.Tensor) -> torch.Tensor:
        """vec_task.py:372-374: actions = noise_lambda(actions) (on a copy: the caller's tensor is kept)."""
        lam = self.dr_randomizations.get("actions", {}).get("noise_lambda") if self.randomize else None
        if lam is None:
            return actions
        if getattr(self, "_dr_act_buf", None) is None or self._dr_act_buf.shape != actions.shape:
            self._dr_act_buf = torch.empty_like(actions)
        self._dr_act_buf.copy_(actions)
        return lam(self._dr_act_buf)

    def _dr_observations(self):
        """vec_task.py:398-400: obs_buf = noise_lambda(obs_buf), then the obs clamp of line 404."""
        lam = self.dr_randomizations.get("observations", {}).get("noise_lambda") if self.randomize else None
        if lam is not None:
            lam(self.obs_buf, self.obs_clamped if self._clamp_obs else None, float(self.clip_obs))
