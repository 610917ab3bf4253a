"""Robot-model loader: MJCF / URDF  ->  flat articulation tables.

Counterpart of the closed ``gym.load_asset`` importer the reference calls in
``tasks/ant.py:154``, ``tasks/humanoid.py:158`` and ``tasks/cartpole.py:89``.
The importer semantics are the build's own (physics parity
unpinned) and follow MuJoCo's MJCF conventions:

* bodies are visited depth first in file order; that order is the gym rigid-body
  order and the order of their joints is the DOF order (what the reference's
  ``dof_limits_lower``/``find_asset_rigid_body_index`` index into);
* every 1-DOF joint becomes one *node* of the dynamics tree.  A body with k
  joints becomes a chain of k nodes; the first k-1 are massless and all k share
  the body's orientation after their own rotation (MuJoCo ``mj_kinematics``
  anchor rule).  A body with no joint is welded into its parent's node
  (masses, geoms and the body frame are composed in);
* node frames sit at the joint anchor; the joint axis is constant in the node
  frame.  A node stores its anchor ``t`` and rest rotation ``r0`` relative to
  its parent node;
* ``inertiafromgeom``: geom volume x density (MJCF default 1000), capsule =
  cylinder + two hemispheres; URDF links without ``<inertia>`` get the
  inertia of their collision box at the given mass (cartpole.urdf has none).

The result is a :class:`ModelSpec`; :func:`pack_model` turns it into the
``mg_model`` POD struct declared in ``include/migym.h`` that both the HIP kernels
and the C oracle consume.  Model tables for the shipped tasks are generated in
the build container by ``tools/build_models.py`` into ``migym/assets/*.json``
so the GPU box never needs the reference checkout.
"""
from __future__ import annotations

import json
import math
import os
import xml.etree.ElementTree as ET
from dataclasses import dataclass, field, asdict
from typing import Dict, List, Optional

import numpy as np

# ---------------------------------------------------------------------------------------------
# constants shared with include/migym.h (checked at load time against mg_model_sizeof())
MAX_NODES = 40
MAX_BODIES = 40
MAX_GEOMS = 48
MAX_PAIRS = 192
MAX_SENSORS = 8
MAX_TENDONS = 8
MAX_HULL_VERTS = 160
MAX_HULL_PLANES = 320
COLLIDE_GROUND, COLLIDE_OBJECT = 1, 2

JT_FREE, JT_FIXED, JT_HINGE, JT_SLIDE = 0, 1, 2, 3
GT_PLANE, GT_SPHERE, GT_CAPSULE, GT_BOX, GT_CYLINDER, GT_ELLIPSOID, GT_CONVEX = 0, 1, 2, 3, 4, 5, 6
_GEOM_TYPES = {"plane": GT_PLANE, "sphere": GT_SPHERE, "capsule": GT_CAPSULE, "box": GT_BOX,
               "cylinder": GT_CYLINDER, "ellipsoid": GT_ELLIPSOID}


# ---------------------------------------------------------------------------------------------
# small rigid-transform helpers (quaternions are xyzw, like the gym root state)
def qmul(a, b):
    ax, ay, az, aw = a
    bx, by, bz, bw = b
    return np.array([aw * bx + ax * bw + ay * bz - az * by,
                     aw * by - ax * bz + ay * bw + az * bx,
                     aw * bz + ax * by - ay * bx + az * bw,
                     aw * bw - ax * bx - ay * by - az * bz])


def qrot(q, v):
    x, y, z, w = q
    u = np.array([x, y, z])
    v = np.asarray(v, dtype=np.float64)
    t = 2.0 * np.cross(u, v)
    return v + w * t + np.cross(u, t)


def qmat(q):
    x, y, z, w = q
    return np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)],
                     [2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)],
                     [2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)]])


def qnorm(q):
    q = np.asarray(q, dtype=np.float64)
    return q / np.linalg.norm(q)


def quat_from_wxyz(w, x, y, z):
    return qnorm([x, y, z, w])


def quat_from_axis_angle(axis, ang):
    axis = np.asarray(axis, dtype=np.float64)
    axis = axis / np.linalg.norm(axis)
    s = math.sin(ang / 2)
    return np.array([axis[0] * s, axis[1] * s, axis[2] * s, math.cos(ang / 2)])


def quat_from_euler(e, seq="xyz"):
    """MJCF default eulerseq 'xyz' = rotations about the moving x, then y, then z axes."""
    q = np.array([0, 0, 0, 1.0])
    for ang, ax in zip(e, seq):
        axis = {"x": [1, 0, 0], "y": [0, 1, 0], "z": [0, 0, 1]}[ax.lower()]
        q = qmul(q, quat_from_axis_angle(axis, ang))
    return q


def quat_from_rpy(r, p, y):
    """URDF rpy = fixed-axis X-Y-Z, i.e. R = Rz(y) Ry(p) Rx(r)."""
    return qmul(quat_from_axis_angle([0, 0, 1], y),
                qmul(quat_from_axis_angle([0, 1, 0], p), quat_from_axis_angle([1, 0, 0], r)))


def quat_from_zaxis(z):
    """Minimal rotation taking +z onto ``z`` (MuJoCo fromto/zaxis convention)."""
    z = np.asarray(z, dtype=np.float64)
    z = z / np.linalg.norm(z)
    c = z[2]
    if c > 1 - 1e-12:
        return np.array([0, 0, 0, 1.0])
    if c < -1 + 1e-12:
        return np.array([1.0, 0, 0, 0])
    axis = np.cross([0, 0, 1.0], z)
    return quat_from_axis_angle(axis, math.acos(max(-1.0, min(1.0, c))))


@dataclass
class Xform:
    pos: np.ndarray = field(default_factory=lambda: np.zeros(3))
    rot: np.ndarray = field(default_factory=lambda: np.array([0, 0, 0, 1.0]))

    def compose(self, other: "Xform") -> "Xform":
        return Xform(self.pos + qrot(self.rot, other.pos), qnorm(qmul(self.rot, other.rot)))

    def apply(self, p):
        return self.pos + qrot(self.rot, p)


# ---------------------------------------------------------------------------------------------
@dataclass
class Node:
    name: str
    parent: int
    jtype: int
    t: List[float]
    r0: List[float]
    axis: List[float]
    body: int                      # gym body index whose joint this is (-1 root handled separately)
    mass: float = 0.0
    com: List[float] = field(default_factory=lambda: [0.0, 0.0, 0.0])
    inertia: List[float] = field(default_factory=lambda: [0.0] * 6)   # about COM, node frame: xx yy zz xy xz yz
    armature: float = 0.0
    damping: float = 0.0
    stiffness: float = 0.0
    lower: float = 0.0
    upper: float = 0.0
    limited: int = 0
    drive_kp: float = 0.0          # MJCF <position kp>: PD position drive (DOF_MODE_POS)
    effort_limit: float = 0.0      # actuator forcerange (|force| clamp of the drive)
    frictionloss: float = 0.0      # MJCF joint frictionloss: dry friction torque bound (mg_model.frictionloss)


@dataclass
class Body:
    name: str
    node: int
    pos: List[float]               # body origin in node frame
    quat: List[float]              # body orientation in node frame
    parent_body: int
    mass: float = 0.0
    com: List[float] = field(default_factory=lambda: [0.0, 0.0, 0.0])   # body COM in body frame


@dataclass
class Geom:
    name: str
    gtype: int
    node: int
    body: int
    size: List[float]              # sphere r | capsule r,half | box half-extents | cylinder r,half
    pos: List[float]               # center in node frame
    quat: List[float]              # orientation in node frame (capsule/cylinder axis = local z)
    contype: int = 1
    conaffinity: int = 1
    filter: int = 3                # MG_COLLIDE_GROUND | MG_COLLIDE_OBJECT


@dataclass
class ModelSpec:
    name: str
    fixed_base: int
    nodes: List[Node]
    bodies: List[Body]
    geoms: List[Geom]
    pairs: List[List[int]]         # self-collision geom pairs (i, j)
    actuators: List[Dict]          # MJCF actuator order: {joint, gear, kind, kp, forcerange}
    dof_names: List[str]
    sensors: List[int] = field(default_factory=list)
    self_collision: int = 0
    tendons: List[Dict] = field(default_factory=list)   # {name, dofs[2], coefs[2], range[2], limit_stiffness, damping}
    gravity_off: int = 0
    obj: Optional[Dict] = None     # free object sharing the env: {type, size, mass, inertia, lin_damping, ...}
    pair_mjcf: int = 0             # 1: the pairs are explicit MJCF <pair>s (condim 1: frictionless; margin 0)
    hull: Optional[Dict] = None    # the convex-mesh geom: {geom, verts [[x,y,z]], planes [[nx,ny,nz,d]]}, geom frame
    # gym AssetOptions of the articulation's links (ASSET_OPTIONS; gym defaults until a task sets them)
    angular_damping: float = 0.5
    max_angular_velocity: float = 64.0

    @property
    def num_dofs(self):
        return len(self.nodes) - 1

    def dof_index(self, joint_name):
        return self.dof_names.index(joint_name)

    def body_index(self, name):
        return [b.name for b in self.bodies].index(name)

    # -------------------------------------------------------------------------------------
    def to_json(self, path):
        d = asdict(self)
        with open(path, "w") as f:
            json.dump(d, f, indent=1)

    @staticmethod
    def from_json(path) -> "ModelSpec":
        with open(path) as f:
            d = json.load(f)
        d["nodes"] = [Node(**n) for n in d["nodes"]]
        d["bodies"] = [Body(**b) for b in d["bodies"]]
        d["geoms"] = [Geom(**g) for g in d["geoms"]]
        return ModelSpec(**d)

    def total_mass(self):
        return sum(n.mass for n in self.nodes)


# ---------------------------------------------------------------------------------------------
# mass properties of primitive geoms (inertia about the geom center, geom frame)
def geom_mass_inertia(gtype, size, density):
    if gtype == GT_SPHERE:
        r = size[0]
        m = density * 4.0 / 3.0 * math.pi * r ** 3
        i = 0.4 * m * r * r
        return m, np.diag([i, i, i])
    if gtype == GT_CAPSULE:
        r, hl = size[0], size[1]
        h = 2 * hl
        mc = density * math.pi * r * r * h
        ms = density * 4.0 / 3.0 * math.pi * r ** 3
        ixx = mc * (3 * r * r + h * h) / 12.0 + ms * (0.4 * r * r + 0.375 * r * h + 0.25 * h * h)
        izz = mc * r * r / 2.0 + ms * 0.4 * r * r
        return mc + ms, np.diag([ixx, ixx, izz])
    if gtype == GT_BOX:
        x, y, z = size
        m = density * 8 * x * y * z
        return m, np.diag([m * (y * y + z * z) / 3, m * (x * x + z * z) / 3, m * (x * x + y * y) / 3])
    if gtype == GT_ELLIPSOID:
        a, b, c = size
        m = density * 4.0 / 3.0 * math.pi * a * b * c
        return m, np.diag([m * (b * b + c * c) / 5, m * (a * a + c * c) / 5, m * (a * a + b * b) / 5])
    if gtype == GT_CYLINDER:
        r, hl = size[0], size[1]
        h = 2 * hl
        m = density * math.pi * r * r * h
        return m, np.diag([m * (3 * r * r + h * h) / 12, m * (3 * r * r + h * h) / 12, m * r * r / 2])
    return 0.0, np.zeros((3, 3))


class _MassAccum:
    """Accumulates point masses with inertia in a common frame (parallel-axis)."""

    def __init__(self):
        self.m = 0.0
        self.mc = np.zeros(3)
        self.I0 = np.zeros((3, 3))   # inertia about the frame origin

    def add(self, m, c, Ic_frame):
        c = np.asarray(c, dtype=np.float64)
        self.m += m
        self.mc += m * c
        self.I0 += Ic_frame + m * (np.dot(c, c) * np.eye(3) - np.outer(c, c))

    def result(self):
        if self.m <= 0:
            return 0.0, np.zeros(3), np.zeros((3, 3))
        c = self.mc / self.m
        Ic = self.I0 - self.m * (np.dot(c, c) * np.eye(3) - np.outer(c, c))
        return self.m, c, Ic


def _inertia6(I):
    return [float(I[0, 0]), float(I[1, 1]), float(I[2, 2]), float(I[0, 1]), float(I[0, 2]), float(I[1, 2])]


# ---------------------------------------------------------------------------------------------
def _floats(s, n=None):
    v = [float(x) for x in s.split()]
    return v if n is None else v[:n]


class _Defaults:
    def __init__(self):
        self.classes: Dict[str, Dict[str, Dict[str, str]]] = {"main": {}}
        self.parent: Dict[str, Optional[str]] = {"main": None}

    def parse(self, elem, cls="main", parent=None):
        if cls not in self.classes:
            self.classes[cls] = {}
        self.parent[cls] = parent
        for child in elem:
            if child.tag == "default":
                self.parse(child, child.get("class", "main"), cls)
            else:
                self.classes[cls].setdefault(child.tag, {}).update(child.attrib)

    def attrs(self, tag, cls):
        chain = []
        c = cls
        while c is not None:
            chain.append(c)
            c = self.parent.get(c)
        out = {}
        for c in reversed(chain):
            out.update(self.classes.get(c, {}).get(tag, {}))
        return out


def _geom_size_and_frame(a, angle_scale):
    gtype = _GEOM_TYPES.get(a.get("type", "sphere"), None)
    size = _floats(a.get("size", "0 0 0"))
    if "fromto" in a:
        ft = _floats(a["fromto"])
        p0, p1 = np.array(ft[:3]), np.array(ft[3:])
        center = 0.5 * (p0 + p1)
        half = 0.5 * np.linalg.norm(p1 - p0)
        rot = quat_from_zaxis(p1 - p0)
        return gtype, [size[0], half, 0.0], Xform(center, rot)
    pos = np.array(_floats(a.get("pos", "0 0 0")))
    rot = _orientation(a, angle_scale)
    sz = (size + [0, 0, 0])[:3]
    return gtype, sz, Xform(pos, rot)


def _orientation(a, angle_scale):
    if "quat" in a:
        w, x, y, z = _floats(a["quat"])
        return quat_from_wxyz(w, x, y, z)
    if "euler" in a:
        return quat_from_euler([v * angle_scale for v in _floats(a["euler"])])
    if "axisangle" in a:
        v = _floats(a["axisangle"])
        return quat_from_axis_angle(v[:3], v[3] * angle_scale)
    if "zaxis" in a:
        return quat_from_zaxis(_floats(a["zaxis"]))
    return np.array([0, 0, 0, 1.0])


def load_mjcf(path, name=None, self_collision=False, merge_world_bodies=True, collapse_fixed=False,
              mesh_boxes=None, mesh_hulls=None) -> ModelSpec:
    """Parse an MJCF file (with <include>) into a :class:`ModelSpec`.

    ``collapse_fixed``: a jointless body is merged into its parent *body* (gym
    ``AssetOptions.collapse_fixed_joints``, shadow_hand.py:236) instead of becoming a
    rigid body of its own.  ``mesh_hulls``: {mesh name: {center, half, verts, planes}} convex
    hulls of mesh collision geoms (mesh frame about ``center``; tools/build_models.py), imported as
    one MG_GT_CONVEX geom (``spec.hull``); ``mesh_boxes``: {mesh name: (center, half extents)} box
    stand-ins for the others.
    A fixed-base root body keeps its MJCF orientation (its translation is replaced by the
    actor start pose): the reference places the object on the palm with the hand mount's
    rotation applied and its position ignored (shadow_hand.py:306-318, robot.xml:3)."""
    root = _read_mjcf_tree(path)
    compiler = root.find("compiler")
    angle_scale = math.pi / 180.0
    if compiler is not None and compiler.get("angle", "degree") == "radian":
        angle_scale = 1.0
    defaults = _Defaults()
    for d in root.findall("default"):
        defaults.parse(d)
    world = root.find("worldbody")
    bodies_xml = [b for b in world.findall("body")]
    if len(bodies_xml) != 1:
        raise ValueError("expected exactly one top-level body")
    top = bodies_xml[0]

    nodes: List[Node] = []
    bodies: List[Body] = []
    geoms: List[Geom] = []
    dof_names: List[str] = []
    mass_acc: Dict[int, _MassAccum] = {}
    body_mass: Dict[int, _MassAccum] = {}
    hulls: List[Dict] = []

    def joint_list(b, cls):
        out = []
        for j in b:
            if j.tag == "freejoint":
                out.append(("free", j.attrib, cls))
            elif j.tag == "joint":
                a = defaults.attrs("joint", j.get("class", cls))
                a.update(j.attrib)
                out.append((a.get("type", "hinge"), a, cls))
        return out

    def add_body_content(b, cls, node_idx, body_idx, T_node_body: Xform, T_acc: Xform = None):
        # geoms and mass, expressed in node frame; T_acc: this MJCF body in the frame of the gym
        # body it is accumulated into (identity unless collapsed into its parent)
        T_acc = T_acc or Xform()
        explicit = b.find("inertial")
        acc = mass_acc.setdefault(node_idx, _MassAccum())
        bacc = body_mass.setdefault(body_idx, _MassAccum())
        for g in b.findall("geom"):
            a = defaults.attrs("geom", g.get("class", cls))
            a.update(g.attrib)
            if a.get("type", "sphere") == "plane":
                continue
            collides = not (a.get("contype", "1") == "0" and a.get("conaffinity", "1") == "0")
            if a.get("type") == "mesh" and mesh_hulls and a.get("mesh") in mesh_hulls and collides:
                mh = mesh_hulls[a["mesh"]]
                Xm = Xform(np.array(_floats(a.get("pos", "0 0 0"))), _orientation(a, angle_scale))
                gtype, size, Xg = GT_CONVEX, [float(v) for v in mh["half"]], Xm.compose(Xform(np.array(mh["center"])))
                hulls.append(dict(geom=len(geoms), verts=[list(map(float, v)) for v in mh["verts"]],
                                  planes=[list(map(float, q)) for q in mh["planes"]]))
            elif a.get("type") == "mesh" and mesh_boxes and a.get("mesh") in mesh_boxes and collides:
                ctr, half = mesh_boxes[a["mesh"]]
                Xm = Xform(np.array(_floats(a.get("pos", "0 0 0"))), _orientation(a, angle_scale))
                gtype, size, Xg = GT_BOX, [float(v) for v in half], Xm.compose(Xform(np.array(ctr)))
            else:
                gtype, size, Xg = _geom_size_and_frame(a, angle_scale)
            if gtype is None:
                continue   # visual meshes
            Xg = T_acc.compose(Xg)
            Xn = T_node_body.compose(Xg)
            contype = int(a.get("contype", "1"))
            conaff = int(a.get("conaffinity", "1"))
            if explicit is None:
                density = float(a.get("density", "1000"))
                if "mass" in a:
                    m0, _ = geom_mass_inertia(gtype, size, 1.0)
                    density = float(a["mass"]) / m0 if m0 > 0 else 0.0
                m, Ig = geom_mass_inertia(gtype, size, density)
                R = qmat(Xn.rot)
                acc.add(m, Xn.pos, R @ Ig @ R.T)
                Rb = qmat(Xg.rot)
                bacc.add(m, Xg.pos, Rb @ Ig @ Rb.T)
            if contype == 0 and conaff == 0:
                continue
            geoms.append(Geom(name=a.get("name", f"g{len(geoms)}"), gtype=gtype, node=node_idx, body=body_idx,
                              size=[float(s) for s in size], pos=[float(v) for v in Xn.pos],
                              quat=[float(v) for v in Xn.rot], contype=contype, conaffinity=conaff))
        if explicit is not None:
            m = float(explicit.get("mass"))
            ipos = np.array(_floats(explicit.get("pos", "0 0 0")))
            irot = _orientation(explicit.attrib, angle_scale)
            if "diaginertia" in explicit.attrib:
                Id = np.diag(_floats(explicit.get("diaginertia")))
            else:
                f = _floats(explicit.get("fullinertia"))
                Id = np.array([[f[0], f[3], f[4]], [f[3], f[1], f[5]], [f[4], f[5], f[2]]])
            Xib = T_acc.compose(Xform(ipos, irot))
            Xi = T_node_body.compose(Xib)
            R = qmat(Xi.rot)
            acc.add(m, Xi.pos, R @ Id @ R.T)
            Rb = qmat(Xib.rot)
            bacc.add(m, Xib.pos, Rb @ Id @ Rb.T)

    def visit(b, cls, parent_node, T_parent: Xform, parent_body, T_acc_parent: Xform = None):
        """T_parent: parent gym-body frame expressed in parent_node frame; T_acc_parent: parent MJCF
        body in its gym body's frame (non-identity only inside a collapsed chain)."""
        cls = b.get("childclass", cls)
        bpos = np.array(_floats(b.get("pos", "0 0 0")))
        brot = _orientation(b.attrib, angle_scale)
        joints = joint_list(b, cls)
        if parent_node >= 0 and not joints and collapse_fixed:
            # welded into the parent gym body (collapse_fixed_joints)
            T_acc = (T_acc_parent or Xform()).compose(Xform(bpos, brot))
            add_body_content(b, cls, parent_node, parent_body, T_parent, T_acc)
            for c in b.findall("body"):
                visit(c, cls, parent_node, T_parent, parent_body, T_acc)
            return
        if T_acc_parent is not None:
            # child of a collapsed body: its pose is relative to the collapsed MJCF body
            T_rel = T_acc_parent.compose(Xform(bpos, brot))
            bpos, brot = T_rel.pos, T_rel.rot
        body_idx = len(bodies)
        if parent_node < 0:
            # root body: its frame is the actor frame (start pose supplied by the task); a fixed
            # base keeps the MJCF orientation of the root body
            jt = JT_FREE if (joints and joints[0][0] == "free") else JT_FIXED
            nodes.append(Node(name=b.get("name", "root"), parent=-1, jtype=jt, t=[0, 0, 0], r0=[0, 0, 0, 1],
                              axis=[0, 0, 1], body=body_idx))
            node_idx = 0
            T_body = Xform(np.zeros(3), brot) if jt == JT_FIXED else Xform()
        elif not joints:
            node_idx = parent_node
            T_body = T_parent.compose(Xform(bpos, brot))
        else:
            prev_anchor = None
            node_idx = parent_node
            for k, (jt, a, _) in enumerate(joints):
                if jt not in ("hinge", "slide"):
                    raise ValueError(f"joint type {jt} unsupported inside the tree")
                p = np.array(_floats(a.get("pos", "0 0 0")))
                axis = np.array(_floats(a.get("axis", "0 0 1")))
                axis = axis / np.linalg.norm(axis)
                if k == 0:
                    Xa = T_parent.compose(Xform(bpos, brot))
                    t = Xa.apply(p)
                    r0 = Xa.rot
                else:
                    t = p - prev_anchor
                    r0 = np.array([0, 0, 0, 1.0])
                limited = a.get("limited", "false") == "true"
                rng = _floats(a.get("range", "0 0"))
                scale = angle_scale if jt == "hinge" else 1.0
                lo, hi = rng[0] * scale, rng[1] * scale
                nodes.append(Node(name=a.get("name", f"j{len(nodes)}"), parent=node_idx,
                                  jtype=JT_HINGE if jt == "hinge" else JT_SLIDE,
                                  t=[float(v) for v in t], r0=[float(v) for v in r0],
                                  axis=[float(v) for v in axis], body=body_idx,
                                  armature=float(a.get("armature", "0")), damping=float(a.get("damping", "0")),
                                  stiffness=float(a.get("stiffness", "0")), lower=lo, upper=hi,
                                  limited=int(limited), frictionloss=float(a.get("frictionloss", "0"))))
                dof_names.append(nodes[-1].name)
                node_idx = len(nodes) - 1
                prev_anchor = p
            T_body = Xform(-prev_anchor, np.array([0, 0, 0, 1.0]))
        bodies.append(Body(name=b.get("name", f"b{body_idx}"), node=node_idx, pos=[float(v) for v in T_body.pos],
                           quat=[float(v) for v in T_body.rot], parent_body=parent_body))
        add_body_content(b, cls, node_idx, body_idx, T_body)
        for c in b.findall("body"):
            visit(c, cls, node_idx, T_body, body_idx)

    visit(top, "main", -1, Xform(), -1)

    for i, n in enumerate(nodes):
        if i in mass_acc:
            m, c, Ic = mass_acc[i].result()
            n.mass, n.com, n.inertia = float(m), [float(v) for v in c], _inertia6(Ic)
    for i, b in enumerate(bodies):
        if i in body_mass:
            m, c, _ = body_mass[i].result()
            b.mass, b.com = float(m), [float(v) for v in c]

    actuators = []
    act = root.find("actuator")
    if act is not None:
        for a0 in act:
            a = defaults.attrs(a0.tag, a0.get("class", "main"))
            a.update(a0.attrib)
            actuators.append(dict(kind=a0.tag, joint=a.get("joint"), gear=float(_floats(a.get("gear", "1"))[0]),
                                  kp=float(a.get("kp", "0")),
                                  forcerange=_floats(a.get("forcerange", "0 0"))))
            if a0.tag == "position" and a.get("joint") in dof_names:
                # gym maps an MJCF position actuator to a DOF_MODE_POS drive: stiffness = kp, damping =
                # the joint damping, effort = forcerange (shadow_hand.py:241-242, 268-280)
                nd = nodes[1 + dof_names.index(a["joint"])]
                nd.drive_kp = float(a.get("kp", "0"))
                fr = _floats(a.get("forcerange", "0 0"))
                nd.effort_limit = float(max(abs(fr[0]), abs(fr[1]))) if a.get("forcelimited", "true") != "false" \
                    else float("inf")
    tendons = []
    ten = root.find("tendon")
    if ten is not None:
        for t0 in ten.findall("fixed"):
            js = t0.findall("joint")
            if len(js) > 2:
                raise ValueError("fixed tendons with more than two joints are not supported")
            dofs = [dof_names.index(j.get("joint")) for j in js]
            coefs = [float(j.get("coef", "1")) for j in js]
            while len(dofs) < 2:
                dofs.append(dofs[0])
                coefs.append(0.0)
            rng = _floats(t0.get("range", "0 0"))
            tendons.append(dict(name=t0.get("name", f"t{len(tendons)}"), dofs=dofs, coefs=coefs, range=rng,
                                limited=int(t0.get("limited", "false") == "true"),
                                limit_stiffness=float(t0.get("stiffness", "0")), damping=float(t0.get("damping", "0"))))

    spec = ModelSpec(name=name or os.path.splitext(os.path.basename(path))[0],
                     fixed_base=int(nodes[0].jtype == JT_FIXED), nodes=nodes, bodies=bodies, geoms=geoms,
                     pairs=[], actuators=actuators, dof_names=dof_names, self_collision=int(self_collision),
                     tendons=tendons)
    if len(hulls) > 1:
        raise ValueError("mg_model holds one convex-mesh geom")
    spec.hull = hulls[0] if hulls else None
    if self_collision:
        spec.pairs = self_collision_pairs(spec)
    explicit, spec.pair_mjcf = mjcf_contact_pairs(root, geoms)
    for pr in explicit:
        if pr not in spec.pairs and pr[::-1] not in spec.pairs:
            spec.pairs.append(pr)
    return spec


def mjcf_contact_pairs(root, geoms):
    """Explicit ``<contact><pair geom1 geom2 condim margin>`` elements of an MJCF: geom index pairs in file order
    (a repeated pair once), and ``mg_model.pair_mjcf``.  MuJoCo collides these pairs whatever contype /
    conaffinity say (the ShadowHand's collision geoms are contype 1 / conaffinity 0, so its only hand-hand
    contacts are the 19 finger / thumb pairs of shared.xml:31-51), with the pair's own attributes: condim 1 =
    frictionless, margin (default 0) = the distance below which the pair is in contact -- not the sim's
    contact offset (at rest the hand's adjacent proximal capsules sit exactly 2 mm apart).  Pairs name sphere
    / capsule geoms, or one box and one sphere / capsule (the kernel's pair narrowphase)."""
    contact = root.find("contact")
    if contact is None:
        return [], 0
    names = [g.name for g in geoms]
    out, condims = [], set()
    for pe in contact.findall("pair"):
        g1, g2 = pe.get("geom1"), pe.get("geom2")
        if g1 not in names or g2 not in names:
            raise ValueError(f"MJCF contact pair names a geom that is not a collision geom: {g1!r}, {g2!r}")
        pr = [names.index(g1), names.index(g2)]
        if pr in out or pr[::-1] in out:
            continue
        types = sorted(geoms[i].gtype for i in pr)
        if types[0] not in (GT_SPHERE, GT_CAPSULE) or types[1] not in (GT_SPHERE, GT_CAPSULE, GT_BOX):
            raise NotImplementedError(f"MJCF contact pair {g1!r} / {g2!r}: geom types {types} have no pair narrowphase")
        out.append(pr)
        condims.add(int(pe.get("condim", "3")))
        if float(pe.get("margin", "0")) != 0.0:
            raise NotImplementedError(f"MJCF contact pair {g1!r} / {g2!r}: margin != 0")
    if condims != {1}:
        raise NotImplementedError(f"MJCF contact pairs with condim {sorted(condims)} (only condim 1 is built)")
    return out, 1


def _read_mjcf_tree(path):
    tree = ET.parse(path)
    root = tree.getroot()
    base = os.path.dirname(path)

    def expand(elem):
        out = []
        for child in list(elem):
            if child.tag == "include":
                inc = ET.parse(os.path.join(base, child.get("file"))).getroot()
                out.extend(expand(inc))
            else:
                child[:] = expand(child)
                out.append(child)
        return out

    root[:] = expand(root)
    # merge repeated top-level sections (several <default>/<worldbody> after includes)
    return root


def self_collision_pairs(spec: ModelSpec):
    """Geom pairs that may collide inside one articulation.

    PhysX never collides two links joined by a joint; the build additionally
    skips geoms of the same body.  (Humanoid: humanoid.py:194 filter 0.)"""
    pairs = []
    for i, gi in enumerate(spec.geoms):
        for j in range(i + 1, len(spec.geoms)):
            gj = spec.geoms[j]
            bi, bj = gi.body, gj.body
            if bi == bj:
                continue
            if spec.bodies[bi].parent_body == bj or spec.bodies[bj].parent_body == bi:
                continue
            if spec.bodies[bi].node == spec.bodies[bj].node:
                continue
            pairs.append([i, j])
    return pairs


# ---------------------------------------------------------------------------------------------
def load_urdf(path, name=None, fix_base=True) -> ModelSpec:
    """URDF loader (prismatic / revolute / continuous / fixed joints)."""
    root = ET.parse(path).getroot()
    links = {l.get("name"): l for l in root.findall("link")}
    joints = root.findall("joint")
    child_of = {j.find("child").get("link"): j for j in joints}
    children: Dict[str, List] = {}
    for j in joints:
        children.setdefault(j.find("parent").get("link"), []).append(j)
    root_link = [n for n in links if n not in child_of][0]

    nodes: List[Node] = []
    bodies: List[Body] = []
    geoms: List[Geom] = []
    dof_names: List[str] = []
    accs: Dict[int, _MassAccum] = {}
    baccs: Dict[int, _MassAccum] = {}

    def origin(e):
        o = e.find("origin") if e is not None else None
        if o is None:
            return Xform()
        xyz = np.array(_floats(o.get("xyz", "0 0 0")))
        rpy = _floats(o.get("rpy", "0 0 0"))
        return Xform(xyz, quat_from_rpy(*rpy))

    def link_content(link, node_idx, body_idx, T: Xform):
        col_boxes = []
        for c in link.findall("collision"):
            Xc = origin(c)
            geo = c.find("geometry")
            box = geo.find("box")
            sph = geo.find("sphere")
            cyl = geo.find("cylinder")
            if box is not None:
                half = [0.5 * v for v in _floats(box.get("size"))]
                g = (GT_BOX, half)
                col_boxes.append((Xc, half))
            elif sph is not None:
                g = (GT_SPHERE, [float(sph.get("radius")), 0, 0])
            elif cyl is not None:
                g = (GT_CYLINDER, [float(cyl.get("radius")), 0.5 * float(cyl.get("length")), 0])
            else:
                continue
            Xn = T.compose(Xc)
            geoms.append(Geom(name=f"{link.get('name')}_col{len(geoms)}", gtype=g[0], node=node_idx, body=body_idx,
                              size=[float(v) for v in g[1]], pos=[float(v) for v in Xn.pos],
                              quat=[float(v) for v in Xn.rot]))
        inert = link.find("inertial")
        if inert is None:
            return
        Xi = origin(inert)
        mass_e = inert.find("mass")
        ie = inert.find("inertia")
        dens = inert.find("density")
        if mass_e is not None:
            m = float(mass_e.get("value"))
            if ie is not None:
                f = {k: float(ie.get(k, "0")) for k in ("ixx", "iyy", "izz", "ixy", "ixz", "iyz")}
                I = np.array([[f["ixx"], f["ixy"], f["ixz"]], [f["ixy"], f["iyy"], f["iyz"]],
                              [f["ixz"], f["iyz"], f["izz"]]])
            elif col_boxes:
                _, half = col_boxes[0]
                x, y, z = half
                I = np.diag([m * (y * y + z * z) / 3, m * (x * x + z * z) / 3, m * (x * x + y * y) / 3])
            else:
                I = np.eye(3) * 1e-4 * m
        elif dens is not None and col_boxes:
            Xc, half = col_boxes[0]
            m, I = geom_mass_inertia(GT_BOX, half, float(dens.get("value")))
            Xi = Xc
        else:
            return
        Xn = T.compose(Xi)
        R = qmat(Xn.rot)
        accs.setdefault(node_idx, _MassAccum()).add(m, Xn.pos, R @ I @ R.T)
        Rb = qmat(Xi.rot)
        baccs.setdefault(body_idx, _MassAccum()).add(m, Xi.pos, Rb @ I @ Rb.T)

    def visit(link_name, parent_node, T_parent: Xform, parent_body):
        body_idx = len(bodies)
        link = links[link_name]
        if parent_node < 0:
            nodes.append(Node(name=link_name, parent=-1, jtype=JT_FIXED if fix_base else JT_FREE, t=[0, 0, 0],
                              r0=[0, 0, 0, 1], axis=[0, 0, 1], body=body_idx))
            node_idx, T = 0, Xform()
        else:
            j = child_of[link_name]
            jt = j.get("type")
            Xj = T_parent.compose(origin(j))
            if jt == "fixed":
                node_idx, T = parent_node, Xj
            else:
                ax = j.find("axis")
                axis = np.array(_floats(ax.get("xyz"))) if ax is not None else np.array([1.0, 0, 0])
                axis = axis / np.linalg.norm(axis)
                lim = j.find("limit")
                lo = float(lim.get("lower", "0")) if lim is not None else 0.0
                hi = float(lim.get("upper", "0")) if lim is not None else 0.0
                dyn = j.find("dynamics")
                nodes.append(Node(name=j.get("name"), parent=parent_node,
                                  jtype=JT_SLIDE if jt == "prismatic" else JT_HINGE,
                                  t=[float(v) for v in Xj.pos], r0=[float(v) for v in Xj.rot],
                                  axis=[float(v) for v in axis], body=body_idx,
                                  damping=float(dyn.get("damping", "0")) if dyn is not None else 0.0,
                                  lower=lo, upper=hi, limited=int(jt in ("prismatic", "revolute"))))
                dof_names.append(j.get("name"))
                node_idx, T = len(nodes) - 1, Xform()
        bodies.append(Body(name=link_name, node=node_idx, pos=[float(v) for v in T.pos],
                           quat=[float(v) for v in T.rot], parent_body=parent_body))
        link_content(link, node_idx, body_idx, T)
        for j in children.get(link_name, []):
            visit(j.find("child").get("link"), node_idx, T, body_idx)

    visit(root_link, -1, Xform(), -1)
    for i, n in enumerate(nodes):
        if i in accs:
            m, c, Ic = accs[i].result()
            n.mass, n.com, n.inertia = float(m), [float(v) for v in c], _inertia6(Ic)
    for i, b in enumerate(bodies):
        if i in baccs:
            m, c, _ = baccs[i].result()
            b.mass, b.com = float(m), [float(v) for v in c]
    return ModelSpec(name=name or root.get("name"), fixed_base=int(fix_base), nodes=nodes, bodies=bodies,
                     geoms=geoms, pairs=[], actuators=[], dof_names=dof_names)


# ---------------------------------------------------------------------------------------------
# packing into the mg_model POD struct (layout mirrors include/migym.h)
def _model_dtype():
    f4, i4 = np.float32, np.int32
    N, B, G, P, S, TD = MAX_NODES, MAX_BODIES, MAX_GEOMS, MAX_PAIRS, MAX_SENSORS, MAX_TENDONS
    return np.dtype([
        ("num_nodes", i4), ("num_dofs", i4), ("fixed_base", i4), ("num_bodies", i4),
        ("num_geoms", i4), ("num_pairs", i4), ("num_sensors", i4), ("nv", i4),
        ("parent", i4, N), ("jtype", i4, N), ("limited", i4, N), ("node_body", i4, N),
        ("t", f4, (N, 3)), ("r0", f4, (N, 4)), ("axis", f4, (N, 3)),
        ("mass", f4, N), ("com", f4, (N, 3)), ("inertia", f4, (N, 6)),
        ("armature", f4, N), ("damping", f4, N), ("stiffness", f4, N), ("lower", f4, N), ("upper", f4, N),
        ("body_node", i4, B), ("body_parent", i4, B),
        ("body_pos", f4, (B, 3)), ("body_quat", f4, (B, 4)), ("body_com", f4, (B, 3)),
        ("geom_type", i4, G), ("geom_node", i4, G), ("geom_body", i4, G), ("geom_filter", i4, G),
        ("geom_size", f4, (G, 3)), ("geom_pos", f4, (G, 3)), ("geom_quat", f4, (G, 4)),
        ("pair", i4, (P, 2)),
        ("sensor_body", i4, S),
        ("drive_kp", f4, N), ("effort_limit", f4, N),
        ("num_tendons", i4), ("gravity_off", i4),
        ("tendon_dof", i4, (TD, 2)), ("tendon_coef", f4, (TD, 2)), ("tendon_range", f4, (TD, 2)),
        ("tendon_limit_stiffness", f4, TD), ("tendon_damping", f4, TD),
        ("obj_type", i4), ("pair_mjcf", i4), ("obj_mass", f4), ("obj_inertia", f4, 3), ("obj_size", f4, 3),
        ("obj_lin_damping", f4), ("obj_ang_damping", f4), ("obj_gravity", f4),
        ("hull_num_verts", i4), ("hull_num_planes", i4),
        ("hull_vert", f4, (MAX_HULL_VERTS, 3)), ("hull_plane", f4, (MAX_HULL_PLANES, 4)),
        ("link_ang_damping", f4), ("link_max_ang_vel", f4), ("obj_max_ang_vel", f4), ("pad_model", i4),
        ("frictionloss", f4, N),
    ])


MODEL_DTYPE = _model_dtype()


def pack_model(spec: ModelSpec) -> np.ndarray:
    if len(spec.nodes) > MAX_NODES or len(spec.bodies) > MAX_BODIES or len(spec.geoms) > MAX_GEOMS:
        raise ValueError("model exceeds mg_model capacity")
    if len(spec.pairs) > MAX_PAIRS or len(spec.sensors) > MAX_SENSORS or len(spec.tendons) > MAX_TENDONS:
        raise ValueError("model exceeds mg_model pair/sensor capacity")
    m = np.zeros((), dtype=MODEL_DTYPE)
    m["num_nodes"] = len(spec.nodes)
    m["num_dofs"] = len(spec.nodes) - 1
    m["fixed_base"] = spec.fixed_base
    m["num_bodies"] = len(spec.bodies)
    m["num_geoms"] = len(spec.geoms)
    m["num_pairs"] = len(spec.pairs)
    m["pair_mjcf"] = int(getattr(spec, "pair_mjcf", 0))
    m["num_sensors"] = len(spec.sensors)
    m["nv"] = (0 if spec.fixed_base else 6) + len(spec.nodes) - 1
    m["parent"][:] = -1
    for i, n in enumerate(spec.nodes):
        m["parent"][i] = n.parent
        m["jtype"][i] = n.jtype
        m["limited"][i] = n.limited
        m["node_body"][i] = n.body
        m["t"][i] = n.t
        m["r0"][i] = n.r0
        m["axis"][i] = n.axis
        m["mass"][i] = n.mass
        m["com"][i] = n.com
        m["inertia"][i] = n.inertia
        m["armature"][i] = n.armature
        m["damping"][i] = n.damping
        m["stiffness"][i] = n.stiffness
        m["lower"][i] = n.lower
        m["upper"][i] = n.upper
        m["drive_kp"][i] = n.drive_kp
        m["effort_limit"][i] = n.effort_limit
        m["frictionloss"][i] = n.frictionloss
    for i, b in enumerate(spec.bodies):
        m["body_node"][i] = b.node
        m["body_parent"][i] = b.parent_body
        m["body_pos"][i] = b.pos
        m["body_quat"][i] = b.quat
        m["body_com"][i] = b.com
    for i, g in enumerate(spec.geoms):
        m["geom_type"][i] = g.gtype
        m["geom_node"][i] = g.node
        m["geom_body"][i] = g.body
        m["geom_size"][i] = g.size
        m["geom_pos"][i] = g.pos
        m["geom_quat"][i] = g.quat
        m["geom_filter"][i] = g.filter
    for i, p in enumerate(spec.pairs):
        m["pair"][i] = p
    for i, s in enumerate(spec.sensors):
        m["sensor_body"][i] = s
    m["num_tendons"] = len(spec.tendons)
    m["gravity_off"] = int(spec.gravity_off)
    for i, t in enumerate(spec.tendons):
        m["tendon_dof"][i] = t["dofs"]
        m["tendon_coef"][i] = t["coefs"]
        m["tendon_range"][i] = t["range"] if t.get("limited", 1) else [-np.inf, np.inf]
        m["tendon_limit_stiffness"][i] = t["limit_stiffness"]
        m["tendon_damping"][i] = t["damping"]
    if spec.obj:
        o = spec.obj
        m["obj_type"] = o["type"]
        m["obj_mass"] = o["mass"]
        m["obj_inertia"] = o["inertia"]
        m["obj_size"] = o["size"]
        m["obj_lin_damping"] = o.get("lin_damping", 0.0)
        m["obj_ang_damping"] = o.get("ang_damping", 0.0)
        m["obj_gravity"] = o.get("gravity", 1)
    if spec.hull:
        h = spec.hull
        if len(h["verts"]) > MAX_HULL_VERTS or len(h["planes"]) > MAX_HULL_PLANES:
            raise ValueError("convex hull exceeds mg_model capacity")
        if spec.geoms[h["geom"]].gtype != GT_CONVEX:
            raise ValueError("hull geom index does not name an MG_GT_CONVEX geom")
        m["hull_num_verts"] = len(h["verts"])
        m["hull_num_planes"] = len(h["planes"])
        m["hull_vert"][:len(h["verts"])] = h["verts"]
        m["hull_plane"][:len(h["planes"])] = h["planes"]
    m["link_ang_damping"] = spec.angular_damping
    m["link_max_ang_vel"] = spec.max_angular_velocity
    m["obj_max_ang_vel"] = spec.obj.get("max_ang_vel", GYM_MAX_ANGULAR_VELOCITY) if spec.obj else 0.0
    return m


ASSET_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "assets")


GYM_ANGULAR_DAMPING = 0.5          # gymapi.AssetOptions defaults (Isaac Gym Preview 4)
GYM_MAX_ANGULAR_VELOCITY = 64.0
# The link options each task's create_sim sets on its articulation asset; the rest keep gym's defaults.
ASSET_OPTIONS = {
    "ant": {"angular_damping": 0.0},                                       # ant.py:152
    "humanoid": {"angular_damping": 0.01, "max_angular_velocity": 100.0},  # humanoid.py:153-154
    "shadow_hand": {"angular_damping": 0.01},                              # shadow_hand.py:240
    "cartpole": {},                                                        # cartpole.py:86-87 (defaults)
}


def apply_asset_options(spec: ModelSpec, name: str) -> ModelSpec:
    """the task's link options (ASSET_OPTIONS) on gym's defaults; tools/build_models.py writes them into the
    shipped tables"""
    spec.angular_damping = GYM_ANGULAR_DAMPING
    spec.max_angular_velocity = GYM_MAX_ANGULAR_VELOCITY
    for k, v in ASSET_OPTIONS.get(name, {}).items():
        setattr(spec, k, v)
    return spec


def load_builtin(name) -> ModelSpec:
    """Load one of the shipped model tables (generated by tools/build_models.py, asset options included)."""
    return ModelSpec.from_json(os.path.join(ASSET_DIR, name + ".json"))


def hand_object(kind: str) -> Dict:
    """The free object of ShadowHand's objectType (shadow_hand.py:86-100): block = cube_multicolor.urdf,
    egg = open_ai_assets/hand/egg.xml (ellipsoid), pen = open_ai_assets/hand/pen.xml (capsule).  Shipped
    as migym/assets/hand_objects.json (tools/build_models.py)."""
    with open(os.path.join(ASSET_DIR, "hand_objects.json")) as f:
        objs = json.load(f)
    if kind not in objs:
        raise ValueError(f"objectType must be one of {sorted(objs)}, got {kind!r}")
    return dict(objs[kind])
