#!/usr/bin/env python3
"""Regenerate the shipped model tables from the reference's robot files.

Build-container only (reads /root/reference/assets).  The tables are derived
data (the build's own importer output, see migym/model.py); the GPU box loads
them from migym/assets/*.json.

  Ant       assets/mjcf/nv_ant.xml        (tasks/ant.py:142-197; feet force sensors :170-178)
  Humanoid  assets/mjcf/nv_humanoid.xml   (tasks/humanoid.py:142-196; foot sensors :163-168;
                                           self-collision filter 0 :194)
  Cartpole  assets/urdf/cartpole.urdf     (tasks/cartpole.py:78-113; fix_base_link :88)
  ShadowHand assets/mjcf/open_ai_assets/hand/shadow_hand.xml + assets/urdf/objects/cube_multicolor.urdf
            (tasks/shadow_hand.py:220-396: fix_base_link, collapse_fixed_joints, disable_gravity,
             tendon limit_stiffness 30 / damping 0.1 on the four T_*J1c tendons, fingertip force
             sensors; the object keeps gym's default AssetOptions: angular_damping 0.5, gravity on).
            The forearm's convex collision mesh (forearm_electric_cvx.stl, 455 hull vertices) is
            imported as a convex hull of 160 of its vertices (greedy: the 26 axis / diagonal extremes,
            then repeatedly the vertex farthest outside the current hull; every dropped vertex lies
            within 0.46 mm of the kept hull; PhysX cooks such meshes to <= 255 vertices) with its face
            planes (coplanar facets merged).
  hand_objects.json  the free object of each ShadowHand objectType (shadow_hand.py:86-100):
            block = urdf/objects/cube_multicolor.urdf, egg = mjcf/open_ai_assets/hand/egg.xml
            (ellipsoid), pen = mjcf/open_ai_assets/hand/pen.xml (capsule along the body z); mass and
            principal inertia from the geom at MJCF's default density 1000; the object body's own
            MJCF pose is replaced by the actor pose (as the cube's URDF origin is).
"""
import json
import os
import struct
import sys
import xml.etree.ElementTree as ET

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "isaacgymenvs-ma_amd"))
from migym import model as M  # noqa: E402

REF = os.environ.get("MIGYM_REFERENCE", "/root/reference")


def stl_vertices(path, scale=(1.0, 1.0, 1.0)):
    """unique vertices of an STL mesh (binary or ASCII), mesh frame, scaled."""
    data = open(path, "rb").read()
    n = struct.unpack("<I", data[80:84])[0] if len(data) >= 84 else 0
    if len(data) == 84 + 50 * n:
        rec = np.frombuffer(data[84:], dtype=np.dtype([("n", "<f4", 3), ("v", "<f4", (3, 3)), ("a", "<u2")]))
        v = rec["v"].reshape(-1, 3).astype(np.float64)
    else:
        v = np.array([[float(x) for x in ln.split()[1:4]] for ln in data.decode().splitlines()
                      if ln.strip().startswith("vertex")])
    return np.unique(v * np.asarray(scale), axis=0)


def reduced_hull(v, max_verts=160, tol=1e-5):
    """a convex hull of at most max_verts of the points v: the extremes along the 26 axis / diagonal
    directions, then greedily the point farthest outside the current hull.  Returns (kept vertices,
    merged outward face planes [n, d] with n.x <= d inside, largest distance of a dropped point
    outside the kept hull)."""
    from scipy.spatial import ConvexHull
    v = v[ConvexHull(v).vertices]
    dirs = [np.array(d, float) - 1.0 for d in np.ndindex(3, 3, 3) if d != (1, 1, 1)]
    sel = []
    for d in dirs:
        i = int(np.argmax(v @ d))
        if i not in sel:
            sel.append(i)
    while True:
        eq = ConvexHull(v[sel]).equations          # n.x + off <= 0 inside
        out = (v @ eq[:, :3].T + eq[:, 3]).max(1)
        i = int(np.argmax(out))
        if out[i] < tol or len(sel) >= max_verts:
            break
        sel.append(i)
    planes = []
    for e in eq:
        q = [float(e[0]), float(e[1]), float(e[2]), float(-e[3])]
        if not any(np.allclose(q, p2, atol=1e-7) for p2 in planes):
            planes.append(q)
    return v[sel], planes, float(max(out.max(), 0.0))


HAND_FINGERTIPS = ["robot0:ffdistal", "robot0:mfdistal", "robot0:rfdistal", "robot0:lfdistal", "robot0:thdistal"]
HAND_TENDONS = ["robot0:T_FFJ1c", "robot0:T_MFJ1c", "robot0:T_RFJ1c", "robot0:T_LFJ1c"]


def shadow_hand():
    hand_dir = os.path.join(REF, "assets/mjcf/open_ai_assets/hand")
    mesh_dir = os.path.join(hand_dir, "../stls/hand")
    hulls = {}
    for m in ET.parse(os.path.join(hand_dir, "shared_asset.xml")).getroot().iter("mesh"):
        if "cvx" not in m.get("file", ""):
            continue
        sc = [float(x) for x in m.get("scale", "1 1 1").split()]
        v = stl_vertices(os.path.join(mesh_dir, m.get("file")), sc)
        lo, hi = v.min(0), v.max(0)
        ctr = (lo + hi) / 2
        kept, planes, err = reduced_hull(v - ctr)
        print(f"{m.get('name')}: {len(v)} vertices -> hull of {len(kept)} ({len(planes)} planes), "
              f"max dropped-vertex distance {err * 1e3:.2f} mm")
        hulls[m.get("name")] = dict(center=ctr.tolist(), half=((hi - lo) / 2).tolist(), verts=kept.tolist(),
                                    planes=planes)
    hand = M.load_mjcf(os.path.join(hand_dir, "shadow_hand.xml"), "shadow_hand", collapse_fixed=True,
                       mesh_hulls=hulls)
    hand.sensors = [hand.body_index(n) for n in HAND_FINGERTIPS]
    hand.gravity_off = 1
    for t in hand.tendons:
        if t["name"] in HAND_TENDONS:
            t["limit_stiffness"], t["damping"] = 30.0, 0.1
    cube = M.load_urdf(os.path.join(REF, "assets/urdf/objects/cube_multicolor.urdf"), "cube", fix_base=False)
    g = cube.geoms[0]
    hand.obj = dict(type=M.GT_BOX, size=list(g.size), mass=cube.nodes[0].mass, inertia=cube.nodes[0].inertia[:3],
                    lin_damping=0.0, ang_damping=0.5, gravity=1)
    return hand


def hand_objects(hand):
    objs = {"block": hand.obj}
    for kind in ("egg", "pen"):
        root = ET.parse(os.path.join(REF, f"assets/mjcf/open_ai_assets/hand/{kind}.xml")).getroot()
        body = next(b for b in root.iter("body") if b.get("name") == "object")
        geom = body.find("geom")
        gtype = M._GEOM_TYPES[geom.get("type")]
        size = [float(x) for x in geom.get("size").split()]
        size = (size + [0.0, 0.0])[:3]
        mass, inertia = M.geom_mass_inertia(gtype, size, float(geom.get("density", "1000")))
        objs[kind] = dict(type=gtype, size=size, mass=mass, inertia=[float(x) for x in np.diag(inertia)],
                          lin_damping=0.0, ang_damping=0.5, gravity=1)
    return objs


def main():
    out = M.ASSET_DIR
    ant = M.load_mjcf(os.path.join(REF, "assets/mjcf/nv_ant.xml"), "ant")
    M.apply_asset_options(ant, "ant")
    ant.sensors = [i for i, b in enumerate(ant.bodies) if "foot" in b.name]
    ant.to_json(os.path.join(out, "ant.json"))
    hum = M.load_mjcf(os.path.join(REF, "assets/mjcf/nv_humanoid.xml"), "humanoid", self_collision=True)
    hum.sensors = [hum.body_index("right_foot"), hum.body_index("left_foot")]
    M.apply_asset_options(hum, "humanoid")
    hum.to_json(os.path.join(out, "humanoid.json"))
    cp = M.load_urdf(os.path.join(REF, "assets/urdf/cartpole.urdf"), "cartpole", fix_base=True)
    M.apply_asset_options(cp, "cartpole")
    cp.to_json(os.path.join(out, "cartpole.json"))
    sh = shadow_hand()
    M.apply_asset_options(sh, "shadow_hand")
    sh.to_json(os.path.join(out, "shadow_hand.json"))
    objs = hand_objects(sh)
    with open(os.path.join(out, "hand_objects.json"), "w") as f:
        json.dump(objs, f, indent=1)
    print("hand objects:", {k: (v["type"], v["size"], round(v["mass"], 5)) for k, v in objs.items()})
    for s in (ant, hum, cp, sh):
        print(f"{s.name}: nodes={len(s.nodes)} dofs={s.num_dofs} bodies={len(s.bodies)} geoms={len(s.geoms)} "
              f"pairs={len(s.pairs)} mass={s.total_mass():.4f} sensors={s.sensors}")


if __name__ == "__main__":
    main()
