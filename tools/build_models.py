#!/usr/bin/env python3
"""Regenerate the shipped model tables from the reference's robot files.

Build-container only (reads /root/reference/assets).  The tables are derived
data (the build's own importer output, see migym/model.py); the GPU box loads
them from migym/assets/*.json.

  Ant       assets/mjcf/nv_ant.xml        (tasks/ant.py:142-197; feet force sensors :170-178)
  Humanoid  assets/mjcf/nv_humanoid.xml   (tasks/humanoid.py:142-196; foot sensors :163-168;
                                           self-collision filter 0 :194)
  Cartpole  assets/urdf/cartpole.urdf     (tasks/cartpole.py:78-113; fix_base_link :88)
"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "isaacgymenvs-ma_amd"))
from migym import model as M  # noqa: E402

REF = os.environ.get("MIGYM_REFERENCE", "/root/reference")


def main():
    out = M.ASSET_DIR
    ant = M.load_mjcf(os.path.join(REF, "assets/mjcf/nv_ant.xml"), "ant")
    ant.sensors = [i for i, b in enumerate(ant.bodies) if "foot" in b.name]
    ant.to_json(os.path.join(out, "ant.json"))
    hum = M.load_mjcf(os.path.join(REF, "assets/mjcf/nv_humanoid.xml"), "humanoid", self_collision=True)
    hum.sensors = [hum.body_index("right_foot"), hum.body_index("left_foot")]
    hum.to_json(os.path.join(out, "humanoid.json"))
    cp = M.load_urdf(os.path.join(REF, "assets/urdf/cartpole.urdf"), "cartpole", fix_base=True)
    cp.to_json(os.path.join(out, "cartpole.json"))
    for s in (ant, hum, cp):
        print(f"{s.name}: nodes={len(s.nodes)} dofs={s.num_dofs} bodies={len(s.bodies)} geoms={len(s.geoms)} "
              f"pairs={len(s.pairs)} mass={s.total_mass():.4f} sensors={s.sensors}")


if __name__ == "__main__":
    main()
