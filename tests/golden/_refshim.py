"""Import shim for generating golden vectors from the reference's own Python.

Used ONLY by ``tests/golden/make_golden.py`` in the build container (where the
read-only reference checkout lives at ``/root/reference``).  It never runs on the
GPU box and nothing in the product imports it.

The reference's obs/reward half is plain ``@torch.jit.script`` Python
(SURVEY.md §8(c)); it becomes importable once the closed ``isaacgym`` wheel and
the ``gym`` package are replaced by inert module objects and the heavy package
``__init__`` files (hydra, the all-tasks import) are bypassed with namespace
shells whose ``__path__`` points at the real directories.
"""
import os
import sys
import types

import numpy as np

REF = os.environ.get("MIGYM_REFERENCE", "/root/reference")


def _module(name):
    m = types.ModuleType(name)
    sys.modules[name] = m
    return m


class _Box:
    def __init__(self, low, high, *a, **k):
        self.low = np.asarray(low, dtype=np.float32)
        self.high = np.asarray(high, dtype=np.float32)
        self.shape = self.low.shape


def install():
    if getattr(install, "_done", False):
        return
    np.Inf = np.inf  # the reference uses the NumPy-1 alias (vec_task.py:108-117)
    ig = _module("isaacgym")
    for sub in ("gymapi", "gymtorch", "gymutil", "torch_utils"):
        m = _module("isaacgym." + sub)
        setattr(ig, sub, m)
    gym = _module("gym")
    spaces = _module("gym.spaces")
    spaces.Box = _Box
    gym.spaces = spaces
    gym.Space = object
    for pkg, rel in (("isaacgymenvs", "isaacgymenvs"),
                     ("isaacgymenvs.tasks", "isaacgymenvs/tasks"),
                     ("isaacgymenvs.tasks.base", "isaacgymenvs/tasks/base"),
                     ("isaacgymenvs.utils", "isaacgymenvs/utils")):
        m = _module(pkg)
        m.__path__ = [os.path.join(REF, rel)]
    fill_gymapi(ig.gymapi)
    install._done = True


def fill_gymapi(gymapi):
    """Constants/classes the task modules touch at construction time (Appendix D)."""
    class Vec3:
        def __init__(self, x=0.0, y=0.0, z=0.0):
            self.x, self.y, self.z = x, y, z

        def __add__(self, o):
            return Vec3(self.x + o.x, self.y + o.y, self.z + o.z)

    class Quat:
        def __init__(self, x=0.0, y=0.0, z=0.0, w=1.0):
            self.x, self.y, self.z, self.w = x, y, z, w

    class Transform:
        def __init__(self, p=None, r=None):
            self.p = p or Vec3()
            self.r = r or Quat()

    class _Bag:
        def __init__(self, *a, **k):
            pass

    class SimParams:
        def __init__(self):
            self.physx = _Bag()
            self.flex = _Bag()
            self.gravity = Vec3()

    for k, v in dict(SIM_PHYSX=0, SIM_FLEX=1, UP_AXIS_Z=1, UP_AXIS_Y=0, DOF_MODE_NONE=0,
                     DOF_MODE_POS=1, DOF_MODE_VEL=2, DOF_MODE_EFFORT=3, MESH_VISUAL=1,
                     DOMAIN_SIM=0, LOCAL_SPACE=0, ENV_SPACE=1, CC_NEVER=0).items():
        setattr(gymapi, k, v)
    gymapi.Vec3, gymapi.Quat, gymapi.Transform = Vec3, Quat, Transform
    gymapi.SimParams = SimParams
    gymapi.PlaneParams = _Bag
    gymapi.AssetOptions = _Bag
    gymapi.CameraProperties = _Bag
    gymapi.ContactCollection = lambda x: x
