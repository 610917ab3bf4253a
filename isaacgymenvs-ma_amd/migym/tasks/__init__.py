"""Task map (counterpart of isaacgymenvs/tasks/__init__.py:94-127, restricted to the hot path)."""
from .locomotion import Ant, Humanoid, MAAnt
from .cartpole import Cartpole
from .shadow_hand import ShadowHand

isaacgym_task_map = {
    "Ant": Ant,
    "Humanoid": Humanoid,
    "Cartpole": Cartpole,
    "MAAnt": MAAnt,
    "ShadowHand": ShadowHand,
}
