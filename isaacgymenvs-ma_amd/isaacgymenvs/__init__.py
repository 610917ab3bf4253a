"""Drop-in import name: ``import isaacgymenvs; isaacgymenvs.make(...)`` resolves to
the MI355X path (migym).  Only the hot-path surface is provided."""
from migym import make, __version__  # noqa: F401
