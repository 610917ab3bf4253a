"""Minimal ``gym.spaces.Box`` stand-in (the reference imports gym, vec_task.py:36-37;
gym is not a dependency of this build).  If ``gym`` is importable its Box is used."""
import numpy as np

try:  # pragma: no cover - optional
    from gym.spaces import Box, Dict  # type: ignore
except Exception:  # noqa: BLE001
    class Dict(dict):
        """``gym.spaces.Dict`` stand-in: a mapping of named sub-spaces."""

        def __init__(self, spaces=None):
            super().__init__(spaces or {})

        @property
        def spaces(self):
            return dict(self)

        def __repr__(self):
            return f"Dict({', '.join(f'{k}: {v!r}' for k, v in self.items())})"

    class Box:
        def __init__(self, low, high, shape=None, dtype=np.float32):
            self.low = np.asarray(low, dtype=dtype)
            self.high = np.asarray(high, dtype=dtype)
            self.shape = self.low.shape if shape is None else tuple(shape)
            self.dtype = np.dtype(dtype)

        def __repr__(self):
            return f"Box({self.shape})"
