"""gym.spaces stand-ins (``Box``, ``Discrete``) used when gym itself is not installed.

The reference only touches ``Box(low, high, shape).shape`` / ``.low`` / ``.high`` and ``Discrete(n).n``
(environments/gym_flock_v2.py:58-60, gym_flock_uw_discrete.py:98-99); if gym is importable its classes are used.
"""
import numpy as np

try:  # pragma: no cover - gym is absent in this image
    from gym.spaces import Box, Discrete  # type: ignore
except Exception:  # noqa: BLE001

    class Box:
        def __init__(self, low, high, shape=None, dtype=np.float32):
            self.low, self.high, self.dtype = low, high, dtype
            self.shape = tuple(shape) if shape is not None else np.shape(low)

        def sample(self):
            return np.random.uniform(self.low, self.high, size=self.shape).astype(self.dtype)

        def __repr__(self):
            return f"Box({self.low}, {self.high}, {self.shape}, {np.dtype(self.dtype).name})"

    class Discrete:
        def __init__(self, n):
            self.n = int(n)
            self.shape = ()

        def sample(self):
            return int(np.random.randint(self.n))

        def __repr__(self):
            return f"Discrete({self.n})"
