"""gymnasium.spaces when installed, else a minimal stand-in with the same surface.

The reference only declares spaces and reads ``.n`` / ``.shape`` / ``.spaces`` (a2c.py:118-135)
and calls ``.sample()`` in train.py:268; Dict keys are sorted like gymnasium does for a plain
dict argument.
"""
import numpy as np

try:  # pragma: no cover - depends on the environment
    from gymnasium import spaces as _gym_spaces
    Discrete = _gym_spaces.Discrete
    MultiDiscrete = _gym_spaces.MultiDiscrete
    Box = _gym_spaces.Box
    Dict = _gym_spaces.Dict
    HAVE_GYMNASIUM = True
except ImportError:
    HAVE_GYMNASIUM = False

    class _Space:
        def seed(self, seed=None):
            self._rng = np.random.default_rng(seed)

        @property
        def np_random(self):
            if not hasattr(self, "_rng"):
                self._rng = np.random.default_rng()
            return self._rng

    class Discrete(_Space):
        def __init__(self, n, start=0):
            self.n = int(n)
            self.start = int(start)
            self.shape = ()
            self.dtype = np.int64

        def sample(self):
            return int(self.np_random.integers(self.n)) + self.start

        def contains(self, x):
            return self.start <= int(x) < self.start + self.n

        def __repr__(self):
            return f"Discrete({self.n})"

    class MultiDiscrete(_Space):
        def __init__(self, nvec, dtype=np.int64):
            self.nvec = np.asarray(nvec, dtype=dtype)
            self.shape = self.nvec.shape
            self.dtype = dtype

        def sample(self):
            return (self.np_random.random(self.nvec.shape) * self.nvec).astype(self.dtype)

        def __repr__(self):
            return f"MultiDiscrete({self.nvec.tolist()})"

    class Box(_Space):
        def __init__(self, low, high, shape=None, dtype=np.float32):
            self.dtype = np.dtype(dtype)
            self.shape = tuple(shape) if shape is not None else np.shape(low)
            self.low = np.full(self.shape, low, dtype=self.dtype)
            self.high = np.full(self.shape, high, dtype=self.dtype)

        def sample(self):
            if self.dtype.kind in "iu":
                return self.np_random.integers(self.low, self.high + 1).astype(self.dtype)
            return self.np_random.uniform(self.low, self.high).astype(self.dtype)

        def __repr__(self):
            return f"Box({self.low.min()}, {self.high.max()}, {self.shape}, {self.dtype})"

    class Dict(_Space):
        def __init__(self, spaces=None, **kw):
            d = dict(spaces or {}, **kw)
            self.spaces = dict(sorted(d.items()))

        def __getitem__(self, k):
            return self.spaces[k]

        def keys(self):
            return self.spaces.keys()

        def items(self):
            return self.spaces.items()

        def sample(self):
            return {k: s.sample() for k, s in self.spaces.items()}

        def __repr__(self):
            return "Dict(" + ", ".join(f"{k}: {v}" for k, v in self.spaces.items()) + ")"
