"""Minimal gymnasium.spaces stand-in: Discrete / MultiDiscrete / Box / Dict (keys sorted
for a plain-dict argument, as gymnasium does)."""
import numpy as np


class Space:
    pass


class Discrete(Space):
    def __init__(self, n, start=0):
        self.n = int(n)
        self.start = start
        self.shape = ()
        self.dtype = np.int64

    def sample(self):
        return int(np.random.randint(self.n)) + self.start


class MultiDiscrete(Space):
    def __init__(self, nvec, dtype=np.int64):
        self.nvec = np.asarray(nvec, dtype=dtype)
        self.shape = self.nvec.shape
        self.dtype = dtype


class Box(Space):
    def __init__(self, low, high, shape=None, dtype=np.float32):
        self.low = low
        self.high = high
        self.shape = tuple(shape) if shape is not None else np.shape(low)
        self.dtype = dtype


class Dict(Space):
    def __init__(self, spaces=None, **kw):
        spaces = dict(spaces or {}, **kw)
        self.spaces = dict(sorted(spaces.items()))

    def __getitem__(self, k):
        return self.spaces[k]

    def keys(self):
        return self.spaces.keys()
