"""Minimal action / observation spaces with gymnasium's semantics (gymnasium is not a dependency).

`Discrete.contains` follows gymnasium.spaces.Discrete.contains, which is what the reference's
`assert self.action_space.contains(action)` (k8s_multi_cloud_env.py:116) evaluates: a python
int (bool included) or a 0-d numpy integer, with start <= x < start + n.  Pinned by
tests/golden/action_validity.json (generated from the reference env).
"""
from __future__ import annotations

import numpy as np


class Discrete:
    def __init__(self, n: int, start: int = 0, seed=None):
        self.n = int(n)
        self.start = int(start)
        self.shape = ()
        self.dtype = np.int64
        self._rng = np.random.default_rng(seed)

    def contains(self, x) -> bool:
        if isinstance(x, int):
            as_int64 = np.int64(x)
        elif isinstance(x, (np.generic, np.ndarray)) and (np.issubdtype(x.dtype, np.integer) and x.shape == ()):
            as_int64 = np.int64(x)
        else:
            return False
        return bool(self.start <= as_int64 < self.start + self.n)

    def __contains__(self, x) -> bool:
        return self.contains(x)

    def sample(self) -> int:
        return int(self.start + self._rng.integers(self.n))

    def seed(self, seed=None):
        self._rng = np.random.default_rng(seed)

    def __repr__(self) -> str:
        return f"Discrete({self.n})" if self.start == 0 else f"Discrete({self.n}, start={self.start})"


class Box:
    def __init__(self, low, high, shape=None, dtype=np.float32):
        self.shape = tuple(shape) if shape is not None else np.shape(low)
        self.dtype = np.dtype(dtype)
        self.low = np.full(self.shape, low, dtype=self.dtype)
        self.high = np.full(self.shape, high, dtype=self.dtype)

    def contains(self, x) -> bool:
        x = np.asarray(x)
        return x.shape == self.shape and bool(np.all(x >= self.low) and np.all(x <= self.high))

    def __repr__(self) -> str:
        return f"Box({self.low.min()}, {self.high.max()}, {self.shape}, {self.dtype})"
