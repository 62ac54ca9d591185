"""Observation/action space types.

The reference builds ``gym.spaces.Box``/``Dict`` (e.g. ``gridworld/base.py:95-99``).
When ``gym`` (or ``gymnasium``) is importable its classes are used directly;
otherwise these minimal stand-ins with the same attributes (low, high, shape,
dtype, sample) are used -- gym is an optional dependency of the env API, not of
the step kernels.
"""
import numpy as np

try:  # pragma: no cover - depends on the environment
    import gym as _gym
    Box, Dict, Discrete = _gym.spaces.Box, _gym.spaces.Dict, _gym.spaces.Discrete
    Env = _gym.Env
except Exception:  # gym is not installed in this image
    class Env(object):
        pass

    class Box(object):
        def __init__(self, low=None, high=None, shape=None, dtype=np.float32, seed=None):
            dtype = np.dtype(dtype)
            if shape is None:
                shape = np.shape(low) if np.ndim(low) > 0 else np.shape(high)
            shape = tuple(shape)
            self.low = np.broadcast_to(np.asarray(low, dtype=dtype), shape).copy()
            self.high = np.broadcast_to(np.asarray(high, dtype=dtype), shape).copy()
            self.shape = shape
            self.dtype = dtype
            self._rng = np.random.default_rng(seed)

        def seed(self, seed=None):
            self._rng = np.random.default_rng(seed)

        def sample(self):
            return self._rng.uniform(self.low, self.high).astype(self.dtype)

        def contains(self, x):
            x = np.asarray(x)
            return x.shape == self.shape and bool(np.all(x >= self.low) and np.all(x <= self.high))

        def __repr__(self):
            return "Box(%s, %s, %s, %s)" % (self.low, self.high, self.shape, self.dtype)

    class Discrete(object):
        def __init__(self, n, seed=None):
            self.n = n
            self.shape = ()
            self.dtype = np.int64
            self._rng = np.random.default_rng(seed)

        def sample(self):
            return int(self._rng.integers(self.n))

    class Dict(object):
        def __init__(self, spaces=None, **kw):
            self.spaces = dict(spaces or {}, **kw)

        def __getitem__(self, k):
            return self.spaces[k]

        def __iter__(self):
            return iter(self.spaces)

        def __len__(self):
            return len(self.spaces)

        def keys(self):
            return self.spaces.keys()

        def items(self):
            return self.spaces.items()

        def values(self):
            return self.spaces.values()

        def sample(self):
            return {k: v.sample() for k, v in self.spaces.items()}

        def __repr__(self):
            return "Dict(%r)" % (self.spaces,)
