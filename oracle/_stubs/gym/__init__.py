"""Minimal stand-in for the ``gym`` package, used ONLY by ``oracle/make_golden.py``
to import the reference (``/root/reference/gridworld/base.py:6`` imports gym, which
is not installed in this image).  Test infrastructure; never imported by the
product package.

Implements just what the reference touches: ``gym.Env``, ``gym.spaces.Box``
(low/high/shape/dtype/sample), ``gym.spaces.Dict`` and ``gym.spaces.Discrete``.
"""
import numpy as np


class Env(object):
    def __init__(self, *args, **kwargs):
        pass


class _Space(object):
    _rng = np.random.default_rng(0)

    def seed(self, seed=None):
        _Space._rng = np.random.default_rng(seed)


class Box(_Space):
    def __init__(self, low=None, high=None, shape=None, dtype=np.float32):
        dtype = np.dtype(dtype)
        if shape is None:
            shape = np.shape(low) if np.ndim(low) > 0 else np.shape(high)
        shape = tuple(shape)
        self.low = np.broadcast_to(np.asarray(low, dtype=dtype), shape).copy()
        self.high = np.broadcast_to(np.asarray(high, dtype=dtype), shape).copy()
        self.shape = shape
        self.dtype = dtype

    def sample(self):
        return self._rng.uniform(self.low, self.high).astype(self.dtype)

    def __repr__(self):
        return "Box(%s, %s, %s)" % (self.low, self.high, self.shape)


class Discrete(_Space):
    def __init__(self, n):
        self.n = n
        self.shape = ()
        self.dtype = np.int64

    def sample(self):
        return int(self._rng.integers(self.n))


class Dict(_Space):
    def __init__(self, spaces=None, **kw):
        self.spaces = dict(spaces or {}, **kw)

    def __getitem__(self, k):
        return self.spaces[k]

    def __iter__(self):
        return iter(self.spaces)

    def keys(self):
        return self.spaces.keys()

    def items(self):
        return self.spaces.items()

    def sample(self):
        return {k: v.sample() for k, v in self.spaces.items()}


class _SpacesModule(object):
    Box = Box
    Dict = Dict
    Discrete = Discrete
    Space = _Space


spaces = _SpacesModule()
