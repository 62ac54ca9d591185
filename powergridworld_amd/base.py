"""Batched ComponentEnv / MultiComponentEnv (reference: gridworld/base.py:12-182).

Every env object here simulates ``num_envs`` independent copies of the
reference env in lockstep on the GPU.  The API is the reference's -- same
constructor arguments, ``reset``/``step``/``step_reward``/``get_obs``,
``real_power``/``reactive_power``/``obs_labels`` -- with these batch rules:

* observations, rewards and real powers are fp64 device tensors with a leading
  env axis ([N, dim] / [N]); they are VIEWS of persistent buffers that the next
  ``step``/``reset`` overwrites (clone them to keep them);
* actions may be [N, dim] tensors (any strides, zero-copy when fp64 on the
  device), a single [dim] action broadcast to all envs, or numpy/lists;
* ``done`` is a Python bool: all copies share the time axis, so they finish
  together exactly as the reference's single env does.
"""
from abc import ABC, abstractmethod
from typing import Dict, List, Tuple

import numpy as np
import torch

from powergridworld_amd import _lib
from powergridworld_amd import spaces
from powergridworld_amd.log import logger


def as_env_tensor(x, n, device, what="value"):
    """Scalar / [N] / [N,1] input -> fp64 [N] device tensor (broadcast allowed)."""
    if x is None:
        return None
    if (type(x) is torch.Tensor and x.dtype == torch.float64 and x.dim() == 1 and x.shape[0] == n
            and x.device == device and x.is_contiguous()):
        return x                                   # already an [N] fp64 device vector
    t = x if isinstance(x, torch.Tensor) else torch.as_tensor(np.asarray(x, dtype=np.float64))
    if t.dtype != torch.float64 or t.device != device:
        t = t.to(device=device, dtype=torch.float64)
    t = t.reshape(-1)
    if t.numel() == 1:
        return t.expand(n).contiguous()
    if t.numel() != n:
        raise ValueError("%s: expected %d values, got shape %s" % (what, n, tuple(t.shape)))
    return t.contiguous()


def as_action(a, n, dim, device, dtype=torch.float64):
    """Normalise an action to a [n, dim] device tensor of `dtype` (views where possible)."""
    if a is None:
        return None
    t = a if isinstance(a, torch.Tensor) else torch.as_tensor(np.asarray(a, dtype=np.float64))
    if t.dtype != dtype or t.device != device:
        t = t.to(device=device, dtype=dtype)
    if t.dim() == 0:
        return t.reshape(1, 1).expand(n, dim)
    if t.dim() == 1:
        if t.shape[0] == dim:
            return t.reshape(1, dim).expand(n, dim)   # one reference-shaped action for all envs
        if dim == 1 and t.shape[0] == n:
            return t.reshape(n, 1)
    if t.dim() == 2 and tuple(t.shape) == (n, dim):
        return t
    raise ValueError("action of shape %s does not fit (num_envs=%d, action_dim=%d)"
                     % (tuple(t.shape), n, dim))


def oob_poll(counter):
    """The reference warns on every out-of-bounds action (utils.py:35-37); the
    kernels count them on the device instead (PGW_OOB).  Called at resets: logs
    the count a previous call copied to pinned host memory, if that copy has
    landed and the count grew, then starts the next asynchronous copy -- never
    a synchronization, so a warning arrives one reset late."""
    st = getattr(counter, "_pgw_oob", None)
    if st is None:
        st = {"host": torch.zeros(1, dtype=torch.int64).pin_memory(), "ev": None, "seen": 0}
        counter._pgw_oob = st
    ev = st["ev"]
    if ev is not None:
        if not ev.query():
            return
        st["ev"] = None
        v = int(st["host"][0])
        if v > st["seen"]:
            logger.warning("argument out of bounds: %d action(s) outside [-1 - 1e-4, 1 + 1e-4] were "
                           "clipped (counted on the device)", v - st["seen"])
            st["seen"] = v
    st["host"].copy_(counter, non_blocking=True)
    ev = torch.cuda.Event()
    ev.record(torch.cuda.current_stream(counter.device))
    st["ev"] = ev


class ComponentEnv(spaces.Env, ABC):
    """Base class for any environment used in the multiagent simulation
    (gridworld/base.py:12-71), batched over ``num_envs`` copies."""

    # storage dtypes the subclass's kernels implement (fp32 = the _f32 entries)
    supported_dtypes = (torch.float64,)

    def __new__(cls, *args, **kwargs):
        # checked here, before any subclass __init__ could swallow `dtype` in **kwargs
        dt = kwargs.get("dtype")
        if dt is not None and _lib.storage_dtype(dt) not in cls.supported_dtypes:
            raise NotImplementedError("%s has no %s storage variant" % (cls.__name__, dt))
        return super().__new__(cls)

    def __init__(self, name: str = None, num_envs: int = 1, device=None, dtype=None, **kwargs):
        super().__init__()
        self.name = name
        self.num_envs = int(num_envs)
        if self.num_envs < 1:
            raise ValueError("num_envs must be >= 1")
        self.device = _lib.require_device(device)
        self.dtype = _lib.storage_dtype(dtype)
        if self.dtype not in self.supported_dtypes:
            raise NotImplementedError("%s has no %s storage variant" % (type(self).__name__, self.dtype))
        n = self.num_envs
        self._real_power = torch.zeros(n, dtype=self.dtype, device=self.device)
        self._reactive_power = torch.zeros(n, dtype=self.dtype, device=self.device)
        self._zero_reward = torch.zeros(n, dtype=self.dtype, device=self.device)
        self._obs_labels = []
        self._in_multicomponent = False
        # out-of-bounds actions (gridworld/utils.py:35-37; PGW_OOB in pgw.h): the
        # kernels count every to_raw call the reference would have warned on
        self.oob_count = torch.zeros(1, dtype=torch.int64, device=self.device)

    # ---- out-of-bounds action counter -----------------------------------------
    def _bind_oob(self, counter):
        """Count this env's out-of-bounds actions into `counter` (a [1] int64
        device tensor; a composite env hands its own to every component)."""
        self.oob_count = counter
        p = self.__dict__.get("params")
        if p is not None and hasattr(p, "oob"):
            p.oob = counter.data_ptr()

    def oob_actions(self) -> torch.Tensor:
        """Out-of-bounds actions clipped so far: the number of warnings the
        reference's to_raw would have logged (one per env, component and step).
        A device tensor -- reading its value synchronizes."""
        return self.oob_count

    # ---- buffers ------------------------------------------------------------
    def _new_obs(self, dim):
        """Env-minor obs buffer [dim, N]; the returned [N, dim] view is what
        step()/reset() hand out (coalesced device writes, zero-copy for the caller)."""
        buf = torch.zeros((dim, self.num_envs), dtype=self.dtype, device=self.device)
        return buf.t()

    def _stream(self):
        return _lib.stream_ptr(self.device)

    def _mat(self, t2d):
        """pgw_mat / pgw_matf of one of this env's [N, dim] buffers (its dtype;
        None: the null matrix)."""
        return (_lib.matf if self.dtype == torch.float32 else _lib.mat)(t2d)

    def _kernel(self, name):
        """The ABI entry for this env's storage dtype (name + "_f32" for fp32)."""
        return getattr(_lib.lib(), name + ("_f32" if self.dtype == torch.float32 else ""))

    # ---- per-step host-cost caches ------------------------------------------
    # _bufv counts re-pointings of the env's device buffers (_adopt): cached
    # launch arguments that hold their pointers are rebuilt when it changes.
    _bufv = 0
    _bufv_gen = 0      # any env's re-pointing (one int for a whole agent set to check)

    def _act_mat(self, a):
        """pgw_mat of an action tensor, cached per (pointer, strides): a policy
        writes its actions into a few buffers that the caching allocator hands
        out in turn, or the caller cycles a preallocated pool."""
        key = (a.data_ptr(), a.stride(0), a.stride(1), a.dtype)
        c = self.__dict__.get("_act_mat_c")
        if c is None:
            c = self._act_mat_c = {}
        m = c.get(key)
        if m is None:
            if len(c) >= 64:
                c.clear()
            m = c[key] = (_lib.matf if a.dtype == torch.float32 else _lib.mat)(a)
        return m

    def _action_mat(self, action, dim):
        """(action as an [N, dim] tensor, its pgw_mat) for the fused MC step.  A
        tensor the kernels can read in place is looked up by (pointer, strides,
        shape, dtype, device) first -- a policy's output buffers and the benches'
        pools repeat -- so the per-step cost is a few attribute reads instead of
        as_action's checks plus _act_mat."""
        key = None
        if type(action) is torch.Tensor:
            key = (action.data_ptr(), action.stride(), action.shape, action.dtype, action.get_device())
            c = self.__dict__.get("_am_c")
            if c is not None:
                hit = c.get(key)
                if hit is not None:
                    # the caller's own tensor: the cache keeps only the pgw_mat
                    # (pointer + strides), never a reference that would pin the
                    # allocation
                    return action, hit
        a = as_action(action, self.num_envs, dim, self.device, self.dtype)
        m = self._act_mat(a)
        if key is not None and a is action:
            c = self.__dict__.get("_am_c")
            if c is None:
                c = self._am_c = {}
            if len(c) >= 64:
                c.clear()
            c[key] = m
        return a, m

    def state_dict(self):
        """The env's whole state (device tensors, generator states, clocks):
        powergridworld_amd.checkpoint.state_dict."""
        from powergridworld_amd.checkpoint import state_dict
        return state_dict(self)

    def load_state_dict(self, sd, strict=False):
        """Restore a state_dict() of an env of the same configuration (in place)."""
        from powergridworld_amd.checkpoint import load_state_dict
        return load_state_dict(self, sd, strict)

    @abstractmethod
    def reset(self, **kwargs):
        """Standard gym reset method but with kwargs."""

    @abstractmethod
    def step(self, action, **kwargs) -> Tuple[torch.Tensor, torch.Tensor, bool, dict]:
        """Standard gym step method but with kwargs."""

    @abstractmethod
    def step_reward(self, **kwargs) -> Tuple[torch.Tensor, dict]:
        """Returns the current step reward and metadata dict."""

    @abstractmethod
    def get_obs(self, **kwargs) -> Tuple[torch.Tensor, dict]:
        """Returns the current observation (state) and any metadata."""

    @property
    def real_power(self) -> torch.Tensor:
        """Real power per env, positive for load and negative for generation."""
        return self._real_power

    @property
    def reactive_power(self) -> torch.Tensor:
        return self._reactive_power

    @property
    def obs_labels(self) -> list:
        return self._obs_labels

    # For the fused multi-agent kernel: which kernel component this env is.
    fused_kind = None


# The hooks a fused kernel implements for a component: a subclass that overrides
# any of them (e.g. a PV with a nonzero reactive_power) must take the generic
# path, which calls them.
FUSED_HOOKS = ("step", "step_reward", "get_obs", "is_terminal", "real_power", "reactive_power")


def owns_fused_hooks(env, attr, hooks=FUSED_HOOKS, skip=()):
    """True when every hook of ``type(env)`` is the one of the class that declares
    ``attr`` (fused_kind / mc_kind), i.e. the code the kernel restates."""
    cls = type(env)
    owner = next((c for c in cls.__mro__ if attr in c.__dict__), None)
    if owner is None:
        return False
    return all(getattr(cls, h, None) is getattr(owner, h, None) for h in hooks if h not in skip)


def resolve_env_class(cls):
    """Accept this package's classes, or reference classes by name (drop-in for
    configs built against gridworld.*)."""
    if isinstance(cls, type) and issubclass(cls, (ComponentEnv,)):
        return cls
    from powergridworld_amd import agents   # noqa: F401  (registers classes)
    name = getattr(cls, "__name__", str(cls))
    reg = ENV_REGISTRY.get(name)
    if reg is None:
        raise TypeError("no MI355X implementation for env class %r" % (name,))
    return reg


ENV_REGISTRY = {}


def register_env(cls):
    ENV_REGISTRY[cls.__name__] = cls
    return cls


@register_env
class MultiComponentEnv(ComponentEnv):
    """Single agent composed of several component envs (gridworld/base.py:74-182):
    the action/observation spaces are the union, real power and reward the sum
    over components (reward recomputed after all components stepped, base.py:137).
    dtype=torch.float32: fp32 storage for every component (fp64 arithmetic),
    stepped by pgw_mc_agent_step_f32; the fused component kinds only."""

    supported_dtypes = (torch.float64, torch.float32)

    def __init__(self, name: str = None, components: List[dict] = None, num_envs: int = 1,
                 device=None, **kwargs):
        super().__init__(name=name, num_envs=num_envs, device=device, **kwargs)
        self.envs = []
        for c in components:
            cls = resolve_env_class(c["cls"])
            cfg = dict(c["config"])
            if self.dtype != torch.float64:
                cfg.setdefault("dtype", self.dtype)
            env = cls(name=c["name"], num_envs=self.num_envs, device=self.device, **cfg)
            env._in_multicomponent = True
            if env.dtype != self.dtype:
                raise NotImplementedError("MultiComponentEnv: component %s is %s, the agent %s"
                                          % (env.name, env.dtype, self.dtype))
            self.envs.append(env)
        self._bind_oob(self.oob_count)
        self.observation_space = spaces.Dict({e.name: e.observation_space for e in self.envs})
        self.action_space = spaces.Dict({e.name: e.action_space for e in self.envs})
        self._obs_labels_dict = {e.name: e.obs_labels for e in self.envs}
        obs_labels = []
        for e in self.envs:
            obs_labels += e.obs_labels
        self._obs_labels = list(set(obs_labels))
        self._reward = torch.zeros(self.num_envs, dtype=self.dtype, device=self.device)
        if len(self.envs) > _lib.MAX_COMP:
            raise ValueError("at most %d components per agent" % _lib.MAX_COMP)
        if self.dtype != torch.float64 and not self._mc_fusable():
            raise NotImplementedError("MultiComponentEnv dtype=%s needs every component to be a fused kind "
                                      "(pgw_mc_agent_step_f32)" % self.dtype)

    def _bind_oob(self, counter):
        super()._bind_oob(counter)
        for e in self.__dict__.get("envs", ()):
            e._bind_oob(counter)

    def reset(self, **kwargs):
        """Resets each component and returns (obs dict, meta dict) (base.py:108-111)."""
        oob_poll(self.oob_count)
        for e in self.envs:
            e.reset(**kwargs)
        self._real_power.zero_()
        self._ep_step = 0                 # episode step (the captured steps' clock, graph.py)
        return self.get_obs(**kwargs)

    def _mc_clock(self):
        """Per-block device clocks of the captured fused step
        (pgw_mc_step_args.clock, one int32 per 64 envs) and the host's record of
        the episode step they hold (None: not known to match)."""
        c = self.__dict__.get("_clock")
        if c is None:
            c = self._clock = torch.zeros(max(1, (self.num_envs + 63) // 64), dtype=torch.int32, device=self.device)
            self._clock_k = None
        return c

    def _reduce(self):
        a = _lib.ReduceArgs()
        a.n_comp = len(self.envs)
        for i, e in enumerate(self.envs):
            a.real_power[i] = e.real_power.data_ptr()
            r = e._current_reward()
            a.reward[i] = None if r is None else r.data_ptr()
        _lib.check(_lib.lib().pgw_agent_reduce(a, self.num_envs, _lib.dptr(self._real_power),
                                               _lib.dptr(self._reward), self._stream()))

    def _mc_fusable(self):
        """Every component is one of the kinds pgw_mc_agent_step implements
        (building with the thermal-energy reward, PV, storage, EV), each once,
        and none overrides its step."""
        if getattr(self, "_mc_fuse", None) is None:
            # the class that declares mc_kind must also provide every hook the
            # kernel restates (step, reward, obs, powers, terminal test)
            kinds = [getattr(type(e), "mc_kind", None) for e in self.envs]
            ok = all(k is not None for k in kinds) and len(set(kinds)) == len(kinds) and len(kinds) <= 4
            self._mc_fuse = ok and all(owns_fused_hooks(e, "mc_kind") for e in self.envs)
        return self._mc_fuse

    def step(self, action: dict, **kwargs):
        obs, dones, metas = {}, [], {}
        if self._mc_fusable():
            # the whole agent in one launch (pgw_mc_agent_step), same arithmetic
            # launch arguments: the static part (parameters, state pointers, obs
            # views) is built once per buffer layout, only the per-step fields
            # (actions, exogenous rows, schedules) are written each step; the
            # library copies the struct into the launch, so reuse is safe
            key = (self._real_power.data_ptr(), self._reward.data_ptr(), [e._bufv for e in self.envs])
            args = self.__dict__.get("_mc_args")
            if args is None or self._mc_args_key != key:
                f32 = self.dtype == torch.float32
                args = (_lib.MCStepArgsF32 if f32 else _lib.MCStepArgs)()
                args.n_comp = len(self.envs)
                for c, env in enumerate(self.envs):
                    env._mc_static(args, c)
                args.real_power, args.reward = self._real_power.data_ptr(), self._reward.data_ptr()
                self._mc_args, self._mc_args_key = args, key
                self._mc_call = (_lib.lib().pgw_mc_agent_step_f32 if f32 else _lib.lib().pgw_mc_agent_step,
                                 self.num_envs)
            keep = []
            if kwargs:
                kws = [{k: v for k, v in kwargs.items() if k in env.obs_labels} for env in self.envs]
            else:
                kws = self.__dict__.get("_mc_nokw")
                if kws is None:
                    kws = self._mc_nokw = [{} for _ in self.envs]
            for c, env in enumerate(self.envs):
                keep.append(env._mc_prepare(args, c, action[env.name], kws[c]))
            fn, n = self._mc_call
            rc = fn(args, n, self._stream())      # (the caller's current stream, every step)
            if rc:
                _lib.check(rc)
            self._ep_step = self.__dict__.get("_ep_step", 0) + 1
            for env, env_kwargs in zip(self.envs, kws):
                ob, _, done, meta = env._mc_finish(env_kwargs)
                obs[env.name] = ob
                dones.append(done)
                metas[env.name] = meta
            return obs, self._reward, any(dones), metas
        for env in self.envs:
            env_kwargs = {k: v for k, v in kwargs.items() if k in env.obs_labels}
            ob, _, done, meta = env.step(action[env.name], **env_kwargs)
            obs[env.name] = ob
            dones.append(done)
            metas[env.name] = meta
        self._reduce()
        return obs, self._reward, any(dones), metas

    def capture_step(self, action, steps=1, clocked=False, **kwargs):
        """A StepGraph (graph.py) of the fused step reading `action` (a dict of
        the components' [N, dim] device tensors, or a list of `steps` such
        dicts): call it to run the captured step(s) with whatever the caller
        wrote into those tensors.  Default: one graph per episode position,
        captured on first use; clocked=True: one graph for every position, the
        per-step values read through the device clocks."""
        from powergridworld_amd.graph import StepGraph
        return StepGraph(self, action, steps, kwargs, clocked)

    def step_reward(self, **kwargs):
        meta = {e.name: e.step_reward()[1] for e in self.envs}
        return self._reward, meta

    def get_obs(self, **kwargs):
        obs, meta = {}, {}
        for env in self.envs:
            env_kwargs = {k: v for k, v in kwargs.items() if k in env.obs_labels}
            obs[env.name], meta[env.name] = env.get_obs(**env_kwargs)
        return obs, meta

    @property
    def obs_labels_dict(self) -> Dict[str, list]:
        return self._obs_labels_dict

    @property
    def env_dict(self) -> Dict[str, ComponentEnv]:
        return {e.name: e for e in self.envs}

    def _current_reward(self):
        return self._reward
