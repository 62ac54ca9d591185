"""RLlib-shaped vectorized adapter over one batched MultiAgentEnv (SURVEY 8(f)
rank 3; reference: gridworld/multiagent_env.py:13-17 makes MultiAgentEnv an
RLlib MultiAgentEnv, examples/marl/rllib/heterogeneous/train.py:12-17 hands it
to RLlib, which vectorizes by stepping `num_envs_per_worker` Python copies).

Here the N copies already step together on the GPU, so the adapter only
reshapes: RLlib's per-sub-env structures are row views of [N, dim] device
tensors (row i of every observation / reward is sub-env i; the observations
stay on the device for a torch policy).  The engine overwrites its buffers in
place every step, while RLlib's collectors keep each step's observations until
they build a batch, so by default the adapter clones every batched tensor ONCE
per step (one device copy per buffer, not per row) and hands out rows of the
copy.  ``zero_copy=True`` hands out rows of the engine's own buffers instead:
valid only until the next step, for callers that consume them at once.

Two RLlib interfaces are provided:

* VectorEnv style -- ``vector_reset()``, ``reset_at(i)``,
  ``vector_step(actions)``, ``get_sub_environments()``;
* BaseEnv style (how RLlib's sampler drives multi-agent envs) --
  ``poll()``, ``send_actions({env_id: {agent: action}})``, ``try_reset(env_id)``.

Lockstep semantics: all copies share one clock, so they
finish their episode on the same step.  ``reset_at(i)`` / ``try_reset(i)``
therefore reset the whole batch on the first call after an episode ended and
return sub-env i's fresh observation on every call of that episode boundary;
asking to reset a sub-env in the middle of an episode raises (it cannot leave
the shared clock).

``vector_step_batched(action)`` is the fast path: the engine's own batched
action format in, batched tensors out, no per-sub-env Python objects.
"""
from typing import Any, Dict, List

import numpy as np
import torch

try:      # the same optional base as the reference's multiagent_env.py:13-17
    from ray.rllib.env.base_env import BaseEnv as _Base
except ImportError:
    _Base = object


def _row(x, i, n):
    """Sub-env i of a batched structure: rows of [N, ...] tensors are views; dicts
    recurse; anything else (lockstep dones, batch-wide counters) is shared."""
    if isinstance(x, torch.Tensor):
        return x[i] if x.dim() >= 1 and x.shape[0] == n else x
    if isinstance(x, dict):
        return {k: _row(v, i, n) for k, v in x.items()}
    return x


def _snapshot(x):
    """One clone per batched tensor (dicts recurse; bools and others are shared)."""
    if isinstance(x, torch.Tensor):
        return x.clone()
    if isinstance(x, dict):
        return {k: _snapshot(v) for k, v in x.items()}
    return x


def _stack(items, device):
    """Per-sub-env actions -> the batched action (dicts recurse; arrays and
    tensors are stacked along a new leading env axis on `device`)."""
    first = items[0]
    if isinstance(first, dict):
        return {k: _stack([it[k] for it in items], device) for k in first}
    if isinstance(first, torch.Tensor):
        return torch.stack([t.to(device=device, dtype=torch.float64) for t in items])
    return torch.as_tensor(np.stack([np.asarray(a, dtype=np.float64) for a in items]), device=device)


class MultiAgentVectorEnv(_Base):
    """RLlib VectorEnv / BaseEnv view of a batched MultiAgentEnv."""

    def __init__(self, env, zero_copy=False):
        self.env = env
        self.zero_copy = bool(zero_copy)
        self.num_envs = env.num_envs
        self.observation_space = env.observation_space
        self.action_space = env.action_space
        self._obs = self._rew = self._done = self._info = None
        self._episode_over = True        # nothing to step before the first reset
        self._reset_done = False         # the batch reset of this boundary happened
        self._pending = None             # BaseEnv: results not yet polled

    # ---------------------------------------------------------------- batched
    def vector_step_batched(self, action):
        """One engine step in its own batched format (dict {agent: ...} of [N, dim]
        tensors, or the fused path's packed buffer); returns the engine's
        (obs, rew, dones, meta)."""
        if self._episode_over:
            raise RuntimeError("step after the episode ended: reset first")
        obs, rew, dones, meta = self.env.step(action)
        if not self.zero_copy:
            obs, rew, meta = _snapshot(obs), _snapshot(rew), _snapshot(meta)
        self._obs, self._rew, self._done, self._info = obs, rew, dones, meta
        self._episode_over = bool(dones["__all__"])
        self._reset_done = False
        return obs, rew, dones, meta

    def _reset_batch(self):
        obs = self.env.reset()
        self._obs = obs if self.zero_copy else _snapshot(obs)
        self._episode_over = False
        self._reset_done = True
        return self._obs

    # ---------------------------------------------------------------- VectorEnv
    def vector_reset(self) -> List[Dict[str, Any]]:
        obs = self._reset_batch()
        return [_row(obs, i, self.num_envs) for i in range(self.num_envs)]

    def reset_at(self, index: int = None) -> Dict[str, Any]:
        index = 0 if index is None else int(index)
        if not 0 <= index < self.num_envs:
            raise IndexError("sub-env %d of %d" % (index, self.num_envs))
        if not self._reset_done:
            if not self._episode_over:
                raise RuntimeError("reset_at(%d) in the middle of an episode: the %d sub-envs share "
                                   "one clock (lockstep) and reset together" % (index, self.num_envs))
            self._reset_batch()
        return _row(self._obs, index, self.num_envs)

    def vector_step(self, actions: List[Dict[str, Any]]):
        """actions: one {agent: action} per sub-env.  Returns per-sub-env lists
        (obs, rewards, dones, infos) as RLlib's VectorEnv does; rewards are
        {agent: scalar tensor view}, dones {agent: bool, "__all__": bool}."""
        if len(actions) != self.num_envs:
            raise ValueError("expected %d actions, got %d" % (self.num_envs, len(actions)))
        obs, rew, dones, meta = self.vector_step_batched(_stack(actions, self.env.device))
        n = self.num_envs
        return ([_row(obs, i, self.num_envs) for i in range(n)], [_row(rew, i, self.num_envs) for i in range(n)],
                [dict(dones) for _ in range(n)], [_row(meta, i, self.num_envs) for i in range(n)])

    def get_sub_environments(self):
        """The engine holds the N copies as one batch, not N objects."""
        return [self.env]

    # ---------------------------------------------------------------- BaseEnv
    def poll(self):
        """(obs, rewards, dones, infos, off_policy_actions), each {env_id: {agent: ...}}:
        after a reset the fresh observations (no rewards yet), after
        send_actions the step's results."""
        if self._pending is None:
            if self._obs is None:
                self._reset_batch()
            self._pending = (self._obs, None, None, None)
        obs, rew, dones, meta = self._pending
        self._pending = ({}, None, None, None)
        ids = range(self.num_envs)
        if not obs:
            return {}, {}, {}, {}, {}
        o = {i: _row(obs, i, self.num_envs) for i in ids}
        r = {i: _row(rew, i, self.num_envs) for i in ids} if rew is not None else {i: {} for i in ids}
        d = {i: dict(dones) for i in ids} if dones is not None else {i: {"__all__": False} for i in ids}
        info = {i: _row(meta, i, self.num_envs) for i in ids} if meta is not None else {i: {} for i in ids}
        return o, r, d, info, {}

    def send_actions(self, action_dict: Dict[int, Dict[str, Any]]):
        missing = set(range(self.num_envs)) - set(action_dict)
        if missing:
            raise ValueError("lockstep batch: actions needed for every sub-env (missing %d)" % len(missing))
        self._pending = self.vector_step_batched(
            _stack([action_dict[i] for i in range(self.num_envs)], self.env.device))

    def try_reset(self, env_id=None):
        """{env_id: obs} of the fresh episode (the whole batch resets once)."""
        i = 0 if env_id is None else int(env_id)
        return {i: self.reset_at(i)}
