"""Captured steps: a hipGraph of an env's step launch(es), replayed per step
("hipGraph-captured step"; pgw_graph_* in include/pgw.h).

The fused MultiComponentEnv step (pgw_mc_agent_step) has per-step arguments
(the building's exogenous rows, the PV's profile value, the EV schedule).  By
default it is captured once per episode position, on first use, each graph's
launches holding that position's values as the eager step writes them (the
unclocked kernel; one graph per position and action buffer set).  With
clocked=True one graph serves every position, through device clocks: those
values are written once per env into a device table of pgw_mc_step_dyn
records, one per episode step, and each block of the kernel reads record
k = its clock and advances the clock (a ~1.3 us dependent prologue in the
kernel).  The host sets the clocks to the episode step before a call when they
may not hold it (after a reset or eager steps: the eager step does not touch
them).  The actions are read from the tensors given at capture: the caller writes each
step's actions into them (a policy's static output buffers), then calls the
graph.  EnergyStorageEnv's step has no per-step values at all.

On this runtime a graph launch costs about twice an eager launch of host time
(DESIGN.md section 7), so graphs of several steps are the ones that pay.

A graph of `steps` > 1 launches runs that many steps per call (one action
buffer set per step; obs / reward are those of the last step) -- open-loop
rollouts, where one graph launch replaces `steps` kernel launches.

Host state (the components' clocks, the EV's schedule cache, `done`) advances
in the call exactly as the eager step advances it, so captured and eager steps
can be mixed freely; the results are bit-identical to the eager step's
(tests/test_gpu_graph.py).
"""
import atexit
import ctypes as C
import weakref

import torch

from powergridworld_amd import _lib

_LIVE = weakref.WeakSet()       # executable graphs still alive


@atexit.register
def _destroy_all():
    """Destroy the graphs still alive at exit while the HIP runtime is (its
    teardown runs after the interpreter's; a graph freed then would call
    into a runtime that is gone)."""
    for g in list(_LIVE):
        g._release()


class _Graph:
    """An executable hipGraph of the library's launches (pgw_graph_*): launch()
    issues it on torch's current stream."""

    def __init__(self, device, launch):
        h = _lib.lib()
        torch.cuda.synchronize(device)
        side = torch.cuda.Stream(device)           # (capture needs a created stream)
        ex = C.c_void_p()
        with torch.cuda.device(device), torch.cuda.stream(side):
            st = _lib.stream_ptr(device)
            _lib.check(h.pgw_graph_begin(st))
            try:
                launch()
            finally:
                rc = h.pgw_graph_end(st, C.byref(ex))
            _lib.check(rc)
        torch.cuda.synchronize(device)
        self._exec, self._device, self._launch = ex, device, h.pgw_graph_launch
        self._destroy = h.pgw_graph_destroy
        _LIVE.add(self)

    def launch(self, stream):
        if not self._exec:
            raise RuntimeError("capture_step: the graph was released")
        rc = self._launch(self._exec, stream)
        if rc:
            _lib.check(rc)

    def _release(self):
        if getattr(self, "_exec", None):
            self._destroy(self._exec)
            self._exec = None

    def __del__(self):
        self._release()


def _capture(device, launch):
    return _Graph(device, launch)


def _in_place(env, action, dim):
    """pgw_mat of an action tensor the kernel reads in place (a graph keeps the
    pointer: a converted copy would be a dead temporary)."""
    if not isinstance(action, torch.Tensor) or action.device != torch.device(env.device):
        raise ValueError("capture_step: actions must be device tensors on %s" % (env.device,))
    a, m = env._action_mat(action, dim)
    if a.data_ptr() != action.data_ptr():
        raise ValueError("capture_step: an action must be a float64 [N, %d] tensor the kernel can read "
                         "in place (got %s %s)" % (dim, tuple(action.shape), action.dtype))
    return m


class StepGraph:
    """Call it to run the captured step(s) on torch's current stream; returns
    what env.step returns."""

    def __init__(self, env, action, steps, kwargs, clocked=False):
        from powergridworld_amd.base import MultiComponentEnv
        from powergridworld_amd.base_hs import HSMultiComponentEnv
        from powergridworld_amd.agents.energy_storage import EnergyStorageEnv
        steps = int(steps)
        if steps < 1:
            raise ValueError("capture_step: steps >= 1")
        actions = list(action) if isinstance(action, (list, tuple)) else [action] * steps
        if len(actions) != steps:
            raise ValueError("capture_step: %d action sets for %d steps" % (len(actions), steps))
        self.env, self.steps, self._keep = env, steps, (actions, kwargs)
        if isinstance(env, HSMultiComponentEnv):
            if clocked:
                raise NotImplementedError("capture_step: the Home-Steward house is captured per position")
            self._init_hs(env, actions, kwargs)
        elif isinstance(env, MultiComponentEnv):
            self._init_mc(env, actions, kwargs, bool(clocked))
        elif type(env) is EnergyStorageEnv and env.dtype == torch.float64:
            self._init_battery(env, actions)
        else:
            raise NotImplementedError("capture_step: MultiComponentEnv (fused) and EnergyStorageEnv (fp64)")

    # ------------------------------------------------------------ battery
    def _init_battery(self, env, actions):
        if kwargs_given(self._keep[1]):
            raise ValueError("capture_step: EnergyStorageEnv takes no observation inputs")
        fn = _lib.lib().pgw_battery_step
        self._parts, self._bufv = [env], [env._bufv]
        mats = [_in_place(env, a, 1) for a in actions]
        fixed = (C.c_void_p(env.soc.data_ptr()), env._mat(env._obs), C.c_void_p(env._real_power.data_ptr()))

        def launch():
            st = env._stream()
            for m in mats:
                _lib.check(fn(env.params, env.num_envs, m, *fixed, st))
        self.graph = _capture(env.device, launch)
        self._finish = self._finish_battery

    def _finish_battery(self):
        env = self.env
        done = False
        for _ in range(self.steps):
            env.simulation_step += 1
            done = done or env.is_terminal()
        return env._obs, env._zero_reward, done, {"state_of_charge": env.soc.unsqueeze(1)}

    # ------------------------------------------------------------ HS house
    def _init_hs(self, env, actions, kwargs):
        """pgw_hs_step captured per episode position: the house's per-step
        values (PV / device rows, grid cost, EV times and window) come from
        _info_at(k), as the eager step builds them at k."""
        if kwargs_given(kwargs):
            raise ValueError("capture_step: the house's observation inputs are bound at its first step")
        if env.params.pv_grid_aware and env._mv_state is None:
            raise NotImplementedError("capture_step: a grid-aware house PV binds its min_voltage at the "
                                      "first step: step once, then capture")
        k0 = env._hs_step_k()
        for k, e in env._by_kind.items():
            kc = e.index if k in (0, 3) else (e.time_index - 1 if k == 2 else None)
            if kc is not None and kc != k0:
                raise RuntimeError("capture_step: component %s is at step %s, the house at %d" % (e.name, kc, k0))
        n = env.num_envs
        sets = []
        for a in actions:
            if not isinstance(a, torch.Tensor) or tuple(a.shape) != (n, len(env.envs)) or \
                    a.dtype != torch.float64 or a.device != torch.device(env.device):
                raise ValueError("capture_step: house actions must be packed [%d, %d] float64 tensors on %s"
                                 % (n, len(env.envs), env.device))
            b = type(env._bufs).from_buffer_copy(env._bufs)
            b.action = _lib.Mat(a.data_ptr(), a.stride(0), a.stride(1))
            if env.params.pv_grid_aware:
                b.min_voltage = env._mv_state.data_ptr()
            sets.append(b)
        self._hs_sets, self._n_dyn, self._clocked = sets, env._hs_steps(), False
        self._parts, self._bufv = [env], [env._bufv]
        self._pos_graphs = {}
        self._finish = self._finish_hs

    def _hs_graph_at(self, k):
        g = self._pos_graphs.get(k)
        if g is None:
            env = self.env
            infos = [env._info_at(k + i) for i in range(self.steps)]
            fn = _lib.lib().pgw_hs_step

            def launch():
                st = env._stream()
                for info, b in zip(infos, self._hs_sets):
                    _lib.check(fn(env.params, info, env.num_envs, b, st))
            g = self._pos_graphs[k] = _capture(env.device, launch)
        return g

    def _finish_hs(self):
        env = self.env
        done = False
        for _ in range(self.steps):
            _, ev_next = env._pre_step()
            obs, rew, d, meta = env._post_step(ev_next)
            done = done or d
        return obs, rew, done, meta

    # ------------------------------------------------------------ MC
    def _init_mc(self, env, actions, kwargs, clocked):
        if not env._mc_fusable():
            raise NotImplementedError("capture_step: the agent's components are not all fused kinds "
                                      "(pgw_mc_agent_step)")
        env._mc_clock()
        k0 = env.__dict__.setdefault("_ep_step", 0)
        for e in env.envs:
            k = e._mc_dyn_k()
            if k is not None and k != k0:
                raise RuntimeError("capture_step: component %s is at episode step %s, the agent at %d "
                                   "(step the agent, not its components)" % (e.name, k, k0))
        self._dyn, self._n_dyn, self._recs = _dyn_table(env)
        # the graph holds the buffers' pointers: a re-pointed buffer (a fused
        # multi-agent env adopting the component) makes it stale
        self._parts = env.envs
        self._bufv = [e._bufv for e in env.envs]
        kws = [{k: v for k, v in kwargs.items() if k in e.obs_labels} for e in env.envs]
        self._kws = kws
        arg_sets = []
        f32 = env.dtype == torch.float32
        for act in actions:
            a = (_lib.MCStepArgsF32 if f32 else _lib.MCStepArgs)()
            a.n_comp = len(env.envs)
            for c, e in enumerate(env.envs):
                e._mc_static(a, c)
                a.comp[c].action = _in_place(e, act[e.name], e.action_space.shape[0])
                if e.mc_kind == 0 and kws[c]:
                    a.bld_ext, keep = e._ext(kws[c])
                    self._keep += (keep,)
                if e.mc_kind == 1 and e.grid_aware:
                    v = e._min_voltage(kws[c])
                    self._keep += (v,)
                    a.pv_min_voltage = v.data_ptr()
            a.real_power, a.reward = env._real_power.data_ptr(), env._reward.data_ptr()
            if clocked:
                a.clock, a.dyn, a.n_dyn = env._clock.data_ptr(), self._dyn.data_ptr(), self._n_dyn
            arg_sets.append(a)
        self._args, self._clocked = arg_sets, clocked
        self._finish = self._finish_mc
        if clocked:
            self.graph = self._capture_mc(arg_sets)
        else:
            # one graph per episode position k (captured on first use), its
            # launches' arguments holding the step values of k .. k + steps - 1
            # as the eager step writes them: the unclocked kernel, no clock
            self._pos_graphs = {}

    def _capture_mc(self, arg_sets):
        env = self.env
        fn = _lib.lib().pgw_mc_agent_step_f32 if env.dtype == torch.float32 else _lib.lib().pgw_mc_agent_step
        n = env.num_envs

        def launch():
            st = env._stream()
            for a in arg_sets:
                _lib.check(fn(a, n, st))
        return _capture(env.device, launch)

    def _graph_at(self, k):
        g = self._pos_graphs.get(k)
        if g is None:
            sets = []
            for i, a in enumerate(self._args):
                b = type(a).from_buffer_copy(a)
                r = self._recs[k + i]
                b.bld_ex_t, b.bld_ex_next, b.pv_pmax, b.ev_step = r.bld_ex_t, r.bld_ex_next, r.pv_pmax, r.ev_step
                sets.append(b)
            g = self._pos_graphs[k] = self._capture_mc(sets)
        return g

    def _finish_mc(self):
        env = self.env
        dones = []                      # (any step of the call reaching the end)
        for _ in range(self.steps):
            obs, metas = {}, {}
            for e in env.envs:
                e._mc_replayed()
            env._ep_step += 1
            for e, kw in zip(env.envs, self._kws):
                ob, _, done, meta = e._mc_finish(kw)
                obs[e.name] = ob
                dones.append(done)
                metas[e.name] = meta
        return obs, env._reward, any(dones), metas

    def __call__(self):
        env = self.env
        if [e._bufv for e in self._parts] != self._bufv:
            raise RuntimeError("capture_step: the env's buffers moved since the capture (capture again)")
        if hasattr(self, "_hs_sets"):
            k = env._hs_step_k()
            if k + self.steps > self._n_dyn:
                raise IndexError("capture_step: house step %d + %d is past its %d steps of data (reset the env)"
                                 % (k, self.steps, self._n_dyn))
            self._hs_graph_at(k).launch(env._stream())
            return self._finish()
        if hasattr(self, "_n_dyn"):
            k = env._ep_step
            if k + self.steps > self._n_dyn:
                raise IndexError("capture_step: episode step %d + %d is past the %d steps of the episode "
                                 "tables (reset the env)" % (k, self.steps, self._n_dyn))
            if not self._clocked:
                self._graph_at(k).launch(env._stream())
                return self._finish()
            if env._clock_k != k:          # (after a reset or eager steps: set the device clocks)
                env._clock.fill_(k)
            env._clock_k = k + self.steps
        self.graph.launch(env._stream())
        return self._finish()


class CoordStepGraph:
    """Captured steps of the fused multi-agent step (MultiAgentEnv fused path,
    pgw_coord_step / _f32 / _general): `steps` consecutive steps per graph,
    captured once per episode position (and step parity of the fused step's
    list counters) on first use, each step's launches holding that step's
    constants as the eager step builds them (_step_entry: exogenous rows, PV
    value, the hour's PF parameters and tables).  The actions are read from the
    packed [n_agents, N, act_dim] tensors bound at capture: `action` is one
    tensor (every step of every call), a list of `steps`, or a callable k ->
    list of `steps` tensors for the graph at episode position k.  Host state
    (clocks, time, done, the list parity) advances in the call exactly as
    `steps` eager steps advance it, so captured and eager steps mix freely; the
    steps of one call must lie inside the episode (IndexError before any launch
    otherwise).  No history ring (record_history=False)."""

    def __init__(self, env, action, steps):
        steps = int(steps)
        if steps < 1:
            raise ValueError("capture_step: steps >= 1")
        F = env._fused
        if F is None:
            raise NotImplementedError("capture_step: the fused multi-agent step only (fused=True)")
        if env._hist is not None:
            raise NotImplementedError("capture_step: record_history=True writes per-step ring slots")
        self.env, self.steps, self._pos = env, steps, {}
        if callable(action):
            self._bind = action
        else:
            acts = list(action) if isinstance(action, (list, tuple)) else [action] * steps
            if len(acts) != steps:
                raise ValueError("capture_step: %d action sets for %d steps" % (len(acts), steps))
            self._bind = lambda k: acts

    def _step_bufs(self, act, parity):
        env = self.env
        F = env._fused
        na, n = len(env.agents), env.num_envs
        if not isinstance(act, torch.Tensor) or tuple(act.shape) != (na, n, F["act_dim"]) or \
                act.dtype != env.dtype or act.device != torch.device(env.device):
            raise ValueError("capture_step: packed actions must be [%d, %d, %d] %s tensors on %s"
                             % (na, n, F["act_dim"], env.dtype, env.device))
        b = type(F["bufs"]).from_buffer_copy(F["bufs"])
        b.action = F["Mat"](act.data_ptr(), act.stride(1), act.stride(2))
        b.act_stride_agent = act.stride(0)
        if F.get("od_on"):
            b.od_parity = parity
        return b

    def _graph_at(self, k, parity):
        env = self.env
        F, solver = env._fused, env.pf_solver
        key = (k, parity, solver.tables_version, F.get("od_on"))
        g = self._pos.get(key)
        if g is not None:
            return g[0]
        acts = list(self._bind(k))
        if len(acts) != self.steps:
            raise ValueError("capture_step: %d action sets for %d steps" % (len(acts), self.steps))
        bld, pv = F["bld0"], F["pv0"]
        t0 = bld.time_index if bld is not None else None
        p0 = pv.index if pv is not None else None
        launches = []
        for i in range(self.steps):
            skey = (t0 + i if bld is not None else -1, p0 + i if pv is not None else -1,
                    env._time_at(env.episode_step + 1 + i), solver.tables_version)
            ent = F["step_cache"].get(skey) or env._step_entry(skey)
            if solver.tables_version != key[2]:
                raise RuntimeError("capture_step: the power-flow tables changed while capturing")
            launches.append((ent, self._step_bufs(acts[i], (parity + 1 + i) & 1)))
        fn = getattr(_lib.lib(), F["kernel"])
        n = env.num_envs

        def launch():
            st = _lib.stream_ptr(env.device)
            for (info, pfp, pft, _), b in launches:
                _lib.check(fn(F["params"], pfp, pft, info, n, b, st))
        g = _capture(env.device, launch)
        self._pos[key] = (g, launches, acts)          # (the launches' structs live as long as the graph)
        return g

    def release(self):
        """Destroy the captured graphs now (a graph's destruction can wait for the
        device: do it here, not inside someone's timed region at garbage
        collection)."""
        for g in self._pos.values():
            g[0]._release()
        self._pos.clear()

    def __call__(self):
        env = self.env
        F = env._fused
        k = env.episode_step
        last = env._episode_last_step()
        if last is not None and k + self.steps > last:
            raise IndexError("capture_step: steps %d..%d run past the episode's last step %d (step eagerly "
                             "or reset)" % (k + 1, k + self.steps, last))
        parity = F["bufs"].od_parity if F.get("od_on") else 0
        self._graph_at(k, parity).launch(_lib.stream_ptr(env.device))
        for _ in range(self.steps):
            out = env._advance_fused()
        return out


def kwargs_given(kwargs):
    return any(v is not None for v in kwargs.values())


def _dyn_table(env):
    """(device uint8 tensor of pgw_mc_step_dyn[L], L, the host records): the
    agent's shared per-step values for episode steps 0 .. L-1, built on the
    host once per env from the same component code the eager step uses."""
    c = env.__dict__.get("_dyn_cache")
    if c is not None:
        return c
    lens = [n for n in (e._mc_dyn_len() for e in env.envs) if n is not None]
    L = max(1, min(lens)) if lens else 1
    recs = (_lib.MCStepDyn * L)()
    for k in range(L):
        for e in env.envs:
            e._mc_dyn(recs[k], k)
    buf = torch.frombuffer(bytearray(recs), dtype=torch.uint8).to(env.device)
    env._dyn_cache = (buf, L, recs)
    return env._dyn_cache
