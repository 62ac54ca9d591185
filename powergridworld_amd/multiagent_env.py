"""Batched MultiAgentEnv (reference: gridworld/multiagent_env.py:20-230).

Two execution paths behind the reference API:

* generic: each agent steps through its own component kernels, bus loads are
  summed on the device, the batched power flow runs (pgw_pf_solve), then the
  Python hooks ``get_external_obs_vars`` / ``reward_transform`` /
  ``meta_transform`` run on [N] tensors -- any agent mix, any override;
* fused (the BASELINE C4 hot path): when every agent is a MultiComponentEnv of
  {FiveZoneROMThermalEnergyEnv, PVEnv, EnergyStorageEnv} with identical
  configs, no agent observes grid voltages and the reward transform is the
  base pass-through or CoordinatedMultiBuildingControlEnv's, the whole
  MultiAgentEnv.step -- all agents, the power flow and the voltage-violation
  reward -- is ONE kernel launch (pgw_coord_step).  Component envs keep
  their state as views of the fused buffers, so resets and queries still go
  through them.
"""
from abc import abstractmethod
from collections.abc import Mapping
from typing import Dict, Tuple, Union

import ctypes as C
import numpy as np
import pandas as pd
import torch

from powergridworld_amd import _lib
from powergridworld_amd.base import (ComponentEnv, MultiComponentEnv, as_action, oob_poll, owns_fused_hooks,
                                     resolve_env_class)
from powergridworld_amd.log import logger

try:
    from ray.rllib.env.multi_agent_env import MultiAgentEnv as Env      # multiagent_env.py:13-17
except ImportError:
    Env = object
    logger.warning("rllib MultiAgentEnv not found, using generic object class")

_KIND_ID = {"building": 0, "pv": 1, "storage": 2}


def resolve_pf_class(cls):
    from powergridworld_amd.distribution_system.opendss import OpenDSSSolver
    from powergridworld_amd.distribution_system.powerflow import PowerFlowSolver
    if isinstance(cls, type) and issubclass(cls, PowerFlowSolver):
        return cls
    if getattr(cls, "__name__", None) == "OpenDSSSolver":
        return OpenDSSSolver
    raise TypeError("unsupported power flow solver class %r" % (cls,))


class MultiAgentEnv(Env):

    # Subclasses that implement a reward transform the fused kernel knows set this.
    fused_reward_transform = None

    def __init__(self, common_config: dict = {}, pf_config: dict = {}, agents: list = None,
                 max_episode_steps: int = None, rescale_spaces: bool = True, num_envs: int = 1,
                 device=None, fused: Union[bool, str] = "auto", record_history: bool = False,
                 dtype=None, history_capacity: int = None, **kwargs):
        self.common_config = common_config
        self.rescale_spaces = rescale_spaces
        assert len(agents) > 0, "need at least one agent!"
        self.num_envs = int(num_envs)
        self.device = _lib.require_device(device)
        # storage dtype of the per-env buffers: fp64 (the reference's), or fp32 on
        # the fused path (pgw_coord_step_f32: fp32 storage, fp64 arithmetic)
        self.dtype = _lib.storage_dtype(dtype)
        if self.dtype != torch.float64 and fused is False:
            raise ValueError("dtype=%s needs the fused path" % self.dtype)
        self.start_time = pd.Timestamp(common_config["start_time"])
        self.end_time = pd.Timestamp(common_config["end_time"])
        self.control_timedelta = common_config["control_timedelta"]
        self.pf_config = pf_config
        self.max_episode_steps = max_episode_steps if max_episode_steps is not None else np.inf
        self.episode_step = None
        self.time = None
        self.history = None
        self.voltages = None
        self.obs_dict = {}
        self.record_history = record_history
        self._times, self._end_step = [], 10 ** 12
        self._time_at(0)

        self.agents = []
        for a in agents:
            _config = a["config"]
            if "name" in a["config"]:
                _config = {k: v for k, v in _config.items() if k != "name"}
                logger.warning("ignoring 'name' in config dict in favor of constructor argument")
            cls = resolve_env_class(a["cls"])
            new_agent = cls(name=a["name"], num_envs=self.num_envs, device=self.device,
                            **_config, **self.common_config)
            self.agents.append(new_agent)
        # one out-of-bounds action counter for every component of every agent
        self.oob_count = torch.zeros(1, dtype=torch.int64, device=self.device)
        for agent in self.agents:
            agent._bind_oob(self.oob_count)
        self.agent_name_bus_map = {a["name"]: a["bus"] for a in agents}
        self.agent_names = list(set([a.name for a in self.agents]))
        assert len(self.agent_names) == len(agents), "all agents need unique names"

        pf_cls = resolve_pf_class(pf_config["cls"])
        self.pf_solver = pf_cls(**pf_config["config"], num_envs=self.num_envs, device=self.device)

        self.observation_space = {agent.name: agent.observation_space for agent in self.agents}
        self.action_space = {agent.name: agent.action_space for agent in self.agents}

        self._fused = None
        self._ma = None              # fused multi-agent path (pgw_ma_step), see _setup_ma
        self._fused_steps = 0
        self._at_reset = False       # the last call was reset() (env.voltages: the reset solve)
        # every agent reports the base class's reactive power (its zero buffer)
        self._q_zero = all(type(a).reactive_power is ComponentEnv.reactive_power for a in self.agents)
        if fused:
            why = self._fusable()
            if why is None and self.dtype != torch.float64:
                why = self._f32_fusable()
                if why is not None:
                    raise ValueError("dtype=%s: %s" % (self.dtype, why))
            if why is None:
                self._setup_fused()
            else:
                why_ma = self._ma_fusable() if self.dtype == torch.float64 else "fp32 storage"
                if why_ma is None:
                    self._setup_ma()
                elif fused is True:
                    raise ValueError("fused=True but this configuration cannot be fused: %s; "
                                     "multi-agent step: %s" % (why, why_ma))
                else:
                    logger.info("MultiAgentEnv: generic path (%s; %s)", why, why_ma)
        if self._fused is None:
            buses = sorted(set(self.agent_name_bus_map.values()))
            self.pf_solver.set_controllable_loads(buses)
        self._hist = None
        if self.record_history:
            self._init_history(history_capacity)

    # ================================================================ hooks
    @abstractmethod
    def get_external_obs_vars(self, agent: Union[ComponentEnv, MultiComponentEnv]) -> dict:
        """multiagent_env.py:90-115: bus_voltage / max_voltage / min_voltage from the
        PREVIOUS power flow, only when the agent lists them in obs_labels."""
        kwargs = {}
        if "bus_voltage" in agent.obs_labels:
            kwargs["bus_voltage"] = self.pf_solver.get_bus_voltage_by_name(
                self.agent_name_bus_map[agent.name])
        if "max_voltage" in agent.obs_labels or "min_voltage" in agent.obs_labels:
            solver = self.pf_solver
            if self.voltages is getattr(solver, "bus_voltages", None) and hasattr(solver, "voltage_extrema"):
                vmin, vmax = solver.voltage_extrema()          # one reduction per solve
            else:
                stacked = torch.stack(list(self.voltages.values()))
                vmin, vmax = stacked.min(0).values, stacked.max(0).values
            if "max_voltage" in agent.obs_labels:
                kwargs["max_voltage"] = vmax
            if "min_voltage" in agent.obs_labels:
                kwargs["min_voltage"] = vmin
        return kwargs

    def reward_transform(self, rew_dict) -> dict:
        """Pass-through by default (multiagent_env.py:215-218)."""
        return rew_dict

    def meta_transform(self, meta) -> dict:
        """Pass-through by default (multiagent_env.py:221-225)."""
        return meta

    # ================================================================ API
    def _time_at(self, step):
        """start_time + step * control_timedelta (cached: pandas arithmetic is slow)."""
        times = self._times
        if step >= len(times):
            n = max(2 * len(times), step + 1, 512)
            self._times = times = [self.start_time + i * self.control_timedelta for i in range(n)]
            # first step whose time is >= end_time (multiagent_env.py:201)
            self._end_step = next((i for i, t in enumerate(times) if t >= self.end_time), n + 10 ** 9)
        return times[step]

    def reset(self) -> Dict[str, any]:
        """multiagent_env.py:125-140"""
        self.episode_step = 0
        self._resets = self.__dict__.get("_resets", 0) + 1
        oob_poll(self.oob_count)
        self.time = self._time_at(0)
        self.history = {"timestamp": [], "voltage": [], "agent_power_p": []}
        if self._hist is not None:
            self._hist["t"] = 0
            self.pf_solver.bind_output(None)     # the reset solve is not recorded
            if self._fused is not None:          # agents' real power back off the ring
                for ai, agent in enumerate(self.agents):
                    agent._real_power = self._fused["agent_power"][ai]
        self.pf_solver.calculate_power_flow(current_time=self.time)
        self._at_reset = True
        self.voltages = self.pf_solver.get_bus_voltages()
        if self._fused is not None and len(self.pf_solver.output_names) < self.pf_solver.feeder.n:
            # the reset solve's rows, every other node solved on first access
            self.voltages = self.pf_solver.bus_voltages = _FusedVoltages(
                self, self.pf_solver.bus_voltages, self._fused_steps, reset=True)
        f32 = self._fused is not None and self.dtype != torch.float64
        if f32:
            self._f32_sync(up=True)
        for agent in self.agents:
            kwargs = self.get_external_obs_vars(agent)
            _ = agent.reset(**kwargs)
        if self._fused is not None:
            self._prewarm_steps()
        if f32:
            self._f32_sync(up=False)
            return self._fused["obs_dict"]
        return self.get_obs()

    def oob_actions(self) -> torch.Tensor:
        """Out-of-bounds actions clipped so far over every agent's components (the
        warnings utils.py:35-37 would have logged; also meta["oob_actions"]).  A
        [1] int64 device tensor: reading its value synchronizes."""
        return self.oob_count

    def get_obs(self) -> Dict[str, any]:
        obs = {}
        for agent in self.agents:
            kwargs = self.get_external_obs_vars(agent)
            obs[agent.name], _ = agent.get_obs(**kwargs)
        return obs

    def step(self, action) -> Tuple[dict, dict, dict, dict]:
        """multiagent_env.py:151-212.  ``action`` is the reference's
        {agent: {component: [N, d]}} dict, or -- fused path -- one packed tensor
        [n_agents, N, act_dim] (any strides; zero-copy)."""
        self.episode_step += 1
        self.time = self._time_at(self.episode_step)
        self._at_reset = False
        self.obs_dict = {}
        if self._fused is not None:
            obs, rew, done, meta = self._step_fused(action)
        elif self._ma is not None:
            obs, rew, done, meta = self._step_ma(action)
        else:
            obs, rew, done, meta = self._step_generic(action)
        any_done = any(done.values())
        max_steps_reached = (self.episode_step == self.max_episode_steps - 1)
        time_up = self.episode_step >= self._end_step
        d = bool(any_done or max_steps_reached or time_up)
        dones = {a.name: d for a in self.agents}
        dones["__all__"] = d
        return obs, rew, dones, meta

    def _step_generic(self, action):
        obs, rew, done, meta = {}, {}, {}, {}
        load_p, load_q = {}, {}
        agent_power_p = []
        for agent in self.agents:
            name = agent.name
            kwargs = self.get_external_obs_vars(agent)
            # (a view of the agent's reward buffer, like the observations: the next
            # step overwrites it; reward_transform hooks build new tensors)
            obs[name], rew[name], done[name], meta[name] = agent.step(action=action[name], **kwargs)
            agent_power_p.append(agent.real_power)
        if self._hist is not None:                     # this step's history slot
            self.pf_solver.bind_output(self._hist["v"][self._hist["t"] % self._hist["cap"]])
        # No agent class here sets a reactive power (every component's stays the
        # zero buffer), so the q sums would add zeros: the solve takes q = 0.
        q_zero = self._q_zero
        if q_zero:
            load_p = self._bus_loads()
        else:
            for agent in self.agents:
                load_bus = self.agent_name_bus_map[agent.name]
                p = agent.real_power
                if load_bus in load_p:
                    load_p[load_bus] = load_p[load_bus] + p
                    load_q[load_bus] = load_q[load_bus] + agent.reactive_power
                else:
                    load_p[load_bus] = p
                    load_q[load_bus] = agent.reactive_power
        self.pf_solver.calculate_power_flow(current_time=self.time, p_controllable_consumed=load_p,
                                            q_controllable_consumed=None if q_zero else load_q)
        self.voltages = self.pf_solver.get_bus_voltages()
        self._record(agent_power_p)
        rew = self.reward_transform(rew)
        meta = self.meta_transform(meta)
        meta["oob_actions"] = self.oob_count
        return obs, rew, done, meta

    def _bus_loads(self):
        """{bus: [N] real power}: the agents' powers summed per bus in agent order
        (multiagent_env.py:171-181).  A bus with one agent takes its tensor as
        is; several agents go through one pgw_agent_reduce launch (0 + p0 + p1
        + ..., the reference's left-to-right sum) into a per-bus buffer, where
        the reference's `+` made a new tensor per agent."""
        key = tuple(a.real_power.data_ptr() for a in self.agents)
        c = self.__dict__.get("_bus_c")
        if c is None or c[0] != key:
            groups = {}
            for agent in self.agents:
                groups.setdefault(self.agent_name_bus_map[agent.name], []).append(agent.real_power)
            plan = []
            for bus, ps in groups.items():
                if len(ps) == 1 or len(ps) > _lib.MAX_COMP:
                    plan.append((bus, ps, None, None))
                    continue
                ra = _lib.ReduceArgs()
                ra.n_comp = len(ps)
                for i, p in enumerate(ps):
                    ra.real_power[i] = p.data_ptr()
                    ra.reward[i] = None
                out = torch.empty(self.num_envs, dtype=torch.float64, device=self.device)
                plan.append((bus, ps, ra, out))
            c = self._bus_c = (key, plan)
        load_p = {}
        lib, st = _lib.lib(), _lib.stream_ptr(self.device)
        for bus, ps, ra, out in c[1]:
            if ra is not None:
                _lib.check(lib.pgw_agent_reduce(ra, self.num_envs, out.data_ptr(), None, st))
                load_p[bus] = out
            else:
                acc = ps[0]
                for p in ps[1:]:
                    acc = acc + p
                load_p[bus] = acc
        return load_p

    def _init_history(self, capacity):
        """On-device voltage / agent-power history: a ring of
        `capacity` step slots, [cap, n_nodes, N] voltages and [cap, n_agents, N]
        agent powers, in place of the reference's per-step dict copies
        (multiagent_env.py:129, 191-194).  On the fused path the kernels write
        each step's outputs straight into its slot (no copy); the history lists
        hold views of the slots, valid until the ring wraps (clone to keep)."""
        if capacity is None:
            capacity = int(min(self.max_episode_steps, self._end_step, 4096)) + 1
        cap, n = int(capacity), self.num_envs
        if cap < 1:
            raise ValueError("history_capacity must be >= 1")
        solver = self.pf_solver
        rows = {name: i for i, name in enumerate(solver.output_names)}
        names = [x for x in solver.feeder.node_names if x in rows]
        dt = self.dtype if self._fused is not None else torch.float64
        H = {"cap": cap, "t": 0,
             "v": torch.zeros((cap, len(solver.output_names), n), dtype=dt, device=self.device),
             "p": torch.zeros((cap, len(self.agents), n), dtype=dt, device=self.device)}
        # per-slot views, built once: {node: [N]} in the reference's node order
        H["vd"] = [{x: H["v"][s_, rows[x]] for x in names} for s_ in range(cap)]
        H["pl"] = [[H["p"][s_, a] for a in range(len(self.agents))] for s_ in range(cap)]
        self._hist = H

    def voltage_history(self):
        """(voltages [T, n_nodes, N], agent powers [T, n_agents, N], node names) of
        the steps recorded this episode (the last `history_capacity` if more), as
        views of the device ring in step order when it has not wrapped."""
        H = self._hist
        if H is None:
            raise RuntimeError("record_history=False")
        t, cap = H["t"], H["cap"]
        order = list(range(t)) if t <= cap else [(t + i) % cap for i in range(cap)]
        idx = torch.tensor(order, dtype=torch.long, device=self.device)
        v, p = (H["v"][:t], H["p"][:t]) if t <= cap else (H["v"][idx], H["p"][idx])
        rows = {name: i for i, name in enumerate(self.pf_solver.output_names)}
        names = list(H["vd"][0].keys())
        perm = [rows[x] for x in names]
        if perm != list(range(len(perm))):
            v = v[:, perm]
        return v, p, names

    def _record(self, agent_power_p):
        H = self._hist
        if H is None:
            return
        s_ = H["t"] % H["cap"]
        if self._fused is None:                # the fused kernels wrote the slot themselves
            torch.stack(agent_power_p, out=H["p"][s_])
        H["t"] += 1
        self.history["timestamp"].append(self.time)
        self.history["voltage"].append(H["vd"][s_])
        self.history["agent_power_p"].append(H["pl"][s_])

    @property
    def agent_dict(self) -> Dict[str, ComponentEnv]:
        return {a.name: a for a in self.agents}

    # ================================================================ fused path
    def _fusable(self):
        from powergridworld_amd.distribution_system.opendss import OpenDSSSolver
        if not isinstance(self.pf_solver, OpenDSSSolver):
            return "power flow solver is not the batched OpenDSSSolver"
        if self.pf_solver.general and self.dtype != torch.float64:
            return "the general power flow (large feeder or convergence='opendss') has no fp32 fused step"
        if getattr(self.pf_solver, "regulators", None) is not None:
            return "RegControl (the control loop runs in OpenDSSSolver.calculate_power_flow)"
        if getattr(self.pf_solver, "snap_start", "direct") != "direct":
            return "snap_start='previous' (each env's solve starts from its own previous solution)"
        if getattr(self.pf_solver, "yprim", "dss_file") != "dss_file":
            return "yprim='step' (every solve's Y holds its own loads' admittances)"
        if len(self.agents) > _lib.MAX_AGENTS:
            return "more than %d agents" % _lib.MAX_AGENTS
        cls = type(self)
        for hook in ("get_external_obs_vars", "step", "reset", "get_obs"):
            if getattr(cls, hook) is not getattr(MultiAgentEnv, hook):
                return "%s is overridden" % hook
        # reward/meta transforms must be the ones the fused kernel implements: the
        # base pass-through, or those of the class that declares fused_reward_transform
        owner = MultiAgentEnv
        for klass in cls.__mro__:
            if klass.__dict__.get("fused_reward_transform") is not None:
                owner = klass
                break
        for hook in ("reward_transform", "meta_transform", "get_voltage_violation"):
            if getattr(cls, hook, None) is not getattr(owner, hook, None):
                return "%s is overridden" % hook
        kinds0 = None
        for a in self.agents:
            if not isinstance(a, MultiComponentEnv) or type(a) is not MultiComponentEnv:
                return "agent %s is not a plain MultiComponentEnv" % a.name
            kinds = [type(e).fused_kind for e in a.envs]
            if any(k is None for k in kinds) or len(set(kinds)) != len(kinds):
                return "agent %s has components the fused kernel does not implement" % a.name
            if not all(owns_fused_hooks(e, "fused_kind") for e in a.envs):
                return "agent %s has a component that overrides a hook the fused kernel restates" % a.name
            if kinds0 is None:
                kinds0 = kinds
            elif kinds != kinds0:
                return "agents differ in components"
            for e in a.envs:
                if any(l in ("bus_voltage", "min_voltage", "max_voltage") for l in e.obs_labels):
                    return "agent %s observes grid voltages" % a.name
                if getattr(e, "grid_aware", False):
                    return "grid-aware PV"
        ref = self.agents[0]
        for a in self.agents[1:]:
            for e0, e1 in zip(ref.envs, a.envs):
                if bytes(e0.params) != bytes(e1.params):
                    return "agents have different component parameters"
                if hasattr(e0, "data") and not np.array_equal(e0.data, e1.data):
                    return "agents have different PV profiles"
                # the fused step feeds every agent agent 0's per-step exogenous
                # row (BuildingExo: T_oa, Q_solar/int/cool, comfort bounds,
                # time_of_day), so the whole tables must agree, not just T_oa
                if hasattr(e0, "_exo") and (
                        len(e0._exo) != len(e1._exo) or e0.df.index[0] != e1.df.index[0] or
                        e0.max_episode_steps != e1.max_episode_steps or
                        any(not np.array_equal(getattr(e0, t), getattr(e1, t))
                            for t in ("_T_oa", "_q_solar", "_q_int", "_q_cool", "_cb"))):
                    return "agents have different exogenous data or comfort bounds"
        if self.fused_reward_transform not in (None, "coordinated"):
            return "unknown fused reward transform"
        if self.fused_reward_transform == "coordinated" and \
                len(set(self.agent_name_bus_map.values())) != 1:
            return "coordinated reward needs all agents on one bus"
        return None

    def _f32_fusable(self):
        """pgw_coord_step_f32 implements the standard C4 agent only."""
        a0 = self.agents[0]
        kinds = [type(e).fused_kind for e in a0.envs]
        if kinds != ["building", "pv", "storage"]:
            return "the fp32 fused step needs agents of [building, pv, storage] in that order"
        if [e.action_space.shape[0] for e in a0.envs] != [6, 1, 1] or \
                [e.observation_space.shape[0] for e in a0.envs] != [15, 1, 1]:
            return "the fp32 fused step needs the default building action / observation layout"
        return None

    def _f32_sync(self, up):
        """fp32 fused path: the component envs keep fp64 state for their reset
        (it runs once per episode); the step state lives in the fp32 buffers.
        up: fp32 -> components (x_k persists across resets, as in the
        reference); down: components -> fp32 after their reset."""
        F = self._fused
        for ai, agent in enumerate(self.agents):
            bld, pv, bat = agent.envs
            if up:
                bld.x.copy_(F["x"][ai])
                bat.soc.copy_(F["soc"][ai])
            else:
                F["x"][ai].copy_(bld.x)
                F["soc"][ai].copy_(bat.soc)
                for i, e in enumerate(agent.envs):
                    o = int(F["obs_off"][i])
                    F["obs"][ai, o:o + F["obs_dims"][i]].copy_(e._obs.t())
                F["reward"][ai].zero_()
                F["agent_power"][ai].zero_()
        if not up:
            F["v_out"][: self.pf_solver.v_out.shape[0]].copy_(self.pf_solver.v_out)
            self.voltages = F["voltages"]
            if len(self.pf_solver.output_names) < self.pf_solver.feeder.n:
                self.voltages = _FusedVoltages(self, F["voltages"], self._fused_steps, reset=True)

    def _full_voltages(self, step_no, reset=False):
        """Every node's voltage for the fused step `step_no` (_FusedVoltages): the
        same snap solve as the kernel's -- the bus loads summed in agent order
        from the step's agent powers, the same predictor first guess -- on a
        second solver that outputs all nodes, so the values are the ones the
        generic path reports (tests/test_gpu_parity.py checks fused == generic).
        With OpenDSSSolver(warm_start=True) the kernel started each env from its
        previous solution, which its own solve has since overwritten: the second
        solver then starts cold (it keeps no history of its own), so these nodes
        equal the kernel's solve to the solver tolerance, not bit for bit."""
        if step_no != self._fused_steps:
            raise RuntimeError("voltages of an earlier step: the fused path solves the other nodes "
                               "on demand from the step's agent powers, which a later step overwrote")
        F, solver = self._fused, self.pf_solver
        full = self.__dict__.get("_pf_full")
        if full is None:
            cfg = dict(self.pf_config["config"], warm_start=False)
            full = self._pf_full = type(solver)(**cfg, num_envs=self.num_envs, device=self.device)
        ctrl = solver._ctrl_names
        full.set_controllable_loads(ctrl)
        if reset:                                   # the reset solve: no controllable load
            full.calculate_power_flow(current_time=self.time)
        elif self._ma is not None:                  # the step's bus loads, as the kernel summed them
            bus_p = self._ma["bus_p"]
            full.calculate_power_flow(p_controllable_consumed={c: bus_p[k] for k, c in enumerate(ctrl)},
                                      current_time=self.time)
        else:
            sums, p = {}, F["params"]
            for ai in range(len(self.agents)):
                s_ = p.agent_ctrl[ai]
                if s_ >= 0:
                    x = F["agent_power"][ai].double()
                    sums[s_] = sums[s_] + x if s_ in sums else x    # 0 + p0 + p1 ... (kernel order)
            full.calculate_power_flow(p_controllable_consumed={ctrl[k]: v for k, v in sums.items()},
                                      current_time=self.time)
        out = full.get_bus_voltages()
        if self.dtype != torch.float64:
            out = {k: v.to(self.dtype) for k, v in out.items()}
        return out

    def load_component_state(self):
        """fp32 fused path: re-read the component envs' state and observations
        into the fp32 step buffers, after a component was reset directly (e.g.
        ``agent.env_dict["storage"].reset(init_storage=...)``).  No-op otherwise."""
        if self._fused is not None and self.dtype != torch.float64:
            self._f32_sync(up=False)
        return self.packed_obs() if self._fused is not None else None

    def _setup_fused(self):
        n, na = self.num_envs, len(self.agents)
        dev = self.device
        dt = self.dtype
        f32 = dt != torch.float64
        a0 = self.agents[0]
        kinds = [type(e).fused_kind for e in a0.envs]
        act_dims = [e.action_space.shape[0] for e in a0.envs]
        obs_dims = [e.observation_space.shape[0] for e in a0.envs]
        act_off = np.concatenate([[0], np.cumsum(act_dims)])[:-1]
        obs_off = np.concatenate([[0], np.cumsum(obs_dims)])[:-1]
        act_dim, obs_dim = int(sum(act_dims)), int(sum(obs_dims))

        buses = [self.agent_name_bus_map[a.name] for a in self.agents]
        ctrl = sorted(set(b for b in buses if b in self.pf_solver.load_bus_name))
        self.pf_solver.set_controllable_loads(ctrl)
        out_nodes = []
        if self.fused_reward_transform == "coordinated":
            out_nodes = [x for x in _bus_nodes(buses[0])]
        for b in sorted(set(buses)):
            for x in _bus_nodes(b):
                if x in self.pf_solver.feeder.node_index and x not in out_nodes:
                    out_nodes.append(x)
        if not out_nodes:
            out_nodes = [self.pf_solver.feeder.node_names[0]]
        if self.record_history:            # the history holds every node (AllBusMagPu)
            out_nodes += [x for x in self.pf_solver.feeder.node_names if x not in out_nodes]
        self.pf_solver.set_output_nodes(out_nodes)
        if self.fused_reward_transform == "coordinated" and len(_bus_nodes(buses[0])) != 1:
            raise ValueError("coordinated reward needs a single-phase common bus (e.g. '675c')")

        p = _lib.CoordParams()
        p.n_agents, p.act_dim, p.obs_dim, p.n_comp = na, act_dim, obs_dim, len(kinds)
        p.act_bld = p.act_pv = p.act_bat = -1
        p.obs_bld = p.obs_pv = p.obs_bat = -1
        for i, (k, e) in enumerate(zip(kinds, a0.envs)):
            p.comp_order[i] = _KIND_ID[k]
            if k == "building":
                p.bld, p.act_bld, p.obs_bld = e.params, int(act_off[i]), int(obs_off[i])
            elif k == "pv":
                p.pv, p.act_pv, p.obs_pv = e.params, int(act_off[i]), int(obs_off[i])
            else:
                p.bat, p.act_bat, p.obs_bat = e.params, int(act_off[i]), int(obs_off[i])
        for i, b in enumerate(buses):
            p.agent_ctrl[i] = ctrl.index(b) if b in ctrl else -1
        p.coordinated = int(self.fused_reward_transform == "coordinated")
        p.vv_row = 0
        p.vv_lo, p.vv_hi = [float(v) for v in getattr(self, "VOLTAGE_LIMITS", [0.95, 1.05])]
        p.vv_penalty = float(getattr(self, "VV_UNIT_PENALTY", 1e4))

        F = dict(params=p, kinds=kinds, act_off=act_off, obs_off=obs_off, act_dims=act_dims,
                 obs_dims=obs_dims, act_dim=act_dim, obs_dim=obs_dim)
        F["obs"] = torch.zeros((na, obs_dim, n), dtype=dt, device=dev)
        F["act"] = torch.zeros((na, act_dim, n), dtype=dt, device=dev)
        F["x"] = torch.zeros((na, 5, n), dtype=dt, device=dev)
        F["soc"] = torch.zeros((na, n), dtype=dt, device=dev)
        F["reward"] = torch.zeros((na, n), dtype=dt, device=dev)
        F["agent_power"] = torch.zeros((na, n), dtype=dt, device=dev)
        F["vv"] = torch.zeros(n, dtype=dt, device=dev)
        F["iters"] = torch.zeros(n, dtype=torch.int32, device=dev)
        # fp32: own voltage rows; fp64: the solver's v_out (its bus_voltages views)
        F["v_out"] = torch.zeros_like(self.pf_solver.v_out, dtype=dt) if f32 else self.pf_solver.v_out
        F["voltages"] = {name: F["v_out"][i] for i, name in enumerate(self.pf_solver.output_names)}
        F["lazy_v"] = _FusedVoltages(self, F["voltages"], 0)     # reused every step
        for ai, agent in enumerate(self.agents):
            if f32:       # the components keep their fp64 buffers (reset only, _f32_sync)
                F["x"][ai].copy_(agent.envs[0].x)
                F["soc"][ai].copy_(agent.envs[2].soc)
                agent._real_power = F["agent_power"][ai]
                agent._reward = F["reward"][ai]
                continue
            for i, (k, e) in enumerate(zip(kinds, agent.envs)):
                view = F["obs"][ai, int(obs_off[i]):int(obs_off[i]) + obs_dims[i]].t()
                if k == "building":
                    e._adopt(x=F["x"][ai], obs=view)
                elif k == "pv":
                    e._adopt(obs=view)
                else:
                    e._adopt(soc=F["soc"][ai], obs=view)
            agent._real_power = F["agent_power"][ai]
            agent._reward = F["reward"][ai]
        # ---- constant per-step launch state and return values (views)
        bufs = _lib.CoordBuffersF32() if f32 else _lib.CoordBuffers()
        F["Mat"] = _lib.Matf if f32 else _lib.Mat
        F["kernel"] = "pgw_coord_step_f32" if f32 else (
            "pgw_coord_step_general" if self.pf_solver.general else "pgw_coord_step")
        obs = F["obs"]
        bufs.obs = F["Mat"](obs.data_ptr(), 1, obs.stride(1))
        bufs.obs_stride_agent = obs.stride(0)
        bufs.x, bufs.soc = F["x"].data_ptr(), F["soc"].data_ptr()
        bufs.reward, bufs.agent_power = F["reward"].data_ptr(), F["agent_power"].data_ptr()
        bufs.v_out = F["v_out"].data_ptr()
        bufs.vv, bufs.iters = F["vv"].data_ptr(), F["iters"].data_ptr()
        F["bufs"], F["act_key"], F["step_cache"] = bufs, None, {}
        comps = [dict(zip(kinds, agent.envs)) for agent in self.agents]
        F["bld0"], F["pv0"] = comps[0].get("building"), comps[0].get("pv")
        F["bld_envs"] = [c["building"] for c in comps if "building" in c]
        F["pv_envs"] = [c["pv"] for c in comps if "pv" in c]
        F["bat_envs"] = [c["storage"] for c in comps if "storage" in c]
        F["agent0_envs"] = list(self.agents[0].envs)
        if f32:
            F["obs_dict"] = {agent.name: {e.name: F["obs"][ai, int(F["obs_off"][i]):int(F["obs_off"][i]) +
                                                   F["obs_dims"][i]].t()
                                          for i, e in enumerate(agent.envs)}
                             for ai, agent in enumerate(self.agents)}
        else:
            F["obs_dict"] = {agent.name: {e.name: e._obs for e in agent.envs} for agent in self.agents}
        F["rew_dict"] = {agent.name: F["reward"][ai] for ai, agent in enumerate(self.agents)}
        F["done_true"] = {agent.name: True for agent in self.agents}
        F["done_false"] = {agent.name: False for agent in self.agents}
        F["meta"] = {agent.name: {} for agent in self.agents}
        if self.fused_reward_transform == "coordinated":
            F["meta"]["voltage_violation"] = F["vv"]
        F["meta"]["oob_actions"] = self.oob_count
        self._fused = F
        if self._one_launch_ok():
            self.set_pf_list(True)

    # ================================================================ fused multi-agent path
    def _ma_fusable(self):
        """pgw_ma_step runs MultiAgentEnv.step for agents that are plain
        MultiComponentEnvs of fusable components or single PV / storage / EV envs
        (the heterogeneous scenario), with the base class's hooks and transforms,
        at most one building / storage / EV and two PV components in all, and no
        agent observing a bus voltage (min / max voltage are the previous solve's
        extrema, which the power flow's epilogue writes)."""
        from powergridworld_amd.distribution_system.opendss import OpenDSSSolver
        if not isinstance(self.pf_solver, OpenDSSSolver):
            return "power flow solver is not the batched OpenDSSSolver"
        if getattr(self.pf_solver, "regulators", None) is not None:
            return "RegControl (the control loop runs in OpenDSSSolver.calculate_power_flow)"
        if getattr(self.pf_solver, "snap_start", "direct") != "direct":
            return "snap_start='previous' (each env's solve starts from its own previous solution)"
        if getattr(self.pf_solver, "yprim", "dss_file") != "dss_file":
            return "yprim='step' (every solve's Y holds its own loads' admittances)"
        if len(self.agents) > _lib.MAX_AGENTS:
            return "more than %d agents" % _lib.MAX_AGENTS
        cls = type(self)
        for hook in ("get_external_obs_vars", "step", "reset", "get_obs", "reward_transform",
                     "meta_transform"):
            if getattr(cls, hook) is not getattr(MultiAgentEnv, hook):
                return "%s is overridden" % hook
        if set(self.pf_solver.output_names) != set(self.pf_solver.feeder.node_names):
            return "the solver does not output every node"
        if not self._q_zero:
            # the kernel's power flow takes no reactive power; the generic path
            # feeds every agent's reactive_power to the solver
            return "an agent overrides reactive_power"
        kinds, slots = [], 0
        for a in self.agents:
            if "bus_voltage" in a.obs_labels:
                return "agent %s observes its bus voltage" % a.name
            if type(a) is MultiComponentEnv:
                if not a._mc_fusable():
                    return "agent %s has components the fused step does not implement" % a.name
                for e in a.envs:
                    if getattr(type(e), "fused_band_reward", None) is not None:
                        return "a voltage-band PV inside a MultiComponentEnv"
                    kinds.append(type(e).mc_kind)
                slots += len(a.envs)
                continue
            k = getattr(type(a), "mc_kind", None)
            if k not in (1, 2, 3):
                return "agent %s is neither a MultiComponentEnv nor a single PV / storage / EV" % a.name
            owner = next(c for c in type(a).__mro__ if "mc_kind" in c.__dict__)
            band = getattr(type(a), "fused_band_reward", None)
            rew_owner = owner
            if band is not None:
                rew_owner = next(c for c in type(a).__mro__ if "fused_band_reward" in c.__dict__)
                if not a.grid_aware:
                    return "voltage-band PV %s does not observe min_voltage" % a.name
            if type(a).step is not owner.step or type(a).step_reward is not rew_owner.step_reward:
                return "agent %s overrides its step or reward" % a.name
            if not owns_fused_hooks(a, "mc_kind", skip=("step_reward",)):
                return "agent %s overrides a hook the fused step restates" % a.name
            kinds.append(k)
            slots += 1
        if slots > _lib.MA_MAX_SLOTS:
            return "more than %d components" % _lib.MA_MAX_SLOTS
        for k, cap in ((0, 1), (1, 2), (2, 1), (3, 1)):
            if kinds.count(k) > cap:
                return "more than %d component(s) of kind %d" % (cap, k)
        return None

    def _setup_ma(self):
        n, dev = self.num_envs, self.device
        solver = self.pf_solver
        solver.set_controllable_loads(sorted(set(self.agent_name_bus_map.values())))
        ctrl = list(solver._ctrl_names)
        args = _lib.MAStepArgs()
        ext = {"min_voltage": solver._vmin, "max_voltage": solver._vmax}
        plan, slot, n_pv = [], 0, 0
        for g, agent in enumerate(self.agents):
            multi = type(agent) is MultiComponentEnv
            envs = list(agent.envs) if multi else [agent]
            args.agent_first[g], args.agent_count[g], args.agent_sum[g] = slot, len(envs), int(multi)
            bus = self.agent_name_bus_map[agent.name]
            args.agent_bus[g] = ctrl.index(bus) if bus in ctrl else -1
            if multi:
                args.agent_real_power[g] = agent._real_power.data_ptr()
                args.agent_reward[g] = agent._reward.data_ptr()
            # the external obs the agent would get (get_external_obs_vars), per component
            kw_agent = {k: v for k, v in ext.items() if k in agent.obs_labels}
            comps = []
            for e in envs:
                if getattr(type(e), "mc_kind", None) == 1:
                    e._mc_pv_fields = ("pv", "pv_pmax", "pv_min_voltage") if n_pv == 0 else \
                        ("pv2", "pv2_pmax", "pv2_min_voltage")
                    args.slot_pv2[slot] = n_pv
                    n_pv += 1
                e._mc_static(args, slot)
                args.slot_agent[slot] = g
                rew = None
                band = getattr(type(e), "fused_band_reward", None)
                if band is not None:
                    rew = e._band_buffer()
                    args.slot_reward[slot] = rew.data_ptr()
                    args.band_lo, args.band_hi, args.band_scale = [float(x) for x in band]
                kw = {k: v for k, v in kw_agent.items() if k in e.obs_labels} if multi else kw_agent
                comps.append((e, slot, kw, rew))
                slot += 1
            plan.append((agent, multi, comps))
        args.n_comp, args.n_agents, args.n_bus = slot, len(self.agents), len(ctrl)
        # waves of a block: the building and the EV (the long per-env chains) one
        # each, the light PV / storage slots together in one more
        kinds = [args.comp[c].kind for c in range(slot)]
        waves = [[c] for c in range(slot) if kinds[c] in (0, 3)]
        light = [c for c in range(slot) if kinds[c] not in (0, 3)]
        if light:
            waves.append(light)
        args.n_waves = len(waves)
        i = 0
        for w, cs in enumerate(waves):
            args.wave_first[w], args.wave_count[w] = i, len(cs)
            for c in cs:
                args.wave_slot[i] = c
                i += 1
        bus_p = torch.zeros((max(len(ctrl), 1), n), dtype=torch.float64, device=dev)
        args.bus_p = bus_p.data_ptr()
        # per-step calls, flattened: (prepare, slot, agent name, component name or
        # None, kwargs) in slot order
        calls = [(e._mc_prepare, slot, agent.name, e.name if multi else None, kw)
                 for agent, multi, comps in plan for e, slot, kw, _ in comps]
        self._ma = {"args": args, "plan": plan, "bus_p": bus_p, "ctrl": ctrl, "calls": calls,
                    "iters": torch.zeros(n, dtype=torch.int32, device=dev),
                    "lazy_v": _FusedVoltages(self, {}, 0), "bufv": self._ma_bufv(plan),
                    "gen": ComponentEnv._bufv_gen, "fn": _lib.lib().pgw_ma_step,
                    "general": _lib.lib().pgw_pf_solve_general if solver.general else None}

    @staticmethod
    def _ma_bufv(plan):
        return tuple(e._bufv for _, _, comps in plan for e, _, _, _ in comps)

    def _step_ma(self, action):
        """MultiAgentEnv.step (multiagent_env.py:151-212) in one call: the
        components' per-step values into the launch arguments, pgw_ma_step
        (every agent's components + sums + bus loads, then the power flow with the
        extrema epilogue), then the components' clocks and the return dicts."""
        M = self._ma
        if ComponentEnv._bufv_gen != M["gen"]:       # some env re-pointed its buffers
            if self._ma_bufv(M["plan"]) != M["bufv"]:
                self._setup_ma()
            M = self._ma
            M["gen"] = ComponentEnv._bufv_gen
        args = M["args"]
        keep = []
        obs, rew, done, meta = {}, {}, {}, {}
        for prep, slot, aname, cname, kw in M["calls"]:
            act = action[aname]
            keep.append(prep(args, slot, act if cname is None else act[cname], kw))
        solver = self.pf_solver
        pfp, pft = solver.step_params(self.time), solver.solve_tables(self.time, args.n_bus > 0)
        H = self._hist
        v_out = None
        if H is not None:                            # every node into this step's history slot
            s_ = H["t"] % H["cap"]
            v_out = H["v"][s_].data_ptr()
        st = _lib.stream_ptr(self.device)
        if M["general"] is None:
            rc = M["fn"](args, pfp, pft, self.num_envs, v_out, M["iters"].data_ptr(), st)
        else:     # the agents' step, then the general power flow on its bus loads
            rc = M["fn"](args, None, None, self.num_envs, None, None, st) or \
                M["general"](pfp, pft, self.num_envs, M["bus_p"].data_ptr() if args.n_bus else None, None,
                             v_out, M["iters"].data_ptr(), st)
        if rc:
            _lib.check(rc)
        solver.solved(pft)
        agent_power_p = []
        for agent, multi, comps in M["plan"]:
            name = agent.name
            if multi:
                o, d, m = {}, False, {}
                for e, slot, kw, _ in comps:
                    ob, _, de, me = e._mc_finish(kw)
                    o[e.name], m[e.name] = ob, me
                    d = d or de
                obs[name], rew[name], done[name], meta[name] = o, agent._reward, d, m
            else:
                e, slot, kw, band = comps[0]
                ob, r, d, me = e._mc_finish(kw)
                if band is not None:
                    r = band
                elif r is None:
                    r = e._zero_reward
                obs[name], rew[name], done[name], meta[name] = ob, r, d, me
            agent_power_p.append(agent.real_power)
        solver.iterations = M["iters"]
        self._fused_steps += 1
        if H is None:
            # the extrema the epilogue wrote; every node solved on first access
            lazy = M["lazy_v"]
            lazy._step, lazy._reset, lazy._full = self._fused_steps, False, None
            self.voltages = solver.bus_voltages = lazy
        else:
            solver.bind_output(H["v"][s_])
            solver._prepare_bus_voltages()
            self.voltages = solver.bus_voltages
        solver._extrema = (solver._vmin, solver._vmax)
        self._record(agent_power_p)
        meta["oob_actions"] = self.oob_count
        return obs, rew, done, meta

    def _one_launch_ok(self):
        """The fused C4 step can run as one launch (k_coord_step_od): fp64, the
        OpenDSS rule on the fast kernel with the hour's response table and node
        records, the coordinated bus the only output row, the standard agent."""
        s = self.pf_solver
        return (self.dtype == torch.float64 and getattr(s, "convergence", None) == "opendss" and
                bool(getattr(s, "od_table", False)) and bool(getattr(s, "od_node_records", False)) and
                not getattr(s, "general", True) and len(s.output_names) == 1 and
                self.fused_reward_transform == "coordinated" and self._f32_fusable() is None)

    def set_pf_list(self, enabled=True):
        """Fused C4 step under the OpenDSS rule with node records (fp64): True
        (the default where _one_launch_ok) runs it as ONE launch,
        k_coord_step_od -- the agents, the table lookup and, for the rare envs
        the table leaves, the snap solve by the lookup wave (od_wave_solve);
        False the two-kernel step (k_coord_agents_std, then k_coord_pf_od over
        every env).  Bit-identical (tests/test_gpu_pf_od.py); one launch saves
        the second launch's ~4.6 us boundary.
        od_count[od_parity] counts the envs the step left to the solve.  (The
        library's PGW_STEP_LIST=1 runs the older list form instead: those envs
        listed and solved by k_coord_pf_od_list in a second launch.)"""
        F = self._fused
        if F is None or self.dtype != torch.float64:
            return
        b = F["bufs"]
        if enabled:
            if "od_list" not in F:
                # the envs the response table does not serve: k_coord_step_od lists
                # them, k_coord_pf_od_list solves them; od_count is two counters, the
                # step's and the next one's (od_parity, flipped every step)
                F["od_list"] = torch.zeros(self.num_envs, dtype=torch.int32, device=self.device)
                F["od_count"] = torch.zeros(2, dtype=torch.int32, device=self.device)
                b.od_parity = 0
            b.od_list, b.od_count = F["od_list"].data_ptr(), F["od_count"].data_ptr()
        else:
            b.od_list = b.od_count = None
        F["od_on"] = bool(enabled)

    def action_buffer(self):
        """Packed [n_agents, N, act_dim] action tensor the fused step reads
        zero-copy, plus the {agent: {component: [N, d]}} views into it."""
        F = self._fused
        if F is None:
            raise RuntimeError("action_buffer() is only available on the fused path")
        packed = F["act"].transpose(1, 2)
        views = {}
        for ai, agent in enumerate(self.agents):
            views[agent.name] = {e.name: packed[ai, :, int(F["act_off"][i]):int(F["act_off"][i]) + F["act_dims"][i]]
                                 for i, e in enumerate(agent.envs)}
        return packed, views

    def _pack_actions(self, action):
        F = self._fused
        if isinstance(action, torch.Tensor):
            na, n = len(self.agents), self.num_envs
            if action.dim() != 3 or tuple(action.shape) != (na, n, F["act_dim"]):
                raise ValueError("packed action must be [n_agents=%d, N=%d, act_dim=%d], got %s"
                                 % (na, n, F["act_dim"], tuple(action.shape)))
            if action.dtype != self.dtype or action.device != self.device:
                action = action.to(device=self.device, dtype=self.dtype)
            return action
        packed, views = self.action_buffer()
        for ai, agent in enumerate(self.agents):
            for i, e in enumerate(agent.envs):
                src = as_action(action[agent.name][e.name], self.num_envs, F["act_dims"][i], self.device,
                                self.dtype)
                views[agent.name][e.name].copy_(src)
        return packed

    def _step_fused(self, action):
        F = self._fused
        act = self._pack_actions(action)
        key = (act.data_ptr(), act.stride(0), act.stride(1), act.stride(2))
        bufs = F["bufs"]
        if key != F["act_key"]:
            bufs.action = F["Mat"](key[0], key[2], key[3])
            bufs.act_stride_agent = key[1]
            F["act_key"] = key
        bld, pv = F["bld0"], F["pv0"]
        solver = self.pf_solver
        skey = (bld.time_index if bld is not None else -1, pv.index if pv is not None else -1,
                self.time, solver.tables_version)
        ent = F["step_cache"].get(skey)
        if ent is None:
            ent = self._step_entry(skey)
        info, pfp, pft, tv = ent
        if tv != solver.tables_version:    # the table solve above recycled the device tables
            F["step_cache"].clear()
            return self._step_fused(action)
        H = self._hist
        if H is not None:            # outputs straight into this step's history slot
            s_ = H["t"] % H["cap"]
            bufs.v_out, bufs.agent_power = H["v"][s_].data_ptr(), H["p"][s_].data_ptr()
        if F.get("od_on"):
            bufs.od_parity ^= 1
        rc = getattr(_lib.lib(), F["kernel"])(F["params"], pfp, pft, info,
                                              self.num_envs, bufs, _lib.stream_ptr(self.device))
        if rc:
            _lib.check(rc)
        return self._fused_post(H, s_ if H is not None else None)

    def _fused_post(self, H, s_):
        """The fused step's host bookkeeping after its launch."""
        F, solver = self._fused, self.pf_solver
        self.pf_solver.iterations = F["iters"]
        self._fused_steps += 1
        if H is None:
            # the rows the kernel wrote, every other node solved on first access
            lazy = F["lazy_v"]
            lazy._step, lazy._reset, lazy._full = self._fused_steps, False, None
            self.voltages = solver.bus_voltages = lazy
            solver._extrema = None
        else:
            self.voltages = H["vd"][s_]
            for ai, agent in enumerate(self.agents):
                agent._real_power = H["pl"][s_][ai]
            if self.dtype == torch.float64:       # keep the solver's views current
                solver.bind_output(H["v"][s_])
                solver._prepare_bus_voltages()
        # advance the component clocks (their is_terminal() drives `done`)
        for e in F["bld_envs"]:
            e.time_index += 1
        for e in F["pv_envs"]:
            e.index += 1
        for e in F["bat_envs"]:
            e.simulation_step += 1
        d = any(e.is_terminal() for e in F["agent0_envs"])
        if H is not None:
            self._record(None)
        return F["obs_dict"], F["rew_dict"], F["done_true"] if d else F["done_false"], F["meta"]

    def capture_step(self, action, steps=1):
        """A CoordStepGraph (graph.py) of `steps` fused multi-agent steps per
        call, reading the packed actions bound at capture (a [n_agents, N,
        act_dim] tensor, a list of `steps` of them, or a callable k -> such a
        list for the graph at episode position k); returns what the last
        step's env.step returns."""
        from powergridworld_amd.graph import CoordStepGraph
        return CoordStepGraph(self, action, steps)

    def _advance_fused(self):
        """One captured step's host side: step()'s clocks and the fused step's
        bookkeeping (_fused_post), as the eager step does them after its launch."""
        self.episode_step += 1
        self.time = self._time_at(self.episode_step)
        self._at_reset = False
        self.obs_dict = {}
        F = self._fused
        if F.get("od_on"):
            F["bufs"].od_parity ^= 1
        obs, rew, done, meta = self._fused_post(None, None)
        any_done = any(done.values())
        d = bool(any_done or self.episode_step == self.max_episode_steps - 1 or self.episode_step >= self._end_step)
        dones = {a.name: d for a in self.agents}
        dones["__all__"] = d
        return obs, rew, dones, meta

    def _episode_last_step(self):
        """The episode step at which step() returns done (the component clocks
        advanced on copies; cached per reset)."""
        c = self.__dict__.get("_ep_last")
        if c is not None and c[0] == self.__dict__.get("_resets", 0):
            return c[1]
        F = self._fused
        clocks = [(e, "time_index") for e in F["bld_envs"]] + [(e, "index") for e in F["pv_envs"]] + \
                 [(e, "simulation_step") for e in F["bat_envs"]]
        saved = [getattr(e, a) for e, a in clocks]
        last, s = None, self.episode_step
        try:
            for _ in range(1 << 20):
                s += 1
                for e, a in clocks:
                    setattr(e, a, getattr(e, a) + 1)
                if any(e.is_terminal() for e in F["agent0_envs"]) or s == self.max_episode_steps - 1 or \
                        s >= self._end_step:
                    last = s
                    break
        finally:
            for (e, a), v in zip(clocks, saved):
                setattr(e, a, v)
        self._ep_last = (self.__dict__.get("_resets", 0), last)
        return last

    def _step_entry(self, skey):
        """The fused step's per-step constants for skey = (building time index,
        PV index, time, tables version): exogenous rows, PV value, PF parameters
        and tables of the hour; cached per key (every episode repeats them)."""
        F, solver = self._fused, self.pf_solver
        t, p, time = skey[0], skey[1], skey[2]
        bld, pv = F["bld0"], F["pv0"]
        info = _lib.CoordStepInfo()
        if bld is not None:
            if t + 1 >= len(bld._exo):
                raise IndexError("building stepped past the end of its exogenous data")
            info.ex_t, info.ex_next = bld._exo[t], bld._exo[t + 1]
        if pv is not None:
            info.pv_pmax = float(pv.data[p])
        pfp = solver.step_params(time)
        pft = solver.step_tables(time)
        if len(F["step_cache"]) > 1 << 14:
            F["step_cache"].clear()
        ent = F["step_cache"][(t, p, time, solver.tables_version)] = (info, pfp, pft, solver.tables_version)
        return ent

    def _prewarm_steps(self):
        """Fill the step cache for the episode that reset() just started (host
        work once per start state, so that the first episode's steps cost what
        later episodes' do; the constants are the ones each step would build)."""
        F = self._fused
        bld, pv = F["bld0"], F["pv0"]
        t0 = bld.time_index if bld is not None else -1
        p0 = pv.index if pv is not None else -1
        solver = self.pf_solver
        horizon = int(min(self.max_episode_steps if self.max_episode_steps else 0, 1024))
        if bld is not None:
            horizon = min(horizon, len(bld._exo) - 1 - t0)
        if pv is not None:
            horizon = min(horizon, len(pv.data) - p0)
        for k in range(1, horizon + 1):
            time = self._time_at(k)
            if k >= self._end_step + 1:
                break
            key = (t0 + k - 1 if bld is not None else -1, p0 + k - 1 if pv is not None else -1, time,
                   solver.tables_version)
            if key not in F["step_cache"]:
                self._step_entry(key)

    def state_dict(self):
        """The env's whole state (device tensors, generator states, clocks):
        powergridworld_amd.checkpoint.state_dict."""
        from powergridworld_amd.checkpoint import state_dict
        return state_dict(self)

    def load_state_dict(self, sd, strict=False):
        """Restore a state_dict() of an env of the same configuration (in place),
        then point the {node: voltage} mapping at the restored step's outputs."""
        from powergridworld_amd.checkpoint import load_state_dict
        load_state_dict(self, sd, strict)
        self._rearm_voltages()
        return self

    def _rearm_voltages(self):
        """env.voltages / solver.bus_voltages for the restored state: the solver's
        output rows, and on the fused paths the other nodes solved on first
        access for the restored step (or reset) number."""
        solver = self.pf_solver
        if not hasattr(solver, "_prepare_bus_voltages"):
            return
        H = self._hist
        if H is not None or (self._fused is None and self._ma is None):
            solver._prepare_bus_voltages()
            self.voltages = solver.bus_voltages
            return
        if self._at_reset or self._fused_steps == 0:
            solver._prepare_bus_voltages()
            self.voltages = solver.bus_voltages
            if self._fused is not None and len(solver.output_names) < solver.feeder.n:
                self.voltages = solver.bus_voltages = _FusedVoltages(self, solver.bus_voltages,
                                                                     self._fused_steps, reset=True)
            return
        lazy = (self._fused or self._ma)["lazy_v"]
        lazy._step, lazy._reset, lazy._full = self._fused_steps, False, None
        self.voltages = solver.bus_voltages = lazy

    def packed_obs(self):
        """Fused path: the [n_agents, N, obs_dim] observation view (list-interface order)."""
        return self._fused["obs"].transpose(1, 2)


class _FusedVoltages(Mapping):
    """{node: [N] voltage} after a fused step, in the feeder's node order like
    OpenDSS's AllBusMagPu (opendss.py:156-165).  The kernel writes only the rows
    the step needs (the coordinated bus); the others are solved on first access
    (MultiAgentEnv._full_voltages), so the hot path pays nothing for them.  Like
    every per-step output it describes the latest step (one object per env,
    re-armed each step)."""
    __slots__ = ("_env", "_fast", "_step", "_reset", "_full")

    def __init__(self, env, fast, step_no, reset=False):
        self._env, self._fast, self._step, self._reset, self._full = env, fast, step_no, reset, None

    def _all(self):
        if self._full is None:
            self._full = self._env._full_voltages(self._step, self._reset)
        return self._full

    def __getitem__(self, node):
        v = self._fast.get(node)
        return v if v is not None else self._all()[node]

    def __iter__(self):
        return iter(self._env.pf_solver.feeder.node_names)

    def __len__(self):
        return len(self._env.pf_solver.feeder.node_names)

    def copy(self):
        return dict(self.items())


def _bus_nodes(bus):
    from powergridworld_amd.distribution_system.opendss import bus_name_to_nodes
    return bus_name_to_nodes(bus)
