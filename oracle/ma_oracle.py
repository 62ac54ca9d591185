"""CPU oracle for the multi-agent step (TEST INFRASTRUCTURE; see pgw_oracle.py
header for the import rule).

``CoordinatedOracle`` restates the BASELINE C4 scenario end to end:
MultiAgentEnv.step (gridworld/multiagent_env.py:151-212) over n MultiComponentEnv
agents built by gridworld/scenarios/buildings.py:11-72 with the MADDPG
make_env configs (examples/marl/openai/train.py:165-181), the power flow
(oracle/pf_oracle.py) and CoordinatedMultiBuildingControlEnv's shared
voltage-violation penalty (train.py:51-88).
"""
import numpy as np
import pandas as pd

from oracle.exogenous import synthetic_exogenous_frame
from oracle.pf_oracle import BatchedPF
from oracle.pgw_oracle import BatteryOracle, BuildingOracle, MCOracle, PVOracle

START = "08-12-2021 00:00:00"
END = "08-13-2021 00:00:00"
DT = pd.Timedelta(300, "s")


class CoordinatedOracle:
    VOLTAGE_LIMITS = (0.95, 1.05)
    VV_UNIT_PENALTY = 1e4

    def __init__(self, K, n_agents=5, sys_load=1.2, exo=None, bus_node="675.3", bus_load="675c"):
        exo = synthetic_exogenous_frame() if exo is None else exo
        self.K, self.n = K, n_agents
        self.agents = [MCOracle([
            ("building", BuildingOracle(K, exo)),
            ("pv", PVOracle(K, profile_csv="pv_profile.csv", scaling_factor=40.)),
            ("storage", BatteryOracle(K, max_power=15., storage_range=(3., 50.)))])
            for _ in range(n_agents)]
        self.pf = BatchedPF(system_load_rescale_factor=sys_load)
        self.node = self.pf.feeder.idx[bus_node]
        self.bus_load = bus_load
        self.start, self.end = pd.Timestamp(START), pd.Timestamp(END)

    def reset(self, init_soc):
        self.t = self.start
        self.episode_step = 0
        obs = []
        for a, agent in enumerate(self.agents):
            o = agent.reset(init_storage=np.asarray(init_soc)[a])
            obs.append(np.concatenate([o["building"], o["pv"], o["storage"]], 1))
        self.v = self.pf.calculate(self.t, K=self.K)[:, self.node]
        return np.stack(obs)

    def step(self, act):
        """act: (n_agents, K, 8) = building 6 | pv 1 | storage 1."""
        self.t = self.t + DT
        self.episode_step += 1
        obs, rew, load, dones = [], [], 0., []
        for a, agent in enumerate(self.agents):
            o, r, d, _ = agent.step({"building": act[a][:, 0:6], "pv": act[a][:, 6:7],
                                     "storage": act[a][:, 7:8]})
            obs.append(np.concatenate([o["building"], o["pv"], o["storage"]], 1))
            rew.append(r)
            dones.append(d)
            load = load + agent.real_power
        v = self.pf.calculate(self.t, {self.bus_load: load}, K=self.K)[:, self.node]
        self.v = v
        vv = np.maximum(np.maximum(0.0, self.VOLTAGE_LIMITS[0] - v), v - self.VOLTAGE_LIMITS[1])
        rew = np.stack(rew) - (vv * self.VV_UNIT_PENALTY) / self.n
        self.done = bool(np.any(dones) or self.t >= self.end)
        return np.stack(obs), rew, vv


class MultiAgentOracle:
    """MultiAgentEnv (gridworld/multiagent_env.py:24-212) with the base
    pass-through reward / meta transforms, for agents that observe no grid
    voltage (get_external_obs_vars :90-115 then passes nothing): each agent
    steps in list order, its real power is added to its bus load (:171-181,
    the first agent's value then ``+=``), the power flow runs at the advanced
    time (:183-189), and the episode ends when any agent is done, at
    max_episode_steps - 1, or when the time reaches end_time (:199-202).

    agents: list of (name, bus, oracle) with oracle an MCOracle or a component
    oracle.  A standalone building returns its lagged reward
    (five_zone_rom_env.py:215); components in an MCOracle the fresh sum."""

    def __init__(self, K, agents, sys_load, start, end, dt=DT, max_episode_steps=None, semantics="exact"):
        self.K, self.agents = K, agents
        self.pf = BatchedPF(system_load_rescale_factor=sys_load, semantics=semantics)
        self.start, self.end, self.dt = pd.Timestamp(start), pd.Timestamp(end), dt
        self.max_episode_steps = np.inf if max_episode_steps is None else max_episode_steps

    def _obs(self, ag):
        if isinstance(ag, MCOracle):
            return {n: (c.get_obs() if isinstance(c, BuildingOracle) else c.obs()) for n, c in ag.comps}
        return ag.get_obs() if isinstance(ag, BuildingOracle) else ag.obs()

    def reset(self, init_storage=None):
        """init_storage: {agent name: [K] initial SoC} for the agents holding a battery."""
        init_storage = init_storage or {}
        self.t = self.start
        self.episode_step = 0
        self.v = self.pf.calculate(self.t, K=self.K)                     # :131-133
        for name, _, ag in self.agents:
            if isinstance(ag, MCOracle):
                ag.reset(init_storage=init_storage.get(name))
            elif isinstance(ag, BatteryOracle):
                ag.reset(init_storage[name])
            else:
                ag.reset()
        return {name: self._obs(ag) for name, _, ag in self.agents}

    def step(self, action):
        self.episode_step += 1
        self.t = self.t + self.dt
        obs, rew, done, load = {}, {}, [], {}
        for name, bus, ag in self.agents:
            if isinstance(ag, BuildingOracle):
                o, r, d, _ = ag.step(action[name], lagged_reward=True)
            else:
                o, r, d, _ = ag.step(action[name])
            obs[name], rew[name] = o, r
            done.append(np.any(d))
            p = ag.real_power
            load[bus] = load[bus] + p if bus in load else p
        self.v = self.pf.calculate(self.t, load, K=self.K)
        d = bool(any(done) or self.episode_step == self.max_episode_steps - 1 or self.t >= self.end)
        return obs, rew, d
