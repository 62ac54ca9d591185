"""The reference's own multi-agent test configurations
(tests/test_multiagent_env.py:13-107 with the fixtures of tests/conftest.py and
tests/agents/conftest.py) run through the engine's MultiAgentEnv (the three
MC buildings take the fused coordinated kernel with its generic agent code and
on-demand all-node voltages; the others the per-component path) with the
reference test runner's low / high / random policies
(tests/conftest.py:19-97), full episodes, checked step by step against the
oracle's MultiAgentOracle.  The reference tests only assert that the episodes
run; here every observation, reward, done flag and node voltage is compared.
Needs an MI355X."""
import numpy as np
import pandas as pd
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
K = 8
COMMON = {"start_time": "08-12-2020 00:00:00", "end_time": "08-13-2020 00:00:00",
          "control_timedelta": pd.Timedelta(300, "s")}
EV_CFG = {"num_vehicles": 100, "minutes_per_step": 5, "max_charge_rate_kw": 7.,
          "peak_threshold": 250., "vehicle_multiplier": 5., "rescale_spaces": False}
BLD_OBS = {"zone_temp": (18, 34), "p_consumed": (-100, 100)}


def _engine(case, exo):
    from powergridworld_amd import MultiAgentEnv, MultiComponentEnv
    from powergridworld_amd.agents import (EnergyStorageEnv, EVChargingEnv,
                                           FiveZoneROMThermalEnergyEnv, PVEnv)
    from powergridworld_amd.distribution_system.opendss import OpenDSSSolver
    mc = [{"name": "building", "cls": FiveZoneROMThermalEnergyEnv,
           "config": {"start_time": COMMON["start_time"], "end_time": COMMON["end_time"],
                      "rescale_spaces": False, "obs_config": BLD_OBS, "exogenous_data": exo}},
          {"name": "pv", "cls": PVEnv,
           "config": {"profile_csv": "pv_profile.csv", "scaling_factor": 10., "rescale_spaces": False}},
          {"name": "storage", "cls": EnergyStorageEnv, "config": {"rescale_spaces": False}}]
    if case == "ev3":
        agents = [{"name": "ev-charging-%d" % i, "bus": "675c", "cls": EVChargingEnv, "config": EV_CFG}
                  for i in range(3)]
    elif case == "buses":      # two buses, one of them with two agents (a per-bus sum)
        agents = [{"name": "ev-charging-%d" % i, "bus": b, "cls": EVChargingEnv, "config": EV_CFG}
                  for i, b in enumerate(("675c", "671", "675c"))]
    elif case == "mc3":
        agents = [{"name": "building-%d" % i, "bus": "675c", "cls": MultiComponentEnv,
                   "config": {"components": mc}} for i in range(3)]
    else:
        agents = [{"name": "building", "bus": "675c", "cls": MultiComponentEnv, "config": {"components": mc}},
                  {"name": "ev-charging", "bus": "675c", "cls": EVChargingEnv, "config": EV_CFG},
                  {"name": "pv", "bus": "675c", "cls": PVEnv,
                   "config": {"name": "pv", "profile_csv": "pv_profile.csv", "scaling_factor": 400.}}]
    pf = {"cls": OpenDSSSolver, "config": {"feeder_file": "ieee_13_dss/IEEE13Nodeckt.dss",
                                           "loadshape_file": "ieee_13_dss/annual_hourly_load_profile.csv",
                                           "system_load_rescale_factor": 0.7}}
    return MultiAgentEnv(common_config=COMMON, pf_config=pf, agents=agents, num_envs=K, device=DEV)


def _oracle(case, exo):
    from oracle.ma_oracle import MultiAgentOracle
    from oracle.pgw_oracle import BatteryOracle, BuildingOracle, EVOracle, MCOracle, PVOracle

    def mc():
        return MCOracle([("building", BuildingOracle(K, exo, obs_config=BLD_OBS, start_time=COMMON["start_time"],
                                                     end_time=COMMON["end_time"], rescale_spaces=False)),
                         ("pv", PVOracle(K, "pv_profile.csv", 10., rescale_spaces=False)),
                         ("storage", BatteryOracle(K, rescale_spaces=False))])
    if case == "ev3":
        agents = [("ev-charging-%d" % i, "675c", EVOracle(K, **EV_CFG)) for i in range(3)]
    elif case == "buses":
        agents = [("ev-charging-%d" % i, b, EVOracle(K, **EV_CFG)) for i, b in enumerate(("675c", "671", "675c"))]
    elif case == "mc3":
        agents = [("building-%d" % i, "675c", mc()) for i in range(3)]
    else:
        agents = [("building", "675c", mc()), ("ev-charging", "675c", EVOracle(K, **EV_CFG)),
                  ("pv", "675c", PVOracle(K, "pv_profile.csv", 400.))]
    # the engine's pf_config names no stopping rule: OpenDSS's snap solve, the
    # reference's (opendss.py:131-135) and the solver's default
    return MultiAgentOracle(K, agents, 0.7, COMMON["start_time"], COMMON["end_time"], semantics="opendss")


def _policy(space, kind, rng):
    """tests/conftest.py:19-39, with 'random' drawn per env."""
    if hasattr(space, "spaces"):
        return {k: _policy(s, kind, rng) for k, s in space.spaces.items()}
    lo, hi = np.asarray(space.low, float), np.asarray(space.high, float)
    if kind == "low":
        return np.tile(lo, (K, 1))
    if kind == "high":
        return np.tile(hi, (K, 1))
    return rng.uniform(lo, hi, size=(K, lo.shape[0]))


def _close(got, want, rtol, atol, what):
    g = got.detach().cpu().numpy() if isinstance(got, torch.Tensor) else np.asarray(got)
    np.testing.assert_allclose(g, np.asarray(want, float).reshape(g.shape), rtol, atol, err_msg=what)


def _cmp_obs(obs, want, t):
    for name, o in want.items():
        if isinstance(o, dict):
            for c, oc in o.items():
                _close(obs[name][c], oc, 1e-9, 1e-9, "obs %s/%s step %d" % (name, c, t))
        else:
            _close(obs[name], o, 1e-9, 1e-9, "obs %s step %d" % (name, t))


@pytest.mark.parametrize("case", ["ev3", "mc3", "het", "buses"])
def test_reference_multiagent_configs(case, exo_frame):
    env, orc = _engine(case, exo_frame), _oracle(case, exo_frame)
    rng = np.random.default_rng(3)
    nodes = orc.pf.feeder.node_names
    for kind in ("low", "high", "random"):
        env.reset()
        init = {}
        for agent in env.agents:                    # inject the sampled initial SoC
            if hasattr(agent, "env_dict") and "storage" in agent.env_dict:
                init[agent.name] = rng.uniform(3.0, 50.0, K)
                agent.env_dict["storage"].reset(init_storage=init[agent.name])
        want = orc.reset(init_storage=init)
        _cmp_obs(env.get_obs(), want, 0)
        steps = 0
        while True:
            action = {a.name: _policy(env.action_space[a.name], kind, rng) for a in env.agents}
            obs, rew, dones, _ = env.step(action)
            o_obs, o_rew, o_done = orc.step(action)
            steps += 1
            _cmp_obs(obs, o_obs, steps)
            for name in o_rew:
                _close(rew[name], o_rew[name], 1e-9, 1e-9, "reward %s step %d" % (name, steps))
            v = env.pf_solver.get_bus_voltages()
            _close(torch.stack([v[x] for x in nodes], 1), orc.v, 1e-8, 0, "voltages step %d" % steps)
            assert dones["__all__"] == o_done and all(dones[a.name] == o_done for a in env.agents)
            if o_done:
                break
        assert steps >= 280, steps                  # a full day (both sides agree on the end)


def _single(case, exo):
    """(engine env, oracle) for the reference's single-agent tests
    (tests/agents/test_*.py, tests/test_multicomponent_env.py)."""
    from powergridworld_amd import MultiComponentEnv
    from powergridworld_amd.agents import (EnergyStorageEnv, EVChargingEnv,
                                           FiveZoneROMThermalEnergyEnv, PVEnv)
    from oracle.pgw_oracle import BatteryOracle, BuildingOracle, EVOracle, MCOracle, PVOracle
    span = {"start_time": COMMON["start_time"], "end_time": COMMON["end_time"]}
    if case == "building":           # tests/agents/conftest.py:4-9
        return (FiveZoneROMThermalEnergyEnv(**span, exogenous_data=exo, num_envs=K, device=DEV),
                BuildingOracle(K, exo, **span))
    if case == "storage":
        return EnergyStorageEnv(num_envs=K, device=DEV), BatteryOracle(K)
    if case == "ev":
        return EVChargingEnv(**EV_CFG, num_envs=K, device=DEV), EVOracle(K, **EV_CFG)
    if case == "pv":
        return (PVEnv(name="pv", profile_csv="pv_profile.csv", scaling_factor=10., num_envs=K, device=DEV),
                PVOracle(K, "pv_profile.csv", 10.))
    mc = [{"name": "building", "cls": FiveZoneROMThermalEnergyEnv,
           "config": dict(span, rescale_spaces=False, obs_config=BLD_OBS, exogenous_data=exo)},
          {"name": "pv", "cls": PVEnv,
           "config": {"profile_csv": "pv_profile.csv", "scaling_factor": 10., "rescale_spaces": False}},
          {"name": "storage", "cls": EnergyStorageEnv, "config": {"rescale_spaces": False}}]
    orc = MCOracle([("building", BuildingOracle(K, exo, obs_config=BLD_OBS, rescale_spaces=False, **span)),
                    ("pv", PVOracle(K, "pv_profile.csv", 10., rescale_spaces=False)),
                    ("storage", BatteryOracle(K, rescale_spaces=False))])
    return MultiComponentEnv(name="mc", components=mc, num_envs=K, device=DEV), orc


@pytest.mark.parametrize("case", ["building", "storage", "ev", "pv", "mc"])
def test_reference_single_agent_configs(case, exo_frame):
    """tests/agents/test_*.py and tests/test_multicomponent_env.py: the
    single_agent_episode_runner / multi_agent_episode_runner policies (low,
    high, random) over full episodes, every step against the oracle."""
    from oracle.pgw_oracle import BatteryOracle, BuildingOracle, MCOracle
    env, orc = _single(case, exo_frame)
    rng = np.random.default_rng(5)
    for kind in ("low", "high", "random"):
        init = rng.uniform(0.0, 60.0, K)
        if case == "storage":
            ob = env.reset(init_storage=init)[0]
            want = orc.reset(init)
        elif case == "mc":
            ob = env.reset(init_storage=init)[0]
            want = orc.reset(init_storage=init)
        else:
            env.reset()
            ob = env.get_obs()[0]
            want = orc.reset()
            want = orc.obs() if want is None else want
        if isinstance(want, dict):
            for c in want:
                _close(ob[c], want[c], 1e-9, 1e-9, "%s reset obs %s" % (kind, c))
        else:
            _close(ob, want, 1e-9, 1e-9, "%s reset obs" % kind)
        steps = 0
        while True:
            a = _policy(env.action_space, kind, rng)
            ob, rew, done, _ = env.step(a)
            if isinstance(orc, BuildingOracle):
                o_ob, o_rew, o_done, _ = orc.step(a, lagged_reward=True)
            else:
                o_ob, o_rew, o_done, _ = orc.step(a)
            steps += 1
            if isinstance(o_ob, dict):
                for c in o_ob:
                    _close(ob[c], o_ob[c], 1e-9, 1e-9, "%s obs %s step %d" % (kind, c, steps))
            else:
                _close(ob, o_ob, 1e-9, 1e-9, "%s obs step %d" % (kind, steps))
            _close(rew, o_rew, 1e-9, 1e-9, "%s reward step %d" % (kind, steps))
            _close(env.real_power, orc.real_power, 1e-9, 1e-9, "%s real power step %d" % (kind, steps))
            assert done == bool(np.any(o_done)), (kind, steps)
            if done:
                break
        assert steps >= 280, (kind, steps)
