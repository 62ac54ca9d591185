"""The oracle (oracle/pgw_oracle.py) against the reference's own outputs
(tests/golden, written by oracle/make_golden.py) and the EV known answers in
examples/envs/ev-charging.ipynb:130,161,192.  CPU only."""
import json

import numpy as np
import pytest

from oracle import pgw_oracle as O
from tests.conftest import golden_path

RTOL = 1e-12
ATOL = 1e-12


def load(name):
    with np.load(golden_path(name), allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


@pytest.mark.parametrize("case", ["default", "norescale", "big"])
def test_battery(case):
    g = load("battery_" + case)
    cfg = json.loads(str(g["config"]))
    if "storage_range" in cfg:
        cfg["storage_range"] = tuple(cfg["storage_range"])
    K = g["init_storage"].shape[0]
    b = O.BatteryOracle(K, **cfg)
    np.testing.assert_allclose(b.reset(g["init_storage"]), g["obs"][0], RTOL, ATOL)
    for t in range(g["actions"].shape[0]):
        o, r, d, _ = b.step(g["actions"][t])
        np.testing.assert_allclose(o, g["obs"][t + 1], RTOL, ATOL)
        np.testing.assert_allclose(b.real_power, g["real_power"][t], RTOL, ATOL)
        np.testing.assert_allclose(b.soc, g["soc"][t + 1], RTOL, ATOL)
        assert (d == g["done"][t]).all()
        assert (r == g["reward"][t]).all()


@pytest.mark.parametrize("case", ["default", "norescale", "offpeak_short"])
def test_pv(case):
    g = load("pv_" + case)
    cfg = json.loads(str(g["config"]))
    K = g["actions"].shape[1]
    p = O.PVOracle(K, **cfg)
    assert p.reset() is None
    for t in range(g["actions"].shape[0]):
        o, r, d, _ = p.step(g["actions"][t])
        np.testing.assert_allclose(o, g["obs"][t], RTOL, ATOL)
        np.testing.assert_allclose(p.real_power, g["real_power"][t], RTOL, ATOL)
        assert (d == g["done"][t]).all()


@pytest.mark.parametrize("case", ["default", "tests_obs", "allobs"])
def test_building_two_episodes(case, exo_frame):
    g0 = load("building_%s_ep0" % case)
    cfg = json.loads(str(g0["config"]))
    if "obs_config" in cfg:
        cfg["obs_config"] = {k: tuple(v) for k, v in cfg["obs_config"].items()}
    K = g0["actions"].shape[1]
    b = O.BuildingOracle(K, exo_frame, **cfg)
    assert b.max_episode_steps == int(g0["max_episode_steps"])
    for ep in range(2):    # second episode checks the x_k carry-over across reset
        g = load("building_%s_ep%d" % (case, ep))
        np.testing.assert_allclose(b.reset(), g["obs"][0], 1e-10, 1e-10)
        np.testing.assert_allclose(b.x, g["x_k"][0], 1e-10, 1e-10)
        for t in range(g["actions"].shape[0]):
            o, r, d, _ = b.step(g["actions"][t], lagged_reward=True)
            np.testing.assert_allclose(o, g["obs"][t + 1], 1e-10, 1e-10)
            np.testing.assert_allclose(r, g["reward"][t], 1e-10, 1e-10)
            np.testing.assert_allclose(b.real_power, g["real_power"][t], 1e-10, 1e-10)
            np.testing.assert_allclose(b.x, g["x_k"][t + 1], 1e-10, 1e-10)
            assert (d == g["done"][t]).all()


@pytest.mark.parametrize("case", ["notebook", "rescaled", "hetero25"])
def test_ev(case):
    g = load("ev_" + case)
    cfg = json.loads(str(g["config"]))
    K = g["actions"].shape[1]
    e = O.EVOracle(K, **cfg)
    np.testing.assert_allclose(e.reset(), g["obs"][0], RTOL, ATOL)
    for t in range(g["actions"].shape[0]):
        o, r, d, _ = e.step(g["actions"][t])
        np.testing.assert_allclose(o, g["obs"][t + 1], RTOL, ATOL)
        np.testing.assert_allclose(r, g["reward"][t], RTOL, ATOL)
        np.testing.assert_allclose(e.real_power, g["real_power"][t], RTOL, ATOL)
        assert (d == g["done"][t]).all()


@pytest.mark.parametrize("case", ["hetero25", "v100"])
def test_ev_randomize(case):
    """randomize=True: each env's sampled vehicle rows (recorded from the
    reference's DataFrame.sample) injected into the oracle, two episodes."""
    g = load("ev_random_" + case)
    cfg = json.loads(str(g["config"]))
    assert cfg.pop("randomize") is True
    EP, T, K = g["reward"].shape
    e = O.EVOracle(K, **cfg)
    for ep in range(EP):
        ids = g["vehicle_ids"][ep]
        assert len(set(ids[0])) == ids.shape[1] and not (ids == np.arange(ids.shape[1])).all()
        np.testing.assert_allclose(e.reset(ids), g["obs"][ep, 0], RTOL, ATOL)
        for t in range(T):
            o, r, d, _ = e.step(g["actions"][ep, t])
            np.testing.assert_allclose(o, g["obs"][ep, t + 1], RTOL, ATOL)
            np.testing.assert_allclose(r, g["reward"][ep, t], RTOL, ATOL)
            np.testing.assert_allclose(e.real_power, g["real_power"][ep, t], RTOL, ATOL)


EV_KNOWN = {"high":-934170.2851237846, "low": -2659771.95782906, "0.8": -1161670.9270816303}


@pytest.mark.parametrize("policy", list(EV_KNOWN))
def test_ev_notebook_known_answers(policy):
    """examples/envs/ev-charging.ipynb:130,161,192 (num_vehicles=100, x5, thr 250)."""
    e = O.EVOracle(1, num_vehicles=100, minutes_per_step=5, max_charge_rate_kw=7.,
                   peak_threshold=250., vehicle_multiplier=5., rescale_spaces=False)
    a = {"high": 1.0, "low": 0.0, "0.8": 0.8}[policy]
    e.reset()
    total, done = 0.0, False
    while not done:
        _, r, d, _ = e.step(np.array([[a]]))
        total += r[0]
        done = d[0]
    np.testing.assert_allclose(total * 1e5, EV_KNOWN[policy], rtol=1e-12)


def test_mc_c3(exo_frame):
    g = load("mc_c3")
    K = g["init_storage"].shape[0]
    comps = [("building", O.BuildingOracle(K, exo_frame)),
             ("pv", O.PVOracle(K, profile_csv="pv_profile.csv", scaling_factor=40.)),
             ("storage", O.BatteryOracle(K)),
             ("ev", O.EVOracle(K, num_vehicles=100, minutes_per_step=5, max_charge_rate_kw=7.,
                               peak_threshold=250., vehicle_multiplier=5., rescale_spaces=True))]
    names = [str(n) for n in g["names"]]
    assert names == [c[0] for c in comps]
    mc = O.MCOracle(comps)
    obs = mc.reset(init_storage=g["init_storage"])
    for n in names:
        np.testing.assert_allclose(obs[n], g["obs_" + n][0], 1e-10, 1e-10)
    for t in range(g["reward"].shape[0]):
        obs, r, d, _ = mc.step({n: g["act_" + n][t] for n in names})
        for n in names:
            np.testing.assert_allclose(obs[n], g["obs_" + n][t + 1], 1e-10, 1e-10)
        np.testing.assert_allclose(r, g["reward"][t], 1e-10, 1e-10)
        np.testing.assert_allclose(mc.real_power, g["real_power"][t], 1e-10, 1e-10)
        assert (d == g["done"][t]).all()


def _c4_oracle(K, NA, semantics):
    from oracle.ma_oracle import CoordinatedOracle
    from oracle.pf_oracle import BatchedPF
    orc = CoordinatedOracle(K, n_agents=NA)
    orc.pf = BatchedPF(system_load_rescale_factor=1.2, semantics=semantics)
    return orc


# golden of each power-flow rule: OpenDSS's snap solve (the reference's) and the fixed point
GOLD_SUFFIX = {"opendss": "_od", "exact": ""}


@pytest.mark.parametrize("semantics", ["opendss", "exact"])
def test_c4_coordinated_oracle(semantics):
    """MultiAgentEnv + CoordinatedMultiBuildingControlEnv (reference, oracle PF behind
    its PowerFlowSolver ABC) vs the oracle's end-to-end C4 restatement."""
    g = load("c4_coordinated" + GOLD_SUFFIX[semantics])
    T, NA, K, _ = g["actions"].shape
    orc = _c4_oracle(K, NA, semantics)
    obs0 = orc.reset(g["init_storage"])
    np.testing.assert_allclose(obs0, g["obs"][0], 1e-10, 1e-10)
    np.testing.assert_allclose(orc.v, g["v675"][0], 1e-12, 1e-12)
    for t in range(T):
        obs, rew, vv = orc.step(g["actions"][t])
        np.testing.assert_allclose(obs, g["obs"][t + 1], 1e-10, 1e-10)
        np.testing.assert_allclose(rew, g["reward"][t], 1e-9, 1e-9)
        np.testing.assert_allclose(vv, g["voltage_violation"][t], 1e-12, 1e-12)
        np.testing.assert_allclose(orc.v, g["v675"][t + 1], 1e-12, 1e-12)
        assert orc.done == bool(g["done"][t, 0])


@pytest.mark.parametrize("semantics", ["opendss", "exact"])
def test_c4_two_episodes_oracle(semantics):
    """C4 across the episode boundary (reference run, two episodes per env): the
    SoC the reference drew at each reset is injected; x_k carries over."""
    g = load("c4_two_episodes" + GOLD_SUFFIX[semantics])
    E, T, NA, K, _ = g["actions"].shape
    orc = _c4_oracle(K, NA, semantics)
    for e in range(E):
        obs0 = orc.reset(g["init_storage"][e])
        np.testing.assert_allclose(obs0, g["obs"][e, 0], 1e-10, 1e-10)
        xk = np.stack([a.comps[0][1].x for a in orc.agents])          # [NA, K, 5]
        np.testing.assert_allclose(xk, g["x_k"][e, 0], 1e-12, 1e-12)
        for t in range(T):
            obs, rew, vv = orc.step(g["actions"][e, t])
            np.testing.assert_allclose(obs, g["obs"][e, t + 1], 1e-10, 1e-10)
            np.testing.assert_allclose(rew, g["reward"][e, t], 1e-9, 1e-9)
            np.testing.assert_allclose(vv, g["voltage_violation"][e, t], 1e-12, 1e-12)
            xk = np.stack([a.comps[0][1].x for a in orc.agents])
            np.testing.assert_allclose(xk, g["x_k"][e, t + 1], 1e-12, 1e-12)
            assert orc.done == bool(g["done"][e, t, 0])
