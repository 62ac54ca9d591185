"""HIP path vs the reference (golden fixtures) and the oracle.  Needs an MI355X.

Tolerances (BASELINE.json north_star): fp64 continuous state/reward within
1e-6 relative -- the tests use tighter bounds where the arithmetic is restated
op-for-op (1e-12..1e-9); done flags and integer counts exactly.
"""
import json

import numpy as np
import pytest
import torch

from tests.conftest import golden_path

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def load(name):
    with np.load(golden_path(name), allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


def T(x):
    return torch.tensor(np.asarray(x), dtype=torch.float64, device=DEV)


def N(t):
    return t.detach().cpu().numpy()


def close(got, want, rtol=1e-12, atol=1e-12):
    np.testing.assert_allclose(N(got) if isinstance(got, torch.Tensor) else got, want, rtol, atol)


# ------------------------------------------------------------------ components
@pytest.mark.parametrize("case", ["default", "norescale", "big"])
def test_battery_golden(case):
    from powergridworld_amd.agents import EnergyStorageEnv
    g = load("battery_" + case)
    cfg = json.loads(str(g["config"]))
    if "storage_range" in cfg:
        cfg["storage_range"] = tuple(cfg["storage_range"])
    K = g["init_storage"].shape[0]
    env = EnergyStorageEnv(name="storage", num_envs=K, device=DEV, **cfg)
    obs, meta = env.reset(init_storage=g["init_storage"])
    close(obs, g["obs"][0])
    for t in range(g["actions"].shape[0]):
        obs, rew, done, meta = env.step(T(g["actions"][t]))
        close(obs, g["obs"][t + 1])
        close(env.real_power, g["real_power"][t])
        close(env.soc, g["soc"][t + 1])
        assert (N(rew) == g["reward"][t]).all()
        assert done == bool(g["done"][t, 0])


@pytest.mark.parametrize("case", ["default", "norescale", "offpeak_short"])
def test_pv_golden(case):
    from powergridworld_amd.agents import PVEnv
    g = load("pv_" + case)
    cfg = json.loads(str(g["config"]))
    K = g["actions"].shape[1]
    env = PVEnv(name="pv", num_envs=K, device=DEV, **cfg)
    assert env.reset() is None
    for t in range(g["actions"].shape[0]):
        obs, rew, done, meta = env.step(T(g["actions"][t]))
        close(obs, g["obs"][t])
        close(env.real_power, g["real_power"][t])
        assert done == bool(g["done"][t, 0])


@pytest.mark.parametrize("case", ["default", "tests_obs", "allobs"])
def test_building_golden_two_episodes(case, exo_frame):
    from powergridworld_amd.agents import FiveZoneROMThermalEnergyEnv
    g0 = load("building_%s_ep0" % case)
    cfg = json.loads(str(g0["config"]))
    if "obs_config" in cfg:
        cfg["obs_config"] = {k: tuple(v) for k, v in cfg["obs_config"].items()}
    K = g0["actions"].shape[1]
    env = FiveZoneROMThermalEnergyEnv(name="building", num_envs=K, device=DEV,
                                      exogenous_data=exo_frame, **cfg)
    assert env.max_episode_steps == int(g0["max_episode_steps"])
    for ep in range(2):                       # x_k carries over across reset()
        g = load("building_%s_ep%d" % (case, ep))
        close(env.reset(), g["obs"][0], 1e-10, 1e-10)
        close(env.x.t(), g["x_k"][0], 1e-10, 1e-10)
        for t in range(g["actions"].shape[0]):
            obs, rew, done, meta = env.step(T(g["actions"][t]))
            close(obs, g["obs"][t + 1], 1e-10, 1e-10)
            close(rew, g["reward"][t], 1e-10, 1e-10)
            close(env.real_power, g["real_power"][t], 1e-10, 1e-10)
            close(env.x.t(), g["x_k"][t + 1], 1e-10, 1e-10)
            assert done == bool(g["done"][t, 0])


@pytest.mark.parametrize("case", ["notebook", "rescaled", "hetero25"])
def test_ev_golden(case):
    from powergridworld_amd.agents import EVChargingEnv
    g = load("ev_" + case)
    cfg = json.loads(str(g["config"]))
    K = g["actions"].shape[1]
    env = EVChargingEnv(num_envs=K, device=DEV, **cfg)
    obs, _ = env.reset()
    close(obs, g["obs"][0])
    for t in range(g["actions"].shape[0]):
        obs, rew, done, meta = env.step(T(g["actions"][t]))
        close(obs, g["obs"][t + 1])
        close(rew, g["reward"][t])
        close(env.real_power, g["real_power"][t])
        assert done == bool(g["done"][t, 0])


def test_ev_notebook_known_answers_batched():
    """examples/envs/ev-charging.ipynb:130,161,192 -- the three policies as three envs
    of one batch."""
    from powergridworld_amd.agents import EVChargingEnv
    env = EVChargingEnv(num_vehicles=100, minutes_per_step=5, max_charge_rate_kw=7.,
                        peak_threshold=250., vehicle_multiplier=5., rescale_spaces=False,
                        num_envs=3, device=DEV)
    env.reset()
    a = T([[1.0], [0.0], [0.8]])
    total = torch.zeros(3, dtype=torch.float64, device=DEV)
    done = False
    while not done:
        _, r, done, _ = env.step(a)
        total += r
    np.testing.assert_allclose(N(total) * 1e5, [-934170.2851237846, -2659771.95782906,
                                                -1161670.9270816303], rtol=1e-12)


@pytest.mark.parametrize("case", ["hetero25", "v100"])
def test_ev_randomize_golden(case):
    """randomize=True (ev_charging_env.py:154-156): the reference's sampled
    vehicle rows injected per env, two episodes against its outputs."""
    from powergridworld_amd.agents import EVChargingEnv
    g = load("ev_random_" + case)
    cfg = json.loads(str(g["config"]))
    EP, steps, K = g["reward"].shape
    env = EVChargingEnv(num_envs=K, device=DEV, **cfg)
    for ep in range(EP):
        obs, _ = env.reset(vehicle_ids=g["vehicle_ids"][ep])
        close(obs, g["obs"][ep, 0])
        for t in range(steps):
            obs, rew, done, _ = env.step(T(g["actions"][ep, t]))
            close(obs, g["obs"][ep, t + 1])
            close(rew, g["reward"][ep, t])
            close(env.real_power, g["real_power"][ep, t])


def test_ev_randomize_sampled_vs_oracle():
    """randomize=True with the engine's own per-env draw (seeded): every env's
    subset is V distinct rows, envs differ, reseeding repeats the draw, and a
    full episode equals the oracle run on the drawn subsets."""
    from oracle.pgw_oracle import EVOracle
    from powergridworld_amd.agents import EVChargingEnv
    n, V = 512, 25
    cfg = dict(num_vehicles=V, minutes_per_step=5, max_charge_rate_kw=7., peak_threshold=200.,
               vehicle_multiplier=40., rescale_spaces=True)
    env = EVChargingEnv(num_envs=n, device=DEV, randomize=True, **cfg)
    env.seed(3)
    obs, _ = env.reset()
    ids = N(env.vehicle_ids)
    assert all(len(set(r)) == V for r in ids) and len({tuple(r) for r in ids}) == n
    assert ids.min() >= 0 and ids.max() < len(env._all_req)
    env.seed(3)
    env.reset()
    assert (N(env.vehicle_ids) == ids).all()
    orc = EVOracle(n, **cfg)
    close(obs, orc.reset(ids))
    rng = np.random.default_rng(7)
    done = False
    while not done:
        a = rng.uniform(-1.2, 1.2, (n, 1))
        obs, rew, done, _ = env.step(T(a))
        o, r, d, _ = orc.step(a)
        close(obs, o)
        close(rew, r)
        close(env.real_power, orc.real_power)
        assert done == bool(d[0])


def test_mc_c3_golden(exo_frame):
    from powergridworld_amd import MultiComponentEnv
    from powergridworld_amd.agents import (EnergyStorageEnv, EVChargingEnv,
                                           FiveZoneROMThermalEnergyEnv, PVEnv)
    g = load("mc_c3")
    K = g["init_storage"].shape[0]
    comps = [
        {"name": "building", "cls": FiveZoneROMThermalEnergyEnv, "config": {"exogenous_data": exo_frame}},
        {"name": "pv", "cls": PVEnv, "config": {"profile_csv": "pv_profile.csv", "scaling_factor": 40.}},
        {"name": "storage", "cls": EnergyStorageEnv, "config": {}},
        {"name": "ev", "cls": EVChargingEnv,
         "config": dict(num_vehicles=100, minutes_per_step=5, max_charge_rate_kw=7.,
                        peak_threshold=250., vehicle_multiplier=5., rescale_spaces=True)},
    ]
    env = MultiComponentEnv(name="mc", components=comps, num_envs=K, device=DEV)
    names = [str(x) for x in g["names"]]
    obs, _ = env.reset(init_storage=g["init_storage"])
    for n in names:
        close(obs[n], g["obs_" + n][0], 1e-10, 1e-10)
    for t in range(g["reward"].shape[0]):
        obs, rew, done, meta = env.step({n: T(g["act_" + n][t]) for n in names})
        for n in names:
            close(obs[n], g["obs_" + n][t + 1], 1e-10, 1e-10)
        close(rew, g["reward"][t], 1e-10, 1e-10)
        close(env.real_power, g["real_power"][t], 1e-10, 1e-10)
        assert done == bool(g["done"][t, 0])


def test_battery_c2_vs_oracle():
    """C2 shape (batch 4096): seeded random episode vs the oracle, incl. clamps."""
    from oracle.pgw_oracle import BatteryOracle
    from powergridworld_amd.agents import EnergyStorageEnv
    n = 4096
    rng = np.random.default_rng(7)
    init = rng.uniform(0.0, 60.0, n)
    env = EnergyStorageEnv(num_envs=n, device=DEV)
    orc = BatteryOracle(n)
    close(env.reset(init_storage=init)[0], orc.reset(init))
    for t in range(300):
        a = rng.uniform(-1.3, 1.3, (n, 1))
        o, _, d, _ = env.step(T(a))
        oo, _, od, _ = orc.step(a)
        close(o, oo)
        close(env.real_power, orc.real_power)
        assert d == bool(od[0])


# ------------------------------------------------------------------ power flow
@pytest.mark.parametrize("semantics", ["opendss", "exact"])
def test_pf_vs_oracle(semantics):
    """Two controllable loads (the general kernel under OpenDSS's rule, the
    fast one for the fixed point) against the oracle with the same rule."""
    from oracle.pf_oracle import BatchedPF
    from powergridworld_amd.distribution_system.opendss import OpenDSSSolver
    n = 1024
    rng = np.random.default_rng(11)
    pf = OpenDSSSolver("ieee_13_dss/IEEE13Nodeckt.dss", "ieee_13_dss/annual_hourly_load_profile.csv",
                       system_load_rescale_factor=1.2, num_envs=n, device=DEV, convergence=semantics)
    orc = BatchedPF(system_load_rescale_factor=1.2, semantics=semantics)
    for ts in ["2021-08-12 00:05", "2021-08-12 15:00", "2021-01-01 05:00"]:
        p675 = rng.uniform(-300, 600, n)
        q675 = rng.uniform(-50, 50, n)
        p671 = rng.uniform(-100, 300, n)
        pf.calculate_power_flow({"675c": T(p675), "671": T(p671)}, {"675c": T(q675)}, current_time=ts)
        v = pf.get_bus_voltages()
        want = orc.calculate(ts, {"675c": p675, "671": p671}, {"675c": q675}, K=n)
        got = np.stack([N(v[name]) for name in orc.feeder.node_names], 1)
        np.testing.assert_allclose(got, want, rtol=1e-8, atol=0)
        close(pf.get_bus_voltage_by_name("675c"), want[:, orc.feeder.idx["675.3"]], 1e-8, 0)
        assert (N(pf.iterations) == orc.last_iters).mean() > 0.99


@pytest.mark.parametrize("semantics", ["opendss", "exact"])
def test_pf_regcap_feeder_vs_oracle(semantics):
    """A feeder beyond IEEE-13 (tests/data/regcap_feeder.dss: fixed-tap
    regulators, capacitors, model-2 loads; parity unpinned, no OpenDSS) through
    the batched solver against the oracle, two controllable loads."""
    import os
    from oracle.pf_oracle import BatchedPF
    from powergridworld_amd.distribution_system.dss import parse_dss
    from powergridworld_amd.distribution_system.opendss import OpenDSSSolver
    from tests.conftest import REPO
    path = os.path.join(REPO, "tests", "data", "regcap_feeder.dss")
    n = 512
    rng = np.random.default_rng(12)
    pf = OpenDSSSolver(path, "ieee_13_dss/annual_hourly_load_profile.csv", system_load_rescale_factor=1.1,
                       num_envs=n, device=DEV, convergence=semantics)
    assert pf.load_bus_name == ["d1", "a1", "c1"]        # model-1 loads only
    orc = BatchedPF(spec=parse_dss(path), system_load_rescale_factor=1.1, semantics=semantics)
    for ts in ["2021-08-12 15:00", "2021-01-01 05:00"]:
        pa = rng.uniform(-100, 300, n)
        pc = rng.uniform(-50, 200, n)
        pf.calculate_power_flow({"a1": T(pa), "c1": T(pc)}, {}, current_time=ts)
        v = pf.get_bus_voltages()
        want = orc.calculate(ts, {"a1": pa, "c1": pc}, {}, K=n)
        got = np.stack([N(v[name]) for name in orc.feeder.node_names], 1)
        np.testing.assert_allclose(got, want, rtol=1e-8, atol=0)
        if semantics == "opendss":
            np.testing.assert_array_equal(N(pf.iterations), orc.last_iters)


@pytest.mark.parametrize("semantics", ["opendss", "exact"])
@pytest.mark.parametrize("loads", [("675c",), ("675c", "671")])
def test_pf_all_rows_ragged_and_extrema_only(loads, semantics):
    """All output rows at a ragged batch (the last wave part-empty: the rows'
    DPP broadcasts read every lane, past-n lanes included, and store nothing);
    the epilogue's min/max equal Python's min/max over the rows in order; an
    extrema-only solve (v_out = NULL) gives the same extrema."""
    from oracle.pf_oracle import BatchedPF
    from powergridworld_amd import _lib
    from powergridworld_amd.distribution_system.opendss import OpenDSSSolver
    n = 1000
    rng = np.random.default_rng(21)
    pf = OpenDSSSolver("ieee_13_dss/IEEE13Nodeckt.dss", "ieee_13_dss/annual_hourly_load_profile.csv",
                       system_load_rescale_factor=0.65, num_envs=n, device=DEV, convergence=semantics)
    orc = BatchedPF(system_load_rescale_factor=0.65, semantics=semantics)
    ts = "2020-08-12 13:00"
    p_np = {k: rng.uniform(-400, 300, n) for k in loads}
    pf.calculate_power_flow({k: T(v) for k, v in p_np.items()}, None, current_time=ts)
    want = orc.calculate(ts, p_np, K=n)
    v = pf.get_bus_voltages()
    got = np.stack([N(v[name]) for name in orc.feeder.node_names], 1)
    np.testing.assert_allclose(got, want, rtol=1e-8, atol=0)
    rows = [N(v[name]) for name in pf.output_names]
    vmn, vmx = rows[0].copy(), rows[0].copy()
    for r in rows[1:]:
        vmn = np.where(r < vmn, r, vmn)
        vmx = np.where(r > vmx, r, vmx)
    lo, hi = pf.voltage_extrema()
    assert np.array_equal(N(lo), vmn) and np.array_equal(N(hi), vmx)
    # the same solve with the extrema only
    p = pf.step_params(ts)
    tb = pf.step_tables(ts)
    t = type(tb).from_buffer_copy(tb)
    if hasattr(tb, "_od_ref"):
        t._od_ref = tb._od_ref
    mn = torch.full((n,), -1.0, dtype=torch.float64, device=DEV)
    mx = torch.full((n,), -1.0, dtype=torch.float64, device=DEV)
    t.v_min_out, t.v_max_out = mn.data_ptr(), mx.data_ptr()
    cp = torch.stack([T(p_np[k]) for k in pf._ctrl_names])
    fn = _lib.lib().pgw_pf_solve_general if pf.general else _lib.lib().pgw_pf_solve
    _lib.check(fn(p, t, n, cp.data_ptr(), None, None, None, _lib.stream_ptr(DEV)))
    assert torch.equal(mn, lo) and torch.equal(mx, hi)


def test_pf_predictor_vs_oracle_and_cold_start():
    """Single controllable load: the per-hour predictor grid (warm start) must
    converge to the oracle's fixed point -- inside the grid, across band kinks and
    outside it (extrapolated stencil) -- and agree with the cold start."""
    from oracle.pf_oracle import BatchedPF
    from powergridworld_amd.distribution_system.opendss import OpenDSSSolver
    n = 2048
    rng = np.random.default_rng(5)
    mk = lambda pred: OpenDSSSolver("ieee_13_dss/IEEE13Nodeckt.dss",
                                    "ieee_13_dss/annual_hourly_load_profile.csv",
                                    system_load_rescale_factor=1.2, num_envs=n, device=DEV,
                                    predictor=pred, convergence="exact")
    warm, cold = mk(True), mk(False)
    orc = BatchedPF(system_load_rescale_factor=1.2)
    for ts in ["2021-08-12 01:00", "2021-08-12 14:00", "2021-08-12 15:00", "2021-08-12 18:00"]:
        p675 = np.concatenate([rng.uniform(0, 1000, n - 64), rng.uniform(-3000, 5000, 64)])
        want = orc.calculate(ts, {"675c": p675}, K=n)
        # past ~4.5 MW on one phase the fixed point barely contracts and the
        # oracle stops at max_iter unconverged: compare converged envs only
        ok = orc.last_iters < 100
        assert ok[:n - 64].all() and ok.sum() > n - 32
        for pf in (warm, cold):
            pf.calculate_power_flow({"675c": T(p675)}, {}, current_time=ts)
            v = pf.get_bus_voltages()
            got = np.stack([N(v[name]) for name in orc.feeder.node_names], 1)
            np.testing.assert_allclose(got[ok], want[ok], rtol=1e-9, atol=0)
        it_w, it_c = N(warm.iterations), N(cold.iterations)
        assert np.median(it_w[:n - 64]) < np.median(it_c) / 2, (np.median(it_w), np.median(it_c))


# ------------------------------------------------------------------ C4 (coordinated)
# golden of each power-flow rule: the reference's MultiAgentEnv over the oracle PF
# with OpenDSS's snap rule (the reference's, the default) or the fixed point
GOLD_SUFFIX = {"opendss": "_od", "exact": ""}


@pytest.mark.parametrize("semantics", ["opendss", "exact"])
@pytest.mark.parametrize("fused", [True, False])
def test_c4_golden(fused, semantics):
    from powergridworld_amd.scenarios.coordinated import (CoordinatedMultiBuildingControlEnv,
                                                          make_c4_config)
    g = load("c4_coordinated" + GOLD_SUFFIX[semantics])
    Tn, NA, K, _ = g["actions"].shape
    env = CoordinatedMultiBuildingControlEnv(**make_c4_config(pf_convergence=semantics), num_envs=K, device=DEV,
                                             fused=fused)
    assert (env._fused is not None) == fused
    env.reset()
    for a, agent in enumerate(env.agents):
        agent.env_dict["storage"].reset(init_storage=T(g["init_storage"][a]))
    obs0 = torch.stack([torch.cat([agent.get_obs()[0][c] for c in ("building", "pv", "storage")], 1)
                        for agent in env.agents])
    close(obs0, g["obs"][0], 1e-10, 1e-10)
    close(env.pf_solver.get_bus_voltage_by_name("675c"), g["v675"][0], 1e-8, 0)
    names = [a.name for a in env.agents]
    for t in range(Tn):
        if fused:
            obs, rew, dones, meta = env.step(T(g["actions"][t]))
            got_obs = env.packed_obs()
        else:
            act = {nm: {"building": T(g["actions"][t, a, :, :6]), "pv": T(g["actions"][t, a, :, 6:7]),
                        "storage": T(g["actions"][t, a, :, 7:8])} for a, nm in enumerate(names)}
            obs, rew, dones, meta = env.step(act)
            got_obs = torch.stack([torch.cat([obs[nm][c] for c in ("building", "pv", "storage")], 1)
                                   for nm in names])
        close(got_obs, g["obs"][t + 1], 1e-10, 1e-10)
        close(torch.stack([rew[nm] for nm in names]), g["reward"][t], 1e-7, 1e-7)
        close(meta["voltage_violation"], g["voltage_violation"][t], 1e-8, 1e-11)
        close(env.pf_solver.get_bus_voltage_by_name("675c"), g["v675"][t + 1], 1e-8, 0)
        assert dones["__all__"] == bool(g["done"][t, 0])


@pytest.mark.parametrize("semantics", ["opendss", "exact"])
def test_c4_fused_equals_generic_full_batch(semantics):
    """Size-independent property at the BASELINE batch (65,536): the one-kernel
    fused step and the generic per-component path are bit-identical."""
    from powergridworld_amd.scenarios.coordinated import (CoordinatedMultiBuildingControlEnv,
                                                          make_c4_config)
    n = 65536
    envs = [CoordinatedMultiBuildingControlEnv(**make_c4_config(pf_convergence=semantics), num_envs=n, device=DEV,
                                               fused=f) for f in (True, False)]
    init = torch.rand((5, n), dtype=torch.float64, device=DEV, generator=torch.Generator(DEV).manual_seed(1)) * 50
    for e in envs:
        e.reset()
        for a, agent in enumerate(e.agents):
            agent.env_dict["storage"].reset(init_storage=init[a])
    gen = torch.Generator(DEV).manual_seed(2)
    names = [a.name for a in envs[0].agents]
    for t in range(4):
        act = torch.rand((5, n, 8), dtype=torch.float64, device=DEV, generator=gen) * 2.2 - 1.1
        _, r_f, d_f, m_f = envs[0].step(act)
        o_f = envs[0].packed_obs().clone()
        dict_act = {nm: {"building": act[a, :, :6], "pv": act[a, :, 6:7], "storage": act[a, :, 7:8]}
                    for a, nm in enumerate(names)}
        o_g, r_g, d_g, m_g = envs[1].step(dict_act)
        o_g = torch.stack([torch.cat([o_g[nm][c] for c in ("building", "pv", "storage")], 1)
                           for nm in names])
        assert torch.equal(o_f, o_g)
        for nm in names:
            assert torch.equal(r_f[nm], r_g[nm])
        assert torch.equal(m_f["voltage_violation"], m_g["voltage_violation"])
        assert d_f == d_g




@pytest.mark.parametrize("semantics", ["opendss", "exact"])
def test_c4_batch_one_and_ragged(semantics):
    """Batch 1 and a batch that is not a multiple of the 256-thread block."""
    from powergridworld_amd.scenarios.coordinated import (CoordinatedMultiBuildingControlEnv,
                                                          make_c4_config)
    from oracle.ma_oracle import CoordinatedOracle
    from oracle.pf_oracle import BatchedPF
    for n in (1, 257):
        env = CoordinatedMultiBuildingControlEnv(**make_c4_config(pf_convergence=semantics), num_envs=n,
                                                 device=DEV)
        rng = np.random.default_rng(n)
        init = rng.uniform(3, 50, (5, n))
        env.reset()
        for a, agent in enumerate(env.agents):
            agent.env_dict["storage"].reset(init_storage=T(init[a]))
        orc = CoordinatedOracle(n)
        orc.pf = BatchedPF(system_load_rescale_factor=1.2, semantics=semantics)
        orc.reset(init)
        for t in range(5):
            act = rng.uniform(-1, 1, (5, n, 8))
            _, rew, _, meta = env.step(T(act))
            o, r, vv = orc.step(act)
            close(env.packed_obs(), o, 1e-10, 1e-10)
            close(torch.stack([rew[a.name] for a in env.agents]), r, 1e-7, 1e-7)


# ------------------------------------------------------------------ heterogeneous
@pytest.mark.parametrize("semantics", ["opendss", "exact"])
@pytest.mark.parametrize("fused", ["auto", False])
def test_heterogeneous_scenario_golden(fused, semantics):
    """The reference's 3-agent heterogeneous scenario (MC building, grid-aware
    PV farm rewarded on min_voltage, EV 25x40) on the fused multi-agent path
    (pgw_ma_step, the default) and the generic path, against the reference run
    (tests/golden/het_scenario{_od}.npz, PF = the oracle behind the reference's
    PowerFlowSolver ABC with OpenDSS's rule or the fixed point), a whole
    286-step episode."""
    from powergridworld_amd.multiagent_env import MultiAgentEnv
    from powergridworld_amd.scenarios.heterogeneous import make_env_config
    g = load("het_scenario" + GOLD_SUFFIX[semantics])
    Tn, K, _ = g["actions"].shape
    env = MultiAgentEnv(**make_env_config(pf_convergence=semantics), num_envs=K, device=DEV, fused=fused)
    assert env._fused is None
    assert (env._ma is not None) == (fused == "auto")
    env.reset()
    bld = env.agent_dict["building"]
    bld.env_dict["storage"].reset(init_storage=T(g["init_storage"]))

    def flat(o):
        return torch.cat([o["building"]["building"], o["building"]["pv"], o["building"]["storage"],
                          o["pv"], o["ev-charging"]], 1)

    close(flat(env.get_obs()), g["obs"][0], 1e-10, 1e-10)
    names = [str(x) for x in g["node_names"]]
    volts = lambda: torch.stack([env.pf_solver.get_bus_voltages()[nm] for nm in names], 1)
    close(volts(), g["voltages"][0], 1e-9, 0)
    for t in range(Tn):
        a = T(g["actions"][t])
        act = {"building": {"building": a[:, :6], "pv": a[:, 6:7], "storage": a[:, 7:8]},
               "pv": a[:, 8:9], "ev-charging": a[:, 9:10]}
        obs, rew, dones, _ = env.step(act)
        close(flat(obs), g["obs"][t + 1], 1e-9, 1e-9)
        close(volts(), g["voltages"][t + 1], 1e-9, 0)
        close(torch.stack([rew[nm] for nm in ("building", "pv", "ev-charging")], 1), g["reward"][t],
              1e-7, 1e-7)
        assert dones["__all__"] == bool(g["done"][t, 0])


def _het_actions(rng, n, T_):
    """Seeded uniform actions, 20 % pushed past the box (the kernels clip them)."""
    a = rng.uniform(-1.2, 1.2, size=(T_, n, 10))
    return torch.tensor(a, device=DEV)


def _het_act(a):
    return {"building": {"building": a[:, :6], "pv": a[:, 6:7], "storage": a[:, 7:8]},
            "pv": a[:, 8:9], "ev-charging": a[:, 9:10]}


@pytest.mark.parametrize("record_history,n,semantics", [(False, 4096, "opendss"), (True, 4096, "opendss"),
                                                        (False, 1000, "opendss"), (False, 1, "opendss"),
                                                        (False, 4096, "exact"), (True, 1000, "exact")])
def test_het_multiagent_step_equals_generic(record_history, n, semantics):
    """pgw_ma_step (the heterogeneous scenario's fused path: every agent's
    components in one launch, the per-bus sums, the power flow with the
    extrema epilogue) against the generic per-agent path, bit for bit, over a
    whole episode and across the reset into a second one, at 4 096 envs:
    observations, rewards, dones, real powers, min/max voltage, iterations and
    every node voltage (solved on first access on the fused path, or written
    into the history ring); also at a ragged batch (1000: a partial last block)
    and at batch 1."""
    from powergridworld_amd.multiagent_env import MultiAgentEnv
    from powergridworld_amd.scenarios.heterogeneous import make_env_config
    envs = [MultiAgentEnv(**make_env_config(pf_convergence=semantics), num_envs=n, device=DEV, fused=f,
                          record_history=record_history) for f in ("auto", False)]
    assert envs[0]._ma is not None and envs[1]._ma is None
    rng = np.random.default_rng(11)
    acts = _het_actions(rng, n, 300)
    soc0 = T(rng.uniform(5.0, 240.0, size=n))

    def flat(o):
        return torch.cat([o["building"]["building"], o["building"]["pv"], o["building"]["storage"],
                          o["pv"], o["ev-charging"]], 1)

    nodes = envs[0].pf_solver.feeder.node_names
    t_act = 0
    for ep in range(2):
        outs = []
        for env in envs:
            env.reset()
            env.agent_dict["building"].env_dict["storage"].reset(init_storage=soc0)
            outs.append(flat(env.get_obs()))
        assert torch.equal(outs[0], outs[1])
        steps = 0
        while True:
            res = [env.step(_het_act(acts[t_act % len(acts)])) for env in envs]
            (o0, r0, d0, m0), (o1, r1, d1, m1) = res
            assert torch.equal(flat(o0), flat(o1))
            for nm in ("building", "pv", "ev-charging"):
                assert torch.equal(r0[nm], r1[nm]), nm
                assert torch.equal(envs[0].agent_dict[nm].real_power, envs[1].agent_dict[nm].real_power), nm
            assert d0 == d1
            e0, e1 = envs[0].pf_solver.voltage_extrema(), envs[1].pf_solver.voltage_extrema()
            assert torch.equal(e0[0], e1[0]) and torch.equal(e0[1], e1[1])
            assert torch.equal(envs[0].pf_solver.iterations, envs[1].pf_solver.iterations)
            if steps % 97 == 0 or d0["__all__"]:
                v0, v1 = envs[0].pf_solver.get_bus_voltages(), envs[1].pf_solver.get_bus_voltages()
                for x in nodes:
                    assert torch.equal(v0[x], v1[x]), x
            t_act += 1
            steps += 1
            if d0["__all__"] or (ep == 1 and steps == 5):
                break
    assert (envs[0].pf_solver.iterations > 0).all()
    if record_history:
        h0, h1 = envs[0].voltage_history(), envs[1].voltage_history()
        assert torch.equal(h0[0], h1[0]) and torch.equal(h0[1], h1[1]) and h0[2] == h1[2]


@pytest.mark.parametrize("semantics", ["opendss", "exact"])
def test_heterogeneous_golden_full_batch_tiled(semantics):
    """The heterogeneous golden's 2 reference trajectories tiled over 65 536 envs
    on the fused multi-agent path: every env reproduces its trajectory for the
    whole episode (obs incl. the PV farm's min_voltage, all three rewards, the
    done flags, and the node voltages at a few steps), compared on the device."""
    from powergridworld_amd.multiagent_env import MultiAgentEnv
    from powergridworld_amd.scenarios.heterogeneous import make_env_config
    g = load("het_scenario" + GOLD_SUFFIX[semantics])
    Tn, K, _ = g["actions"].shape
    n = 65536
    rep = n // K
    env = MultiAgentEnv(**make_env_config(pf_convergence=semantics), num_envs=n, device=DEV)
    assert env._ma is not None
    env.reset()
    env.agent_dict["building"].env_dict["storage"].reset(init_storage=T(np.tile(g["init_storage"], rep)))
    G_obs, G_rew = T(g["obs"]), T(g["reward"])
    names = [str(x) for x in g["node_names"]]

    def flat(o):
        return torch.cat([o["building"]["building"], o["building"]["pv"], o["building"]["storage"],
                          o["pv"], o["ev-charging"]], 1)

    def check(got, want, rtol, atol, what):
        want = want.unsqueeze(0).expand(rep, *want.shape).reshape(got.shape)
        bad = ~torch.isclose(got, want, rtol=rtol, atol=atol)
        assert not bool(bad.any()), "%s: %d mismatches" % (what, int(bad.sum()))

    check(flat(env.get_obs()), G_obs[0], 1e-10, 1e-10, "reset obs")
    acts = T(np.tile(g["actions"], (1, rep, 1)))
    for t in range(Tn):
        a = acts[t]
        act = {"building": {"building": a[:, :6], "pv": a[:, 6:7], "storage": a[:, 7:8]},
               "pv": a[:, 8:9], "ev-charging": a[:, 9:10]}
        obs, rew, dones, _ = env.step(act)
        check(flat(obs), G_obs[t + 1], 1e-9, 1e-9, "obs step %d" % t)
        check(torch.stack([rew[nm] for nm in ("building", "pv", "ev-charging")], 1), G_rew[t], 1e-7, 1e-7,
              "reward step %d" % t)
        assert dones["__all__"] == bool(g["done"][t, 0])
        if t % 95 == 0:
            v = torch.stack([env.pf_solver.get_bus_voltages()[nm] for nm in names], 1)
            check(v, T(g["voltages"][t + 1]), 1e-9, 0, "voltages step %d" % t)


# ------------------------------------------------------------------ Home-Steward house
def _hs_run(env, g, names, n_rep=1, meta_every=1):
    """Step `env` (batch K * n_rep, golden actions tiled) through the golden's
    two episodes; compare obs, reward, real power, done, meta and SoC."""
    A, O = g["actions"], g["obs"]
    K = A.shape[1]
    tile = lambda x: np.tile(x, (n_rep,) + (1,) * (x.ndim - 1))
    dims = [env.env_dict[n]._observation_space.shape[0] for n in names]
    flat = lambda o: torch.cat([o[n] for n in names], 1)
    t_obs, t_act = 0, 0
    for ep in range(int(g["episodes"])):
        o = env.reset()
        close(flat(o), tile(O[t_obs]), 1e-12, 1e-12)
        close(env.env_dict["storage"].current_storage, tile(g["soc"][t_obs]), 0, 0)
        t_obs += 1
        while True:
            a = tile(A[t_act])
            o, r, d, m = env.step({n: T(a[:, i:i + 1]) for i, n in enumerate(names)})
            close(flat(o), tile(O[t_obs]), 1e-12, 1e-12)
            close(r, tile(g["reward"][t_act]), 1e-12, 1e-12)
            close(env.real_power, tile(g["real_power"][t_act]), 1e-12, 1e-12)
            close(torch.stack([m["pv_power"], m["es_power"], m["grid_power"]], 1), tile(g["meta"][t_obs]),
                  1e-12, 1e-12)
            close(env.env_dict["storage"].current_storage, tile(g["soc"][t_obs]), 1e-12, 1e-12)
            if t_act % meta_every == 0:
                _hs_step_meta(m, g, t_act, names, tile)
            assert d == bool(g["done"][t_act, 0])
            t_obs += 1
            t_act += 1
            if d:
                break
    assert t_act == A.shape[0] and sum(dims) == O.shape[2]


def _hs_step_meta(m, g, t, names, tile):
    """meta["step_meta"] (base_hs.py:133-164) against the reference's records:
    device ids, timestamp, custom-info keys and every numeric field."""
    from powergridworld_amd.base_hs import HS_COMMON_FIELDS
    recs = m["step_meta"]
    assert [r["device_id"] for r in recs] == names
    want = tile(g["step_meta"][t])                    # [N, n_comp, 13]
    for c, r in enumerate(recs):
        assert r["timestamp"] == str(g["step_meta_timestamp"][t])
        keys = str(g["step_meta_custom_keys"][c]).split(",")
        assert list(r["device_custom_info"]) == keys
        got = [r[f] for f in HS_COMMON_FIELDS] + [r["device_custom_info"][k] for k in keys]
        close(torch.stack(got, 1), want[:, c, :len(got)], 1e-12, 1e-12)
        assert np.isnan(want[:, c, len(got):]).all()


def test_hs_house_golden_two_episodes():
    """The reference's Home-Steward house (HSMultiComponentEnv + the shipped
    JSON scenario) against the reference's own run: 4 envs, two 288-step
    episodes each (the battery's stored-energy cost and the meta_state es_power
    carried across reset), actions partly outside [-1, 1] and exact zeros."""
    from powergridworld_amd.base_hs import HSMultiComponentEnv
    from powergridworld_amd.scenarios.heterogeneous_hs import make_env_config
    g = load("hs_scenario")
    names = [str(x) for x in g["names"]]
    K = g["actions"].shape[1]
    env = HSMultiComponentEnv(**make_env_config(), num_envs=K, device=DEV)
    assert [e.name for e in env.envs] == names
    _hs_run(env, g, names)


def test_hs_house_reordered_grid_aware_golden():
    """The reference's house with the chain [PV (grid-aware), EV, devices,
    storage] and a min_voltage keyword at every reset / step (golden
    hs_order, oracle/make_golden.py gen_hs_order): the components' draws in
    that order, the grid-aware PV's min_voltage observation, the storage's
    reward over the resources the EV and devices left; 3 envs, two episodes."""
    from powergridworld_amd.base_hs import HSMultiComponentEnv
    from powergridworld_amd.scenarios.heterogeneous_hs import make_env_config
    g = load("hs_order")
    names = [str(x) for x in g["names"]]
    cfg = make_env_config()
    by = {c["name"]: c for c in cfg["components"]}
    cfg["components"] = [by[n] for n in names]
    by["pv"]["config"]["grid_aware"] = True
    A, O, MV = g["actions"], g["obs"], g["min_voltage"]
    K = A.shape[1]
    env = HSMultiComponentEnv(**cfg, num_envs=K, device=DEV, step_meta=False)
    flat = lambda o: torch.cat([o[n] for n in names], 1)
    t_obs, t_act = 0, 0
    for ep in range(int(g["episodes"])):
        o = env.reset(min_voltage=T(MV[t_obs]))
        close(flat(o), O[t_obs], 1e-12, 1e-12)
        t_obs += 1
        while True:
            a = A[t_act]
            o, r, d, m = env.step({n: T(a[:, i:i + 1]) for i, n in enumerate(names)}, min_voltage=T(MV[t_obs]))
            close(flat(o), O[t_obs], 1e-12, 1e-12)
            close(r, g["reward"][t_act], 1e-12, 1e-12)
            close(env.real_power, g["real_power"][t_act], 1e-12, 1e-12)
            close(torch.stack([m["pv_power"], m["es_power"], m["grid_power"]], 1), g["meta"][t_obs], 1e-12, 1e-12)
            close(env.env_dict["storage"].current_storage, g["soc"][t_obs], 1e-12, 1e-12)
            assert d == bool(g["done"][t_act, 0])
            t_obs += 1
            t_act += 1
            if d:
                break
    assert t_act == A.shape[0]
    fresh = HSMultiComponentEnv(**cfg, num_envs=K, device=DEV, step_meta=False)
    fresh.reset(min_voltage=1.0)
    with pytest.raises(KeyError, match="min_voltage"):      # the first step needs the keyword
        fresh.step({n: T(A[0][:, i:i + 1]) for i, n in enumerate(names)})


def test_hs_house_full_batch_tiled():
    """Size-independent property at 65 536 envs: envs are independent, so the
    golden's 4 trajectories tiled over the batch reproduce it everywhere."""
    from powergridworld_amd.base_hs import HSMultiComponentEnv
    from powergridworld_amd.scenarios.heterogeneous_hs import make_env_config
    g = load("hs_scenario")
    names = [str(x) for x in g["names"]]
    K = g["actions"].shape[1]
    env = HSMultiComponentEnv(**make_env_config(), num_envs=65536, device=DEV)
    _hs_run(env, g, names, n_rep=65536 // K, meta_every=37)


# ------------------------------------------------------------------ list interface
def test_list_interface_fused_zero_copy_equals_dict():
    """MultiAgentListInterfaceEnv over C4: on the fused path the per-agent
    observations are views of the packed buffer (no copy), and list actions give
    the same obs / rewards / dones as the dict API of a second engine."""
    from powergridworld_amd import MultiAgentListInterfaceEnv
    from powergridworld_amd.scenarios.coordinated import (CoordinatedMultiBuildingControlEnv,
                                                          make_c4_config)
    n = 1024
    cfg = make_c4_config()
    le = MultiAgentListInterfaceEnv(CoordinatedMultiBuildingControlEnv,
                                    dict(cfg, num_envs=n, device=torch.device(DEV)))
    de = CoordinatedMultiBuildingControlEnv(**cfg, num_envs=n, device=DEV)
    assert le.ma_env._fused is not None and le._packed()
    init = torch.rand((5, n), dtype=torch.float64, device=DEV, generator=torch.Generator(DEV).manual_seed(9)) * 40 + 5
    lo = le.reset()
    de.reset()
    for a, (la, da) in enumerate(zip(le.ma_env.agents, de.agents)):
        la.env_dict["storage"].reset(init_storage=init[a])
        da.env_dict["storage"].reset(init_storage=init[a])
    lo = le.convert_to_list_obs(None)
    packed = le.ma_env.packed_obs()
    assert all(o.data_ptr() == packed[i].data_ptr() for i, o in enumerate(lo))
    assert [s.shape[0] for s in le.observation_space] == [17] * 5
    assert [s.shape[0] for s in le.action_space] == [8] * 5
    gen = torch.Generator(DEV).manual_seed(10)
    names = [a.name for a in de.agents]
    for t in range(6):
        act = [torch.rand((n, 8), dtype=torch.float64, device=DEV, generator=gen) * 2 - 1 for _ in range(5)]
        lo, lr, ld, _ = le.step(act)
        do, dr, dd, _ = de.step({nm: {"building": act[i][:, :6], "pv": act[i][:, 6:7], "storage": act[i][:, 7:8]}
                                 for i, nm in enumerate(names)})
        for i, nm in enumerate(names):
            want = torch.cat([do[nm][c] for c in ("building", "pv", "storage")], 1)
            assert torch.equal(lo[i], want)
            assert torch.equal(lr[i], dr[nm])
            assert ld[i] == dd[nm]


# ------------------------------------------------------------------ fused MC agent step
@pytest.mark.parametrize("randomize", [False, True])
def test_mc_fused_equals_generic_c3(randomize):
    """pgw_mc_agent_step (the whole building + PV + storage + EV agent in one
    launch) against the per-component kernels + reduce, bit for bit, at the C3
    batch; the golden test above already runs the fused path.  randomize: the
    EV draws per-env vehicle subsets (both envs seeded alike)."""
    from powergridworld_amd import MultiComponentEnv
    from powergridworld_amd.agents import EnergyStorageEnv, EVChargingEnv, FiveZoneROMThermalEnergyEnv, PVEnv
    n = 16384
    comps = [
        {"name": "building", "cls": FiveZoneROMThermalEnergyEnv, "config": {}},
        {"name": "pv", "cls": PVEnv, "config": {"profile_csv": "pv_profile.csv", "scaling_factor": 40.}},
        {"name": "storage", "cls": EnergyStorageEnv, "config": {}},
        {"name": "ev", "cls": EVChargingEnv,
         "config": dict(num_vehicles=100, minutes_per_step=5, max_charge_rate_kw=7.,
                        peak_threshold=250., vehicle_multiplier=5., rescale_spaces=True,
                        randomize=randomize)},
    ]
    fused, generic = [MultiComponentEnv(name="mc", components=comps, num_envs=n, device=DEV) for _ in range(2)]
    generic._mc_fuse = False
    assert fused._mc_fusable()
    init = torch.rand(n, dtype=torch.float64, device=DEV, generator=torch.Generator(DEV).manual_seed(11)) * 60
    for e in (fused, generic):
        if randomize:
            e.env_dict["ev"].seed(5)
        e.reset(init_storage=init)
    if randomize:
        assert torch.equal(fused.env_dict["ev"].vehicle_ids, generic.env_dict["ev"].vehicle_ids)
    gen = torch.Generator(DEV).manual_seed(12)
    dims = {"building": 6, "pv": 1, "storage": 1, "ev": 1}
    for t in range(40):
        act = {c: torch.rand((n, d), dtype=torch.float64, device=DEV, generator=gen) * 2.4 - 1.2
               for c, d in dims.items()}
        of, rf, df, _ = fused.step(act)
        og, rg, dg, _ = generic.step(act)
        for c in dims:
            assert torch.equal(of[c], og[c]), c
            assert torch.equal(fused.env_dict[c].real_power, generic.env_dict[c].real_power), c
        assert torch.equal(rf, rg) and torch.equal(fused.real_power, generic.real_power)
        assert df == dg


# ------------------------------------------------------------------ voltage history
@pytest.mark.parametrize("semantics", ["opendss", "exact"])
def test_history_ring_fused_and_generic(semantics):
    """record_history=True: the on-device ring holds every node's voltage and
    every agent's power per step (the reference's self.history,
    multiagent_env.py:129, 191-194).  Fused (kernels write the slot) and generic
    (solver bound to the slot) agree bit for bit, recording does not change the
    step results, and the ring wraps at its capacity."""
    from powergridworld_amd.scenarios.coordinated import (CoordinatedMultiBuildingControlEnv,
                                                          make_c4_config)
    n, steps = 1000, 12
    mk = lambda **kw: CoordinatedMultiBuildingControlEnv(**make_c4_config(pf_convergence=semantics), num_envs=n,
                                                         device=DEV, **kw)
    envs = [mk(fused=True, record_history=True), mk(fused=False, record_history=True),
            mk(fused=True), mk(fused=True, record_history=True, history_capacity=5)]
    init = torch.rand((5, n), dtype=torch.float64, device=DEV, generator=torch.Generator(DEV).manual_seed(4)) * 50
    for e in envs:
        e.reset()
        for a, agent in enumerate(e.agents):
            agent.env_dict["storage"].reset(init_storage=init[a])
    names = [a.name for a in envs[0].agents]
    gen = torch.Generator(DEV).manual_seed(6)
    nodes = envs[1].pf_solver.feeder.node_names
    for t in range(steps):
        act = torch.rand((5, n, 8), dtype=torch.float64, device=DEV, generator=gen) * 2 - 1
        dict_act = {nm: {"building": act[a, :, :6], "pv": act[a, :, 6:7], "storage": act[a, :, 7:8]}
                    for a, nm in enumerate(names)}
        outs = [e.step(act if e._fused is not None else dict_act) for e in envs]
        for o in outs[1:]:
            for nm in names:
                assert torch.equal(outs[0][1][nm], o[1][nm])
        hf, hg = envs[0].history, envs[1].history
        assert list(hf["voltage"][t].keys()) == list(nodes) == list(hg["voltage"][t].keys())
        for x in nodes:
            assert torch.equal(hf["voltage"][t][x], hg["voltage"][t][x]), x
        for a in range(5):
            assert torch.equal(hf["agent_power_p"][t][a], hg["agent_power_p"][t][a])
        # the solver and env views follow the newest slot
        assert torch.equal(envs[0].pf_solver.get_bus_voltage_by_name("675c"),
                           envs[2].pf_solver.get_bus_voltage_by_name("675c"))
        assert torch.equal(envs[0].voltages["675.3"], hf["voltage"][t]["675.3"])
    v, p, vn = envs[0].voltage_history()
    assert tuple(v.shape) == (steps, len(nodes), n) and tuple(p.shape) == (steps, 5, n) and vn == list(nodes)
    for t in (0, steps - 1):
        assert torch.equal(v[t, vn.index("675.3")], envs[0].history["voltage"][t]["675.3"])
    v5, p5, _ = envs[3].voltage_history()          # wrapped: the last 5 steps in order
    assert tuple(v5.shape) == (5, len(nodes), n)
    assert torch.equal(v5, v[-5:]) and torch.equal(p5, p[-5:])
    vg, pg, _ = envs[1].voltage_history()
    assert torch.equal(vg, v) and torch.equal(pg, p)


@pytest.mark.parametrize("semantics", ["opendss", "exact"])
def test_fused_voltages_on_demand_only(semantics):
    """The fused step writes only the rows it needs; the all-node solve runs
    only when a caller reads another node (never on the step / reset path)."""
    from powergridworld_amd.scenarios.coordinated import (CoordinatedMultiBuildingControlEnv,
                                                          make_c4_config)
    n = 300
    cfg = make_c4_config(pf_convergence=semantics)
    env = CoordinatedMultiBuildingControlEnv(**cfg, num_envs=n, device=DEV, fused=True)
    ref = CoordinatedMultiBuildingControlEnv(**cfg, num_envs=n, device=DEV, fused=False)
    init = torch.rand((5, n), dtype=torch.float64, device=DEV, generator=torch.Generator(DEV).manual_seed(8)) * 50
    for e in (env, ref):
        e.reset()
        for a, agent in enumerate(e.agents):
            agent.env_dict["storage"].reset(init_storage=init[a])
    gen = torch.Generator(DEV).manual_seed(9)
    names = [a.name for a in env.agents]
    for t in range(3):
        act = torch.rand((5, n, 8), dtype=torch.float64, device=DEV, generator=gen) * 2 - 1
        env.step(act)
        ref.step({nm: {"building": act[a, :, :6], "pv": act[a, :, 6:7], "storage": act[a, :, 7:8]}
                  for a, nm in enumerate(names)})
    env.reset()
    ref.reset()
    for a, agent in enumerate(env.agents):
        agent.env_dict["storage"].reset(init_storage=init[a])
        ref.agents[a].env_dict["storage"].reset(init_storage=init[a])
    act = torch.rand((5, n, 8), dtype=torch.float64, device=DEV, generator=gen) * 2 - 1
    env.step(act)
    ref.step({nm: {"building": act[a, :, :6], "pv": act[a, :, 6:7], "storage": act[a, :, 7:8]}
              for a, nm in enumerate(names)})
    assert "_pf_full" not in env.__dict__
    assert torch.equal(env.voltages["675.3"], ref.voltages["675.3"])
    assert "_pf_full" not in env.__dict__                  # a row the kernel wrote
    got = env.pf_solver.get_bus_voltages()
    assert list(got.keys()) == list(ref.voltages.keys())
    for x in ref.voltages:
        assert torch.equal(got[x], ref.voltages[x]), x        # the on-demand rows: bit-identical
    assert "_pf_full" in env.__dict__


def test_pf_warm_start_multi_bus():
    """OpenDSSSolver(warm_start=True), for layouts without a predictor table (two
    controllable buses): every env's solve starts from its previous solution, as
    OpenDSS's snap solve does (opendss.py:134).  Same fixed point as the cold
    start (rtol 1e-9 on every node over 40 steps), in fewer iterations."""
    from powergridworld_amd.distribution_system.opendss import OpenDSSSolver
    n = 4096
    kw = dict(feeder_file="ieee_13_dss/IEEE13Nodeckt.dss",
              loadshape_file="ieee_13_dss/annual_hourly_load_profile.csv",
              system_load_rescale_factor=0.7, num_envs=n, device=DEV, convergence="exact")
    cold, warm = OpenDSSSolver(**kw), OpenDSSSolver(**kw, warm_start=True)
    rng = np.random.default_rng(21)
    base = rng.uniform(0, 400, size=(2, n))
    it_c, it_w = [], []
    for t in range(40):
        p = base + rng.normal(0, 15, size=(2, n))            # loads drift step to step
        loads = {"675c": T(p[0]), "671": T(p[1])}
        time = "2020-08-12 %02d:%02d:00" % (t // 12, 5 * (t % 12))
        for s_, its in ((cold, it_c), (warm, it_w)):
            s_.calculate_power_flow(p_controllable_consumed=loads, current_time=time)
            its.append(float(s_.iterations.double().mean()))
        assert cold.unconverged() == 0 and warm.unconverged() == 0
        vc, vw = cold.get_bus_voltages(), warm.get_bus_voltages()
        for x in cold.feeder.node_names:
            close(vw[x], N(vc[x]), 1e-9, 0)
    assert it_w[0] == it_c[0]                                 # the first solve starts cold
    assert np.mean(it_w[1:]) < np.mean(it_c[1:]) - 1.0, (np.mean(it_w[1:]), np.mean(it_c[1:]))


@pytest.mark.parametrize("randomize", [False, True])
def test_mc_ev_split_walk_equals_one_lane_walk(randomize):
    """k_mc_step's EV walk split over kEvGroups waves (pgw_mc_ev_split_mode(1);
    the default splits below 257 blocks on steps of 2+ chunks) against the same
    kernel with the walk in one lane (pgw_mc_ev_split_mode(0)) and against
    the generic k_ev_step, bit for bit, over a whole episode of 300 vehicles (5
    scan words, up to ~40 chunks: every group boundary and word-crossing case)."""
    from powergridworld_amd import MultiComponentEnv, _lib
    from powergridworld_amd.agents import EnergyStorageEnv, EVChargingEnv
    n = 2048
    comps = [
        {"name": "storage", "cls": EnergyStorageEnv, "config": {}},
        {"name": "ev", "cls": EVChargingEnv,
         "config": dict(num_vehicles=300, minutes_per_step=5, max_charge_rate_kw=7.,
                        peak_threshold=250., vehicle_multiplier=5., rescale_spaces=True,
                        randomize=randomize)},
    ]
    split, lane, generic = [MultiComponentEnv(name="mc", components=comps, num_envs=n, device=DEV)
                            for _ in range(3)]
    generic._mc_fuse = False
    assert split._mc_fusable()
    init = torch.rand(n, dtype=torch.float64, device=DEV, generator=torch.Generator(DEV).manual_seed(3)) * 60
    for e in (split, lane, generic):
        if randomize:
            e.env_dict["ev"].seed(7)
        e.reset(init_storage=init)
    gen = torch.Generator(DEV).manual_seed(13)
    for t in range(400):
        act = {"storage": torch.rand((n, 1), dtype=torch.float64, device=DEV, generator=gen) * 2 - 1,
               "ev": torch.rand((n, 1), dtype=torch.float64, device=DEV, generator=gen) * 2.4 - 1.2}
        try:
            _lib.check(_lib.lib().pgw_mc_ev_split_mode(1, None))
            os_ = split.step(act)
            _lib.check(_lib.lib().pgw_mc_ev_split_mode(0, None))
            ol = lane.step(act)
        finally:
            _lib.check(_lib.lib().pgw_mc_ev_split_mode(-1, None))
        og = generic.step(act)
        for o in (ol, og):
            for c in ("storage", "ev"):
                assert torch.equal(os_[0][c], o[0][c]), (t, c)
            assert torch.equal(os_[1], o[1]), t
            assert os_[2] == o[2]
        for e in (lane, generic):
            assert torch.equal(split.env_dict["ev"].real_power, e.env_dict["ev"].real_power), t
        if os_[2]:
            break
    assert t > 250, t                                     # a whole episode
