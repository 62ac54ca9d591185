"""The EV's integer outputs at the full batch, every kernel that walks the
vehicles.  A dropped round-3 build (lanes over vehicles,
profiles/r03/ev_lanes_rebuild.patch) returned num_active_vehicles = 0 in
37-62 % of the envs at 65,536, varying run to run; DESIGN.md section 4 item 5
records what was found.  These tests pin the live kernels: at 65,536 envs
(64 oracle envs tiled) every env's vehicle count -- obs column 1, the
reference's num_active_vehicles * multiplier (ev_charging_env.py:186-247,
253-254) -- must equal the oracle's bit for bit at every step of a whole
episode, and the other EV outputs within 1e-12.  Paths: the standalone
k_ev_step, k_mc_step's one-lane and split walks, and the heterogeneous
scenario's k_ma_step.  Needs an MI355X."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
N_ENVS, K = 65536, 64
HET_EV = dict(num_vehicles=25, minutes_per_step=5, max_charge_rate_kw=7., peak_threshold=200.,
              vehicle_multiplier=40., rescale_spaces=True)
C3_EV = dict(num_vehicles=100, minutes_per_step=5, max_charge_rate_kw=7., peak_threshold=250.,
             vehicle_multiplier=5., rescale_spaces=True)


def _episode(step_fn, cfg, seed, check_done=True):
    """Run one episode: step_fn(action [N, 1] tensor) -> (EV obs [N, 6], EV real power [N],
    done); compare with EVOracle on the K distinct action streams tiled over N."""
    from oracle.pgw_oracle import EVOracle
    orc = EVOracle(K, **cfg)
    orc.reset()
    idx = torch.arange(N_ENVS, device=DEV) % K
    rng = np.random.default_rng(seed)
    bad_count = torch.zeros((), dtype=torch.int64, device=DEV)
    worst = torch.zeros((), dtype=torch.float64, device=DEV)
    steps, done = 0, False
    while not done:
        a = rng.uniform(-1.2, 1.2, (K, 1))
        obs, rp, done = step_fn(torch.tensor(a, device=DEV)[idx])
        o, _, d, _ = orc.step(a)
        want = torch.tensor(o, device=DEV)[idx]
        bad_count += (obs[:, 1] != want[:, 1]).sum()
        rel = ((obs - want).abs() / (1e-12 + 1e-12 * want.abs())).max()
        rel_p = ((rp - torch.tensor(orc.real_power, device=DEV)[idx]).abs() /
                 (1e-12 + 1e-12 * torch.tensor(np.abs(orc.real_power), device=DEV)[idx])).max()
        worst = torch.maximum(worst, torch.maximum(rel, rel_p))
        if check_done:
            assert done == bool(d[0])
        done = done or bool(d[0])
        steps += 1
    assert steps > 250, steps
    assert int(bad_count) == 0, "num_active_vehicles differs in %d env-steps" % int(bad_count)
    assert float(worst) <= 1.0, float(worst)


@pytest.mark.parametrize("cfg", [HET_EV, C3_EV], ids=["v25", "v100"])
def test_ev_step_counts_full_batch(cfg):
    from powergridworld_amd.agents import EVChargingEnv
    env = EVChargingEnv(num_envs=N_ENVS, device=DEV, **cfg)
    env.reset()

    def step(a):
        obs, _, d, _ = env.step(a)
        return obs, env.real_power, d
    _episode(step, cfg, 1)


@pytest.mark.parametrize("split", [-1, 1])
def test_mc_ev_counts_full_batch(split):
    """k_mc_step at 65,536 envs: the one-lane walk (automatic: 1,024 blocks) and
    the walk split over 4 waves (forced)."""
    from powergridworld_amd import MultiComponentEnv, _lib
    from powergridworld_amd.agents import EnergyStorageEnv, EVChargingEnv
    comps = [{"name": "storage", "cls": EnergyStorageEnv, "config": {}},
             {"name": "ev", "cls": EVChargingEnv, "config": C3_EV}]
    env = MultiComponentEnv(name="mc", components=comps, num_envs=N_ENVS, device=DEV)
    assert env._mc_fusable()
    env.reset(init_storage=torch.full((N_ENVS,), 20.0, dtype=torch.float64, device=DEV))
    zero = torch.zeros((N_ENVS, 1), dtype=torch.float64, device=DEV)

    def step(a):
        obs, _, d, _ = env.step({"storage": zero, "ev": a})
        return obs["ev"], env.env_dict["ev"].real_power, d
    _lib.check(_lib.lib().pgw_mc_ev_split_mode(split, None))
    try:
        _episode(step, C3_EV, 2)
    finally:
        _lib.check(_lib.lib().pgw_mc_ev_split_mode(-1, None))


def test_het_ev_counts_full_batch():
    """The heterogeneous scenario's fused step (k_ma_step: the EV agent on its own
    wave) at 65,536 envs."""
    from powergridworld_amd.multiagent_env import MultiAgentEnv
    from powergridworld_amd.scenarios.heterogeneous import make_env_config
    env = MultiAgentEnv(**make_env_config(), num_envs=N_ENVS, device=DEV)
    env.reset()
    assert env._ma is not None
    g = torch.Generator(DEV).manual_seed(4)
    ev = env.agent_dict["ev-charging"]

    def step(a):
        o = torch.rand((N_ENVS, 9), dtype=torch.float64, device=DEV, generator=g) * 2 - 1
        act = {"building": {"building": o[:, :6], "pv": o[:, 6:7], "storage": o[:, 7:8]}, "pv": o[:, 8:9],
               "ev-charging": a}
        obs, _, d, _ = env.step(act)
        return obs["ev-charging"], ev.real_power, d["__all__"]
    _episode(step, HET_EV, 3, check_done=False)
