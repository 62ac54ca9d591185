"""Out-of-bounds action counter (PGW_OOB, include/pgw.h).  The reference's
to_raw warns whenever a rescaled action leaves [-1 - 1e-4, 1 + 1e-4] and clips
it (gridworld/utils.py:35-40); the kernels count those warnings on the device,
one per (env, component, step).  Expected counts are computed here from the
actions with the reference's own condition.  Needs an MI355X."""
import logging

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
EPS = 1e-4


def bad(a):
    """utils.py:36 -- per element: not (a >= -1 - eps and a <= 1 + eps)."""
    a = np.asarray(a)
    return ~((a >= -np.ones_like(a) - EPS) & (a <= np.ones_like(a) + EPS))


def actions(rng, shape):
    """Mostly inside the box; some within eps of it (no warning), some past it."""
    a = rng.uniform(-1, 1, shape)
    r = rng.random(shape)
    a[r < 0.05] = 1.0 + 0.5 * EPS
    a[(r >= 0.05) & (r < 0.10)] = -1.0 - 0.5 * EPS
    a[(r >= 0.10) & (r < 0.15)] *= 1.3
    a[(r >= 0.15) & (r < 0.17)] = -1.0 - 2 * EPS
    return a


def count(env):
    return int(env.oob_actions().item())


def test_oob_battery_standalone_and_no_rescale():
    from powergridworld_amd.agents import EnergyStorageEnv
    n, steps = 4096, 40
    rng = np.random.default_rng(1)
    env = EnergyStorageEnv(num_envs=n, device=DEV)
    env.reset()
    want = 0
    for _ in range(steps):
        a = actions(rng, (n, 1))
        env.step(torch.tensor(a, device=DEV))
        want += int(bad(a).sum())
    assert want > 0 and count(env) == want
    # rescale_spaces=False: no to_raw, hence no warning (energy_storage_env.py:136)
    raw = EnergyStorageEnv(num_envs=n, device=DEV, rescale_spaces=False)
    raw.reset()
    raw.step(torch.full((n, 1), 3.0, dtype=torch.float64, device=DEV))
    assert count(raw) == 0


@pytest.mark.parametrize("randomize", [False, True])
def test_oob_mc_c3_fused_and_generic(randomize):
    """C3 agent: one count per component whose action vector has any element
    past the bound (the building's six elements are one to_raw call)."""
    from powergridworld_amd import MultiComponentEnv
    from powergridworld_amd.agents import EnergyStorageEnv, EVChargingEnv, FiveZoneROMThermalEnergyEnv, PVEnv
    n, steps = 2048, 12
    comps = [
        {"name": "building", "cls": FiveZoneROMThermalEnergyEnv, "config": {}},
        {"name": "pv", "cls": PVEnv, "config": {"profile_csv": "pv_profile.csv", "scaling_factor": 40.}},
        {"name": "storage", "cls": EnergyStorageEnv, "config": {}},
        {"name": "ev", "cls": EVChargingEnv,
         "config": dict(num_vehicles=100, minutes_per_step=5, max_charge_rate_kw=7., peak_threshold=250.,
                        vehicle_multiplier=5., rescale_spaces=True, randomize=randomize)},
    ]
    fused, generic = [MultiComponentEnv(name="mc", components=comps, num_envs=n, device=DEV) for _ in range(2)]
    generic._mc_fuse = False
    assert fused._mc_fusable()
    for e in (fused, generic):
        e.reset()
        assert all(c.oob_count is e.oob_count for c in e.envs)
    rng = np.random.default_rng(2)
    dims = {"building": 6, "pv": 1, "storage": 1, "ev": 1}
    want = 0
    for _ in range(steps):
        act = {c: actions(rng, (n, d)) for c, d in dims.items()}
        want += sum(int(bad(a).any(1).sum()) for a in act.values())
        ta = {c: torch.tensor(a, device=DEV) for c, a in act.items()}
        fused.step(ta)
        generic.step(ta)
    assert want > 0 and count(fused) == want and count(generic) == want


@pytest.mark.parametrize("conv", ["opendss", "exact"])
@pytest.mark.parametrize("fused", [True, False])
def test_oob_c4_meta(fused, conv):
    """C4 (5 agents x [building, PV, storage]): the fused kernels and the generic
    path count the same warnings; meta["oob_actions"] is the running total."""
    from powergridworld_amd.scenarios.coordinated import CoordinatedMultiBuildingControlEnv, make_c4_config
    n, steps = 1024, 10
    env = CoordinatedMultiBuildingControlEnv(**make_c4_config(pf_convergence=conv), num_envs=n, device=DEV,
                                             fused=fused)
    assert (env._fused is not None) == fused
    env.reset()
    rng = np.random.default_rng(3)
    want = 0
    for _ in range(steps):
        act = {}
        for agent in env.agents:
            a = actions(rng, (n, 8))
            want += int(bad(a[:, :6]).any(1).sum() + bad(a[:, 6]).sum() + bad(a[:, 7]).sum())
            act[agent.name] = {"building": torch.tensor(a[:, :6], device=DEV),
                               "pv": torch.tensor(a[:, 6:7], device=DEV),
                               "storage": torch.tensor(a[:, 7:8], device=DEV)}
        _, _, _, meta = env.step(act)
    assert want > 0 and int(meta["oob_actions"].item()) == want == count(env)


def test_oob_hs_house():
    from powergridworld_amd.base_hs import HSMultiComponentEnv
    from powergridworld_amd.scenarios.heterogeneous_hs import make_env_config
    n, steps = 512, 20
    env = HSMultiComponentEnv(**make_env_config(), num_envs=n, device=DEV)
    env.reset()
    names = [e.name for e in env.envs]
    rng = np.random.default_rng(4)
    want = 0
    for _ in range(steps):
        a = actions(rng, (n, len(names)))
        want += int(bad(a).sum())
        env.step({nm: torch.tensor(a[:, i:i + 1], device=DEV) for i, nm in enumerate(names)})
    assert want > 0 and count(env) == want


def test_oob_warning_logged_at_a_later_reset(caplog):
    """The host learns the count without a synchronization: the copy started
    at one reset is read (and warned about) at the next."""
    from powergridworld_amd.agents import PVEnv
    env = PVEnv(profile_csv="pv_profile.csv", scaling_factor=40., num_envs=8, device=DEV)
    env.reset()
    env.step(torch.full((8, 1), 1.5, dtype=torch.float64, device=DEV))
    with caplog.at_level(logging.WARNING, logger="default"):
        env.reset()                    # starts the copy of 8
        torch.cuda.synchronize()
        env.reset()                    # reads it
    assert any("8 action(s)" in r.getMessage() for r in caplog.records)


@pytest.mark.parametrize("conv", ["opendss", "exact"])
def test_oob_heterogeneous_fused_and_generic(conv):
    """The heterogeneous scenario on the fused multi-agent step (pgw_ma_step) and
    on the generic path: one warning per (env, component, step) whose rescaled
    action is out of the box -- the building's six actions count once."""
    from powergridworld_amd.multiagent_env import MultiAgentEnv
    from powergridworld_amd.scenarios.heterogeneous import make_env_config
    n, steps = 2048, 20
    rng = np.random.default_rng(9)
    A = actions(rng, (steps, n, 10))
    want = 0
    for t in range(steps):
        want += int(bad(A[t, :, :6]).any(1).sum())                       # building
        want += sum(int(bad(A[t, :, j]).sum()) for j in range(6, 10))   # pv, storage, pv farm, EV
    got = []
    for fused in ("auto", False):
        env = MultiAgentEnv(**make_env_config(pf_convergence=conv), num_envs=n, device=DEV, fused=fused)
        assert (env._ma is not None) == (fused == "auto")
        env.reset()
        for t in range(steps):
            a = torch.tensor(A[t], device=DEV)
            env.step({"building": {"building": a[:, :6], "pv": a[:, 6:7], "storage": a[:, 7:8]},
                      "pv": a[:, 8:9], "ev-charging": a[:, 9:10]})
        got.append(count(env))
    assert got == [want, want], (got, want)
