"""fp32-storage variants (pgw_*_f32): state, actions and outputs
stored as fp32, arithmetic in fp64.  Needs an MI355X.

Two kinds of check:
* one-step parity (bit level): from the same fp32 state and fp32-representable
  actions, every fp32 output equals the fp64 path's output rounded to fp32
  (within 1 fp32 ulp where a second rounding is involved: the coordinated
  reward is RN32(RN32(r) - RN32(share)));
* a free-running episode against the fp64 path within the north-star fp32
  bound, 1e-3 relative (BASELINE.json north_star).
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
F32_ULP = 2.0 ** -23


def rn32(t):
    return t.to(torch.float32)


def assert_f32(got, want64, ulps=1, atol=0.0):
    """got (fp32) == RN32(want64) within `ulps` fp32 ulps."""
    assert got.dtype == torch.float32
    want = rn32(want64).double()
    g = got.double()
    tol = ulps * F32_ULP * want.abs() + atol
    bad = (g - want).abs() > tol
    assert not bad.any(), (int(bad.sum()), g[bad][:5].tolist(), want[bad][:5].tolist())


def test_battery_f32_one_step_and_episode():
    from powergridworld_amd.agents import EnergyStorageEnv
    n = 4096
    gen = torch.Generator(DEV).manual_seed(3)
    init = (torch.rand(n, dtype=torch.float64, device=DEV, generator=gen) * 60.0).float()
    e32 = EnergyStorageEnv(num_envs=n, device=DEV, dtype=torch.float32)
    e64 = EnergyStorageEnv(num_envs=n, device=DEV)
    free = EnergyStorageEnv(num_envs=n, device=DEV)
    o32 = e32.reset(init_storage=init)[0]
    o64 = e64.reset(init_storage=init.double())[0]
    free.reset(init_storage=init.double())
    assert o32.dtype == torch.float32 and e32.soc.dtype == torch.float32
    assert_f32(o32, o64, ulps=0)
    assert_f32(e32.soc, e64.soc, ulps=0)
    for t in range(300):
        a = (torch.rand((n, 1), dtype=torch.float64, device=DEV, generator=gen) * 2.6 - 1.3).float()
        e64.soc.copy_(e32.soc)                      # teacher forcing: same fp32 state
        o32, r32, d32, _ = e32.step(a)
        o64, _, d64, _ = e64.step(a.double())
        _, _, _, _ = free.step(a.double())
        assert_f32(o32, o64, ulps=0)
        assert_f32(e32.soc, e64.soc, ulps=0)
        assert_f32(e32.real_power, e64.real_power, ulps=0)
        assert d32 == d64
    # free-running fp64 vs fp32: SoC is continuous in the state (the clamps end at
    # the bounds), so it stays within the fp32 bound over the whole episode
    np.testing.assert_allclose(e32.soc.double().cpu().numpy(), free.soc.cpu().numpy(), rtol=1e-3, atol=1e-3)


def _c4_pair(n, seed, semantics):
    from powergridworld_amd.scenarios.coordinated import (CoordinatedMultiBuildingControlEnv,
                                                          make_c4_config)
    cfg = make_c4_config(pf_convergence=semantics)
    e32 = CoordinatedMultiBuildingControlEnv(**cfg, num_envs=n, device=DEV, dtype=torch.float32)
    e64 = CoordinatedMultiBuildingControlEnv(**cfg, num_envs=n, device=DEV, fused=True)
    assert e32._fused is not None and e32._fused["kernel"] == "pgw_coord_step_f32"
    # OpenDSS's rule: k_coord_pf_od<14, pgw_coord_buffers_f32>; the fixed point: k_coord_pf
    assert e32.pf_solver._od_fast == (semantics == "opendss") and not e32.pf_solver.general
    gen = torch.Generator(DEV).manual_seed(seed)
    init = (torch.rand((5, n), dtype=torch.float64, device=DEV, generator=gen) * 50.0).float().double()
    for e in (e32, e64):
        e.reset()
        for a, agent in enumerate(e.agents):
            agent.env_dict["storage"].reset(init_storage=init[a])
    e32.load_component_state()
    return e32, e64, gen


@pytest.mark.parametrize("semantics", ["opendss", "exact"])
def test_c4_f32_one_step_parity(semantics):
    """Teacher-forced: each step starts the fp64 fused env from the fp32 env's
    state; every fp32 output is the fp64 output rounded once.  Under OpenDSS's
    rule the power flow stops at an iteration count, which the fp32-rounded
    agent powers (the same values summed in fp64) can move by one for an env
    within ~1e-5 kW of a stopping threshold: such envs (their count differs from
    the fp64 path's, at most a 1e-4 fraction) are excluded from the PF / reward
    comparison of that step."""
    n = 8192
    e32, e64, gen = _c4_pair(n, 5, semantics)
    assert_f32(e32.packed_obs(), e64.packed_obs(), ulps=0)
    F32, F64 = e32._fused, e64._fused
    names = [a.name for a in e32.agents]
    flips = 0
    for t in range(40):
        F64["x"].copy_(F32["x"])
        F64["soc"].copy_(F32["soc"])
        act = (torch.rand((5, n, 8), dtype=torch.float64, device=DEV, generator=gen) * 2.2 - 1.1).float()
        _, r32, d32, m32 = e32.step(act)
        _, r64, d64, m64 = e64.step(act.double())
        assert_f32(e32.packed_obs(), e64.packed_obs(), ulps=0)
        assert_f32(F32["x"], F64["x"], ulps=0)
        assert_f32(F32["soc"], F64["soc"], ulps=0)
        assert_f32(F32["agent_power"], F64["agent_power"], ulps=0)
        # PF from the fp32-rounded agent powers (same values, summed in fp64)
        same = F32["iters"] == F64["iters"]
        flips += int((~same).sum())
        assert_f32(F32["v_out"][0][same], F64["v_out"][0][same], ulps=1)
        assert_f32(m32["voltage_violation"][same], m64["voltage_violation"][same], ulps=1, atol=1e-9)
        for nm in names:
            assert_f32(r32[nm][same], r64[nm][same], ulps=2, atol=1e-6)
        assert d32["__all__"] == d64["__all__"]
    assert flips <= 1e-4 * 40 * n, flips
    if semantics == "exact":
        assert flips == 0


@pytest.mark.parametrize("semantics", ["opendss", "exact"])
def test_c4_f32_episode_within_bound(semantics):
    """Free-running full episode (286 steps + the next reset) at batch 4096
    against the fp64 path: observations within 1e-3 relative (north star).
    The reward contains the reference's discontinuous battery clamp
    (energy_storage_env.py:117-126 omit the efficiency) via the agent power in
    the voltage penalty, so a state 1 fp32 ulp from a clamp threshold can take
    the other branch; rewards are held to the bound on all but a 1e-4 fraction."""
    n = 4096
    e32, e64, gen = _c4_pair(n, 9, semantics)
    names = [a.name for a in e32.agents]
    bad_r, tot_r = 0, 0
    steps = 0
    while True:
        act = (torch.rand((5, n, 8), dtype=torch.float64, device=DEV, generator=gen) * 2 - 1).float()
        _, r32, d32, _ = e32.step(act)
        _, r64, d64, _ = e64.step(act.double())
        steps += 1
        np.testing.assert_allclose(e32.packed_obs().double().cpu().numpy(),
                                   e64.packed_obs().cpu().numpy(), rtol=1e-3, atol=1e-3)
        for nm in names:
            g, w = r32[nm].double(), r64[nm]
            bad_r += int(((g - w).abs() > 1e-3 * w.abs() + 1e-3).sum())
            tot_r += n
        assert d32["__all__"] == d64["__all__"]
        if d64["__all__"]:
            break
    assert steps == 286
    assert bad_r <= 1e-4 * tot_r, (bad_r, tot_r)
    o32, o64 = e32.reset(), e64.reset()      # x_k persists across the reset
    for nm in names:
        for c in ("building", "pv"):         # (storage: each env draws its own initial SoC)
            np.testing.assert_allclose(o32[nm][c].double().cpu().numpy(), o64[nm][c].cpu().numpy(),
                                       rtol=1e-3, atol=1e-3)


def test_f32_refuses_non_standard_layout():
    from powergridworld_amd.scenarios.coordinated import (CoordinatedMultiBuildingControlEnv,
                                                          make_c4_config)
    from powergridworld_amd.agents import EnergyStorageEnv
    from powergridworld_amd.agents.pv import PVEnv
    with pytest.raises(ValueError):
        CoordinatedMultiBuildingControlEnv(**make_c4_config(), num_envs=8, device=DEV,
                                           dtype=torch.float32, fused=False)
    from powergridworld_amd.base import MultiComponentEnv
    # an fp32 MC agent runs pgw_mc_agent_step_f32: its components must all be fused kinds
    m = MultiComponentEnv(name="mc", components=make_c4_config()["agents"][0]["config"]["components"],
                          num_envs=8, device=DEV, dtype=torch.float32)
    assert m.dtype == torch.float32 and m._mc_fusable()

    class OwnStepPV(PVEnv):
        def step(self, *a, **k):
            return super().step(*a, **k)
    with pytest.raises(NotImplementedError):
        MultiComponentEnv(name="mc", components=[{"name": "pv", "cls": OwnStepPV,
                                                  "config": {"profile_csv": "pv_profile.csv"}}],
                          num_envs=8, device=DEV, dtype=torch.float32)
    assert PVEnv(profile_csv="pv_profile.csv", num_envs=8, device=DEV, dtype=torch.float32).dtype == torch.float32
    with pytest.raises(Exception):
        EnergyStorageEnv(num_envs=8, device=DEV, dtype=torch.float16)


def _c4_component(name):
    from powergridworld_amd.scenarios.coordinated import make_c4_config
    comps = make_c4_config()["agents"][0]["config"]["components"]
    c = [x for x in comps if x["name"] == name][0]
    return c["cls"], c["config"]


def test_pv_f32_one_step():
    """pgw_pv_*_f32: obs and real power = RN32 of the fp64 path's, every step."""
    cls, cfg = _c4_component("pv")
    n = 4096
    e32 = cls(**cfg, num_envs=n, device=DEV, dtype=torch.float32)
    e64 = cls(**cfg, num_envs=n, device=DEV)
    e32.reset()
    e64.reset()
    gen = torch.Generator(DEV).manual_seed(11)
    assert_f32(e32._obs, e64._obs, ulps=0)
    for t in range(200):
        a = (torch.rand((n, 1), dtype=torch.float64, device=DEV, generator=gen) * 2.4 - 1.2).float()
        o32, _, d32, _ = e32.step(a)
        o64, _, d64, _ = e64.step(a.double())
        assert o32.dtype == torch.float32
        assert_f32(o32, o64, ulps=0)
        assert_f32(e32.real_power, e64.real_power, ulps=0)
        assert d32 == d64


def test_building_f32_one_step_and_episode():
    """pgw_building_*_f32 (fp32 x_k, p_consumed, rewards, obs; fp64 arithmetic):
    from the same fp32 state (teacher forcing) every output is RN32 of the fp64
    path's; a free-running episode stays within the north-star fp32 bound."""
    cls, cfg = _c4_component("building")
    n = 2048
    e32 = cls(**cfg, num_envs=n, device=DEV, dtype=torch.float32)
    e64 = cls(**cfg, num_envs=n, device=DEV)
    free = cls(**cfg, num_envs=n, device=DEV)
    for e in (e32, e64, free):
        e.reset()
    assert e32.x.dtype == torch.float32
    gen = torch.Generator(DEV).manual_seed(12)
    for t in range(250):
        a = (torch.rand((n, 6), dtype=torch.float64, device=DEV, generator=gen) * 2.2 - 1.1).float()
        e64.x.copy_(e32.x)
        e64._reward_state.copy_(e32._reward_state)
        o32, r32, d32, _ = e32.step(a)
        o64, r64, d64, _ = e64.step(a.double())
        free.step(a.double())
        assert_f32(o32, o64, ulps=0)
        assert_f32(e32.x, e64.x, ulps=0)
        assert_f32(e32.p_consumed, e64.p_consumed, ulps=0)
        assert_f32(r32, r64, ulps=0)
        assert d32 == d64
    np.testing.assert_allclose(e32.x.double().cpu().numpy(), free.x.cpu().numpy(), rtol=1e-3, atol=1e-3)


@pytest.mark.parametrize("randomize", [False, True])
def test_ev_f32_one_step_and_episode(randomize):
    """pgw_ev_*_f32 (fp32 requirements, obs, real power, reward): from the same
    fp32 requirements every output is RN32 of the fp64 path's; a free-running
    episode stays within the fp32 bound."""
    from powergridworld_amd.agents.vehicles import EVChargingEnv
    cfg = dict(num_vehicles=100, minutes_per_step=5, max_charge_rate_kw=7., peak_threshold=250.,
               vehicle_multiplier=5., rescale_spaces=True, randomize=randomize)
    n = 2048
    envs = [EVChargingEnv(**cfg, num_envs=n, device=DEV, dtype=dt)
            for dt in (torch.float32, torch.float64, torch.float64)]
    for e in envs:
        if randomize:
            e.seed(5)
        e.reset()
    e32, e64, free = envs
    assert e32.req.dtype == torch.float32
    if not randomize:      # (reset = req0 stored, then the action-less step: two roundings)
        assert_f32(e32.req, e64.req, ulps=1)
    gen = torch.Generator(DEV).manual_seed(13)
    for t in range(280):
        a = (torch.rand((n, 1), dtype=torch.float64, device=DEV, generator=gen) * 2.2 - 1.1).float()
        e64.req.copy_(e32.req)
        e64.charging.copy_(e32.charging)
        o32, r32, d32, _ = e32.step(a)
        o64, r64, d64, _ = e64.step(a.double())
        free.step(a.double())
        assert_f32(o32, o64, ulps=0)
        assert_f32(r32, r64, ulps=0)
        assert_f32(e32.real_power, e64.real_power, ulps=0)
        assert_f32(e32.req, e64.req, ulps=0)
        assert d32 == d64
        if d32:
            break
    np.testing.assert_allclose(e32.req.double().cpu().numpy(), free.req.cpu().numpy(), rtol=1e-3, atol=1e-2)


def test_mc_f32_c3_one_step_and_episode():
    """pgw_mc_agent_step_f32 (the C3 agent: building + PV + storage + EV(100),
    fp32 state / obs / actions / powers / rewards, fp64 arithmetic): from the
    same fp32 state every component output is RN32 of the fp64 fused step's;
    the agent sums are formed from the stored fp32 component values (so within
    2^-23 (sum |terms| + |sum|)); a free-running episode stays within the
    north-star fp32 bound."""
    from powergridworld_amd import MultiComponentEnv
    from powergridworld_amd.agents import EnergyStorageEnv, EVChargingEnv, FiveZoneROMThermalEnergyEnv, PVEnv
    n = 16384
    comps = [
        {"name": "building", "cls": FiveZoneROMThermalEnergyEnv, "config": {}},
        {"name": "pv", "cls": PVEnv, "config": {"profile_csv": "pv_profile.csv", "scaling_factor": 40.}},
        {"name": "storage", "cls": EnergyStorageEnv, "config": {}},
        {"name": "ev", "cls": EVChargingEnv,
         "config": dict(num_vehicles=100, minutes_per_step=5, max_charge_rate_kw=7.,
                        peak_threshold=250., vehicle_multiplier=5., rescale_spaces=True)},
    ]
    m32 = MultiComponentEnv(name="mc", components=comps, num_envs=n, device=DEV, dtype=torch.float32)
    m64, free = [MultiComponentEnv(name="mc", components=comps, num_envs=n, device=DEV) for _ in range(2)]
    assert m32._mc_fusable() and all(e.dtype == torch.float32 for e in m32.envs)
    init = (torch.rand(n, dtype=torch.float64, device=DEV, generator=torch.Generator(DEV).manual_seed(11)) * 60)
    init = init.float().double()
    m32.reset(init_storage=init.float())
    for e in (m64, free):
        e.reset(init_storage=init)
    b32, s32, v32 = m32.env_dict["building"], m32.env_dict["storage"], m32.env_dict["ev"]
    b64, s64, v64 = m64.env_dict["building"], m64.env_dict["storage"], m64.env_dict["ev"]
    assert b32.x.dtype == s32.soc.dtype == v32.req.dtype == m32.real_power.dtype == torch.float32
    gen = torch.Generator(DEV).manual_seed(12)
    dims = {"building": 6, "pv": 1, "storage": 1, "ev": 1}
    for t in range(280):
        act = {c: (torch.rand((n, d), dtype=torch.float64, device=DEV, generator=gen) * 2.4 - 1.2).float()
               for c, d in dims.items()}
        b64.x.copy_(b32.x)
        b64._reward_state.copy_(b32._reward_state)
        s64.soc.copy_(s32.soc)
        v64.req.copy_(v32.req)
        v64.charging.copy_(v32.charging)
        o32, r32, d32, _ = m32.step(act)
        o64, r64, d64, _ = m64.step({c: a.double() for c, a in act.items()})
        free.step({c: a.double() for c, a in act.items()})
        for c in dims:
            assert_f32(o32[c], o64[c], ulps=0)
            assert_f32(m32.env_dict[c].real_power, m64.env_dict[c].real_power, ulps=0)
        # the sums add the stored (rounded) terms: each term and the sum are off
        # by <= half an fp32 ulp, so the bound is 2^-24 (sum |terms| + |sum|), x2
        big = torch.stack([m64.env_dict[c].real_power.abs() for c in dims]).sum(0)
        assert_f32(m32.real_power, m64.real_power, ulps=0, atol=F32_ULP * (big + m64.real_power.abs()))
        rbig = b64._reward_state.abs() + v64._reward.abs()
        assert_f32(r32, r64, ulps=0, atol=F32_ULP * (rbig + r64.abs()))
        assert d32 == d64
        if d32:
            break
    np.testing.assert_allclose(b32.x.double().cpu().numpy(), free.env_dict["building"].x.cpu().numpy(),
                               rtol=1e-3, atol=1e-3)
    np.testing.assert_allclose(s32.soc.double().cpu().numpy(), free.env_dict["storage"].soc.cpu().numpy(),
                               rtol=1e-3, atol=1e-2)
