"""Captured steps (powergridworld_amd/graph.py): a StepGraph replay is
bit-identical to the eager step it stands for, across an episode boundary, in
1- and multi-step graphs, mixed with eager steps, and for the EV's randomized
schedule and a grid-aware PV.  Needs an MI355X."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
N = 320                      # 5 blocks of 64 envs, the last one partial below


def mc_env(n=N, randomize=False, grid_aware=False):
    from powergridworld_amd import MultiComponentEnv
    from powergridworld_amd.agents import EnergyStorageEnv, EVChargingEnv, FiveZoneROMThermalEnergyEnv, PVEnv
    comps = [
        {"name": "building", "cls": FiveZoneROMThermalEnergyEnv, "config": {}},
        {"name": "pv", "cls": PVEnv, "config": {"profile_csv": "pv_profile.csv", "scaling_factor": 40.,
                                                "grid_aware": grid_aware}},
        {"name": "storage", "cls": EnergyStorageEnv, "config": {}},
        {"name": "ev", "cls": EVChargingEnv,
         "config": dict(num_vehicles=100, minutes_per_step=5, max_charge_rate_kw=7., peak_threshold=250.,
                        vehicle_multiplier=5., rescale_spaces=True, randomize=randomize)},
    ]
    env = MultiComponentEnv(name="mc", components=comps, num_envs=n, device=DEV)
    if randomize:
        env.envs[3].seed(7)
    return env


DIMS = {"building": 6, "pv": 1, "storage": 1, "ev": 1}


def actions(n, steps, seed):
    g = torch.Generator(DEV).manual_seed(seed)
    return [{c: torch.empty((n, d), dtype=torch.float64, device=DEV).uniform_(-1, 1, generator=g)
             for c, d in DIMS.items()} for _ in range(steps)]


def snap(env):
    """Every output and state buffer of the agent, as host arrays."""
    out = [env._reward, env._real_power]
    for e in env.envs:
        out.append(e._obs)
        out.append(e._real_power if e.mc_kind != 0 else e.p_consumed)
    b, s, v = env.envs[0], env.envs[2], env.envs[3]
    out += [b.x, b._reward_state, s.soc, v.req, v.charging, v._reward]
    return [t.detach().cpu().numpy().copy() for t in out]


def same(a, b, what):
    for i, (x, y) in enumerate(zip(a, b)):
        np.testing.assert_array_equal(x, y, err_msg="%s: buffer %d" % (what, i))


def reset(env, n=N):
    init = torch.linspace(5.0, 45.0, n, dtype=torch.float64, device=DEV)
    return env.reset(init_storage=init)


@pytest.mark.parametrize("randomize,clocked", [(False, True), (True, True), (False, False), (True, False)])
def test_mc_graph_step_matches_eager_across_reset(randomize, clocked):
    """One captured step replayed over 1.2 episodes (an episode is 287 steps
    after the reset) == the eager fused step, every buffer after every step;
    device-clocked, and captured per episode position."""
    ea, eb = mc_env(randomize=randomize), mc_env(randomize=randomize)
    acts = actions(N, 16, 1)
    reset(ea)
    reset(eb)
    buf = {c: torch.empty_like(t) for c, t in acts[0].items()}
    g = eb.capture_step(buf, clocked=clocked)
    assert g._clocked == clocked
    steps = 0
    for ep in range(2):
        for t in range(340 if ep == 0 else 60):
            a = acts[t % 16]
            for c in buf:
                buf[c].copy_(a[c])
            _, ra, da, ma = ea.step(a)
            _, rb, db, mb = g()
            assert da == db
            assert ma["pv"] == mb["pv"]
            steps += 1
            if t % 37 == 0 or da:
                same(snap(ea), snap(eb), "step %d" % steps)
            if da:
                break
        reset(ea)
        reset(eb)
    torch.cuda.synchronize()
    same(snap(ea), snap(eb), "end")
    assert eb._ep_step == ea._ep_step == 0
    if clocked:
        assert bool((eb._clock == eb._clock_k).all())      # (every block's clock, as the host records it)
    else:
        assert len(g._pos_graphs) >= 280


@pytest.mark.parametrize("clocked", [True, False])
def test_mc_graph_multi_step_and_mixed_with_eager(clocked):
    """A 4-step graph (four action buffer sets) and eager steps interleaved ==
    eager steps only (the host resets the device clocks after eager steps)."""
    ea, eb = mc_env(), mc_env()
    acts = actions(N, 4, 2)
    reset(ea)
    reset(eb)
    bufs = [{c: t.clone() for c, t in a.items()} for a in acts]
    g4 = eb.capture_step(bufs, steps=4, clocked=clocked)
    for r in range(10):
        for a in acts:
            ea.step(a)
        if r % 3 == 1:
            for a in acts:
                eb.step(a)
        else:
            _, _, done, _ = g4()
            assert not done
        same(snap(ea), snap(eb), "round %d" % r)
    assert eb._ep_step == 40
    if clocked:
        assert bool((eb._clock == 40).all())


def test_mc_graph_grid_aware_pv_reads_the_static_voltage():
    ea, eb = mc_env(grid_aware=True), mc_env(grid_aware=True)
    acts = actions(N, 1, 3)
    vmin = torch.full((N,), 1.0, dtype=torch.float64, device=DEV)
    gen = torch.Generator(DEV).manual_seed(4)
    for e in (ea, eb):
        e.reset(init_storage=torch.linspace(5.0, 45.0, N, dtype=torch.float64, device=DEV), min_voltage=vmin)
    g = eb.capture_step(acts[0], min_voltage=vmin)
    for t in range(20):
        vmin.uniform_(0.92, 1.06, generator=gen)
        ea.step(acts[0], min_voltage=vmin)
        g()
        same(snap(ea), snap(eb), "step %d" % t)


def test_mc_graph_refuses_past_the_tables_and_copies():
    env = mc_env(n=64)
    reset(env, 64)
    a = actions(64, 1, 5)[0]
    with pytest.raises(ValueError):
        env.capture_step({**a, "pv": a["pv"].float()})
    g = env.capture_step(a)
    env._ep_step = g._n_dyn            # (as if stepped to the tables' end)
    with pytest.raises(IndexError):
        g()


def test_battery_graph_matches_eager():
    from powergridworld_amd.agents import EnergyStorageEnv
    n = 4096 + 17
    ea, eb = EnergyStorageEnv(num_envs=n, device=DEV), EnergyStorageEnv(num_envs=n, device=DEV)
    init = torch.linspace(3.0, 50.0, n, dtype=torch.float64, device=DEV)
    ea.reset(init_storage=init)
    eb.reset(init_storage=init)
    gen = torch.Generator(DEV).manual_seed(6)
    acts = [torch.empty((n, 1), dtype=torch.float64, device=DEV).uniform_(-1, 1, generator=gen) for _ in range(8)]
    bufs, one = [a.clone() for a in acts], acts[0].clone()
    g1, g8 = eb.capture_step(one), eb.capture_step(bufs, steps=8)
    for r in range(40):
        da = False
        for a in acts:
            da = ea.step(a)[2] or da       # (a graph call reports any of its steps' ends)
        if r % 2:
            _, _, db, _ = g8()
        else:
            db = False
            for a in acts:
                one.copy_(a)
                db = g1()[2] or db
        assert da == db
        assert ea.simulation_step == eb.simulation_step
        np.testing.assert_array_equal(ea.soc.cpu().numpy(), eb.soc.cpu().numpy())
        np.testing.assert_array_equal(ea._obs.cpu().numpy(), eb._obs.cpu().numpy())
        np.testing.assert_array_equal(ea._real_power.cpu().numpy(), eb._real_power.cpu().numpy())


def test_mc_graph_state_dict_round_trip():
    """state_dict() after captured steps, loaded into a fresh env that then
    captures its own graph: both continue bit-identically."""
    ea, eb = mc_env(), mc_env()
    acts = actions(N, 4, 11)
    reset(ea)
    buf = {c: t.clone() for c, t in acts[0].items()}
    ga = ea.capture_step(buf)
    for t in range(30):
        for c in buf:
            buf[c].copy_(acts[t % 4][c])
        ga()
    sd = ea.state_dict()
    reset(eb)
    eb.load_state_dict(sd)
    bufb = {c: t.clone() for c, t in acts[0].items()}
    gb = eb.capture_step(bufb)
    for t in range(30, 60):
        for c in buf:
            buf[c].copy_(acts[t % 4][c])
            bufb[c].copy_(acts[t % 4][c])
        _, _, da, _ = ga()
        _, _, db, _ = gb()
        assert da == db
    same(snap(ea), snap(eb), "after the round trip")
    assert ea._ep_step == eb._ep_step == 60


def hs_env(n):
    from powergridworld_amd.base_hs import HSMultiComponentEnv
    from powergridworld_amd.scenarios.heterogeneous_hs import make_env_config
    return HSMultiComponentEnv(**make_env_config(), num_envs=n, device=DEV)


@pytest.mark.parametrize("steps", [1, 4])
def test_hs_graph_matches_eager_across_reset(steps):
    """The Home-Steward house captured per episode position (1- and 4-step
    graphs) == its eager step, every output and state buffer, over more than
    an episode and a reset, mixed with eager steps."""
    n = 200
    ea, eb = hs_env(n), hs_env(n)
    gen = torch.Generator(DEV).manual_seed(12)
    acts = [torch.empty((n, len(ea.envs)), dtype=torch.float64, device=DEV).uniform_(-1, 1, generator=gen)
            for _ in range(steps)]
    init = torch.linspace(0.2, 0.9, n, dtype=torch.float64, device=DEV)
    for e in (ea, eb):
        e.reset(init_storage=init)
    g = eb.capture_step(acts if steps > 1 else acts[0], steps=steps)

    def state(e):
        return [t.detach().cpu().numpy().copy() for t in
                (e._obs_buf, e._reward, e._real_power, e._meta, e._ev_req, e._ev_chg, e._ev_cost, e._dev_cost,
                 e._es_last, e._pv_last)]

    total = 0
    for ep in range(2):
        calls = 0
        while True:
            da = False
            for a in acts:
                da = ea.step(a)[2] or da
            if calls % 5 == 3:
                db = False
                for a in acts:
                    db = eb.step(a)[2] or db
            else:
                db = g()[2]
            assert da == db
            calls += 1
            total += steps
            if calls % 17 == 0 or da:
                same(state(ea), state(eb), "ep %d call %d" % (ep, calls))
            if da or eb._hs_step_k() + steps > g._n_dyn:
                break
        for e in (ea, eb):
            e.reset(init_storage=init)
    assert len(g._pos_graphs) > 1


@pytest.mark.parametrize("conv", ["opendss", "exact"])
def test_c4_graph8_equals_eager_across_episodes(conv):
    """The fused C4 step captured 8 steps per graph (MultiAgentEnv.capture_step,
    graph.CoordStepGraph; one graph per episode position, actions bound per
    position from a pool) against the eager step over two whole episodes and
    the resets between them: every output bit for bit at every call; the
    episode's tail (fewer than 8 steps left) runs eagerly, a call past the
    last step is refused before launching."""
    from powergridworld_amd.scenarios.coordinated import CoordinatedMultiBuildingControlEnv, make_c4_config
    n, P, S = 2048, 16, 8
    g = torch.Generator(DEV).manual_seed(21)
    pool = torch.rand((P, 5, 8, n), dtype=torch.float64, device=DEV, generator=g) * 2.2 - 1.1
    packed = pool.transpose(2, 3)
    eager, cap = [CoordinatedMultiBuildingControlEnv(**make_c4_config(pf_convergence=conv), num_envs=n,
                                                     device=DEV, fused=True) for _ in range(2)]
    graph = cap.capture_step(lambda k: [packed[(k + i) % P] for i in range(S)], steps=S)

    def snap(env, r, d):
        return [env.packed_obs().clone(), torch.stack([r[a.name] for a in env.agents]).clone(),
                env.pf_solver.get_bus_voltage_by_name("675c").clone(), env.pf_solver.iterations.clone(),
                torch.tensor(float(d["__all__"]))]
    rng = np.random.default_rng(5)
    for ep in range(2):
        init = torch.tensor(rng.uniform(5.0, 45.0, size=(5, n)), device=DEV)
        for env in (eager, cap):                   # the same random initial SoC in both
            env.reset()
            for ai, agent in enumerate(env.agents):
                agent.env_dict["storage"].reset(init_storage=init[ai])
            env.load_component_state()
        last = cap._episode_last_step()
        assert last is not None and last > S
        k = 0
        while k < last:
            if k + S <= last:
                _, r2, d2, _ = graph()
                for i in range(S):
                    _, r1, d1, _ = eager.step(packed[(k + i) % P])
                k += S
            else:
                with pytest.raises(IndexError):
                    graph()
                _, r2, d2, _ = cap.step(packed[k % P])
                _, r1, d1, _ = eager.step(packed[k % P])
                k += 1
            for i, (x, y) in enumerate(zip(snap(eager, r1, d1), snap(cap, r2, d2))):
                assert torch.equal(x, y), "episode %d step %d output %d" % (ep, k, i)
        assert d1["__all__"] and d2["__all__"] and eager.episode_step == cap.episode_step == last
    assert len(graph._pos) >= (last // S)
